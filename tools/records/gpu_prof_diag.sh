# GPU box: hard-QP queue statistics, then the rocprofv3 recipe (kernel trace + PMC passes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag_hard.py > gpurun_out/diag_hard.log 2>&1 || { tail gpurun_out/diag_hard.log; exit 1; }
cat gpurun_out/diag_hard.log
bash tools/profile.sh || exit 2
