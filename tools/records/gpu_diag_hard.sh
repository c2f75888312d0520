# GPU box: hard-QP queue size over a run + per-launch kernel trace of the same run
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 200 python3 -u tools/diag_hard.py > gpurun_out/diag/hard.log 2>&1 || { tail -20 gpurun_out/diag/hard.log; exit 1; }
cat gpurun_out/diag/hard.log
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/diag/trace -o run -- python3 tools/diag_hard.py > gpurun_out/diag/trace.log 2>&1 || exit 2
echo diag-done
