# GPU box: kernel-trace stats + separate PMC passes for the cfg4 bench in both barrier modes
set -o pipefail
export TMPDIR=/tmp
PROF_OUT=gpurun_out/prof_hocbf BENCH_EXTRA="--barrier euclidean_hocbf" bash tools/profile.sh || exit 1
PROF_OUT=gpurun_out/prof bash tools/profile.sh || exit 2
echo all-profiles-done
