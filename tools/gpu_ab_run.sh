# run(10) per-timestep times of tools/ab_window.py (no profiler) for each tree given, at cfg4 and
# cfg4f spacing, both culls, interleaved twice.  Usage: bash tools/gpu_ab_run.sh <tree>...
set -u
cd /root/repo
for rep in 1 2; do
  for sp in 0.145 0.2; do
    for t in "$@"; do
      timeout -k 10 120 python3 tools/ab_window.py $t window $sp || exit 1
    done
  done
done
