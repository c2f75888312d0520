# GPU box: kernel-trace stats of the sharded path at one rank
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_shard
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 bench.py --shard --steps 96 --warmup 10 --no-cpu-baseline --kernel-iters 5 > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_shard/run_kernel_stats.csv")):
    print(f'{r["Name"][:70]:70s} {r["Calls"]:>6s} {float(r["AverageNs"])/1e3:9.2f} us')
PY
