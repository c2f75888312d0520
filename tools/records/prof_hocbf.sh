# GPU box: stall breakdown of the HOCBF lattice filter (separate PMC passes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/profh
mkdir -p $OUT
B="python3 bench.py --barrier euclidean_hocbf --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES -f csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH -f csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || exit 3
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(list)
for sub in ("p1", "p2"):
    for r in csv.DictReader(open(f"gpurun_out/profh/{sub}/run_counter_collection.csv")):
        if "hocbf" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):.4g}")
for r in csv.DictReader(open("gpurun_out/profh/trace/run_kernel_stats.csv")):
    print(f'{r["Name"][:60]:60s} {float(r["AverageNs"])/1e3:9.2f} us')
PY
