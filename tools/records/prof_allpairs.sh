# GPU box: stall breakdown of the cfg3 split all-pairs kernels (separate PMC passes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/profap
mkdir -p $OUT
B="python3 bench.py --config cfg3 --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT -f csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || exit 3
python3 - <<'PY'
import csv, collections, re
for p in ("p1", "p2"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/profap/{p}/run_counter_collection.csv")):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        if m and "allpairs" in m.group(1):
            agg[(m.group(1), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(p, k, c, sum(v) / len(v))
PY
grep -E "allpairs|ap_stage" $OUT/trace/run_kernel_stats.csv | cut -c1-60,200-400
