# PMC passes (each counter set its own run, kernel trace only) of tools/ab_window.py on one tree at
# cfg4 spacing, plus the counter list of the box.  Usage: bash tools/gpu_pmc_window.sh <out> <tree>
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; T=$2; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for S in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $S -f csv -d $O/pmc$i -o run -- python3 tools/ab_window.py $T window 0.145 > $O/pmc$i.log 2>&1 || echo "pass $i failed"
done
python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob("$O/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "window" not in k and "hard" not in k: continue
    print("==", k)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {v / max(1, n[(k, c)]):.4g} per dispatch (summed over the dispatch's records)")
PY
