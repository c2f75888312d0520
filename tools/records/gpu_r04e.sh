# GPU box, round 4: window build without the prep ticket; PMC comparison of the window and the
# cell-list filters (tools/ab_window.py runs under rocprofv3: trace, SQ counters, TA/TD busy).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -x -q --timeout 240 --timeout-method thread > $O/pytest_window.log 2>&1 || { tail -40 $O/pytest_window.log; exit 1; }
tail -1 $O/pytest_window.log
for rows in 1024 128; do
  for c in cells window; do
    timeout -k 10 120 python tools/ab_window.py . $c 0.145 $rows >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
for c in window cells; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$c/trace -o run -- python3 tools/ab_window.py . $c > $O/$c.trace.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -f csv -d $O/$c/pmc_sq -o run -- python3 tools/ab_window.py . $c > $O/$c.sq.log 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY TA_BUSY_avr TD_BUSY_avr -f csv -d $O/$c/pmc_ta -o run -- python3 tools/ab_window.py . $c > $O/$c.ta.log 2>&1 || exit 5
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/$c/pmc_fetch -o run -- python3 tools/ab_window.py . $c > $O/$c.fetch.log 2>&1 || exit 6
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/$c/pmc_write -o run -- python3 tools/ab_window.py . $c > $O/$c.write.log 2>&1 || exit 7
done
python3 - <<'PY'
import csv, collections, glob
for c in ("window", "cells"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/r04e/{c}/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "filter" not in n and "tile" not in n and "prep" not in n and "scan" not in n:
                continue
            k = n[n.find("k_"):n.find("(")] if "k_" in n else n[:40]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, e in agg.items():
        print(c, k, {cn: round(sum(v) / len(v), 1) for cn, v in sorted(e.items())})
    for r in csv.DictReader(open(glob.glob(f"gpurun_out/r04e/{c}/trace/run_kernel_stats.csv")[0])):
        if any(t in r["Name"] for t in ("filter", "tile", "prep", "scan", "bin")):
            print(c, r["Name"][r["Name"].find("k_"):r["Name"].find("(")], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
echo R04E_OK
