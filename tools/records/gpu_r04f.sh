# GPU box, round 4: window tests, then A/B of tile shapes (tools/_abt) and the cell list, kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -x -q --timeout 240 --timeout-method thread > $O/pytest_window.log 2>&1 || { tail -40 $O/pytest_window.log; exit 1; }
tail -1 $O/pytest_window.log
for rep in 1 2; do
  for rows in 1024 128; do
    timeout -k 10 120 python tools/ab_window.py . cells 0.145 $rows >> $O/ab.txt || exit 2
    for t in . tools/_abt/r8 tools/_abt/r2 tools/_abt/untiled; do
      timeout -k 10 120 python tools/ab_window.py $t window 0.145 $rows >> $O/ab.txt || exit 3
    done
  done
done
cat $O/ab.txt
for t in . tools/_abt/r8; do
  n=$(basename $t); [ "$n" = "." ] && n=main
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$n -o run -- python3 tools/ab_window.py $t window > $O/trace_$n.log 2>&1 || exit 4
done
python3 - <<'PY'
import csv, glob, re
def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^<>()]*>)?)", n)
    return m.group(1) if m else n[:40]
for f in sorted(glob.glob("gpurun_out/r04f/trace_*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if short(r["Name"]).startswith("k_"):
            print(f.split("/")[2], short(r["Name"]), r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
echo R04F_OK
