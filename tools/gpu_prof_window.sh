# Kernel traces (rocprofv3 --kernel-trace --stats) of tools/ab_window.py for each tree given, at
# cfg4 spacing: per-kernel average durations of the window-cull step, one summary per tree.
# Usage: bash tools/gpu_prof_window.sh <out-name> <tree>...
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for t in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/p$i -o run -- python3 tools/ab_window.py $t window 0.145 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name "*kernel_stats.csv" | head -1)
  echo "== $t"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'window' in n or 'hard' in n or 'rowscan' in n:
        print(f\"{n.split('(')[0][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:7.2f} us\")
"
done
