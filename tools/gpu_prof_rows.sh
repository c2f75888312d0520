# Kernel traces of tools/ab_window.py at a given lattice height (window cull, placement auto) for
# each tree given.  Usage: bash tools/gpu_prof_rows.sh <out-name> <rows> <tree>...
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
i=0
for t in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/r$i -o run -- python3 tools/ab_window.py $t window 0.145 $R > $O/r$i.log 2>&1 || { tail -5 $O/r$i.log; exit 1; }
  f=$(find $O/r$i -name "*kernel_stats.csv" | head -1)
  echo "== $t"; grep "run(10)" $O/r$i.log; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'window' in n or 'hard' in n:
        print(f\"{n.split('(')[0][-50:]:50s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:7.2f} us\")
"
done
