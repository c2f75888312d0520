# run(10) per-timestep time and kernel traces of tools/ab_window.py under the cell-list cull for
# each tree given (cfg4 spacing).  Usage: bash tools/gpu_ab_cells.sh <out-name> <tree>...
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for t in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/c$i -o run -- python3 tools/ab_window.py $t cells 0.145 > $O/c$i.log 2>&1 || { tail -5 $O/c$i.log; exit 1; }
  f=$(find $O/c$i -name "*kernel_stats.csv" | head -1)
  echo "== $t"; grep "run(10)" $O/c$i.log; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'lattice' in n or 'hard' in n or 'scatter' in n or 'scan' in n:
        print(f\"{n.split('(')[0][-50:]:50s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:7.2f} us\")
"
done
