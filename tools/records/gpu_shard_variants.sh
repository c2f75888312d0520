# GPU box: sharded bench (one rank) per tree + the scatter / bin kernel averages from a kernel trace.
# usage: bash tools/gpu_shard_variants.sh <tree> ...   ("." = the working tree)
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/shv; mkdir -p $O; : > $O/res.txt
for rep in 1 2; do
  for t in "$@"; do
    timeout -k 10 200 python $t/bench.py --shard --no-cpu-baseline --kernel-iters 2 > $O/b.json 2>/dev/null || exit 2
    python -c "import json; d=json.load(open('$O/b.json')); print('$t', round(d['ms_per_step']*1e3, 2), 'us/step')" >> $O/res.txt
  done
done
for t in "$@"; do
  D=$O/prof_$(basename $t)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $D -o run -- python3 $t/bench.py --shard --steps 96 --warmup 10 --no-cpu-baseline --kernel-iters 2 > $D.log 2>&1 || exit 3
  python3 -c "
import csv
for r in csv.DictReader(open('$D/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('scatter_ordered', 'nominal_bin', 'halo_pack', 'lattice_filter')):
        print('$t', r['Name'][:45], round(float(r['AverageNs'])/1e3, 2))" >> $O/res.txt
done
cat $O/res.txt
