# A/B of the sharded path at one rank (bench.py --shard) for the working tree and variant trees
# (tools/_ab/<name>, built on the CPU), twice, interleaved.
set -u
cd /root/repo
O=gpurun_out/shab; mkdir -p $O; : > $O/ab.txt
for rep in 1 2; do
for t in . "$@"; do
  (cd $t && timeout -k 10 300 python bench.py --shard --no-cpu-baseline --steps 100 --warmup 8 --kernel-iters 2 > /tmp/sb.json 2>/dev/null) || exit 2
  python -c "import json; d=json.load(open('/tmp/sb.json')); print('$t', round(d['ms_per_step']*1e3, 1), 'us/step')" >> $O/ab.txt
done
done
cat $O/ab.txt
