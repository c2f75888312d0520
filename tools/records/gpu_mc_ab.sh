# A/B of the cfg5 Monte-Carlo bench (bench.py --config cfg5) for the working tree and variant trees
# (tools/_ab/<name> with their own bench.py), twice, interleaved.
set -u
cd /root/repo
O=gpurun_out/mcab; mkdir -p $O; : > $O/ab.txt
for rep in 1 2; do
for t in . "$@"; do
  (cd $t && timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 > /tmp/mc.json 2>/dev/null) || exit 2
  python -c "import json; d=json.load(open('/tmp/mc.json')); print('$t', round(d['ms_per_step'], 3), 'ms/step', '%.3g' % d['value'])" >> $O/ab.txt
done
done
cat $O/ab.txt
