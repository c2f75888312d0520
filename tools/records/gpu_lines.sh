# GPU box: the committed bench lines (cfg4 with the CPU baseline, cfg4f, cfg4r, cfg4 HOCBF, cfg3)
set -u
cd /root/repo
O=gpurun_out/lines; mkdir -p $O
for c in "cfg4:--cpu-budget 5" "cfg4f:--no-cpu-baseline" "cfg4r:--no-cpu-baseline" "cfg4_hocbf:--barrier euclidean_hocbf --no-cpu-baseline" "cfg3:--no-cpu-baseline"; do
  n=${c%%:*}; a=${c#*:}; cfg=${n%_hocbf}
  timeout -k 10 400 python bench.py --config $cfg $a > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 3; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], round(d['ms_per_step']*1e3, 2), (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('traffic'))"
done
