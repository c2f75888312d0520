# GPU box: A/B trees given, driver bench line (steps 20, warm-up 5) twice each, interleaved.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
for rep in 1 2; do
  for t in "$@"; do
    timeout -k 10 300 python3 $t/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/b.json')); w=d.get('window_cull') or {}; print('$t', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), round(d['roofline']['kernel_ms']*1e3, 2), d.get('end_state_sha256', '')[:16], {k: v for k, v in w.items() if 'walk' in k or 'stall' in k})"
  done
done
