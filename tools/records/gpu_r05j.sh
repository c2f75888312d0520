# GPU box: nominal controls formed in the window tile (no per-agent u0 from the build): the window
# parity tests, then the driver's bench line and the run(10) timing for the A/B trees.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_window.log 2>&1 || { tail -30 $O/pytest_window.log; exit 1; }
tail -1 $O/pytest_window.log
for rep in 1 2; do
  for t in tools/_abt/base tools/_abt/nomtile; do
    timeout -k 10 300 python3 $t/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/b.json')); print('$t', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), round(d['roofline']['kernel_ms']*1e3, 2), d.get('end_state_sha256', '')[:16])"
  done
done
bash tools/gpu_ab_run.sh tools/_abt/base tools/_abt/nomtile
