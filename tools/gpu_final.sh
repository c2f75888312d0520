# GPU box: round-end rehearsal of the driver's steps: the GPU test suite, smoke(), the bench at the
# driver's arguments and at the defaults, the sharded bench at one rank, and the N>1 bench path
# with 2 and 3 ranks on one GPU (gloo).  Each step has its own time limit; the first failure ends it.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 3; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 4; }
timeout -k 10 300 python bench.py --shard --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_shard.json 2> $O/bench_shard.err || { tail -20 $O/bench_shard.err; exit 5; }
for f in bench_driver bench_default bench_shard; do
  python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], round(d['ms_per_step']*1e3, 2), (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
done
bash tools/gpu_rehearse.sh > $O/rehearse.log 2>&1 || { tail -20 $O/rehearse.log; exit 6; }
tail -2 $O/rehearse.log | cut -c1-300
echo FINAL_OK
