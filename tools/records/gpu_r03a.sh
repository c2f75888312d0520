# GPU box, round 3 first pass: the changed GPU tests, then the bench at the driver's arguments, the
# sharded bench at one rank (1M agents, and a 1/8 stripe), graph vs eager, and --gpus 2 (gloo).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bench.py tests/test_shard_gpu.py tests/test_gpu_torch_ops.py "tests/test_gpu_parity.py::test_lattice_run_output_history" "tests/test_gpu_parity.py::test_lattice_run_matches_steps" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 3; }
for R in 1024 128; do
  for E in "" "--eager"; do
    timeout -k 10 300 python bench.py --shard --rows $R --no-cpu-baseline --steps 48 --warmup 8 $E > $O/shard_${R}${E}.json 2> $O/shard_${R}${E}.err || { tail -20 $O/shard_${R}${E}.err; exit 4; }
  done
done
timeout -k 10 300 python bench.py --rows 128 --no-cpu-baseline --steps 48 --warmup 8 > $O/single_128.json 2> $O/single_128.err || { tail -20 $O/single_128.err; exit 5; }
for f in $O/*.json; do
  python -c "import json,sys; d=json.load(open('$f')); print('$f', '%.3e'%d['value'], round(d['ms_per_step']*1e3, 2), d.get('ms_per_step_outputs_every_step'), (d.get('roofline') or {}).get('frac'), d['config'].get('parallelism'))"
done
echo R03A_OK
