# GPU box: the stats-off timed region (bench) and its tests: the new GPU tests, the bench at the
# driver's arguments, the sharded bench at one rank, and a 2-rank gloo rehearsal.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/statsoff; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "stats_off or replay or run_matches" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 3; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 4; }
timeout -k 10 300 python bench.py --shard --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_shard.json 2> $O/bench_shard.err || { tail -20 $O/bench_shard.err; exit 5; }
for f in bench_driver bench_default bench_shard; do
  python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], round(d['ms_per_step']*1e3, 2), round((d.get('ms_per_step_with_stats') or 0)*1e3, 2), (d.get('roofline') or {}).get('frac'), d['safety']['max_violation_optimal'], d['safety']['solves'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --backend gloo --steps 20 --warmup 4 --rows 256 --no-cpu-baseline > $O/rehearse_2.json 2> $O/rehearse_2.err || { tail -20 $O/rehearse_2.err; exit 6; }
cut -c1-400 $O/rehearse_2.json
echo STATSOFF_OK
