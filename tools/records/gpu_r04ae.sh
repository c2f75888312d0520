# GPU box, round 4: the window cull's row guard as a runtime choice (in the filter launch, or a
# separate kernel for ranks time-sharing a GPU): window, shard and bench tests, then the 2- and
# 4-rank gloo rehearsals at full size (ranks share this GPU: separate guard), which must end in the
# 1-rank state.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_window.py tests/test_shard_gpu.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 2 4; do
  timeout -k 10 900 python bench.py --gpus $n --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/gloo$n.json 2> $O/gloo$n.err || { tail -20 $O/gloo$n.err; exit 2; }
  python -c "import json; d=json.load(open('$O/gloo$n.json')); print('gloo$n', d['config'].get('cull'), d['n_gpus'], '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
done
timeout -k 10 400 python bench.py --shard --steps 48 --warmup 8 --no-cpu-baseline > $O/shard1.json 2> $O/shard1.err || { tail -20 $O/shard1.err; exit 3; }
python -c "import json; d=json.load(open('$O/shard1.json')); print('shard1', d['config'].get('cull'), d['n_gpus'], '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
echo R04AE_OK
