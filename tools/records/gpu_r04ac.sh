# GPU box, round 4: sharded stripes of >= 256 rows take the window cull: the bench GPU tests, then
# full-size gloo rehearsals at 2 and 4 ranks (512 / 256 rows per rank, window cull) that must end in
# the 1-rank state of the driver's command (sha256 3f7acf0a...).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py tests/test_shard_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 2 4; do
  timeout -k 10 900 python bench.py --gpus $n --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/gloo$n.json 2> $O/gloo$n.err || { tail -20 $O/gloo$n.err; exit 2; }
  python -c "import json; d=json.load(open('$O/gloo$n.json')); print('gloo$n', d['config'].get('cull'), d['n_gpus'], '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
done
echo R04AC_OK
