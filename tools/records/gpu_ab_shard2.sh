# GPU box: sharded-path A/B (one rank, RCCL) of the working tree against tools/_ab/base, after the
# shard GPU tests; then a kernel trace of the sharded bench (tools/gpu_prof_shard.sh).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/abs; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_gpu_bench.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/base; do
    timeout -k 10 200 python $t/bench.py --shard --no-cpu-baseline --kernel-iters 2 > $O/b.json 2>/dev/null || exit 2
    python -c "import json; d=json.load(open('$O/b.json')); print('$t', round(d['ms_per_step']*1e3, 2), 'us/step')" >> $O/ab.txt
  done
done
cat $O/ab.txt
bash tools/gpu_prof_shard.sh
