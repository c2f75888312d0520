# GPU box: sharded-path overhead at one rank (graph vs eager) + the sharded GPU parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -2 gpurun_out/shard_tests.log
timeout -k 10 200 python bench.py --shard --no-cpu-baseline > gpurun_out/bench_shard.json 2> gpurun_out/bench_shard.err || { tail gpurun_out/bench_shard.err; exit 2; }
cat gpurun_out/bench_shard.json
timeout -k 10 200 python bench.py --shard --eager --no-cpu-baseline > gpurun_out/bench_shard_eager.json 2> gpurun_out/bench_shard_eager.err || { tail gpurun_out/bench_shard_eager.err; exit 3; }
cat gpurun_out/bench_shard_eager.json
