# GPU box: sharded-path parity tests + per-step cost of the sharded path at one rank (k sub-steps per exchange)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -2 gpurun_out/shard_tests.log
for k in 1 4 8; do
  timeout -k 10 200 python bench.py --shard --substeps $k --no-cpu-baseline > gpurun_out/bench_shard_k$k.json 2> gpurun_out/bench_shard_k$k.err || { tail gpurun_out/bench_shard_k$k.err; exit 2; }
  cat gpurun_out/bench_shard_k$k.json
done
timeout -k 10 200 python bench.py --shard --substeps 4 --eager --no-cpu-baseline > gpurun_out/bench_shard_k4e.json 2> gpurun_out/bench_shard_k4e.err || { tail gpurun_out/bench_shard_k4e.err; exit 3; }
cat gpurun_out/bench_shard_k4e.json
