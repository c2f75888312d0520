set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/ablate.py run > gpurun_out/ablate.json 2> gpurun_out/ablate.err || exit 1
timeout -k 10 200 python bench.py --config cfg3 --steps 20 --warmup 3 > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || exit 2
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || exit 3
cat gpurun_out/ablate.json gpurun_out/bench_cfg3.json gpurun_out/bench_cfg5.json
