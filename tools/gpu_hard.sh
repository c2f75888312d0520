# GPU box: parity suite, a lattice-step A/B of the variant set $SET (tools/ablate.py), cfg4 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
ABLATE_SET=${SET:-hardinline} timeout -k 10 300 python tools/ablate.py run --rounds 5 --iters 20 > gpurun_out/ablate_hard.json 2> gpurun_out/ablate_hard.err || { tail gpurun_out/ablate_hard.err; exit 2; }
cat gpurun_out/ablate_hard.json; grep -v amdgpu.ids gpurun_out/ablate_hard.err
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail gpurun_out/bench_cfg4.err; exit 3; }
cat gpurun_out/bench_cfg4.json
