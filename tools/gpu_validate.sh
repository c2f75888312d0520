# GPU box: re-validate the current tree -- parity suite + smoke, cfg4 bench in both barrier modes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail gpurun_out/bench_cfg4.err; exit 3; }
cat gpurun_out/bench_cfg4.json
timeout -k 10 300 python bench.py --barrier euclidean_hocbf --no-cpu-baseline --steps 100 > gpurun_out/bench_cfg4_hocbf.json 2> gpurun_out/bench_hocbf.err || { tail gpurun_out/bench_hocbf.err; exit 4; }
cat gpurun_out/bench_cfg4_hocbf.json
