# GPU box: parity suite, HOCBF certificate A/B (lattice step in HOCBF mode), HOCBF cfg4 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
ABLATE_HOCBF=1 ABLATE_SET=${SET:-hcert} timeout -k 10 300 python tools/ablate.py run --rounds 4 --iters 10 > gpurun_out/ablate_hcert.json 2> gpurun_out/ablate_hcert.err || { tail gpurun_out/ablate_hcert.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/ablate_hcert.json')); print({k: (round(v['build']['median_us'],1), round(v['advance']['median_us'],1), v.get('bit_identical_to_reg')) for k, v in d.items()})"
timeout -k 10 300 python bench.py --barrier euclidean_hocbf --no-cpu-baseline --steps 100 > gpurun_out/bench_cfg4_hocbf.json 2> gpurun_out/bench_hocbf.err || { tail gpurun_out/bench_hocbf.err; exit 3; }
cat gpurun_out/bench_cfg4_hocbf.json
