# GPU box: parity suite, then all-pairs screen variants (ABLATE_SET=allpairs) at the cfg3 size
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
ABLATE_SET=allpairs timeout -k 10 300 python tools/ablate.py run_allpairs --W 256 --H 256 --rounds 4 --iters 5 > gpurun_out/ablate_ap.json 2> gpurun_out/ablate_ap.err || { tail gpurun_out/ablate_ap.err; exit 2; }
cat gpurun_out/ablate_ap.json; cat gpurun_out/ablate_ap.err
