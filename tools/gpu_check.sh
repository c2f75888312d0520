# GPU box: parity tests, smoke, then the benches named in $BENCHES (default: cfg4)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
for c in ${BENCHES:-cfg4}; do
  case $c in
    cfg3) a="--config cfg3 --steps 20 --warmup 3";;
    cfg5) a="--config cfg5 --steps 5 --warmup 1";;
    *) a="";;
  esac
  timeout -k 10 300 python bench.py $a > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo BENCH_FAILED $c; tail gpurun_out/bench_$c.err; exit 3; }
  cat gpurun_out/bench_$c.json
done
