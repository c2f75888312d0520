# GPU box: HOCBF parity tests then the cfg4 bench in HOCBF mode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hocbf.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hocbf_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/hocbf_tests.log; exit 1; }
tail -2 gpurun_out/hocbf_tests.log
timeout -k 10 300 python bench.py --barrier euclidean_hocbf --no-cpu-baseline --steps 100 > gpurun_out/bench_cfg4_hocbf.json 2> gpurun_out/bench_hocbf.err || { tail gpurun_out/bench_hocbf.err; exit 3; }
cat gpurun_out/bench_cfg4_hocbf.json
if [ -n "$HOCBF_STATS" ]; then
  export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/hstats -o run -- python3 bench.py --barrier euclidean_hocbf --no-cpu-baseline --steps 100 > gpurun_out/hstats.log 2>&1 || exit 4
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/hstats/run_kernel_stats.csv')):
    print(r['Name'][:60].ljust(60), '%9.2f us' % (float(r['AverageNs']) / 1e3))"
fi
