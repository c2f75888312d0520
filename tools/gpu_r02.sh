#!/bin/bash
# Round-2 GPU check: parity suite, cfg4 / cfg4f bench lines, kernel-trace profiles.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
step() { echo "== $*"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step bench cfg4
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --cpu-budget 4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
step bench cfg4f
timeout -k 10 300 python bench.py --config cfg4f --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_cfg4f.json 2> $O/bench_cfg4f.err || { tail -20 $O/bench_cfg4f.err; exit 1; }
step bench cfg5
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
step rocprof cfg4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4 -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/prof_cfg4.log 2>&1 || { tail -20 $O/prof_cfg4.log; exit 1; }
step rocprof cfg4f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4f -o run -- python bench.py --config cfg4f --steps 50 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/prof_cfg4f.log 2>&1 || { tail -20 $O/prof_cfg4f.log; exit 1; }
cat $O/bench_cfg4.json $O/bench_cfg4f.json
echo ALL_OK
