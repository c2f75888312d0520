#!/bin/bash
# Round-2 GPU check: parity suite, profiles (tools/profile.sh), bench lines per config.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
if [ -n "${PROFILE:-}" ]; then
  echo "== profile"
  PROF_OUT=$O/prof bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 2; }
fi
for C in ${BENCH:-cfg4 cfg4f cfg5}; do
  echo "== bench $C"
  EXTRA="--no-cpu-baseline"
  [ $C = cfg4 ] && EXTRA="--cpu-budget 5"
  timeout -k 10 400 python bench.py --config $C $EXTRA > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 3; }
  python -c "import json; d=json.load(open('$O/bench_$C.json')); print('$C', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
echo ALL_OK
