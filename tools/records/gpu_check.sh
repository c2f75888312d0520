#!/bin/bash
# GPU check of the tree: parity suite, then bench lines (driver settings, defaults, sharded at one
# rank with and without the cycle graph).  Every GPU step has its own time limit; the first failure
# ends the script.  OUT=gpurun_out/<name>, SKIP_TESTS=1, BENCH="driver default shard shard_eager".
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${OUT:-gpurun_out/check}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for B in ${BENCH:-driver default shard shard_eager}; do
  case $B in
    driver) A="--steps 20 --warmup 5 --cpu-budget 3" ;;
    default) A="--no-cpu-baseline" ;;
    shard) A="--shard --no-cpu-baseline" ;;
    shard_eager) A="--shard --eager --no-cpu-baseline" ;;
    cfg4f|cfg5|cfg3) A="--config $B --no-cpu-baseline" ;;
    *) A="$B --no-cpu-baseline" ;;
  esac
  echo "== bench $B"
  timeout -k 10 400 python bench.py $A > $O/bench_$B.json 2> $O/bench_$B.err || { tail -20 $O/bench_$B.err; exit 3; }
  python -c "import json; d=json.load(open('$O/bench_$B.json')); print('$B', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('kernel_ms'))"
done
echo ALL_OK
