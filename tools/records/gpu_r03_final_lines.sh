# GPU box, round 3 (final tree): the GPU test suite, smoke(), then every bench line with its CPU
# baseline (the driver's cfg4 command first) and the sharded step at one rank.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); c=d.get('cpu_baseline') or {}; print('$n', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), (d.get('roofline') or {}).get('frac'), c.get('value'), c.get('cores'))"; }
run cfg4_driver --gpus 1 --steps 20 --warmup 5
run cfg4 --cpu-budget 8
run cfg4f --config cfg4f --cpu-budget 8
run cfg4r --config cfg4r --cpu-budget 8
run cfg5 --config cfg5 --steps 20 --warmup 2 --cpu-budget 8
run cfg3 --config cfg3 --steps 20 --warmup 3 --cpu-budget 8
run cert --config cert --steps 5 --warmup 1 --cpu-budget 8
run shard1 --shard --steps 48 --warmup 8 --no-cpu-baseline
run shard128 --shard --weak --rows 128 --steps 96 --warmup 16 --no-cpu-baseline
run rows128 --rows 128 --no-cpu-baseline
echo LINES_OK
