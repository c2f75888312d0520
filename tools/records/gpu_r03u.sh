# GPU box, round 3: the tree after the sub-step default change -- GPU test suite, smoke, the driver's
# cfg4 command, the sharded 128-row stripe (k = 16) and the 2-rank gloo rehearsal of --gpus 2.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['n_gpus'], d['config']['parallelism'][:60])"; }
run cfg4_driver --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run shard128 --shard --weak --rows 128 --steps 96 --warmup 16 --no-cpu-baseline
run shard256 --shard --weak --rows 256 --steps 96 --warmup 16 --no-cpu-baseline
run gloo2 --gpus 2 --backend gloo --steps 32 --warmup 4 --no-cpu-baseline
echo R03U_OK
