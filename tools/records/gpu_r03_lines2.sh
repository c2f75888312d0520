# GPU box, round 3: the GPU test suite, smoke(), then every bench line with its CPU baseline
# (the driver's cfg4 command first), the sharded step at one rank, and the --gpus N launcher
# rehearsed with gloo on this one GPU (2 and 4 ranks, strong scaling of the 1M lattice).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03_lines2; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); c=d.get('cpu_baseline') or {}; print('$n', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), (d.get('roofline') or {}).get('frac'), c.get('value'), c.get('cores'))"; }
run cfg5 --config cfg5 --steps 20 --warmup 2 --cpu-budget 8
run cfg3 --config cfg3 --steps 20 --warmup 3 --cpu-budget 8
run cert --config cert --steps 5 --warmup 1 --cpu-budget 8
run shard1 --shard --steps 48 --warmup 8 --no-cpu-baseline
run shard1_128 --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline
run gloo2 --gpus 2 --backend gloo --steps 24 --warmup 4
run gloo4 --gpus 4 --backend gloo --steps 24 --warmup 4
echo LINES_OK
