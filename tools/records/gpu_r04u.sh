# GPU box, round 4: the other bench lines with their CPU baselines (cfg4 default run, cfg5, cfg3,
# cert, the sharded step at one rank, HOCBF mode), the --gpus 2 gloo rehearsal, and a kernel
# trace of the HOCBF step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); c=d.get('cpu_baseline') or {}; print('$n', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), (d.get('roofline') or {}).get('frac'), c.get('value'), c.get('cores'))"; }
run cfg4 --cpu-budget 8
run cfg5 --config cfg5 --steps 20 --warmup 2 --cpu-budget 8
run cfg3 --config cfg3 --steps 20 --warmup 3 --cpu-budget 8
run cert --config cert --steps 5 --warmup 1 --cpu-budget 8
run shard1 --shard --steps 48 --warmup 8 --no-cpu-baseline
run shard1_128 --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline
run hocbf --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline
run gloo2 --gpus 2 --backend gloo --steps 24 --warmup 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/hocbf_trace -o run -- python3 bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline > $O/hocbf_trace.log 2>&1 || { tail -20 $O/hocbf_trace.log; exit 4; }
echo R04U_OK
