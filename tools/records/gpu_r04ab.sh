# GPU box, round 4: the sharded step at one RCCL rank with the window cull against the cell list,
# 1024 and 512 rows per rank (the weak-scaling share and the N = 2 strong-scaling share).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ab; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['config'].get('cull'), '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"; }
# (first call: 1024 / 512 / 256 rows; this one adds 128)
#run s1024_cells --shard --steps 48 --warmup 8 --no-cpu-baseline --cull cells
#run s1024_win --shard --steps 48 --warmup 8 --no-cpu-baseline --cull window
#run s512_cells --shard --rows 512 --steps 48 --warmup 8 --no-cpu-baseline --cull cells
#run s512_win --shard --rows 512 --steps 48 --warmup 8 --no-cpu-baseline --cull window
#run s256_cells --shard --rows 256 --steps 48 --warmup 8 --no-cpu-baseline --cull cells
#run s256_win --shard --rows 256 --steps 48 --warmup 8 --no-cpu-baseline --cull window
run s128_cells --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --cull cells
run s128_win --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --cull window
run s128_cells2 --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --cull cells
run s128_win2 --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --cull window
echo R04AB_OK
