# GPU box, round 5: the sharded cycle at one rank (1024 / 512 / 256 / 128 rows per rank) and the
# unsharded step at the heights a sub-step window of the N = 8 share spans (128 .. 256 rows), both
# culls: the inputs of DESIGN.md sec. 5's strong-scaling model.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
for R in 1024 512 256 128; do
  timeout -k 10 300 python bench.py --shard --rows $R --no-cpu-baseline --steps 64 --warmup 16 > $O/shard_$R.json 2> $O/shard_$R.err || { tail -20 $O/shard_$R.err; exit 1; }
  python -c "import json; d=json.load(open('$O/shard_$R.json')); c=d['config']; print('shard rows $R', c.get('cull'), c.get('substeps'), '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), d.get('end_state_sha256', '')[:16])"
done
for R in 128 136 144 160 192 224 256; do
  for C in cells window; do
    timeout -k 10 120 python3 tools/ab_window.py . $C 0.145 $R | tee -a $O/heights.txt || exit 2
  done
done
echo R05B_OK
