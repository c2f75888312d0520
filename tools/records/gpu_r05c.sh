# GPU box, round 5: kernel traces of the one-rank sharded cycle at 1024 and 128 rows per rank.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
for R in 1024 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/t$R -o run -- python3 bench.py --shard --rows $R --no-cpu-baseline --steps 64 --warmup 16 > $O/t$R.json 2> $O/t$R.err || { tail -20 $O/t$R.err; exit 1; }
done
echo R05C_OK
