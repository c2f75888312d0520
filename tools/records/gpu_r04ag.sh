# GPU box, round 4: HOCBF mode with solve_rows' inner loops unrolled (the rows' LDS loads issued
# together): the HOCBF GPU tests on this tree (unroll 4), then the HOCBF bench step for unroll 1 /
# 4 / 8 and a kernel trace of this tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ah; mkdir -p $O
true
true
for rep in 1 2; do
  for t in tools/_abt/hu8 tools/_abt/hu16 tools/_abt/hu24; do
    (cd $t && timeout -k 10 400 python bench.py --barrier euclidean_hocbf --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/h.json 2> $GRAFT_REPO_ROOT/$O/h.err) || { tail -20 $O/h.err; exit 2; }
    python -c "import json; d=json.load(open('$O/h.json')); print('$t', round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
  done
done
true
echo R04AG_OK
