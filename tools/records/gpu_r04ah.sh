# GPU box, round 4: HOCBF solve_rows unroll 8 / 16 / 24 (bench step only).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ai; mkdir -p $O


for rep in 1 2; do
  for t in tools/_abt/hu8 .; do
    (cd $t && timeout -k 10 400 python bench.py --barrier euclidean_hocbf --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/h.json 2> $GRAFT_REPO_ROOT/$O/h.err) || { tail -20 $O/h.err; exit 2; }
    python -c "import json; d=json.load(open('$O/h.json')); print('$t', round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
  done
done

echo R04AG_OK
