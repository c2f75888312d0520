# GPU box, round 4: HOCBF solve_rows loading row i + 1 while testing row i, against HEAD; HOCBF tests.
set -u

cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ak; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hocbf.py tests/test_gpu_parity.py -x -v -k "hocbf" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log


for rep in 1 2; do
  for t in tools/_abt/head .; do
    (cd $t && timeout -k 10 400 python bench.py --barrier euclidean_hocbf --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/h.json 2> $GRAFT_REPO_ROOT/$O/h.err) || { tail -20 $O/h.err; exit 2; }
    python -c "import json; d=json.load(open('$O/h.json')); print('$t', round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
  done
done

echo R04AG_OK
