# GPU box, round 4: nominal controls formed in the window tile (prep stops writing u0): window
# tests, then A/B of HEAD / this tree / this tree without the waves-per-SIMD fit.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_shard_gpu.py tests/test_gpu_parity.py -m gpu -x -v -k "window" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in tools/_abt/head . tools/_abt/wpe0; do
    echo "== $t" >> $O/ab.txt
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
  done
done
cat $O/ab.txt
echo R04H_OK
