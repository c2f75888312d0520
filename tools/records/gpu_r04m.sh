# GPU box, round 4: the row guard formed by the tile launch's first block as token-tagged words
# (no k_window_rowscan): window tests, then A/B against HEAD and the rowscan build at 1024 / 128 rows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_shard_gpu.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py -m gpu -x -v -k "window" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in tools/_abt/head tools/_abt/fold0 .; do
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.145 128 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 3; }
  done
done
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 tools/ab_window.py . window > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 4; }
echo R04J_OK
