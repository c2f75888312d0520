# GPU box, round 4: guard extents with the min / max instructions (no compare-and-select): window
# tests, A/B against HEAD, kernel traces.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_shard_gpu.py tests/test_gpu_parity.py -m gpu -x -v -k "window" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in tools/_abt/head .; do
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.2 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 3; }
  done
done
grep -v amdgpu.ids $O/ab.txt
for t in tools/_abt/head .; do
  n=$(basename $(realpath $t))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_window.py $t window > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 4; }
done
echo R04AA_OK
