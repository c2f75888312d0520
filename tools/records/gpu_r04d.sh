# GPU box, round 4: window-cull tests (single GPU and sharded), then A/B of window-filter variants
# (tools/_abt) against the cell list at 1024 and 128 rows, then a kernel trace of the default bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py tests/test_gpu_torch_ops.py -k "window or cell_starts or lattice_step_vs or run_matches or checkpoint or lattice_run_op" -x -q --timeout 240 --timeout-method thread > $O/pytest_window.log 2>&1 || { tail -40 $O/pytest_window.log; exit 1; }
tail -1 $O/pytest_window.log
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py -k "window" -x -q --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1 || { tail -40 $O/pytest_shard.log; exit 1; }
tail -1 $O/pytest_shard.log
for rep in 1 2; do
  for rows in 1024 128; do
    timeout -k 10 120 python tools/ab_window.py . cells 0.145 $rows >> $O/ab.txt || exit 2
    for t in . tools/_abt/untiled tools/_abt/spec; do
      timeout -k 10 120 python tools/ab_window.py $t window 0.145 $rows >> $O/ab.txt || exit 3
    done
  done
done
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --kernel-iters 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 5; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/window_kernel_stats.csv
cut -d, -f1-8 $O/window_kernel_stats.csv | head -8
echo R04D_OK
