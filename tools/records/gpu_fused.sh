# RECORD ONLY: the fused queue + scan kernel this measured was reverted (profiles/r02_hard_scan_fused_ab.txt).
# GPU box: the fused queue + next-scan kernel (CBF_HARD_SCAN_FUSED): lattice run / shard / full-size
# GPU tests, then tools/ab_stats.py A/B against tools/_ab/head (separate launches), cfg4 and cfg4f
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fused; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_torch_ops.py -m gpu -x -v --timeout 200 --timeout-method thread -k "lattice or shard or torch or scan_timeout or workspace" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sp in 0.145 0.2; do
  for rep in 1 2; do
    for t in . tools/_ab/head; do
      timeout -k 10 120 python tools/ab_stats.py $t $sp 2>>$O/ab.err >> $O/ab.txt || { tail -5 $O/ab.err; exit 2; }
    done
  done
done
cat $O/ab.txt
