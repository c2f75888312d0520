# RECORD ONLY: the streaming queue kernel this measured was reverted (profiles/r02_hard_stream_ab.txt); the variant trees no longer exist.
# GPU box: the streaming hard-QP kernel (CBF_HARD_STREAM): lattice GPU tests, then A/B against the
# post-filter queue kernel (tools/_ab/s0) and 1 / 2 blocks per sub-queue (q1, q2), cfg4 and cfg4f.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/stream; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_torch_ops.py -m gpu -x -v --timeout 200 --timeout-method thread -k "lattice or shard or torch or scan_timeout or workspace" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sp in 0.145 0.2; do
  for rep in 1 2; do
    for t in . tools/_ab/s0 tools/_ab/q1 tools/_ab/q2; do
      echo -n "$sp $t " >> $O/ab.txt
      timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>>$O/ab.err >> $O/ab.txt || { tail -5 $O/ab.err; exit 2; }
    done
  done
done
cat $O/ab.txt
