# GPU box: deferred window walks run wave-wide by the queue kernel: window, shard and parity GPU
# tests, then the driver's bench line and run(10) for base (HEAD) and wavewalk, interleaved.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_window.py tests/test_shard_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/gpu_r05k.sh tools/_abt/base tools/_abt/wavewalk tools/_abt/base tools/_abt/wavewalk || exit 2
for rep in 1 2; do
  for t in tools/_abt/base tools/_abt/wavewalk; do
    timeout -k 10 120 python3 tools/ab_window.py $t window 0.145 || exit 3
  done
done
