# GPU box: the window walk's row-guard continuation 4 words per round: window GPU tests, then the
# driver's bench line and run(10) for base (HEAD) and rowchunk, interleaved.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/gpu_r05k.sh tools/_abt/base tools/_abt/rowchunk tools/_abt/base tools/_abt/rowchunk || exit 2
for rep in 1 2; do
  for t in tools/_abt/base tools/_abt/rowchunk; do
    timeout -k 10 120 python3 tools/ab_window.py $t window 0.145 || exit 3
  done
done
