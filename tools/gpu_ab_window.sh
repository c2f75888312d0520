# A/B of the window-cull step: the GPU window tests on the working tree, then tools/ab_window.py
# (run(10) per timestep, build / filter / advance by HIP events) for the working tree and each
# variant tree under tools/_abt, interleaved, at cfg4 (0.145) and cfg4f (0.2) spacing.
# Usage: bash tools/gpu_ab_window.sh <out-name> [variant trees...]
set -u
cd /root/repo
O=gpurun_out/$1; shift; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py -k "window or lattice_step or full_size" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for t in "$@"; do
  for sp in 0.145 0.2; do
    timeout -k 10 120 python tools/ab_window.py $t window $sp >> $O/ab.txt 2>/dev/null || exit 2
  done
done
done
cat $O/ab.txt
