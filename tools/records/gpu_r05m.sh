# GPU box: the window walk reading staged candidates from LDS: window + parity GPU tests, then the
# driver's bench line and run(10) for base (round-5 head) and ldswalk.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu/gpu_r05k.sh tools/_abt/base tools/_abt/ldswalk tools/_abt/base tools/_abt/ldswalk
bash tools/gpu_ab_run.sh tools/_abt/base tools/_abt/ldswalk
