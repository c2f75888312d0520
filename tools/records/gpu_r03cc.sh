# GPU box, round 3: the drop-in get_safe_control with pinned, per-instance buffers (this tree)
# against the one-buffer version (tools/_ab/base): the tests that call it, then per-call time.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03cc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hocbf.py tests/test_gpu_rps.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for t in . tools/_ab/base; do timeout -k 10 120 python tools/compat_call_time.py $t 3000 || exit 2; done; done
echo R03CC_OK
