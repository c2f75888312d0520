# GPU box, round 3 (final tree): the GPU test suite, smoke(), the driver's bench command, and the
# drop-in get_safe_control's per-call time against the previous tree (tools/_ab/base).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${FINAL_OUT:-r03_final2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
python -c "import json; d=json.load(open('$O/cfg4_driver.json')); print('driver', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), d['roofline']['frac'], d['end_state_sha256'][:12])"
for t in . tools/_ab/base; do timeout -k 10 120 python tools/compat_call_time.py $t 2000 || exit 4; done
echo FINAL2_OK
