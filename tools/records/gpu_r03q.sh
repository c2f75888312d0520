# GPU box, round 3: the filter's and the scatter's independent loads issued in one round trip at
# kernel start (this tree) against the committed tree (tools/_ab/base): lattice GPU tests, A/B at
# cfg4 / cfg4f / cfg4r / 128 rows.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03q; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for t in . tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.2 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 128 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
echo R03Q_OK
