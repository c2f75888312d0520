# GPU box, round 3: loads in flight per lane in the small-window filter instantiation (IN) --
# this tree (scan 12 / flush 8) against 24 / 16, 8 / 6 and the round-3 HEAD tree (6 / 4), at the
# strong-scaled stripe sizes (128 and 256 rows of 1024) plus the lattice GPU tests.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for t in . tools/_ab/su24 tools/_ab/su8 tools/_ab/head; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 128 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 160 2>/dev/null >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
echo R03M_OK
