# GPU box, round 3: CBF_INLINE_MAX 196608 -> 131072 (inline solve only while the window is at most
# 2 waves per SIMD): GPU test suite, then run(10) at 128 / 136 / 160 rows against the committed tree.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03g3; mkdir -p $O; : > $O/rows.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for h in 128 136 160 192; do
  for t in . tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 $h 2>/dev/null >> $O/rows.txt || exit 2
  done
done
cat $O/rows.txt
echo R03G3_OK
