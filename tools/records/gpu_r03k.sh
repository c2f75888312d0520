# GPU box, round 3: the x-split lattice grid (CBF_XSUB columns per caller cell, disc-clipped row
# ranges) -- GPU test suite, then A/B of CBF_XSUB = 4 (this tree) against 2, 8 and the round-3
# HEAD tree (tools/_ab/head, square 3 x 3 cells), and a kernel trace of the default cfg4 bench.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/xs2 tools/_ab/xs8 tools/_ab/head; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_cfg4.json 2>$O/prof_cfg4.err || exit 3
echo R03K_OK
