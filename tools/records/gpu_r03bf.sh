# GPU box, round 3: the branch-free exact solve (CBF_SOLVE_BRANCHFREE, this tree) against the
# committed tree (tools/_ab/base): GPU test suite, run(10) A/B at cfg4 / cfg4r / 128 rows, kernel
# traces, cfg5 (the Monte-Carlo kernel solves in every lane) through bench.py.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03bf; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in . tools/_ab/base; do
  n=$(basename $t); [ "$n" = "." ] && n=bf
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 3
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_rw -o run -- python3 tools/ab_lattice.py $t 0.22 60 1024 rw > $O/${n}_rw.txt 2>&1 || exit 4
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_128 -o run -- python3 tools/ab_lattice.py $t 0.145 100 128 > $O/${n}_128.txt 2>&1 || exit 5
done
for rep in 1 2; do
  for t in . tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 128 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 200 python $t/bench.py --config cfg5 --steps 20 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$t cfg5', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 1))" >> $O/ab.txt || exit 6
  done
done
sort $O/ab.txt
echo R03BF_OK
