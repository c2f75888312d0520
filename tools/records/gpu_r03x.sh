# GPU box, round 3: the filter's screened scan over an fp32 pairs copy (two candidates per 16-B
# load, exact re-test in the flush) against the committed tree (tools/_ab/base): GPU test suite,
# A/B at cfg4 / cfg4f / cfg4r / 128 rows, kernel trace and a TD/VMEM counter pass at cfg4.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03x; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.2 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 128 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.json 2>$O/prof.err || exit 3
timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VALU -f csv -d $O/pmc -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/pmc.log 2>&1 || exit 4
echo R03X_OK
