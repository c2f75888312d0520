# GPU box, round 3: queue-kernel spread targets (tools/_ab/s4, s8, s16: a sub-queue's entries
# dealt over ceil(nq / S) lanes per block) against the committed tree (tools/_ab/base): kernel traces
# at cfg4 and cfg4r spacing, then run(10) A/B.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03z2; mkdir -p $O; : > $O/ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k lattice > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in tools/_ab/s4 tools/_ab/s8 tools/_ab/s16 tools/_ab/base; do
  n=$(basename $t)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 3
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_rw -o run -- python3 tools/ab_lattice.py $t 0.22 60 1024 rw > $O/${n}_rw.txt 2>&1 || exit 4
done
for rep in 1 2; do
  for t in tools/_ab/s4 tools/_ab/s8 tools/_ab/s16 tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
echo R03Z2_OK
