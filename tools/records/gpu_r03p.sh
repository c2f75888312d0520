# GPU box, round 3: the queue kernel's Seidel solve with the event points computed up front
# (CBF_HARD_PRE=1, this tree) against the plain incremental solve (tools/_ab/pre0): lattice GPU
# tests, A/B step times, and kernel traces of both at cfg4 and cfg4r.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03p; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/pre0; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.2 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
i=0
for t in . tools/_ab/pre0; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof${i}_cfg4 -o run -- python3 tools/ab_lattice.py $t 0.145 100 > $O/prof${i}_cfg4.txt 2>&1 || exit 3
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof${i}_cfg4r -o run -- python3 tools/ab_lattice.py $t 0.22 100 1024 rw > $O/prof${i}_cfg4r.txt 2>&1 || exit 4
done
echo R03P_OK
