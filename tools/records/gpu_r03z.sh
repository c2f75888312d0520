# GPU box, round 3: the queue kernel's entries spread over all of a sub-queue's blocks
# (CBF_HARD_SPREAD, this tree; tools/_ab/pq64 with 64 blocks per sub-queue) against the committed
# tree (tools/_ab/base): lattice + shard GPU tests, A/B, kernel traces.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/pq64 tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.2 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
for t in . tools/_ab/pq64; do
  n=$(basename $t); [ "$n" = "." ] && n=ship
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 3
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_rw -o run -- python3 tools/ab_lattice.py $t 0.22 60 1024 rw > $O/${n}_rw.txt 2>&1 || exit 4
done
echo R03Z_OK
