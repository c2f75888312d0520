# GPU box, round 3: the strong-scaled stripe (128 rows = 131 k agents, the N = 8 share of cfg4)
# and the coordinate stencil at CBF_XSUB = 1 (this tree) against 4 and the round-3 HEAD tree;
# kernel traces of the 128-row single-GPU run and of the sharded step at one rank on 128 rows.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03l; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/xs4 tools/_ab/head; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 128 2>/dev/null >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_128 -o run -- python3 bench.py --rows 128 --no-cpu-baseline > $O/prof_128.json 2>$O/prof_128.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_shard128 -o run -- python3 bench.py --shard --weak --rows 128 --steps 96 --warmup 16 --no-cpu-baseline > $O/prof_shard128.json 2>$O/prof_shard128.err || exit 4
timeout -k 10 300 python3 bench.py --rows 128 --no-cpu-baseline > $O/b128.json 2>$O/b128.err || exit 5
timeout -k 10 300 python3 bench.py --shard --weak --rows 128 --steps 96 --warmup 16 --no-cpu-baseline > $O/bshard128.json 2>$O/bshard128.err || exit 6
echo R03L_OK
