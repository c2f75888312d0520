set -u
cd /root/repo
O=gpurun_out/ab4; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for t in . tools/_ab/pq8 tools/_ab/pq64; do
  for sp in 0.145 0.2; do
    timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>/dev/null >> $O/ab.txt || exit 2
  done
done
done
timeout -k 10 120 python bench.py --config cfg5 --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('cfg5', d['value'], d['ms_per_step'])" >> $O/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4 -o run -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/prof.log 2>&1 || exit 3
cat $O/ab.txt
