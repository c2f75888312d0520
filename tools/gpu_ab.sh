# A/B of the working tree against variant trees under tools/_ab (built beforehand on the CPU),
# after the GPU test suite: tools/ab_lattice.py step / advance times at cfg4 and cfg4f spacing.
set -u
cd /root/repo
O=gpurun_out/ab; mkdir -p $O; : > $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for t in . "$@"; do
  for sp in 0.145 0.2; do
    timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>/dev/null >> $O/ab.txt || exit 2
  done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4 -o run -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/prof.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4f -o run -- python bench.py --config cfg4f --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 5 > $O/prof.log 2>&1 || exit 4
cat $O/ab.txt
