# GPU box: the GPU test suite on the default build (fused scan + scatter),
# then A/B against tools/_ab/unfused (CBF_FUSED_BUILD=0), and kernel traces.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/unfused; do
    for sp in 0.145 0.2; do
      timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>/dev/null >> $O/ab.txt || exit 2
    done
  done
done
cat $O/ab.txt
for R in 1024 128; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$R -o run -- python3 bench.py --rows $R --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/prof_$R.json 2>$O/prof_$R.err || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4r -o run -- python3 bench.py --config cfg4r --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/prof_cfg4r.json 2>&1 || exit 7
echo R03D_OK
