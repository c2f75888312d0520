# GPU box: the GPU test suite on the cooperative-solve build, then A/B against tools/_ab/queue
# (CBF_HARD_COOP=0: round 2's queue kernel), benches at 1M and at a 1/8 stripe, and kernel traces.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/queue; do
    for sp in 0.145 0.2; do
      timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>/dev/null >> $O/ab.txt || exit 2
    done
  done
done
cat $O/ab.txt
for c in cfg4 cfg4r; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 3; }
done
timeout -k 10 300 python bench.py --rows 128 --no-cpu-baseline --steps 48 --warmup 8 > $O/single_128.json 2> $O/single_128.err || exit 4
for f in $O/*.json; do
  python -c "import json,sys; d=json.load(open('$f')); print('$f', '%.3e'%d['value'], round(d['ms_per_step']*1e3, 2), d.get('ms_per_step_outputs_every_step'), (d.get('roofline') or {}).get('frac'), d['safety']['seidel_fraction'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_full -o run -- python3 bench.py --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/prof_full.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_small -o run -- python3 bench.py --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/prof_small.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4r -o run -- python3 bench.py --config cfg4r --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/prof_cfg4r.log 2>&1 || exit 7
echo R03B_OK
