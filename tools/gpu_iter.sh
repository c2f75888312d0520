# GPU box, one development iteration (round 6): the GPU tests named in $TESTS (default: the window,
# fused and parity suites; "all" = every -m gpu test; "none" = skip), the fused-hard-solve A/B when
# FUSED_AB=1, run(10) of the base tree (tools/_abt/base, HEAD's sources) against this tree when that
# tree exists, the driver's bench line and its kernel trace.
#   O=gpurun_out/<name> bash tools/gpu_iter.sh
set -u
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=${O:-gpurun_out/iter}; mkdir -p $O
T=${TESTS:-tests/test_gpu_fused.py tests/test_gpu_window.py tests/test_gpu_parity.py}
[ "$T" = all ] && T="tests -m gpu"
if [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ "${FUSED_AB:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/ab_fused.py 0.145 0.2 > $O/ab_fused.txt 2>&1 || { tail $O/ab_fused.txt; exit 2; }
  cat $O/ab_fused.txt
fi
if [ -d tools/_abt/base ]; then
  for rep in 1 2; do for t in tools/_abt/base .; do
    timeout -k 10 120 python tools/ab_window.py $t window 0.145 >> $O/ab_walk.txt 2>&1 || { tail $O/ab_walk.txt; exit 3; }
  done; done
  grep run $O/ab_walk.txt
fi
for rep in $(seq 1 ${BENCH_REPS:-1}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$rep.json 2> $O/bench$rep.err || { tail $O/bench$rep.err; exit 4; }
  python -c "import json; d=json.load(open('$O/bench$rep.json')); print('bench', round(d['ms_per_step']*1e3, 2), 'tile', round(d['roofline']['kernel_ms']*1e3, 2), 'cfg4r', round(d['exact_qp_regime']['ms_per_step']*1e3, 2), d.get('end_state_sha256', '')[:8])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || { tail $O/trace.log; exit 5; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | sed 's/(.*)"/"/' | head -12
echo ITER_OK
