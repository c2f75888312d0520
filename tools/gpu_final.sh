# GPU box, a round's closing measurement set: every -m gpu test; the driver's exact bench command
# (with its CPU baseline) twice; its kernel trace; the 200-step default run; the HOCBF line; smoke();
# the PMC passes of tools/profile.sh for $PMC_CONFIGS (default cfg4 cfg4f; "none" skips them),
# summarised afterwards by tools/summarize_profile.py.
#   O=gpurun_out/<name> bash tools/gpu_final.sh
set -u
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=${O:-gpurun_out/final}; mkdir -p $O
if [ "${TESTS:-all}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for rep in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver$rep.json 2> $O/bench_driver$rep.err || { tail $O/bench_driver$rep.err; exit 2; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || { tail $O/trace.log; exit 3; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-exact-qp > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 4; }
timeout -k 10 300 python bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-exact-qp > $O/bench_hocbf.json 2> $O/bench_hocbf.err || { tail $O/bench_hocbf.err; exit 6; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 7; }
if [ "${PMC_CONFIGS:-}" != none ]; then
  PROF_OUT=$O/prof CONFIGS="${PMC_CONFIGS:-cfg4 cfg4f}" bash tools/profile.sh > $O/profile.log 2>&1 || { tail $O/profile.log; exit 5; }
fi
echo FINAL_OK
