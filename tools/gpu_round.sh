# GPU box: parity suite + smoke, A/B of the working tree against the built revisions
# (tools/ablate.py, ABLATE_SET=head), the cfg4 bench line, then the profile recipe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
ABLATE_SET=head timeout -k 10 300 python tools/ablate.py run --rounds 5 --iters 20 > gpurun_out/ablate_head.json 2> gpurun_out/ablate_head.err || { tail gpurun_out/ablate_head.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ablate_head.json')); print({k: (round(v['build']['median_us'],1), round(v['advance']['median_us'],1), v.get('bit_identical_to_tree')) for k, v in d.items()})"
timeout -k 10 300 python bench.py > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail gpurun_out/bench_cfg4.err; exit 4; }
cat gpurun_out/bench_cfg4.json
if [ -n "$PROFILE" ]; then PROF_OUT=gpurun_out/prof timeout -k 10 900 bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail gpurun_out/profile.log; exit 5; }; tail -1 gpurun_out/profile.log; fi
