# GPU box, round 4: the bench tests (incl. the killed-rank test), then the driver's bench command
# (cfg4 with the exact_qp_regime record) and cfg4r alone with the same arguments.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_bench_tests.log 2>&1 || { echo "bench tests failed"; tail -30 gpurun_out/r04a_bench_tests.log; exit 1; }
tail -3 gpurun_out/r04a_bench_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_cfg4_driver.json 2> gpurun_out/r04a_cfg4_driver.err || { tail -20 gpurun_out/r04a_cfg4_driver.err; exit 1; }
timeout -k 10 400 python bench.py --config cfg4r --steps 20 --warmup 5 > gpurun_out/r04a_cfg4r.json 2> gpurun_out/r04a_cfg4r.err || { tail -20 gpurun_out/r04a_cfg4r.err; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r04a_cfg4_driver.json")); b = json.load(open("gpurun_out/r04a_cfg4r.json"))
e = a["exact_qp_regime"]
print("cfg4", a["value"], a["ms_per_step"], "exact", e["value"], e["ms_per_step"], "cfg4r alone", b["value"], b["ms_per_step"])
PY
