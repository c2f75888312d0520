# GPU box, round 4: the filter timed by its own launch's events (hipExtLaunchKernel): the timed
# advance tests, then the driver's bench command and its kernel trace, to compare kernel_ms with
# the trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --cull cells > $O/cfg4_cells.json 2> $O/cfg4_cells.err || { tail -20 $O/cfg4_cells.err; exit 4; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_trace.log 2>&1 || { tail -20 $O/driver_trace.log; exit 5; }
python - <<'PY'
import json
for f in ("cfg4_driver", "cfg4_cells"):
    d = json.load(open(f"gpurun_out/r04z/{f}.json"))
    r = d["roofline"]
    print(f, d["config"]["cull"], round(d["ms_per_step"] * 1e3, 2), "kernel_ms", round(r["kernel_ms"] * 1e3, 2),
          "stream", round(r["kernel_ms_stream_events"] * 1e3, 2), "frac", round(r["frac"], 3))
PY
echo R04Z_OK
