# GPU box, round 4 final (after the runtime guard choice): the whole -m gpu suite, smoke(), the driver's bench command and its
# kernel trace, PMC passes of cfg4 / cfg4f on the final kernels, and a full-size 4-rank gloo
# rehearsal of the strong-scaled split (must end in the 1-rank end state).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04af; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_trace.log 2>&1 || { tail -20 $O/driver_trace.log; exit 4; }
# (PMC passes: see gpu_r04y.sh)
timeout -k 10 900 python bench.py --gpus 4 --backend gloo --steps 20 --warmup 5 > $O/gloo4.json 2> $O/gloo4.err || { tail -20 $O/gloo4.err; exit 6; }
python - <<'PY'
import json
for f in ("cfg4_driver", "gloo4"):
    d = json.load(open(f"gpurun_out/r04af/{f}.json"))
    e = d.get("exact_qp_regime") or {}
    print(f, d["n_gpus"], d["config"].get("cull"), "%.4g" % d["value"], round(d["ms_per_step"] * 1e3, 2),
          round(d["roofline"]["frac"], 3), d["end_state_sha256"][:16], "exact", e.get("value"), e.get("ms_per_step"))
PY
echo R04Y_OK
