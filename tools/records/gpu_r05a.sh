# GPU box, round 5 checkpoint (event deferral, sorted rows): smoke(), the driver's bench command
# and its kernel trace, PMC passes of cfg4 / cfg4f (tools/profile.sh).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_trace.log 2>&1 || { tail -20 $O/driver_trace.log; exit 4; }
PROF_OUT=$O/prof CONFIGS="cfg4 cfg4f" bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 5; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r05a/cfg4_driver.json"))
e = d.get("exact_qp_regime") or {}
print(d["n_gpus"], d["config"].get("cull"), "%.4g" % d["value"], round(d["ms_per_step"] * 1e3, 2),
      round(d["roofline"]["frac"], 3), d["end_state_sha256"][:16], "exact", e.get("value"), e.get("ms_per_step"))
PY
echo R05A_OK
