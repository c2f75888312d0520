# GPU box, round 4: the whole -m gpu suite (both solve placements), smoke(), the driver's bench
# command (cfg4 line with the exact_qp_regime record) and cfg4r alone.  First failure ends it.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 python bench.py --config cfg4r --steps 20 --warmup 5 --no-cpu-baseline > $O/cfg4r.json 2> $O/cfg4r.err || { tail -20 $O/cfg4r.err; exit 4; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r04b/cfg4_driver.json")); b = json.load(open("gpurun_out/r04b/cfg4r.json"))
e = a.get("exact_qp_regime", {})
print("cfg4", a["value"], a["ms_per_step"], a["roofline"]["frac"], "exact", e.get("value"), e.get("ms_per_step"), "cfg4r alone", b["value"], b["ms_per_step"])
PY
echo R04B_OK
