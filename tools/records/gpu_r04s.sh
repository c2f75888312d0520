# GPU box, round 4 (after the row-guard fold): the whole -m gpu suite, smoke(), the driver's bench
# command and its kernel trace, cfg4 with the cell list, cfg4f, cfg4r.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_trace.log 2>&1 || { tail -20 $O/driver_trace.log; exit 4; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --cull cells > $O/cfg4_cells.json 2> $O/cfg4_cells.err || { tail -20 $O/cfg4_cells.err; exit 5; }
timeout -k 10 400 python bench.py --config cfg4f > $O/cfg4f.json 2> $O/cfg4f.err || { tail -20 $O/cfg4f.err; exit 6; }
timeout -k 10 400 python bench.py --config cfg4r > $O/cfg4r.json 2> $O/cfg4r.err || { tail -20 $O/cfg4r.err; exit 7; }
python - <<'PY'
import json
for f in ("cfg4_driver", "cfg4_cells", "cfg4f", "cfg4r"):
    d = json.load(open(f"gpurun_out/r04s/{f}.json"))
    e = d.get("exact_qp_regime") or {}
    print(f, d["config"].get("cull"), d["value"], round(d["ms_per_step"] * 1e3, 2), round(d["roofline"]["frac"], 3),
          round(d["roofline"]["kernel_ms"] * 1e3, 2), d["end_state_sha256"][:16], "exact", e.get("value"), e.get("ms_per_step"))
PY
echo R04S_OK
