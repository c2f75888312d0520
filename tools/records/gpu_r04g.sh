# GPU box, round 4: the whole -m gpu suite, smoke(), the driver's bench command (window cull for
# cfg4, exact_qp_regime on the cell list), cfg4 with the cell list, cfg4f.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/cfg4_driver.json 2> $O/cfg4_driver.err || { tail -20 $O/cfg4_driver.err; exit 3; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --cull cells > $O/cfg4_cells.json 2> $O/cfg4_cells.err || { tail -20 $O/cfg4_cells.err; exit 4; }
timeout -k 10 400 python bench.py --config cfg4f --steps 20 --warmup 5 --no-cpu-baseline > $O/cfg4f.json 2> $O/cfg4f.err || { tail -20 $O/cfg4f.err; exit 5; }
python - <<'PY'
import json
for f in ("cfg4_driver", "cfg4_cells", "cfg4f"):
    d = json.load(open(f"gpurun_out/r04g/{f}.json"))
    e = d.get("exact_qp_regime") or {}
    print(f, d["config"]["cull"], d["value"], round(d["ms_per_step"] * 1e3, 2), round(d["roofline"]["frac"], 3),
          round(d["roofline"]["kernel_ms"] * 1e3, 2), d["end_state_sha256"][:16], d["full_size_check"]["u_bit_identical_to_cell_filter"],
          "exact", e.get("value"), e.get("ms_per_step"))
PY
echo R04G_OK
