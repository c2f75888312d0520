# GPU box, round 4: the window-cull tests and the lattice oracle tests (both culls), then the
# default bench (window cull) and the same with --cull cells, short.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py -x -v --timeout 240 --timeout-method thread > $O/pytest_window.log 2>&1 || { tail -40 $O/pytest_window.log; exit 1; }
tail -1 $O/pytest_window.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "lattice" > $O/pytest_lattice.log 2>&1 || { tail -40 $O/pytest_lattice.log; exit 2; }
tail -1 $O/pytest_lattice.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp > $O/cfg4_window.json 2> $O/cfg4_window.err || { tail -20 $O/cfg4_window.err; exit 3; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --cull cells > $O/cfg4_cells.json 2> $O/cfg4_cells.err || { tail -20 $O/cfg4_cells.err; exit 4; }
python - <<'PY'
import json
for f in ("cfg4_window", "cfg4_cells"):
    d = json.load(open(f"gpurun_out/r04c/{f}.json"))
    print(f, d["value"], round(d["ms_per_step"] * 1e3, 2), d["roofline"]["frac"], round(d["roofline"]["kernel_ms"] * 1e3, 2),
          round(d["roofline"]["advance_phase"]["ms"] * 1e3, 2), d["end_state_sha256"][:16], d["full_size_check"]["u_bit_identical_to_cell_filter"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-qp --kernel-iters 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 5; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/window_kernel_stats.csv
head -12 $O/window_kernel_stats.csv | cut -c1-200
echo R04C_OK
