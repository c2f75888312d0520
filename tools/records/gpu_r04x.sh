# GPU box, round 4: cfg4r (random-walk nominal) with the window cull against the cell list, at the
# driver's arguments and over the default 200-step run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04x; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['config'].get('cull'), '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16], d['full_size_check']['u_bit_identical_to_cell_filter'])"; }
run r_win_20 --config cfg4r --cull window --steps 20 --warmup 5 --no-cpu-baseline
run r_cells_20 --config cfg4r --cull cells --steps 20 --warmup 5 --no-cpu-baseline
run r_win_200 --config cfg4r --cull window --no-cpu-baseline
run r_cells_200 --config cfg4r --cull cells --no-cpu-baseline
echo R04X_OK
