# GPU box, round 5: the full-size strong-scaled split rehearsed with 4 gloo ranks on one GPU
# (256 rows of the 1 M lattice per rank); it must end in the 1-rank driver run's state.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05g4; mkdir -p $O
timeout -k 10 1000 python bench.py --gpus 4 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/gloo4.json 2> $O/gloo4.err || { tail -20 $O/gloo4.err; exit 7; }
python -c "import json; d=json.load(open('$O/gloo4.json')); print('gloo4', d['value'], round(d['ms_per_step']*1e3, 1), d['end_state_sha256'][:16])"
