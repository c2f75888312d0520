# GPU box, round 4: diagnose the 2-rank gloo rehearsal with the window cull (335 ms per step): the
# same with the row guard from the separate scan kernel (no in-launch hand-off: fold0), a kernel
# trace of the slow run, and the 1-rank sharded step at 512 rows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04ad; mkdir -p $O
run() { n=$1; shift; timeout -k 10 600 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['config'].get('cull'), d['n_gpus'], '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"; }
run shard512 --shard --rows 512 --steps 8 --warmup 2 --no-cpu-baseline --cull window --kernel-iters 2
run gloo2_short --gpus 2 --backend gloo --steps 4 --warmup 1 --no-cpu-baseline --cull window --kernel-iters 2
cd tools/_abt/fold0 && ln -sf ../../../bench.py bench.py && ln -sf ../../../oracle oracle && cd ../../..
(cd tools/_abt/fold0 && timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 4 --warmup 1 --no-cpu-baseline --cull window --kernel-iters 2 > ../../../$O/gloo2_fold0.json 2> ../../../$O/gloo2_fold0.err) || { tail -20 $O/gloo2_fold0.err; exit 4; }
python -c "import json; d=json.load(open('$O/gloo2_fold0.json')); print('gloo2_fold0', d['config'].get('cull'), d['n_gpus'], '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
echo R04AD_OK
