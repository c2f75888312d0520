# GPU box, round 4: the HOCBF bench line (100 steps after 20) and its kernel trace after the unroll.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04aj; mkdir -p $O
timeout -k 10 400 python bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline > $O/hocbf.json 2> $O/hocbf.err || { tail -20 $O/hocbf.err; exit 1; }
python -c "import json; d=json.load(open('$O/hocbf.json')); print('hocbf', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2), d['end_state_sha256'][:16])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 2; }
echo R04AJ_OK
