# GPU box, round 5: the HOCBF tests, then the HOCBF bench line and its kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hocbf.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --barrier euclidean_hocbf --steps 60 --warmup 20 --no-cpu-baseline > $O/hocbf.json 2> $O/hocbf.err || { tail -20 $O/hocbf.err; exit 2; }
python -c "import json; d=json.load(open('$O/hocbf.json')); print('hocbf', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), d.get('end_state_sha256', '')[:16])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --barrier euclidean_hocbf --steps 60 --warmup 20 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 3; }
f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]:
    print(f\"{r['Name'][:60]:60s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:8.2f}\")
"
