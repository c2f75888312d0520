# HOCBF-mode bench line (steps 100, warm-up 20, as round 4) for each A/B tree given (a tree holds
# its own copy of bench.py): time and end state.  Usage: bash tools/gpu_ab_hocbf.sh <tree>...
set -u
cd /root/repo
for t in "$@"; do
  timeout -k 10 300 python3 $t/bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/hab.json 2> gpurun_out/hab.err || { tail -5 gpurun_out/hab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hab.json')); print('$t', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2), d.get('end_state_sha256', '')[:16])"
done
