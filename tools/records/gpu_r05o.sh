# GPU box: round-5 bench lines of the other configs on the final tree (README table).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
for C in cfg4f cfg4r cfg5 cfg3 cert; do
  timeout -k 10 400 python3 bench.py --config $C --no-cpu-baseline > $O/$C.json 2> $O/$C.err || { tail -20 $O/$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$C.json')); print('$C', '%.4g' % d['value'], d['unit'], round(d['ms_per_step']*1e3, 2))"
done
timeout -k 10 400 python3 bench.py --barrier euclidean_hocbf --steps 100 --warmup 20 --no-cpu-baseline > $O/hocbf.json 2> $O/hocbf.err || { tail -20 $O/hocbf.err; exit 2; }
python3 -c "import json; d=json.load(open('$O/hocbf.json')); print('hocbf', '%.4g' % d['value'], round(d['ms_per_step']*1e3, 2))"
