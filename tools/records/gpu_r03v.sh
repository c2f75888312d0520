# GPU box, round 3: the HOCBF-mode cfg4 line, and the driver's cfg4 command twice more (run-to-run
# spread of the headline on one box).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 3; }; python -c "import json; d=json.load(open('$O/$n.json')); print('$n', '%.4g'%d['value'], round(d['ms_per_step']*1e3, 2))"; }
run hocbf --barrier euclidean_hocbf --steps 200 --warmup 20 --no-cpu-baseline
run driver_a --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run driver_b --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo R03V_OK
