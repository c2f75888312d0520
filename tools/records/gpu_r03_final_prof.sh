# GPU box, round 3 (final tree): the kernel trace of the driver's exact bench command, then the
# PMC passes of tools/profile.sh for cfg4, cfg4r and cfg5.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03_prof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2>$O/driver.err || exit 1
PROF_OUT=$O CONFIGS="cfg4 cfg4r cfg5" bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 2; }
echo PROF_OK
