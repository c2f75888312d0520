# GPU box: round-5 closing run on the final tree: the round-end rehearsal (tools/gpu_final.sh: GPU
# suite, smoke, bench lines, 3-rank rehearsal), then the driver command's kernel trace and the PMC
# passes (tools/profile.sh) for profiles/.
set -u
cd /root/repo
export TMPDIR=/tmp
bash tools/gpu_final.sh || exit 1
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/driver_trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_trace.log 2>&1 || { tail -20 $O/driver_trace.log; exit 4; }
PROF_OUT=$O/prof CONFIGS="cfg4" bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 5; }
echo R05N_OK
