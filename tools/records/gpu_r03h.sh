# GPU box, round 3 re-entry: where a cfg4 step goes now (scan fused into the scatter).
# Kernel traces of the driver's bench command and of the 200-step default, plus cfg4r.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_driver.json 2>$O/prof_driver.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_default -o run -- python3 bench.py --no-cpu-baseline > $O/prof_default.json 2>$O/prof_default.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_cfg4r -o run -- python3 bench.py --config cfg4r --no-cpu-baseline > $O/prof_cfg4r.json 2>$O/prof_cfg4r.err || exit 3
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_noprof.json 2>$O/driver_noprof.err || exit 4
echo R03H_OK
