# GPU box, round 3: kernel traces of the small windows (128-row lattice, and the sharded 128-row
# stripe at one rank with 16 sub-steps), to see where a strong-scaled step goes.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/rows128 -o run -- python3 bench.py --rows 128 --no-cpu-baseline --steps 100 --warmup 10 > $O/rows128.json 2>$O/rows128.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/shard128 -o run -- python3 bench.py --shard --weak --rows 128 --steps 96 --warmup 16 --no-cpu-baseline > $O/shard128.json 2>$O/shard128.err || exit 2
echo R03S_OK
