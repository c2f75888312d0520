# GPU box: kernel traces of the 1/8-stripe workload (128 x 1024 rows = 131,072 agents, the per-GPU
# share of the 1M lattice at 8 GPUs): single-GPU chained run and the sharded cycle at one rank.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/prof_small; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/single -o run -- python3 bench.py --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/single.json 2> $O/single.err || { tail -20 $O/single.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/shard -o run -- python3 bench.py --shard --rows 128 --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/shard.json 2> $O/shard.err || { tail -20 $O/shard.err; exit 2; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/full -o run -- python3 bench.py --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/full.json 2> $O/full.err || { tail -20 $O/full.err; exit 3; }
find $O -name "*kernel_stats.csv" | head
echo PROF_OK
