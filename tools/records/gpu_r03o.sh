# GPU box, round 3: is the sharded step host-bound?  Host enqueue time per exchange cycle against
# wall time (tools/diag_shard_host.py), at 128 and 1024 rows, one RCCL rank.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 200 python tools/diag_shard_host.py 128 60 > $O/diag128.txt 2>$O/diag128.err || { tail -20 $O/diag128.err; exit 1; }
cat $O/diag128.txt
timeout -k 10 200 python tools/diag_shard_host.py 1024 30 > $O/diag1024.txt 2>$O/diag1024.err || { tail -20 $O/diag1024.err; exit 2; }
cat $O/diag1024.txt
echo R03O_OK
