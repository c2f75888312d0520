# GPU box, round 3: the multi-rank bench paths rehearsed on one GPU with gloo: the bench test file
# (2, 4 and 8 ranks vs the 1-rank end state), then --gpus 4 and --gpus 8 at the full 1 M lattice
# (256 and 128 rows per rank, as the driver's N = 4 / 8 runs split it).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03r; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for n in 4 8; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=2957$n timeout -k 10 300 python bench.py --gpus $n --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/rehearse_$n.json 2> $O/rehearse_$n.err || { tail -20 $O/rehearse_$n.err; exit 2; }
  cat $O/rehearse_$n.json
done
echo R03R_OK
