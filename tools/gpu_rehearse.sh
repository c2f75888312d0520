# GPU box: the N>1 bench path rehearsed with 2 and 3 ranks on one GPU (gloo, host-staged exchange)
set -o pipefail
mkdir -p gpurun_out
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29560 + n)) bench.py --gpus $n --backend gloo --steps 20 --warmup 4 --rows 384 --no-cpu-baseline > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { tail -20 gpurun_out/rehearse_$n.err; exit 1; }
  cat gpurun_out/rehearse_$n.json
done
