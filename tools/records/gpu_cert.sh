# GPU box: batched coupled barrier-certificate throughput (bench.py --config cert) at N = 4, 16, 32
set -o pipefail
mkdir -p gpurun_out
for n in 16 4 8 32; do
  timeout -k 10 200 python bench.py --config cert --cert-agents $n --steps 10 --warmup 2 > gpurun_out/bench_cert$n.json 2> gpurun_out/bench_cert$n.err || { echo CERT_FAILED $n; tail gpurun_out/bench_cert$n.err; exit 1; }
  cat gpurun_out/bench_cert$n.json
done
