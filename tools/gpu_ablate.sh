# GPU box: A/B timings of kernel variants built by tools/ablate.py (ABLATE_SET picks the set)
set -o pipefail
mkdir -p gpurun_out
cmd=${ABLATE_CMD:-run}
timeout -k 10 300 python tools/ablate.py $cmd > gpurun_out/ablate.json 2> gpurun_out/ablate.err || { tail gpurun_out/ablate.err; exit 2; }
cat gpurun_out/ablate.json
