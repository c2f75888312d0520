bash tools/gpu_ab.sh tools/_ab/base || exit 1
mkdir -p gpurun_out/r02 && timeout -k 10 400 python bench.py --shard --no-cpu-baseline > gpurun_out/r02/bench_shard.json 2> gpurun_out/r02/bench_shard.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/r02/bench_shard.json')); print('shard', d['value'], d['ms_per_step'])"
