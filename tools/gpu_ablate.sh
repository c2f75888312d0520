# GPU box: parity tests, then the filter-kernel A/B timings (tools/ablate.py)
set -o pipefail
mkdir -p gpurun_out
true
true
timeout -k 10 300 python tools/ablate.py run > gpurun_out/ablate.json 2> gpurun_out/ablate.err || { tail gpurun_out/ablate.err; exit 2; }
python -c "
import json; d=json.load(open('gpurun_out/ablate.json'))
for k,v in d.items(): print(f'{k:16s} build {v[\"build\"][\"median_us\"]:7.1f}  advance {v[\"advance\"][\"median_us\"]:7.1f}')"
