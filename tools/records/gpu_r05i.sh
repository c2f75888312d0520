# GPU box: HOCBF neighbour histogram, then the main kernel's LDS-rows / unroll A/B (tools/_abt trees).
set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gpu/diag_hocbf_nbrs.py > gpurun_out/hnbrs.txt 2>&1 || { tail -20 gpurun_out/hnbrs.txt; exit 1; }
cat gpurun_out/hnbrs.txt
bash tools/gpu_ab_hocbf.sh tools/_abt/base tools/_abt/u4 tools/_abt/r6u4 tools/_abt/r5u4 tools/_abt/r6u2 tools/_abt/base tools/_abt/r6u4 tools/_abt/r5u4
