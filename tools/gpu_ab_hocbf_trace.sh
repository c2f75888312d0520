# GPU box: kernel traces of tools/ab_hocbf.py (60 HOCBF timesteps of the cfg4 lattice) for this tree and
# tools/_abt/nocert (or the trees in $TREES), twice each; prints per-kernel mean durations and the end state.
#   O=gpurun_out/<name> bash tools/gpu_ab_hocbf_trace.sh
set -u
cd /root/repo
export TMPDIR=/tmp
O=${O:-gpurun_out/hab}; mkdir -p $O
for rep in 1 2; do for t in ${TREES:-. tools/_abt/nocert}; do
  n=$(basename $t); [ "$t" = . ] && n=this
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$n.$rep -o run -- python3 tools/ab_hocbf.py $t > $O/$n.$rep.log 2>&1 || { tail $O/$n.$rep.log; exit 1; }
  echo "$n $(python3 tools/trace_gaps.py $O/$n.$rep/run_kernel_trace.csv 20 | head -1) | $(grep "^end" $O/$n.$rep.log)"
done; done
