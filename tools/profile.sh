#!/bin/bash
# Profiling recipe run on the GPU box (gpurun): per config, a kernel-trace pass and separate PMC
# passes (FETCH_SIZE and WRITE_SIZE never share a pass; MI355X_MICROARCH.md "rocprofv3 PMC slots").
#   CONFIGS="cfg4 cfg4f cfg5" bash tools/profile.sh      -> gpurun_out/prof/<config>/...
#   (cfg4_hocbf: the cfg4 shape with --barrier euclidean_hocbf)
# then, back in the container: python tools/summarize_profile.py gpurun_out/prof r02
set -o pipefail
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
for C in ${CONFIGS:-cfg4 cfg4f cfg5}; do
  D=$OUT/$C
  mkdir -p $D
  if [ $C = cfg5 ]; then
    B="python3 bench.py --config cfg5 --steps 3 --warmup 1"
    SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
  elif [ $C = cfg4_hocbf ]; then
    B="python3 bench.py --config cfg4 --barrier euclidean_hocbf --steps 40 --warmup 10 --no-cpu-baseline --no-exact-qp"
    SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
  else
    B="python3 bench.py --config $C --steps 60 --warmup 20 --no-cpu-baseline --no-exact-qp --kernel-iters 10"
    SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- $B > $D/trace.log 2>&1 || exit 1
  if [ $C != cfg5 ]; then
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $D/pmc_fetch -o run -- $B > $D/pmc_fetch.log 2>&1 || exit 2
    timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $D/pmc_write -o run -- $B > $D/pmc_write.log 2>&1 || exit 3
  fi
  timeout -s KILL 200 rocprofv3 --pmc $SQ -f csv -d $D/pmc_sq -o run -- $B > $D/pmc_sq.log 2>&1 || exit 4
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -f csv -d $D/pmc_grbm -o run -- $B > $D/pmc_grbm.log 2>&1 || exit 5
done
echo profile-done
