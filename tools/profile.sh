#!/bin/bash
# Profiling recipe run on the GPU box (gpurun): kernel-trace stats + separate PMC passes.
set -o pipefail
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
B="python3 bench.py --steps 150 --warmup 40 --no-cpu-baseline --kernel-iters 10 ${BENCH_EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -f csv -d $OUT/pmc_sq -o run -- $B > $OUT/pmc_sq.log 2>&1 || exit 4
echo profile-done
