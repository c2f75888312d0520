# GPU box: stall breakdown + cache counters of the lattice step kernels (separate PMC passes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/proff
mkdir -p $OUT
B="python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --kernel-iters 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum -f csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD -f csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1 || exit 3
echo done
