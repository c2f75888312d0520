# GPU box: kernel trace + SQ counters of the cfg5 Monte-Carlo rollout kernel
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof5
mkdir -p $OUT
B="python3 bench.py --config cfg5 --steps 2 --warmup 1 --mc-scenarios 100000"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -f csv -d $OUT/pmc1 -o run -- $B > $OUT/pmc1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_LDS -f csv -d $OUT/pmc2 -o run -- $B > $OUT/pmc2.log 2>&1 || exit 3
echo done
