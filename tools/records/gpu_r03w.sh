# GPU box, round 3: cache-level counters of the lattice kernels at cfg4 (what bounds the filter):
# vector L1 (TCP) accesses / misses / stalls, L2 (TCC) hits / misses, texture addresser and data
# (TA / TD) busy -- one rocprofv3 --pmc pass per counter group (no pass exceeds a block's limit).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-iters 5"
i=0
for P in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_PENDING_STALL_CYCLES_sum" \
         "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -f csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit $i; }
done
echo R03W_OK
