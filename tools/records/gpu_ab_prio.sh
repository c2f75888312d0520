# RECORD ONLY: the s_setprio variant this measured was not kept (profiles/r02_setprio_ab.txt).
# GPU box: s_setprio after the candidate scan (tools/_ab/p2, CBF_FLUSH_PRIO=2) vs the working tree
set -u
cd /root/repo
O=gpurun_out/abp; mkdir -p $O; : > $O/ab.txt
for sp in 0.145 0.2; do
  for rep in 1 2; do
    for t in . tools/_ab/p2; do
      timeout -k 10 120 python tools/ab_stats.py $t $sp 2>>$O/ab.err >> $O/ab.txt || { tail -5 $O/ab.err; exit 2; }
    done
  done
done
cat $O/ab.txt
