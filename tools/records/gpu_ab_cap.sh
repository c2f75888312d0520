# RECORD ONLY: the hit-list cap variants this measured were not kept (profiles/r02_hitcap_ab.txt).
# GPU box: hit-list cap A/B (tools/_ab/c14, c12 vs the working tree's 16), tools/ab_stats.py, cfg4 and cfg4f
set -u
cd /root/repo
O=gpurun_out/abcap; mkdir -p $O; : > $O/ab.txt
for sp in 0.145 0.2; do
  for rep in 1 2; do
    for t in . tools/_ab/c14 tools/_ab/c12; do
      timeout -k 10 120 python tools/ab_stats.py $t $sp 2>>$O/ab.err >> $O/ab.txt || { tail -5 $O/ab.err; exit 2; }
    done
  done
done
cat $O/ab.txt
