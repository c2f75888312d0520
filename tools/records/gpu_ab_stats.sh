# GPU box: tools/ab_stats.py for the working tree and tools/_ab/head, interleaved, cfg4 and cfg4f
set -u
cd /root/repo
O=gpurun_out/abs; mkdir -p $O; : > $O/ab.txt
for sp in 0.145 0.2; do
  for rep in 1 2; do
    for t in . tools/_ab/head; do
      timeout -k 10 120 python tools/ab_stats.py $t $sp 2>>$O/ab.err >> $O/ab.txt || { tail -5 $O/ab.err; exit 2; }
    done
  done
done
cat $O/ab.txt
