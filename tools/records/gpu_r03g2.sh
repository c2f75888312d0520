# GPU box, round 3: inline-solve filter (this tree, windows <= CBF_INLINE_MAX agents) against the
# queue form (tools/_ab/noin, CBF_INLINE_MAX=0) at the window heights of a strong-scaled interior
# rank, to place the crossover.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03g2; mkdir -p $O; : > $O/rows.txt
for rep in 1 2; do
  for h in 128 136 144 152 160 176 192; do
    for t in . tools/_ab/noin; do
      timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 $h 2>/dev/null >> $O/rows.txt || exit 2
    done
  done
done
sort -k5,5n -s $O/rows.txt
echo R03G2_OK
