# GPU box, round 3: the unsharded lattice step at the window heights an interior rank of the
# N = 8 strong-scaled run computes (128 owned rows + up to 2 x 60 ghost rows at 16 sub-steps), for
# the per-rank cost model of DESIGN.md sec. 5 (a one-rank sharded run has no ghost rows).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O; : > $O/rows.txt
for rep in 1 2; do
  for h in 128 160 192 224 256; do
    timeout -k 10 120 python tools/ab_lattice.py . 0.145 200 $h 2>/dev/null >> $O/rows.txt || exit 2
  done
done
cat $O/rows.txt
echo R03G_OK
