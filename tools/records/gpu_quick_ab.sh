# Quick A/B (no test suite, no profile): tools/ab_lattice.py for the working tree and the variant
# trees given as arguments (tools/_ab/<name>, built beforehand on the CPU), twice, interleaved.
set -u
cd /root/repo
O=gpurun_out/qab; mkdir -p $O; : > $O/ab.txt
for rep in 1 2; do
for t in . "$@"; do
  for sp in 0.145 0.2; do
    timeout -k 10 120 python tools/ab_lattice.py $t $sp 100 2>>$O/err.txt >> $O/ab.txt || exit 2
  done
done
done
cat $O/ab.txt
