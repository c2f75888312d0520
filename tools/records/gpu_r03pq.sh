# GPU box, round 3: queue-kernel grid of 4 or 8 blocks per sub-queue (tools/_ab/pq4, pq8) against
# the shipped 32 (tools/_ab/base = this tree), at strong-scaled window heights and at 1 M agents.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03pq; mkdir -p $O; : > $O/ab.txt
for rep in 1 2; do
  for t in tools/_ab/pq4 tools/_ab/pq8 tools/_ab/base; do
    for h in 136 192; do timeout -k 10 120 python tools/ab_lattice.py $t 0.145 200 $h 2>/dev/null >> $O/ab.txt || exit 2; done
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.2 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
echo R03PQ_OK
