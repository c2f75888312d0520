# GPU box, round 3: timing probes of the queue kernel with the done counter removed (queue reset
# moved into the next scan_scatter; tools/_ab/r16, r32, r64: 3, 2, 1 lanes per wave at cfg4)
# against the committed tree (tools/_ab/base). Probes only: not a shippable queue protocol.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03z3; mkdir -p $O; : > $O/ab.txt
true

for t in tools/_ab/r16 tools/_ab/r32 tools/_ab/r64 tools/_ab/base; do
  n=$(basename $t)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 3
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_rw -o run -- python3 tools/ab_lattice.py $t 0.22 60 1024 rw > $O/${n}_rw.txt 2>&1 || exit 4
done
for rep in 1 2; do
  for t in tools/_ab/r16 tools/_ab/r32 tools/_ab/r64 tools/_ab/base; do
    timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 2>/dev/null >> $O/ab.txt || exit 2
    timeout -k 10 120 python tools/ab_lattice.py $t 0.22 100 1024 rw 2>/dev/null >> $O/ab.txt || exit 2
  done
done
sort $O/ab.txt
echo R03Z3_OK
