# GPU box, round 3: where the queue kernel's ~9.8 us go. Kernel traces of the shipped tree and two
# timing-only probes (tools/_ab/nosolve: the solve replaced by u = 0; tools/_ab/nobin: the chained
# binning atomic replaced by rank 0), cfg4 spacing and cfg4r.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03y; mkdir -p $O
for t in . tools/_ab/nosolve tools/_ab/nobin; do
  n=$(basename $t); [ "$n" = "." ] && n=ship
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/$n.txt 2>&1 || exit 2
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/${n}_rw -o run -- python3 tools/ab_lattice.py $t 0.22 60 1024 rw > $O/${n}_rw.txt 2>&1 || exit 3
done
echo R03Y_OK
