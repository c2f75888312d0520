# GPU box: tools/ab_lattice.py timings (step, advance, run(10)) of the working tree and variant
# trees, interleaved, 2 repetitions.  usage: SP=0.145 bash tools/gpu_ab_quick.sh <tree> ...
set -u
cd /root/repo
O=gpurun_out/abq; mkdir -p $O; : > $O/ab.txt
for rep in ${REPS:-1 2}; do
  for t in . "$@"; do
    timeout -k 10 120 python tools/ab_lattice.py $t ${SP:-0.145} 100 2>/dev/null >> $O/ab.txt || exit 2
  done
done
cat $O/ab.txt
