# GPU box, round 6: A/B of the tile's tail solve (this tree) against the queue kernel (tools/_abt/base,
# built with CBF_TAIL_SOLVE=0), run(10) at 1 M agents (cfg4, cfg4f) and at 128 / 256 rows (inline vs
# queued placement), interleaved, then the driver bench line and its kernel trace.
#   O=gpurun_out/<name> bash tools/gpu_ab_ts.sh
set -u
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=${O:-gpurun_out/ab_ts}; mkdir -p $O
for rep in 1 2; do
  for t in tools/_abt/base .; do
    timeout -k 10 120 python tools/ab_window.py $t window 0.145 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 3; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.2 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 3; }
    for rows in 128 256; do
      for pl in auto queued; do
        timeout -k 10 120 python tools/ab_window.py $t window 0.145 $rows $pl >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 3; }
      done
    done
  done
done
grep run $O/ab.txt
O=$O TESTS=none BENCH_REPS=2 bash tools/gpu_iter.sh
