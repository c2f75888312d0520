# GPU box, round 4: window build blocks of 128 / 64 threads (8 / 16 columns per thread) against
# 256 (this tree), kernel traces.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
for t in . tools/_abt/pb128 tools/_abt/pb64; do
  n=$(basename $(realpath $t))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_window.py $t window > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep "run(10)" $O/$n.log
done
for t in . tools/_abt/pb128 tools/_abt/pb64 .; do timeout -k 10 120 python tools/ab_window.py $t window 2>&1 | grep "run(10)"; done
echo R04W_OK
