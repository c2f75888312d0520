# GPU box, round 4: where the window build's time goes (timing only; px1 = no nominal-control
# stores, px2 = no column-extent stores, px3 = no loads of the rows above and below; their results
# are not the build's), kernel traces.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04v; mkdir -p $O
for t in tools/_abt/head tools/_abt/px1 tools/_abt/px2 tools/_abt/px3; do
  n=$(basename $t)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 tools/ab_window.py $t window > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep "run(10)" $O/$n.log
done
echo R04V_OK
