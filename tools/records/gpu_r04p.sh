# GPU box, round 4: the 128-row window (the N = 8 stripe) in detail: kernel traces of the window
# cull and the cell list, inline and queued solves.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
for c in window cells; do
  for pl in inline queued; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/${c}_$pl -o run -- python3 tools/ab_window.py . $c 0.145 128 $pl > $O/${c}_$pl.log 2>&1 || { tail -20 $O/${c}_$pl.log; exit 1; }
    grep "run(10)" $O/${c}_$pl.log
  done
done
echo R04P_OK
