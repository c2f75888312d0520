# GPU box, round 4: where the per-tile row guard's time goes (timing only: tg1 = no pass over the
# rows, tg2 = no reductions either; their results are not the guard's), against fold0 (rowscan
# kernel) and this tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
for rep in 1 2; do
  for t in tools/_abt/fold0 . tools/_abt/tg1 tools/_abt/tg2; do
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
  done
done
grep -v amdgpu.ids $O/ab.txt
echo R04L_OK
