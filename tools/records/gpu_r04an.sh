# GPU box, round 4: the tile's candidate-row loop unrolled by 2 / 3 against 1 (this tree).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04an; mkdir -p $O
for rep in 1 2; do
  for t in . tools/_abt/ru2 tools/_abt/ru3; do
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.2 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 3; }
  done
done
grep -v amdgpu.ids $O/ab.txt
echo R04AL_OK
