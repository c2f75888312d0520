# GPU box, round 4: window cull against the cell list by window height (the sharded sub-steps'
# windows), auto solve placement.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
for rep in 1 2; do
  for h in 136 192 256 384 512; do
    for c in cells window; do
      timeout -k 10 120 python tools/ab_window.py . $c 0.145 $h >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
    done
  done
done
grep -v amdgpu.ids $O/ab.txt
echo R04R_OK
