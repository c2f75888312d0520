# GPU box, round 4: the inline-solve window tile fitted to 4 / 6 waves per SIMD (spilling the rare
# solve path) against the unfitted one and the queued solve, at 1 M agents and 128 rows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python tools/ab_window.py . window 0.145 1024 queued >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
  for t in . tools/_abt/in4 tools/_abt/in6; do
    timeout -k 10 120 python tools/ab_window.py $t window 0.145 1024 inline >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.145 128 inline >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 3; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.2 1024 inline >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 4; }
  done
  timeout -k 10 120 python tools/ab_window.py . window 0.2 1024 queued >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 5; }
done
grep -v amdgpu.ids $O/ab.txt
echo R04Q_OK
