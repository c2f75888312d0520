# GPU box, round 4: occupancy variants of the window path: tile kernel fitted to 8 waves per SIMD
# (4 blocks per CU, spills), build blocks of 512 threads, both; window tests on this tree first.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
for rep in 1 2; do
  for t in . tools/_abt/tw8 tools/_abt/pb512 tools/_abt/both; do
    timeout -k 10 120 python tools/ab_window.py $t window >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 2; }
    timeout -k 10 120 python tools/ab_window.py $t window 0.2 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 3; }
  done
done
grep -v amdgpu.ids $O/ab.txt
for t in tools/_abt/tw8 tools/_abt/pb512; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$(basename $t) -o run -- python3 tools/ab_window.py $t window > $O/trace_$(basename $t).log 2>&1 || { tail -20 $O/trace_$(basename $t).log; exit 4; }
done
echo R04T_OK
