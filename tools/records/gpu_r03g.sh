# GPU box: the small-window inline-solve filter (CBF_INLINE_MAX): GPU tests of the lattice paths,
# then A/B of the default build against never-inline and always-inline trees over window sizes.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O; : > $O/ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for rows in 64 128 256 512 1024; do
    for t in . tools/_ab/noinline tools/_ab/allinline; do
      timeout -k 10 120 python tools/ab_lattice.py $t 0.145 100 $rows 2>/dev/null >> $O/ab.txt || exit 2
    done
  done
done
cat $O/ab.txt
echo R03G_OK
