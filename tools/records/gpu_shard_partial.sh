# GPU box: shard tests, then the sharded bench at one rank with the driver's arguments
# (--steps 20 --warmup 5) and at the defaults, working tree vs tools/_ab/base, interleaved.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/shp; mkdir -p $O; : > $O/res.txt
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for t in . tools/_ab/base; do
    for A in "--steps 20 --warmup 5" "--steps 200 --warmup 20" ${EXTRA:+"$EXTRA"}; do
      timeout -k 10 200 python $t/bench.py --shard --no-cpu-baseline --kernel-iters 2 $A > $O/b.json 2>/dev/null || exit 2
      python -c "import json; d=json.load(open('$O/b.json')); print('$t', '$A', round(d['ms_per_step']*1e3, 2), 'us/step')" >> $O/res.txt
    done
  done
done
cat $O/res.txt
