# GPU box, round 3: sub-steps per exchange at the strong-scaled stripe (128 rows, one RCCL rank):
# fewer sub-steps = fewer ghost rows recomputed, more exchanges.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03r2; mkdir -p $O; : > $O/k.txt
for rep in 1 2; do
  for k in 8 10 12 16; do
    timeout -k 10 200 python bench.py --shard --weak --rows 128 --substeps $k --steps 96 --warmup 16 --no-cpu-baseline > $O/k$k.json 2>$O/k$k.err || { tail -20 $O/k$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/k$k.json')); print('k $k', round(d['ms_per_step']*1e3, 2), d['config']['parallelism'])" >> $O/k.txt
  done
done
cat $O/k.txt
echo R03R_OK
