# GPU box, round 3: sub-steps per exchange at the N = 4 and N = 2 stripes of the 1 M lattice (256
# and 512 rows, one RCCL rank), 8 against 16 (12 at 256 rows).
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O; : > $O/k.txt
for rep in 1 2; do
  for rk in 256:8 256:12 256:16 512:8 512:16; do
    r=${rk%%:*}; k=${rk##*:}
    timeout -k 10 200 python bench.py --shard --weak --rows $r --substeps $k --steps 96 --warmup 16 --no-cpu-baseline > $O/r${r}k$k.json 2>$O/r${r}k$k.err || { tail -20 $O/r${r}k$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/r${r}k$k.json')); print('rows $r k $k', round(d['ms_per_step']*1e3, 2))" >> $O/k.txt
  done
done
cat $O/k.txt
echo R03S_OK
