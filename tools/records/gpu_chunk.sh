# GPU box: timesteps per cbf_lattice_run graph (bench --chunk), driver arguments and defaults
set -u
cd /root/repo
O=gpurun_out/chunk; mkdir -p $O; : > $O/res.txt
for rep in 1 2; do
  for c in 10 20 50; do
    for a in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --kernel-iters 2 --chunk $c $a > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 2; }
      python -c "import json; d=json.load(open('$O/b.json')); print('chunk $c', '$a', round(d['ms_per_step']*1e3, 2))" >> $O/res.txt
    done
  done
done
cat $O/res.txt
