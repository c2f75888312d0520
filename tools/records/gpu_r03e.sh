# GPU box: where the small-stripe step's time goes: kernel traces at 131k agents with the default
# spacing, with no neighbours at all (spacing 0.5: every queue empty, every ego idle) and with few.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
for sp in 0.5 0.3 0.145; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_sp$sp -o run -- python3 bench.py --rows 128 --spacing $sp --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 2 > $O/sp$sp.json 2>$O/sp$sp.err || exit 1
done
echo R03E_OK
