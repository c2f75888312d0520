# GPU box, round 3: timing probes of the filter's hit flush (tools/_ab/probe<k>, CBF_PROBE: 1 no
# position gather, 2 no velocity gather, 3 neither; results deliberately wrong) against this tree:
# the filter kernel's average duration under a kernel trace at cfg4.
set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r03t; mkdir -p $O; : > $O/probe.txt
for t in . tools/_ab/probe1 tools/_ab/probe2 tools/_ab/probe3; do
  n=$(basename $t)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/p_$n -o run -- python3 tools/ab_lattice.py $t 0.145 60 > $O/p_$n.txt 2>&1 || exit 1
  python3 -c "
import csv
r=list(csv.DictReader(open('$O/p_$n/run_kernel_stats.csv')))
for x in r:
    if 'k_lattice_filter<' in x['Name'] or 'filter_hard' in x['Name']: print('$n', x['Name'][37:70], x['Calls'], round(float(x['AverageNs'])/1e3, 2))
" >> $O/probe.txt
done
cat $O/probe.txt
echo R03T_OK
