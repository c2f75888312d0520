# GPU box: kernel traces of tools/ab_window.py (cfg4 spacing, 1 M agents, window cull) for each
# source tree named in $TREES (default: this tree and every tools/_abt/* variant), one rocprofv3
# --kernel-trace --stats pass each; prints the per-launch averages of the window kernels.
#   O=gpurun_out/<name> TREES=". tools/_abt/x" bash tools/gpu_prof_trees.sh
set -u
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=${O:-gpurun_out/prof_trees}; mkdir -p $O
TREES=${TREES:-". $(ls -d tools/_abt/* 2>/dev/null | tr '\n' ' ')"}
SP=${SPACING:-0.145}
for rep in 1 2; do
  for t in $TREES; do
    n=$(basename $t); [ "$t" = . ] && n=this
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$n.$rep -o run -- python3 tools/ab_window.py $t window $SP > $O/$n.$rep.log 2>&1 || { tail $O/$n.$rep.log; exit 1; }
    f=$(find $O/$n.$rep -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$n" "$(grep run $O/$n.$rep.log)" <<'PY'
import csv, re, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", r["Name"])
    if m and ("window" in m.group(1) or "hard" in m.group(1)):
        out.append(f"{m.group(1)}{m.group(2) or ''} {float(r['AverageNs']) / 1e3:.2f}")
print(sys.argv[2], " | ".join(out), "|", sys.argv[3].split(":")[-1].strip())
PY
  done
done
