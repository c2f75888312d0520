# GPU box: kernel durations per timestep over the first 40 timesteps of cfg4 (one run(40) call)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/steps
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 tools/steps_profile.py > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
python3 - <<'PY'
import csv, glob, re
f = glob.glob("gpurun_out/steps/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "k_lattice" in r["Kernel_Name"] or "k_scan" in r["Kernel_Name"]]
step, cur = [], {}
for r in rows:
    n = re.search(r"(k_[A-Za-z_]+)", r["Kernel_Name"]).group(1)
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n == "k_scan_onepass" and cur:
        step.append(cur); cur = {}
    cur[n] = cur.get(n, 0) + d
step.append(cur)
for i, c in enumerate(step):
    print(i + 1, " ".join(f"{k[2:]}={v:.1f}" for k, v in c.items()), f"sum={sum(c.values()):.1f}")
PY
