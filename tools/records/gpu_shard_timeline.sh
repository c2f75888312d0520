# GPU box: kernel timeline of the sharded path at one rank: one exchange cycle in the timed region,
# every kernel's duration and the gap before it (rocprofv3 kernel trace with timestamps)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/shard_tl
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 bench.py --shard --steps 48 --warmup 8 --no-cpu-baseline --kernel-iters 1 > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
python3 - <<'PY' > gpurun_out/shard_tl/cycle.txt
import csv, glob, re
f = glob.glob("gpurun_out/shard_tl/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
packs = [i for i, r in enumerate(rows) if "halo_pack" in r["Kernel_Name"]]
print("exchanges", len(packs))
i0, i1 = packs[len(packs) // 2], packs[len(packs) // 2 + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = None
tot = {}
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^<>()]*>)?)|(__amd_rocclr_\w+)|(\w+Kernel\w*)", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(f"{(s - t0) / 1e3:9.2f} {name[:44]:44s} dur {(e - s) / 1e3:7.2f} gap {gap:7.2f}")
    tot[name] = tot.get(name, 0) + (e - s) / 1e3
    prev_end = e
print("cycle span us", (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3)
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k[:44]:44s} {v:8.2f}")
PY
cat gpurun_out/shard_tl/cycle.txt
