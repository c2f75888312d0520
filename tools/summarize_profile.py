"""Condense a tools/profile.sh output directory into the committed profiles/ summaries.

  python tools/summarize_profile.py gpurun_out/prof r01

writes profiles/<round>_kernel_stats.csv (rocprofv3 --stats, verbatim), profiles/<round>_pmc.json
(mean counter values per kernel) and profiles/pmc_summary.json (read by bench.py for the
roofline `traffic` field).  HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads,
so the corrected read side is 2 x FETCH_SIZE (the filter kernels' loads are 16-B double2 loads).
"""
from __future__ import annotations

import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name[:40]


def counters(path):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        out[k][c] = sum(v) / len(v)
        out[k]["dispatches"] = len(v)
    return out


def main(prof, rnd):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{rnd}_kernel_stats.csv"))
    dur = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    pmc = collections.defaultdict(dict)
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq"):
        for k, d in counters(os.path.join(prof, sub, "run_counter_collection.csv")).items():
            pmc[k].update(d)
    summary = {}
    for k, d in pmc.items():
        e = dict(d)
        e["avg_duration_ns"] = dur.get(k)
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["fetch_bytes_raw"] = d["FETCH_SIZE"] * 1024
            e["write_bytes"] = d["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        summary[k] = e
    with open(os.path.join(ROOT, "profiles", f"{rnd}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    # merged: kernels of an earlier summary that this run did not profile are kept
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    merged = {}
    if os.path.exists(path):
        merged = {k: v for k, v in json.load(open(path)).items() if isinstance(v, dict)}
    merged.update(summary)
    with open(path, "w") as f:
        json.dump({"round": rnd, **merged}, f, indent=1, sort_keys=True)
    for k, e in sorted(summary.items(), key=lambda kv: -(kv[1].get("avg_duration_ns") or 0)):
        print(f"{k:28s} dur={((e.get('avg_duration_ns') or 0) / 1e3):8.2f} us  "
              f"hbm={(e.get('hbm_bytes_per_launch') or 0) / 1e6:8.2f} MB  valu={e.get('SQ_INSTS_VALU', 0):.3g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
