"""Condense a tools/profile.sh output directory into the committed profiles/ summaries.

  python tools/summarize_profile.py gpurun_out/prof r02

For every config directory (cfg4, cfg4f, cfg5): profiles/<round>_<config>_kernel_stats.csv
(rocprofv3 --stats, verbatim) and one entry per kernel in profiles/<round>_pmc.json (mean counter
values per dispatch).  profiles/pmc_summary.json keeps, per config, what bench.py reads:
  * HBM bytes per launch (the roofline `traffic` field), following MI355X_MICROARCH.md "HBM":
    FETCH_SIZE and WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE counts half the bytes of
    16-B-per-lane streaming reads, so the read side is 2 x FETCH_SIZE (the kernels' loads are
    16-B double2 loads);
  * for cfg5 (k_mc_rollout, state in LDS, VALU-bound), the VALU busy fraction by the gfx9 formula
    rocprofv3 falls back to on gfx950: SQ_ACTIVE_INST_VALU (quad-cycles, summed over SIMDs) x 4 /
    (SIMDs x cycles of the dispatch).  GRBM_GUI_ACTIVE comes summed over the 8 XCDs (per dispatch it
    reads 8 x 2.3 GHz x the kernel's duration), so the dispatch's cycles are GRBM_GUI_ACTIVE / 8;
    the implied clock is recorded beside it.
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
SIMDS = 256 * 4   # MI355X: 256 CUs x 4 SIMDs
XCDS = 8


def short(name: str) -> str:
    """Kernel name with its template arguments (the lattice filter has one instantiation per
    statistics mode: k_lattice_filter<FZ, ST>)."""
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^<>()]*>)?)", name)
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


def summarize(prof, cfg, rnd):
    d = os.path.join(prof, cfg)
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{rnd}_{cfg}_kernel_stats.csv"))
    dur = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    pmc = collections.defaultdict(dict)
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_grbm"):
        for k, e in counters(os.path.join(d, sub, "run_counter_collection.csv")).items():
            pmc[k].update(e)
    out = {}
    for k, e in pmc.items():
        e = dict(e)
        e["avg_duration_ns"] = dur.get(k)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["fetch_bytes_raw"] = e["FETCH_SIZE"] * 1024
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if "SQ_ACTIVE_INST_VALU" in e and e.get("GRBM_GUI_ACTIVE"):
            cyc = e["GRBM_GUI_ACTIVE"] / XCDS
            e["valu_busy"] = e["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc)
            if e.get("avg_duration_ns"):
                e["implied_clock_ghz"] = cyc / e["avg_duration_ns"]
        if "SQ_ACTIVE_INST_VALU" in e and e.get("avg_duration_ns"):
            # clock-corrected form (MI355X_MICROARCH.md, DVFS note: GRBM_GUI_ACTIVE / 8 reads high on
            # dispatches shorter than ~0.3 ms): VALU issue cycles over the SIMD cycles the dispatch's
            # traced duration holds at the 2.4 GHz peak clock -- a lower bound of the busy fraction
            e["valu_busy_2p4ghz"] = e["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * e["avg_duration_ns"] * 2.4)
        out[k] = e
    return out


def main(prof, rnd):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    allk = {}
    for cfg in sorted(os.listdir(prof)):
        if not os.path.exists(os.path.join(prof, cfg, "trace", "run_kernel_stats.csv")):
            continue
        allk[cfg] = summarize(prof, cfg, rnd)
    # merged per config into what is already there (a run may profile a subset of the configs)
    for name, extra in ((f"{rnd}_pmc.json", {}), ("pmc_summary.json", {"round": rnd})):
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as f:
                old = json.load(f)
        except (OSError, ValueError):
            old = {}
        old.update(allk)
        old.update(extra)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)
    for cfg, ks in allk.items():
        print(cfg)
        for k, e in sorted(ks.items(), key=lambda kv: -(kv[1].get("avg_duration_ns") or 0)):
            print(f"  {k:30s} dur={((e.get('avg_duration_ns') or 0) / 1e3):8.2f} us  "
                  f"hbm={(e.get('hbm_bytes_per_launch') or 0) / 1e6:8.2f} MB  valu_busy={e.get('valu_busy')} "
                  f"(at 2.4 GHz {e.get('valu_busy_2p4ghz')})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
