"""Idle gaps between consecutive dispatches of a rocprofv3 kernel trace (run_kernel_trace.csv):
per (previous kernel -> next kernel) pair, the count and mean / median gap in us, and the mean
duration of each kernel.  `python tools/trace_gaps.py <kernel_trace.csv> [min_count]`."""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+|spin_kernel|copyBuffer|fillBuffer\w*|\w+_kernel)", name)
    return m.group(1) if m else name[:30]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    min_count = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    gaps, durs = defaultdict(list), defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = short(r["Kernel_Name"])
        durs[n].append((e - s) / 1e3)
        if prev is not None:
            gaps[(prev[0], n)].append((s - prev[1]) / 1e3)
        prev = (n, e)
    print("kernel durations (us): " + ", ".join(f"{k} {statistics.mean(v):.2f} x{len(v)}" for k, v in durs.items()
                                                 if len(v) >= min_count))
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        if len(v) >= min_count:
            print(f"{a:>34} -> {b:<34} n={len(v):5d} mean {statistics.mean(v):8.2f} median {statistics.median(v):8.2f}")


if __name__ == "__main__":
    main()
