#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): count, average duration,
and the gaps between consecutive dispatches.  Usage: trace_summary.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def short(name):
    name = name.replace("fea::", "").replace("(fea::MgArgs<double>)", "").replace("(fea::MgArgs<float>)", "")
    return name.replace("void ", "")[:60]


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups = defaultdict(list)
    for r in rows:
        g = (short(r["Kernel_Name"]), int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
        groups[g].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':60s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s}")
    for (k, grid), d in sorted(groups.items(), key=lambda x: -sum(x[1])):
        print(f"{k:60s} {grid:9d} {len(d):6d} {sum(d) / len(d) / 1e3:9.2f} {min(d) / 1e3:9.2f}")
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
    gaps = [g for g in gaps if 0 <= g < 50_000]
    if gaps:
        gaps.sort()
        print(f"inter-dispatch gaps (<50us): n={len(gaps)} median={gaps[len(gaps) // 2] / 1e3:.2f}us "
              f"mean={sum(gaps) / len(gaps) / 1e3:.2f}us")


if __name__ == "__main__":
    main(sys.argv[1])
