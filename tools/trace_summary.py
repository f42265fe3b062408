#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace per (kernel, grid size): count, average duration, and the
gaps between consecutive dispatches.  Accepts the CSV (`*_kernel_trace.csv`) or the rocpd SQLite
output (`*_results.db`, rocprofv3's default format in ROCm 7), or a directory holding either.
Usage: trace_summary.py <csv | db | dir>"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = name.replace("fea::", "").replace("(fea::MgArgs<double>)", "").replace("(fea::MgArgs<float>)", "")
    return name.replace("void ", "")[:60]


def load(path):
    """-> list of (name, grid_x, start_ns, end_ns)."""
    if os.path.isdir(path):
        cand = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) +
                      glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
        if not cand:
            raise SystemExit(f"no kernel trace under {path}")
        path = cand[0]
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        return [(n, int(g), int(s), int(e)) for n, g, s, e in
                con.execute("select name, grid_x, start, end from kernels")]
    rows = list(csv.DictReader(open(path)))
    return [(r["Kernel_Name"], int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
             int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]


def main(path):
    rows = sorted(load(path), key=lambda r: r[2])
    groups = defaultdict(list)
    for name, grid, s, e in rows:
        groups[(short(name), grid)].append(e - s)
    print(f"{'kernel':60s} {'grid':>9s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s}")
    for (k, grid), d in sorted(groups.items(), key=lambda x: -sum(x[1])):
        print(f"{k:60s} {grid:9d} {len(d):6d} {sum(d) / len(d) / 1e3:9.2f} {min(d) / 1e3:9.2f}")
    gaps = [b[2] - a[3] for a, b in zip(rows, rows[1:])]
    gaps = [g for g in gaps if 0 <= g < 50_000]
    if gaps:
        gaps.sort()
        print(f"inter-dispatch gaps (<50us): n={len(gaps)} median={gaps[len(gaps) // 2] / 1e3:.2f}us "
              f"mean={sum(gaps) / len(gaps) / 1e3:.2f}us")


if __name__ == "__main__":
    main(sys.argv[1])
