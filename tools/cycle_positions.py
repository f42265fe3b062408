"""Per-position view of a V-cycle from a rocprofv3 kernel trace: the cycle is cut at every launch of the
finest level's kernel (default: the cycle join), and for each position in the cycle the median duration
and the median gap from the previous kernel's end are printed (separates levels that share one kernel
name, e.g. the level-1 and level-2 residual-restriction launches).
    python tools/cycle_positions.py <trace dir or run_kernel_trace.csv> [anchor substring]"""
import csv
import glob
import os
import statistics
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_mg_cycle_join"
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    cycles, cur = [], None
    for s, e, n in rows:
        if anchor in n:
            if cur:
                cycles.append(cur)
            cur = []
        if cur is not None:
            cur.append((s, e, n))
    # keep the most common cycle shape
    shapes = {}
    for c in cycles:
        shapes.setdefault(tuple(n for _, _, n in c), []).append(c)
    shape, cs = max(shapes.items(), key=lambda kv: len(kv[1]))
    print(f"{len(cs)} cycles of {len(shape)} launches")
    tot = []
    for i, name in enumerate(shape):
        d = statistics.median((c[i][1] - c[i][0]) / 1e3 for c in cs)
        g = statistics.median((c[i][0] - c[i - 1][1]) / 1e3 for c in cs) if i else float("nan")
        tot.append(d)
        short = name.split("(")[0][:70]
        print(f"{i:3d}  {d:8.2f} us  gap {g:6.2f} us  {short}")
    span = statistics.median((c[-1][1] - c[0][0]) / 1e3 for c in cs)
    print(f"sum of medians {sum(tot):.2f} us, median first-start to last-end {span:.2f} us")


if __name__ == "__main__":
    main()
