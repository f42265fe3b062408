#!/usr/bin/env python3
"""Per-kernel mean of every counter in one or more rocprofv3 --pmc counter_collection.csv files.
usage: pmc_table.py CSV [CSV ...]   (rows: kernel (short name) x grid; columns: counters)"""
import csv
import sys
from collections import defaultdict


def short(n):
    return n.replace("void ", "").replace("fea::", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            vals[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cols = sorted({c for v in vals.values() for c in v})
    print("kernel".ljust(62) + "grid".rjust(10) + "".join(c[:28].rjust(30) for c in cols))
    for (k, g), v in sorted(vals.items(), key=lambda x: x[0]):
        if k.startswith("at::"):
            continue
        print(k.ljust(62) + str(g).rjust(10) +
              "".join((f"{sum(v[c]) / len(v[c]):.4g}" if c in v else "-").rjust(30) for c in cols))


if __name__ == "__main__":
    main(sys.argv[1:])
