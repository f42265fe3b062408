#!/usr/bin/env python3
"""HBM traffic per launch from two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read -> doubled here;
WRITE_SIZE is exact for 16 B/lane streaming stores.  Every load/store of the framed kernels is
16 B/lane (halo loads included).

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [SUMMARY_TXT]
"""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict

KERNEL_SOURCE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multigrid-feanet_amd", "csrc",
                             "framed_ops.hip")


def kernel_source_sha():
    """First 16 hex digits of the SHA-256 of the level kernels' source: bench.py reports stored PMC traffic
    only for the kernels it was measured on."""
    return hashlib.sha256(open(KERNEL_SOURCE, "rb").read()).hexdigest()[:16]


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


def short(n):
    return n.replace("void ", "").replace("fea::", "").split("(")[0]


def main(fcsv, wcsv, out_json, summary=None, src="profiles/r01_pmc"):
    """FETCH/WRITE csv: rocprofv3 --pmc counter_collection.csv of the two passes."""
    fetch = load(fcsv, "FETCH_SIZE")
    write = load(wcsv, "WRITE_SIZE")
    rows = []
    for key in sorted(set(fetch) & set(write), key=lambda k: -sum(fetch[k])):
        name, grid = key
        f = 2 * 1024 * sum(fetch[key]) / len(fetch[key])
        w = 1024 * sum(write[key]) / len(write[key])
        rows.append((short(name), grid, len(fetch[key]), f, w))
    res = {}
    nodes, cnodes = 4095 * 4095, 2047 * 2047
    for name, grid, n, f, w in rows:
        key = alg = None
        if name.startswith("k_mg_sweep<double, false, false") and grid == 262144:
            key, alg = "mg_sweep_f64_4097", 24 * nodes
        elif name.startswith("k_mg_cycle_join<double, false") and n >= 10:  # the 4097^2 join (most launches)
            key, alg = "mg_cycle_join_f64_4097", 24 * nodes + 16 * cnodes
        if key and (key not in res or res[key]["launches"] < n):
            res[key] = {
                "hbm_bytes_per_launch": f + w, "read_bytes_per_launch": f, "write_bytes_per_launch": w,
                "algorithmic_bytes_per_launch": alg, "launches": n, "grid": grid,
                "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streaming reads), KiB -> bytes",
                "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({src})",
                "kernel_source_sha256": kernel_source_sha()}
    json.dump(res, open(out_json, "w"), indent=1)
    if summary:
        with open(summary, "w") as fh:
            fh.write(f"{'kernel':45s} {'grid':>8s} {'n':>4s} {'read MB':>9s} {'write MB':>9s}\n")
            for name, grid, n, f, w in rows:
                fh.write(f"{name:45s} {grid:8d} {n:4d} {f / 1e6:9.2f} {w / 1e6:9.2f}\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
