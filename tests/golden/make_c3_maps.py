#!/usr/bin/env python3
"""Pattern maps of the C3 hierarchy (2049^2 two-material circle, every level down to 3^2) computed by
the ORACLE's element/node loop (oracle/feanet_oracle.py interface_mesh, a restatement of
FEANet/mesh.py:62-101 pinned by the reference-generated maps N = 5..129 in tables.npz).

The loop takes ~90 s for the whole hierarchy, too slow for a GPU test; the GPU test of config C3
(tests/test_gpu_configs.py) builds its oracle hierarchy from this fixture, and the CPU suite
(tests/test_setup.py::test_c3_maps_fixture_is_oracle) re-runs the loop at 2049^2 and checks the
fixture against it and against the product's vectorised builder.

Usage:  python tests/golden/make_c3_maps.py      (writes tests/golden/c3_pattern_maps.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import feanet_oracle as orc  # noqa: E402

N_FINE = 2049


def levels(N=N_FINE):
    out = []
    while N >= 3:
        out.append(N)
        N = (N + 1) // 2
    return out


def main():
    maps = {}
    for N in levels():
        ktab, pid = orc.interface_mesh(N, (1, 20), 0)
        maps[f"pid_{N}"] = pid
        print(N, int(pid.max()), flush=True)
    maps["ktab"] = ktab
    np.savez_compressed(os.path.join(HERE, "c3_pattern_maps.npz"), **maps)


if __name__ == "__main__":
    main()
