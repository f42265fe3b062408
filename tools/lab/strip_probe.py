"""Is the fine-level cycle join bound by its wave count or by its bytes?  Isolated joins on H = 4097 grids
whose width W gives a ragged last strip (4097: 35 strips, the last owns 15 of 120 columns) or full
strips only (4081: 34 strips), fp64; and the C5 shape (256 x 1025^2 fp32: 5 strips, the last owns 47 of
244) against 977-wide rows (4 full strips).  GPU box: python tools/lab/strip_probe.py"""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
import bench
from feanet_amd.solver import MultigridSolver

import sys as _s
CASES = {"a": ((4096, 4096, 1, torch.float64), (4096, 4080, 1, torch.float64),
               (1024, 1024, 256, torch.float32), (1024, 976, 256, torch.float32)),
         # C5 rows of 1025 / 1017 (both 5 strips, last strip 47 / 39 owned columns) and 977 / 969 (4 strips):
         # separates the ragged strip from the row pitch
         "b": ((1024, 1024, 256, torch.float32), (1024, 1016, 256, torch.float32),
               (1024, 976, 256, torch.float32), (1024, 968, 256, torch.float32))}
for (m, n, B, T) in CASES[_s.argv[1] if len(_s.argv) > 1 else "a"]:
    s = MultigridSolver(n, rows=m, dtype=T, batch=B, levels=4)
    s.set_rhs(f=torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=T))
    s.load()
    r = bench.time_fine_kernels(s, 20 if B == 1 else 5)
    t, by = r["fea_mg_cycle_join"]
    ts, bys = r["fea_mg_sweep"]
    print(f"{B} x {m + 1} x {n + 1} {T} (ld {s.levels[0].ld}): join {t * 1e6:.1f} us ({by / t / 1e9:.0f} GB/s), "
          f"sweep {ts * 1e6:.1f} us ({bys / ts / 1e9:.0f} GB/s)", flush=True)
    del s
    torch.cuda.empty_cache()
