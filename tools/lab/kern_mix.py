"""Launch the three fine-level kernels at 4097^2 fp64 (sweep, sweep+restrict, prolong+sweep) a few
times each, for rocprofv3 counter collection."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
import bench
from feanet_amd.solver import MultigridSolver

s = MultigridSolver(4096, dtype=torch.float64)
g = torch.Generator(device="cuda"); g.manual_seed(0)
s.set_rhs(f=torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
s.load(torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
r = bench.time_fine_kernels(s, 8)
for k, (t, b) in r.items():
    print(f"{k:24s} {t * 1e6:7.1f} us  {b / t / 1e9:6.0f} GB/s")
