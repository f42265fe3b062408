"""Achievable HBM streaming rate on this GPU: torch device copy (read + write) of large fp64 buffers,
and the fine sweep at 8193^2 (fields ~537 MB, no Infinity-Cache reuse) for comparison."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
import bench
from feanet_amd.solver import MultigridSolver

for mb in (512, 1024, 2048):
    n = mb * 2 ** 20 // 8
    a = torch.randn(n, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"copy {mb} MiB: {2 * n * 8 / t / 1e12:.2f} TB/s", flush=True)
    del a, b
for n in (4096, 8192):
    s = MultigridSolver(n, dtype=torch.float64)
    s.levels[0].f.normal_()
    s.levels[0].a.normal_()
    r = bench.time_fine_kernels(s, 20)
    print(n + 1, {k: f"{b / t / 1e12:.2f} TB/s" for k, (t, b) in r.items()}, flush=True)
    del s
