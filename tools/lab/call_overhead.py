"""Host cost of one vcycle(k) call on a warmed-up 4097^2 solver (graph replay path; no synchronisation inside
the timed calls), and the synchronised per-call time, for k = 1, 4, 20, 32."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402

from feanet_amd.solver import MultigridSolver  # noqa: E402

s = MultigridSolver(4096, dtype=torch.float64)
g = torch.Generator(device="cuda")
g.manual_seed(1)
s.set_rhs(f=torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
s.load()
for k in (1, 4, 20, 32):
    for _ in range(8):
        s.vcycle(k)
    torch.cuda.synchronize()
    host = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.vcycle(k)
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    tot = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.vcycle(k)
        torch.cuda.synchronize()
        tot.append(time.perf_counter() - t0)
    host.sort()
    tot.sort()
    print(f"k={k:3d}: host call {host[len(host) // 2] * 1e6:7.1f} us (min {host[0] * 1e6:6.1f}), synchronised call "
          f"{tot[len(tot) // 2] * 1e6:8.1f} us = {tot[len(tot) // 2] * 1e6 / k:6.1f} us per cycle", flush=True)
