"""Lab: one DD projection configuration (interior rank of P ranks), for a kernel trace: warm-up, then
`--cycles` V-cycles in one vcycle() call.  Modes: cap (captured, split join), nosplit, seg (segment graphs)."""
import argparse
import os
import sys
import time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402
from tools.dd_projection import PackComm, interior_rank  # noqa: E402
from feanet_amd.dd import DDSolver, default_grid  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8192)
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--ld", type=int, default=4)
ap.add_argument("--mode", default="cap", choices=["cap", "nosplit", "seg"])
ap.add_argument("--cycles", type=int, default=100)
a = ap.parse_args()
Pr, Pc = default_grid(a.ranks)
r = interior_rank(Pr, Pc)
comm = PackComm()
comm.capturable = a.mode != "seg"
s = DDSolver(a.n, a.n, r, a.ranks, comm=comm, agglomerate=a.ld, grid=(Pr, Pc), split_join=a.mode == "cap")
g = torch.Generator(device="cuda")
g.manual_seed(0)
s.set_rhs(torch.randn(1, 1, a.n + 1, a.n + 1, dtype=torch.float64, device="cuda", generator=g))
s.load()
for _ in range(4):
    s.vcycle(a.cycles)
torch.cuda.synchronize()
t0 = time.perf_counter()
s.vcycle(a.cycles)
th = time.perf_counter() - t0
torch.cuda.synchronize()
t = time.perf_counter() - t0
print(f"{a.mode} P={a.ranks} Ld={a.ld}: {t / a.cycles * 1e6:.1f} us/cycle, host {th / a.cycles * 1e6:.1f} us/cycle")
