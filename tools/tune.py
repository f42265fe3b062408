"""Interleaved A/B timing of V-cycle variants in one process (guide §5.4 rule 24)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
import torch
from feanet_amd.solver import MultigridSolver

def make(n, **kw):
    s = MultigridSolver(n, dtype=torch.float64, **kw)
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    s.set_rhs(f=torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g))
    s.load(); s.vcycle(3); torch.cuda.synchronize()
    return s

def timeit(s, k=30):
    torch.cuda.synchronize(); t = time.perf_counter(); s.vcycle(k); torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e6

variants = {"fuse": dict(fuse=True), "nofuse": dict(fuse=False), "notail": dict(coarse_tail=False)}
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ss = {k: make(n, **v) for k, v in variants.items()}
res = {k: [] for k in ss}
for r in range(5):
    for k, s in ss.items():
        res[k].append(timeit(s))
for k, v in res.items():
    v.sort()
    print(f"TW={os.environ.get('FEANET_TARGET_WAVES','default')} {k:8s} median {v[2]:8.1f} us  min {v[0]:8.1f} us")
