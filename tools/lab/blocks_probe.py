"""Same-process A/B of the vcycle(k) block decomposition at k = 20 (the driver's step count): median
synchronised call time over rounds of alternating variants (see blocks_ab.py for the variants)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402

from feanet_amd.solver import MultigridSolver  # noqa: E402

base = MultigridSolver.pipe_blocks


def head(h):
    return lambda njoin, G: [njoin] if njoin <= h else [h] + base(njoin - h, G)


VARIANTS = {"new": base, "old": MultigridSolver.graph_blocks, "head1": head(1), "head2": head(2), "head4": head(4)}
K = int(os.environ.get("K", "20"))
s = MultigridSolver(4096, dtype=torch.float64)
g = torch.Generator(device="cuda")
g.manual_seed(1)
s.set_rhs(f=torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
s.load()
names = sys.argv[1:] or list(VARIANTS)
for nm in names:  # warm-up: every variant's graphs captured
    MultigridSolver.pipe_blocks = staticmethod(VARIANTS[nm])
    for _ in range(6):
        s.vcycle(K)
torch.cuda.synchronize()
res = {nm: [] for nm in names}
for r in range(25):
    for nm in names:
        MultigridSolver.pipe_blocks = staticmethod(VARIANTS[nm])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.vcycle(K)
        torch.cuda.synchronize()
        res[nm].append(time.perf_counter() - t0)
for nm in names:
    v = sorted(res[nm])
    print(f"{nm:6s} k={K}: median {v[len(v) // 2] * 1e6 / K:7.2f} us per cycle, min {v[0] * 1e6 / K:7.2f}, "
          f"max {v[-1] * 1e6 / K:7.2f}", flush=True)
