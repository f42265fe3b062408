import sys, os, gc
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
from oracle import feanet_oracle as orc
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib
mode = sys.argv[1]
def run(n, B, tail, T=torch.float64, check_steps=False):
    N = n + 1
    rng = np.random.default_rng(n)
    mg_o = orc.OracleMultigrid(n, "poisson", np.float64)
    geo, _ = orc.square_geometry(N, np.float64)
    bc = (rng.random((B, N, N)) * (1 - geo))
    mg_o.set_boundary(geo, bc)
    u0 = rng.standard_normal((B, N, N)); f = rng.standard_normal((B, N, N))
    s = MultigridSolver(n, dtype=T, batch=B, coarse_tail=tail, graph=False)
    s.set_boundary(torch.from_numpy(bc).cuda().reshape(B, 1, N, N))
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, N, N))
    s.load(torch.from_numpy(u0).cuda().reshape(B, 1, N, N))
    if check_steps:
        for l, L in enumerate(s.levels):
            for b in ("a", "b", "f"):
                x = L.buf(b)[: L.B * L.bs].view(L.B, L.N + 2, L.ld)
                # everything outside the N x N nodes must be zero (ghost ring + padding)
                m = x.clone(); m[:, 1:L.N + 1, 15:15 + L.N] = 0
                nz = (m != 0).sum().item()
                if nz:
                    print(f"   level {l} buf {b}: {nz} nonzero ghost/pad entries", flush=True)
    s.vcycle()
    got = s.solution().cpu().numpy()[:, 0]
    ref = mg_o.step(u0 * geo + bc, f)
    print(n, B, tail, np.abs(got - ref).max(axis=(1, 2)), flush=True)
    return s
keep = []
for n in (32, 64):
    for B in (1, 2):
        for tail in (True, False):
            s = run(n, B, tail, check_steps=True)
            if mode == "keep":
                keep.append(s)
            del s
            if mode == "empty":
                gc.collect(); torch.cuda.empty_cache()
