import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
from oracle import feanet_oracle as orc
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib
T = torch.float64; n = 64; B = 2; N = n + 1
rng = np.random.default_rng(n)
mg_o = orc.OracleMultigrid(n, "poisson", np.float64)
geo, _ = orc.square_geometry(N, np.float64)
bc = (rng.random((B, N, N)) * (1 - geo))
mg_o.set_boundary(geo, bc)
u0 = rng.standard_normal((B, N, N)); f = rng.standard_normal((B, N, N))
ref = mg_o.step(u0 * geo + bc, f)
for mode in ("plain", "sync_after_load", "sync_each_step", "sync_before_tail", "sync_after_tail", "plain"):
    s = MultigridSolver(n, dtype=T, batch=B, coarse_tail=True, graph=False)
    s.set_boundary(torch.from_numpy(bc).cuda().reshape(B, 1, N, N))
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, N, N))
    s.load(torch.from_numpy(u0).cuda().reshape(B, 1, N, N))
    if mode != "plain":
        torch.cuda.synchronize()
    plan, end = s._plan("a")
    stream = torch.cuda.current_stream().cuda_stream
    for name, args in plan:
        if mode == "sync_before_tail" and name == "mg_coarse_tail":
            torch.cuda.synchronize()
        _lib.call(name, T, *args, stream)
        if mode == "sync_each_step" or (mode == "sync_after_tail" and name == "mg_coarse_tail"):
            torch.cuda.synchronize()
    s._state = end
    got = s.solution().cpu().numpy()[:, 0]
    print(mode, np.abs(got - ref).max(axis=(1, 2)), flush=True)
