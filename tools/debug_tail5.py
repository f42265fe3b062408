import sys, os, gc
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from oracle import feanet_oracle as orc
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib
from test_schedule import tail_oracle
keep = []
for n in (32, 64):
    for B in (1, 2):
        for tail in (True, False):
            N = n + 1
            rng = np.random.default_rng(n)
            mg_o = orc.OracleMultigrid(n, "poisson", np.float64)
            geo, _ = orc.square_geometry(N, np.float64)
            bc = (rng.random((B, N, N)) * (1 - geo))
            u0 = rng.standard_normal((B, N, N)); f = rng.standard_normal((B, N, N))
            s = MultigridSolver(n, dtype=torch.float64, batch=B, coarse_tail=tail, graph=False)
            s.set_boundary(torch.from_numpy(bc).cuda().reshape(B, 1, N, N))
            s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, N, N))
            s.load(torch.from_numpy(u0).cuda().reshape(B, 1, N, N))
            plan, end = s._plan("a")
            st = torch.cuda.current_stream().cuda_stream
            for name, args in plan:
                if name == "mg_coarse_tail":
                    torch.cuda.synchronize()
                    t = s.tail_from
                    L = s.levels[t]
                    f1 = L.view(L.f).cpu().numpy()
                    before = L.view(L.a).cpu().numpy().copy()
                    _lib.call(name, torch.float64, *args, st)
                    torch.cuda.synchronize()
                    got = L.view(L.a).cpu().numpy()
                    ref = tail_oracle(mg_o, t, f1, None, B, nu1=1, nu2=1, q2=False)
                    print(n, B, "tail_from", t, "|f1|", np.abs(f1).max(axis=(1, 2)), "err", np.abs(got - ref).max(axis=(1, 2)),
                          "|got|", np.abs(got).max(axis=(1, 2)), "args", args[2:6], flush=True)
                else:
                    _lib.call(name, torch.float64, *args, st)
            keep.append(s)
