import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np, torch
from oracle import feanet_oracle as orc
from feanet_amd.solver import MultigridSolver
for T in (torch.float64, torch.float32):
  for n in (32, 64, 128):
    for B in (1, 2):
      for tail in (True, False):
        npdt = np.float64 if T == torch.float64 else np.float32
        rng = np.random.default_rng(n); N = n + 1
        mg_o = orc.OracleMultigrid(n, "poisson", npdt)
        geo, _ = orc.square_geometry(N, npdt)
        bc = (rng.random((B, N, N)) * (1 - geo)).astype(npdt)
        mg_o.set_boundary(geo, bc)
        u0 = rng.standard_normal((B, N, N)).astype(npdt); f = rng.standard_normal((B, N, N)).astype(npdt)
        s = MultigridSolver(n, dtype=T, batch=B, coarse_tail=tail, graph=False)
        s.set_boundary(torch.from_numpy(bc).cuda().reshape(B, 1, N, N))
        s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, N, N))
        s.load(torch.from_numpy(u0).cuda().reshape(B, 1, N, N))
        v = u0 * geo + bc
        s.vcycle(); v = mg_o.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        err = np.abs(got - v).max(axis=(1, 2)) / np.abs(v).max()
        print(T, n, B, "tail" if tail else "notail", s.tail_from, err)
