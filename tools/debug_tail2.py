import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from oracle import feanet_oracle as orc
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib
from test_schedule import tail_oracle
T = torch.float64; n = 64; B = 2; N = n + 1
rng = np.random.default_rng(n)
mg_o = orc.OracleMultigrid(n, "poisson", np.float64)
geo, _ = orc.square_geometry(N, np.float64)
bc = (rng.random((B, N, N)) * (1 - geo))
mg_o.set_boundary(geo, bc)
u0 = rng.standard_normal((B, N, N)); f = rng.standard_normal((B, N, N))
s = MultigridSolver(n, dtype=T, batch=B, coarse_tail=True, graph=False)
s.set_boundary(torch.from_numpy(bc).cuda().reshape(B, 1, N, N))
s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, N, N))
s.load(torch.from_numpy(u0).cuda().reshape(B, 1, N, N))
plan, end = s._plan("a")
lv = s.levels
v = u0 * geo + bc
stream = torch.cuda.current_stream().cuda_stream
for i, (name, args) in enumerate(plan):
    print("step", i, name, flush=True)
    _lib.call(name, T, *args, stream)
    torch.cuda.synchronize()
    for l in range(2):
        for buf in ("a", "b", "f"):
            x = lv[l].view(lv[l].buf(buf)).cpu().numpy()
            print(f"   L{l}.{buf}: max|.| per sample", np.abs(x).max(axis=(1, 2)))
# oracle tail for level 1 from the GPU's f_1
f1 = lv[1].view(lv[1].f).cpu().numpy()
ref = tail_oracle(mg_o, 1, f1, None, B, nu1=1, nu2=1, q2=False)
got = lv[1].view(lv[1].a).cpu().numpy()
print("tail err per sample", np.abs(got - ref).max(axis=(1, 2)), np.abs(ref).max())
# restriction check
r = f - mg_o.levels[0].K(u0 * geo + bc)
