"""Lab: where does the captured DD path (PackComm, capturable) leave the segment-wise path?"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402
from tools.dd_projection import PackComm  # noqa: E402
from feanet_amd.dd import DDSolver  # noqa: E402

P, grid, rank, n = 8, (4, 2), 3, 1024
g = torch.Generator(device="cuda")
g.manual_seed(1)
f = torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
runs = {}
for name, capture, split, gmin in (("seg", False, False, 5), ("seg_eager", False, False, 10**6), ("cap", True, False, 5),
                                   ("cap_split", True, True, 5)):
    comm = PackComm()
    comm.capturable = capture
    s = DDSolver(n, n, rank, P, comm=comm, agglomerate=2, grid=grid, split_join=split, graph_min=gmin)
    s.set_rhs(f)
    s.load()
    hist = []
    for k in (1, 1, 1, 3, 3, 3, 2):
        s.vcycle(k)
        torch.cuda.synchronize()
        L0 = s.local.levels[0]
        hist.append((k, s._state, L0.view(L0.buf(s._state)).clone(), s.local.levels[1].view(s.local.levels[1].f).clone()))
    runs[name] = hist
ref = runs["seg"]
for name, hist in runs.items():
    print(name, [(k, st, bool(torch.equal(a, r[2])), bool(torch.equal(b, r[3]))) for (k, st, a, b), r in zip(hist, ref)])
