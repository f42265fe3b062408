"""Lab: the launch list of one joined DD cycle (interior rank), with each launch's name."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402
from tools.dd_projection import PackComm, interior_rank  # noqa: E402
from feanet_amd.dd import DDSolver, default_grid  # noqa: E402

P, n, Ld = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
Pr, Pc = default_grid(P)
s = DDSolver(n, n, interior_rank(Pr, Pc), P, comm=PackComm(), agglomerate=Ld, grid=(Pr, Pc))
print("local levels", [(L.H, L.W) for L in s.local.levels], "coarse levels", [(L.H, L.W) for L in s.coarse.levels])
segs, end = s.chunk(("join", "a"))
for kind, st, lvl0 in segs:
    if kind == "k":
        print("K", lvl0, [x[0] for x in st])
    else:
        print("C", st[0], st[1] if st[0] != "exchanges" else [tuple(i) for i in st[1]])
print("coarse plan", [x[0] for x in s.coarse_plan])
