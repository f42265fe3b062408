"""Find the first V-cycle step whose output depends on the batch size (rows-per-task)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
import torch
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
g = torch.Generator(device="cuda"); g.manual_seed(0)
f = torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
s1 = MultigridSolver(n, dtype=torch.float64, batch=1, graph=False)
s3 = MultigridSolver(n, dtype=torch.float64, batch=3, graph=False)
s1.set_rhs(f=f); s3.set_rhs(f=f.expand(3, 1, n + 1, n + 1).contiguous())
s1.load(); s3.load()
stream = torch.cuda.current_stream().cuda_stream
for cyc in range(2):
    p1, e1 = s1._plan(s1._state); p3, e3 = s3._plan(s3._state)
    for i, ((nm, a1), (_, a3)) in enumerate(zip(p1, p3)):
        _lib.call(nm, s1.dtype, *a1, stream); _lib.call(nm, s3.dtype, *a3, stream)
        torch.cuda.synchronize()
        bad = []
        for l, (L1, L3) in enumerate(zip(s1.levels, s3.levels)):
            for name in ("f", "a", "b"):
                x1 = L1.view(L1.buf(name))[0]; x3 = L3.view(L3.buf(name))[0]
                if not torch.equal(x1, x3):
                    d = (x1 - x3).abs()
                    rows = torch.nonzero(d.amax(dim=-1).flatten() > 0).flatten().tolist()
                    cols = torch.nonzero(d.amax(dim=-2).flatten() > 0).flatten().tolist()
                    bad.append(f"L{l}.{name} max {d.max().item():.3e} rows {rows[:12]} cols {cols[:12]}")
        print(f"cycle {cyc} step {i} {nm}: {'OK' if not bad else '; '.join(bad)}", flush=True)
        if bad:
            sys.exit(0)
    s1._state = e1; s3._state = e3
