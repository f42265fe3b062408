"""Same-process A/B of the row-task height rule of the overlapped-strip kernels (cycle join, sweep+restriction):
the balanced choice (FEANET_BALANCE unset) against the power-of-two choice (FEANET_BALANCE=0), per configuration,
alternating, on the same buffers.  GPU box: python3 tools/lab/balance_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from feanet_amd import _lib  # noqa: E402
from feanet_amd.solver import MultigridSolver  # noqa: E402

CONFIGS = [(4096, 1, torch.float64, "poisson", 20), (8192, 1, torch.float64, "poisson", 8),
           (2048, 1, torch.float64, "interface", 20), (2048, 1, torch.float32, "poisson", 20),
           (1024, 1, torch.float64, "poisson", 30), (1024, 256, torch.float32, "poisson", 5),
           (1024, 16, torch.float32, "poisson", 10), (2048, 8, torch.float64, "poisson", 10)]
for n, B, T, prob, reps in CONFIGS:
    s = MultigridSolver(n, dtype=T, batch=B, levels=3, problem=prob)
    L0, L1 = s.levels[0], s.levels[1]
    for t in (L0.f, L0.a, L1.a):
        t.normal_()
    res = {}
    for rnd in range(3):
        for env in ("bal", "pow2"):
            if env == "pow2":
                os.environ["FEANET_BALANCE"] = "0"
            else:
                os.environ.pop("FEANET_BALANCE", None)
            r = bench.time_fine_kernels(s, reps)
            for k in ("fea_mg_cycle_join", "fea_mg_sweep_restrict"):
                res.setdefault((k, env), []).append(r[k][0])
    os.environ.pop("FEANET_BALANCE", None)
    esz = 4 if T == torch.float32 else 8
    for k in ("fea_mg_cycle_join", "fea_mg_sweep_restrict"):
        tb, tp = min(res[(k, "bal")]), min(res[(k, "pow2")])
        print(f"{B} x {n + 1}^2 {prob} {T}: {k:22s} balanced {tb * 1e6:8.1f} us   pow2 {tp * 1e6:8.1f} us   "
              f"({(tb / tp - 1) * 100:+.1f} %)", flush=True)
    del s
    torch.cuda.empty_cache()
