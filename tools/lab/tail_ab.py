# (historical record: written for the former FEANET_LIB_OVERRIDE variable; run variant builds through tools/lab/with_lib.py now)
"""Bitwise A/B of two library builds on V-cycles that use the coarse tail (run once per build,
FEANET_LIB_OVERRIDE selects the build; the second run compares against the first's saved output).
usage: python tools/lab/tail_ab.py OUT.npz [REF.npz]"""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import numpy as np
import torch
from feanet_amd.solver import MultigridSolver

res = {}
for T in (torch.float64, torch.float32):
    for problem, n, B in (("poisson", 256, 2), ("interface", 128, 2), ("poisson", 64, 1), ("poisson", 4096, 1)):
        rng = np.random.default_rng(n)
        f = torch.from_numpy(rng.standard_normal((B, 1, n + 1, n + 1))).cuda().to(T)
        s = MultigridSolver(n, problem=problem, dtype=T, batch=B)
        s.set_rhs(f=f)
        s.load()
        s.vcycle(3)
        res[f"{problem}_{n}_{str(T)[-7:]}"] = s.solution().cpu().numpy()
np.savez(sys.argv[1], **res)
if len(sys.argv) > 2:
    ref = np.load(sys.argv[2])
    bad = [k for k in res if not np.array_equal(res[k], ref[k])]
    print("bitwise equal" if not bad else f"DIFFER: {bad}", flush=True)
    sys.exit(1 if bad else 0)
