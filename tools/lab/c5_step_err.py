"""C5 fp32: each GPU V-cycle against the fp32 oracle's cycle from the GPU's own previous iterate (lab measurement
behind the tolerance of tests/test_gpu_configs.py::test_c5_batch256_1025_fp32)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "multigrid-feanet_amd")]
from feanet_amd.solver import MultigridSolver  # noqa: E402
from oracle import feanet_oracle as orc  # noqa: E402
from tools import rhs_families  # noqa: E402

n = 1024
F = rhs_families.batch(256, n + 1, torch.float32, "cuda", seed=5)
s = MultigridSolver(n, dtype=torch.float32, batch=256)
s.set_rhs(F=F)
idx = [0, 97, 255]
f = s.levels[0].view(s.levels[0].f).unsqueeze(1).clone()[idx]
s3 = MultigridSolver(n, dtype=torch.float32, batch=3)
s3.set_rhs(f=f)
s3.load()
fb = f[:, 0].cpu().numpy()
mg32 = orc.OracleMultigrid(n, "poisson", np.float32)
prev = np.zeros_like(fb)
for k in range(6):
    s3.vcycle()
    got = s3.solution().cpu().numpy()[:, 0]
    one = mg32.step(prev, fb)
    errs = [float(np.abs(got[i] - one[i]).max() / np.abs(one[i]).max()) for i in range(3)]
    chg = [float(np.abs(got[i] - prev[i]).max() / np.abs(got[i]).max()) for i in range(3)]
    print(f"cycle {k + 1}: rel err vs fp32 oracle step {errs}  cycle change {chg}", flush=True)
    prev = got.copy()
