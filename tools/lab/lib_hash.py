"""Bitwise fingerprint of a solver run (lab A/B of library builds: run under tools/lab/with_lib.py, compare lines).
  python3 tools/lab/with_lib.py LIB.so tools/lab/lib_hash.py [n] [cycles] [problem] [dtype]
Prints one line: the sha256 of the solution after `cycles` joined V-cycles (seeded randn rhs, zero guess)."""
import hashlib
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
from feanet_amd.solver import MultigridSolver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 37
problem = sys.argv[3] if len(sys.argv) > 3 else "poisson"
T = torch.float64 if (sys.argv[4] if len(sys.argv) > 4 else "f64") == "f64" else torch.float32
s = MultigridSolver(n, problem=problem, dtype=T)
g = torch.Generator(device="cuda")
g.manual_seed(1234)
s.set_rhs(f=torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=T, generator=g))
s.load()
out = []
for k in (1, cycles, 2):  # a single cycle, a joined block + remainder, then two more
    s.vcycle(k)
    torch.cuda.synchronize()
    out.append(hashlib.sha256(s.solution().cpu().numpy().tobytes()).hexdigest()[:16])
print(f"n={n} {problem} {T} hashes {' '.join(out)} resid {float(s.residual_norm().max()):.6e}")
