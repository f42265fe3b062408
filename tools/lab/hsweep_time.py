"""Time fea_mg_hsweep at 4097^2 fp64 (LDS-tile multi-stage kernel) vs fea_mg_sweep."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import numpy as np
import torch
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib

n = 4096
hw = np.random.default_rng(0).standard_normal((3, 3, 3)).astype(np.float32) * 0.1
s = MultigridSolver(n, dtype=torch.float64, smoother="hjac", hnet=hw)
g = torch.Generator(device="cuda"); g.manual_seed(0)
s.set_rhs(f=torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g))
s.load()
L0 = s.levels[0]
st = torch.cuda.current_stream()

def ev_time(fn, reps=30):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st); fn(); e1.record(st)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return t[len(t) // 2] * 1e3

for nl in (0, 1, 3):
    fn = lambda: _lib.call("mg_hsweep", s.dtype, L0.a.data_ptr(), None, L0.f.data_ptr(), L0.b.data_ptr(), None,
                           s.ktab.data_ptr(), s.omd.data_ptr(), 1, s.hw.data_ptr(), nl, *L0.geom(), st.cuda_stream)
    t = ev_time(fn)
    print(f"hsweep nl={nl}: {t:7.1f} us  {24 * 4095**2 / t / 1e3:6.0f} GB/s algorithmic")
fn = lambda: _lib.call("mg_sweep", s.dtype, L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), None,
                       s.ktab.data_ptr(), s.omd.data_ptr(), 1, *L0.geom(), st.cuda_stream)
t = ev_time(fn)
print(f"sweep      : {t:7.1f} us  {24 * 4095**2 / t / 1e3:6.0f} GB/s")
