"""Isolated timing of the level-1 streaming kernels at 2049^2 fp64 (zero-guess residual+restriction,
recompute prolongation+sweep) for several rows-per-task targets (GPU box)."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import torch
from feanet_amd import _lib
from test_gpu_mg import Frame, tables

T = torch.float64
ktab, omd, R, P, kt, om, rt, pt = tables("poisson", T)
n = int(os.environ.get("N", 2048))
fr, co = Frame(n, 1, T, "poisson"), Frame(n // 2, 1, T, "poisson")
for x in (fr, co):
    x.L.f.normal_()
    x.L.a.normal_()


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


rr = lambda: _lib.call("mg_residual_restrict", T, None, fr.L.f.data_ptr(), None, co.L.f.data_ptr(), None,
                       kt.data_ptr(), om.data_ptr(), 1, rt.data_ptr(), 1, 1.0, *fr.args(), co.L.ld, co.L.bs, None)
ps = lambda: _lib.call("mg_prolong_sweep", T, None, co.L.a.data_ptr(), fr.L.f.data_ptr(), fr.L.b.data_ptr(), None,
                       None, kt.data_ptr(), om.data_ptr(), 1, pt.data_ptr(), 1, 1.0, *fr.args(), co.L.ld, co.L.bs, None)
nodes = (n - 1) ** 2
print(f"N={n + 1} target={os.environ.get('FEANET_TARGET_WAVES', 2048)}: RR {timeit(rr):.2f} us "
      f"({10 * nodes / timeit(rr) / 1e3:.0f} GB/s alg)  PS {timeit(ps):.2f} us ({18 * nodes / timeit(ps) / 1e3:.0f} GB/s alg)")
