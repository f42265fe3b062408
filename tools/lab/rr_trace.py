# (historical record: written for the former FEANET_LIB_OVERRIDE variable; run variant builds through tools/lab/with_lib.py now)
"""Per-wave start / end of the level-1 residual-restriction kernel (2049^2 fp64, zero-guess) from a
lab build with -DFEA_RR_TRACE (s_memrealtime, 10 ns ticks): is the launch dispatch-, latency- or
tail-bound?  Build: python multigrid-feanet_amd/feanet_amd/build.py --out=tools/lab/lib_rrtrace.so -DFEA_RR_TRACE
Run (GPU box): FEANET_LIB_OVERRIDE=tools/lab/lib_rrtrace.so python tools/lab/rr_trace.py"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np
import torch
from feanet_amd import _lib
from test_gpu_mg import Frame, tables

T = torch.float64
ktab, omd, R, P, kt, om, rt, pt = tables("poisson", T)
n = int(os.environ.get("N", 2048))
fr, co = Frame(n, 1, T, "poisson"), Frame(n // 2, 1, T, "poisson")
fr.L.f.normal_()
rr = lambda: _lib.call("mg_residual_restrict", T, None, fr.L.f.data_ptr(), None, co.L.f.data_ptr(), None,
                       kt.data_ptr(), om.data_ptr(), 1, rt.data_ptr(), 1, 1.0, *fr.args(), co.L.ld, co.L.bs, None)
for _ in range(20):
    rr()
torch.cuda.synchronize()
buf = (ctypes.c_longlong * (2 * 8192))()
_lib.lib().fea_rr_trace_read(buf)
a = np.array(buf[:8192]); b = np.array(buf[8192:])
m = (a > 0) & (b > 0)
a, b = a[m], b[m]
t0 = a.min()
print(f"N={n + 1}: {m.sum()} waves; span {(b.max() - t0) * 10} ns; start spread {(a.max() - t0) * 10} ns; "
      f"wave duration median {np.median(b - a) * 10:.0f} ns, min {(b - a).min() * 10} ns, max {(b - a).max() * 10} ns")
for q in (0.1, 0.5, 0.9, 1.0):
    print(f"  start quantile {q}: {(np.quantile(a, q) - t0) * 10:.0f} ns, end quantile {q}: {(np.quantile(b, q) - t0) * 10:.0f} ns")
