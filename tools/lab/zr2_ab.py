"""Launch time of fea_mg_zero_restrict2 against the two single-level zero-guess restrictions it replaces
(levels 1-2 of the 4097^2 cycle: 2049^2 -> 1025^2 -> 513^2, fp64; and the C5 batch shape in fp32).
Run against A/B builds of the task height:  python3 tools/lab/with_lib.py LIB.so tools/lab/zr2_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from feanet_amd import _lib  # noqa: E402
from feanet_amd.solver import MultigridSolver  # noqa: E402

for n, B, T in ((4096, 1, torch.float64), (8192, 1, torch.float64), (1024, 64, torch.float32)):
    s = MultigridSolver(n, dtype=T, batch=B, pair_levels=False)
    lv = s.levels
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    lv[1].f.normal_(generator=g)
    kt, om, rt = s.ktab.data_ptr(), s.omd.data_ptr(), s.rtab.data_ptr()
    st = torch.cuda.current_stream()
    a1 = (None, lv[1].f.data_ptr(), None, lv[2].f.data_ptr(), None, kt, om, 1, rt, 1, s.w[0]) + lv[1].geom() + (lv[2].ld, lv[2].bs)
    a2 = (None, lv[2].f.data_ptr(), None, lv[3].f.data_ptr(), None, kt, om, 1, rt, 1, s.w[0]) + lv[2].geom() + (lv[3].ld, lv[3].bs)
    t1 = bench.time_kernel("mg_residual_restrict", T, a1, 200, st)
    t2 = bench.time_kernel("mg_residual_restrict", T, a2, 200, st)
    a3 = (lv[1].f.data_ptr(), lv[2].f.data_ptr(), lv[3].f.data_ptr(), None, None, kt, om, 1, rt, 1, s.w[0]) + lv[1].geom() + (lv[2].ld, lv[2].bs, lv[3].ld, lv[3].bs)
    t3 = bench.time_kernel("mg_zero_restrict2", T, a3, 200, st)
    print(f"{_lib.LIB.split('/')[-1]:24s} {B} x {lv[1].H}^2 {str(T)[6:]}: levels 1+2 separately {t1 * 1e6:6.2f} + {t2 * 1e6:6.2f} = "
          f"{(t1 + t2) * 1e6:6.2f} us, fused {t3 * 1e6:6.2f} us", flush=True)
    del s
    torch.cuda.empty_cache()
