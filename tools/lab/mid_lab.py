"""Time the multi-level launches (fea_mg_mid_down / _up) against the per-level chains they replace,
for a few (top size, k, tile) choices (GPU box): python3 tools/lab/mid_lab.py"""
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


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for n, k, Td, Tu in [(512, 3, 4, 32), (512, 4, 2, 32), (256, 3, 4, 32), (256, 2, 8, 32), (1024, 2, 8, 32),
                     (512, 1, 16, 32), (128, 1, 4, 16)]:
    lv = [Frame(n >> j, 1, T, "poisson") for j in range(k + 1)]
    for x in lv:
        x.L.f.normal_()
        x.L.a.normal_()
    fs = _lib.PtrArray([x.L.f.data_ptr() for x in lv])
    fu = _lib.PtrArray([x.L.f.data_ptr() for x in lv[:k]])

    def chain_down():
        for j in range(k):
            _lib.call("mg_residual_restrict", T, None, lv[j].L.f.data_ptr(), None, lv[j + 1].L.f.data_ptr(), None,
                      kt.data_ptr(), om.data_ptr(), 1, rt.data_ptr(), 1, 1.0, *lv[j].args(), lv[j + 1].L.ld,
                      lv[j + 1].L.bs, None)

    def chain_up():
        for j in range(k - 1, -1, -1):
            _lib.call("mg_prolong_sweep", T, None, lv[j + 1].L.a.data_ptr(), lv[j].L.f.data_ptr(), lv[j].L.a.data_ptr(),
                      None, None, kt.data_ptr(), om.data_ptr(), 1, pt.data_ptr(), 1, 1.0, *lv[j].args(),
                      lv[j + 1].L.ld, lv[j + 1].L.bs, None)

    def mid_down():
        _lib.call("mg_mid_down", T, fs, None, k, 1, lv[0].H, lv[0].W, kt.data_ptr(), om.data_ptr(), 1,
                  rt.data_ptr(), 1, 1.0, Td, Td, None)

    def mid_up():
        _lib.call("mg_mid_up", T, fu, lv[k].L.a.data_ptr(), lv[0].L.b.data_ptr(), None, k, 1, lv[0].H, lv[0].W,
                  kt.data_ptr(), om.data_ptr(), 1, pt.data_ptr(), 1, 1.0, Tu, Tu, None)

    r = {}
    for name, fn in (("chain_down", chain_down), ("mid_down", mid_down), ("chain_up", chain_up), ("mid_up", mid_up)):
        try:
            r[name] = f"{timeit(fn):7.2f}"
        except RuntimeError as e:
            r[name] = "   n/a"
    print(f"n={n:5d} k={k} Td={Td:3d} Tu={Tu:3d}  " + "  ".join(f"{a} {b} us" for a, b in r.items()), flush=True)
