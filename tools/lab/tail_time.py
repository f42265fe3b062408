"""Time fea_mg_coarse_tail alone (f64, Poisson) for Ht = Wt = 65, 33, 17 and every nlev: where the
coarse tail's ~39 us go.  Usage (GPU box): python tools/lab/tail_time.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "multigrid-feanet_amd"))
from feanet_amd import _lib  # noqa: E402

dev = torch.device("cuda")
T = torch.float64
k = torch.tensor([[-1, -1, -1], [-1, 8, -1], [-1, -1, -1]], dtype=T) / 3
ktab = k.reshape(1, 9).to(dev)
omd = torch.tensor([2 / 3 / (8 / 3)], dtype=T, device=dev)
lin = torch.tensor([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=T) / 4
rtab = lin.reshape(1, 9).to(dev)
ptab = rtab.clone()
s = torch.cuda.current_stream().cuda_stream
for Ht in (65, 33, 17):
    ld, bs = _lib.mg_layout(Ht, Ht, 8)
    f = torch.randn(bs, dtype=T, device=dev)
    v = torch.zeros(bs, dtype=T, device=dev)
    nl = 1
    while nl <= 8 and ((Ht - 1) >> (nl - 1)) >= 2:
        args = (f.data_ptr(), v.data_ptr(), Ht, Ht, nl, ld, bs, None, ktab.data_ptr(), omd.data_ptr(), 1,
                rtab.data_ptr(), ptab.data_ptr(), 1.0, 1.0, 1, 1, 0, 1, s)
        for _ in range(20):
            _lib.call("mg_coarse_tail", T, *args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 200
        e0.record()
        for _ in range(n):
            _lib.call("mg_coarse_tail", T, *args)
        e1.record()
        torch.cuda.synchronize()
        print(f"Ht={Ht:3d} nlev={nl}: {e0.elapsed_time(e1) / n * 1e3:7.2f} us")
        nl += 1
