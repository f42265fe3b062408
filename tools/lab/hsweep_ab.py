"""The streaming learned-smoother sweep (hnet_ops.hip, round 3) against the round-2 LDS-tile form, loaded side by
side from the previous build (tools/lab/lib_hnet_old.so, built from the previous commit's sources): bitwise
outputs over sizes, dtypes, both problems, 0..3 layers, zero guess and the raw-iterate first sweep; then the
launch times.   GPU box: python3 tools/lab/hsweep_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from feanet_amd import _lib  # noqa: E402
from feanet_amd.solver import MultigridSolver  # noqa: E402

new = _lib.lib()
_lib._lib = None
_lib.LIB = os.path.join(HERE, "lib_hnet_old.so")
old = _lib.lib()
_lib._lib = new
hw = np.random.default_rng(0).standard_normal((3, 3, 3)) * 0.1
bad = 0
for n, B, T, prob in [(4, 1, torch.float32, "poisson"), (8, 2, torch.float64, "poisson"), (32, 1, torch.float32, "poisson"),
                      (64, 3, torch.float64, "interface"), (128, 1, torch.float32, "interface"),
                      (256, 2, torch.float64, "poisson"), (1024, 1, torch.float64, "interface"),
                      (1024, 1, torch.float32, "poisson"), (4096, 1, torch.float64, "poisson")]:
    s = MultigridSolver(n, dtype=T, batch=B, problem=prob, levels=2, smoother="hjac", hnet=hw)
    L0 = s.levels[0]
    g = torch.Generator(device="cuda")
    g.manual_seed(n)
    for t in (L0.f, L0.a, L0.b):
        t.normal_(generator=g)
    raw = torch.randn(L0.a.shape, dtype=T, device="cuda", generator=g)
    pid = None if L0.pid is None else L0.pid.data_ptr()
    for nl in (0, 1, 2, 3):
        for mode in ("u", "zero", "raw"):
            u = None if mode == "zero" else L0.a.data_ptr()
            r = raw.data_ptr() if mode == "raw" else None
            outs = []
            for h in (old, new):
                _lib._lib = h
                o = torch.full_like(L0.a, 7.0)
                _lib.call("mg_hsweep", T, u, r, L0.f.data_ptr(), o.data_ptr(), pid, s.ktab.data_ptr(), s.omd.data_ptr(),
                          s.ntab, s.hw.data_ptr(), nl, *L0.geom(), torch.cuda.current_stream().cuda_stream)
                outs.append(L0.view(o).clone())
            _lib._lib = new
            if not torch.equal(outs[0], outs[1]):
                bad += 1
                print(f"MISMATCH n={n} B={B} {T} {prob} nl={nl} {mode}: {(outs[0] - outs[1]).abs().max().item():.3e}",
                      flush=True)
    if n >= 1024:
        for name, h in (("round-2 tile", old), ("streaming", new)):
            _lib._lib = h
            args = (L0.a.data_ptr(), None, L0.f.data_ptr(), L0.b.data_ptr(), pid, s.ktab.data_ptr(), s.omd.data_ptr(),
                    s.ntab, s.hw.data_ptr(), 3) + L0.geom()
            t = bench.time_kernel("mg_hsweep", T, args, 20, torch.cuda.current_stream())
            by = (3 * L0.f.element_size() + (1 if pid else 0)) * B * (L0.H - 2) * (L0.W - 2)
            print(f"{B} x {n + 1}^2 {T} {prob} hsweep (3 layers) {name:13s}: {t * 1e6:8.1f} us  {by / t / 1e12:.2f} TB/s",
                  flush=True)
        _lib._lib = new
    del s
    torch.cuda.empty_cache()
print("bitwise mismatches:", bad)
