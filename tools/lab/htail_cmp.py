"""Lab: outputs of fea_mg_hjac_tail on seeded inputs over a grid of shapes (run under tools/lab/with_lib.py, once per
library build; then `python3 tools/lab/htail_cmp.py --compare A.npz B.npz`).
  python3 tools/lab/with_lib.py LIB.so tools/lab/htail_cmp.py OUT.npz"""
import os
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        d = np.abs(a[k] - b[k])
        print(f"{k:40s} max|diff| {d.max():.3e}  equal {np.array_equal(a[k], b[k])}  first bad {np.argwhere(d > 0)[:3].tolist()}")
    sys.exit(0)

import torch  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
from feanet_amd import _lib, mesh_setup as ms  # noqa: E402
from feanet_amd.solver import _Level  # noqa: E402

out = {}
for T in (torch.float32, torch.float64):
    npdt = np.float32 if T == torch.float32 else np.float64
    ktab = ms.stencil_table(None)
    kt = torch.from_numpy(ktab.reshape(-1, 9).astype(npdt)).cuda()
    om = torch.from_numpy(ms.omega_over_d(ktab, 2 / 3., npdt)).cuda()
    lin = (ms.linear_transfer_kernel() / 4).reshape(1, 9).astype(npdt)
    rt = torch.from_numpy(lin).cuda()
    pt = torch.from_numpy(lin).cuda()
    for Nt, nlev in ((5, 2), (9, 2), (9, 3), (17, 2), (17, 4), (33, 2), (33, 5), (65, 2), (65, 6)):
        for B in (1, 2):
            for nl in (1, 3):
                if T == torch.float64 and Nt == 65 and _lib.hjac_tail_lds_bytes(Nt, Nt, nlev, 8, False) > _lib.TAIL_LDS_LIMIT:
                    continue
                rng = np.random.default_rng(Nt * 100 + nlev * 10 + B + nl)
                hw = torch.from_numpy((0.25 * rng.standard_normal((nl, 9))).astype(npdt)).cuda()
                L = _Level(Nt - 1, Nt - 1, B, T, torch.device("cuda"))
                f = rng.standard_normal((B, Nt, Nt)).astype(npdt)
                L.view(L.f).copy_(torch.from_numpy(f))
                L.view(L.a).zero_()
                rc = _lib.call("mg_hjac_tail", T, L.f.data_ptr(), L.a.data_ptr(), Nt, Nt, nlev, L.ld, L.bs, None,
                               kt.data_ptr(), om.data_ptr(), 1, rt.data_ptr(), pt.data_ptr(), hw.data_ptr(), nl, 1.0,
                               1.0, 1, 1, B, None)
                torch.cuda.synchronize()
                out[f"{str(T)[6:]}_N{Nt}_l{nlev}_B{B}_nl{nl}"] = L.view(L.a).cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", len(out))
