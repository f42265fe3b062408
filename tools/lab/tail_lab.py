"""Per-phase timing of the coarse-tail kernel: builds coarse_tail.hip with -DFEA_TAIL_TRACE into
tools/lab/tail_lab.so (clock64() after every workgroup barrier) and prints the cycles per phase.
Usage: python tools/lab/tail_lab.py build   (here)   /   python tools/lab/tail_lab.py (GPU box)"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
SO = os.path.join(ROOT, "lab_libs", "tail_lab.so")  # (lab_libs/ travels to the GPU box; tools/lab/*.so does not)
SRC = os.path.join(ROOT, "multigrid-feanet_amd", "csrc", "coarse_tail.hip")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=on", "-std=c++17", "-fPIC",
           "-shared", "-DFEA_TAIL_TRACE", f"-I{os.path.join(ROOT, 'include')}",
           f"-I{os.path.join(ROOT, 'multigrid-feanet_amd', 'csrc')}", SRC, "-o", SO] + sys.argv[2:]
    subprocess.check_call(cmd)
    sys.exit(0)

import torch  # noqa: E402

L = ctypes.CDLL(SO)
P, I, LL, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_double
L.fea_mg_coarse_tail_f64.argtypes = [P, P, I, I, I, I, LL, P, P, P, I, P, P, D, D, I, I, I, I, P]
dev = torch.device("cuda")
T = torch.float64
k = torch.tensor([[-1, -1, -1], [-1, 8, -1], [-1, -1, -1]], dtype=T) / 3
ktab = k.reshape(1, 9).to(dev)
omd = torch.tensor([2 / 3 / (8 / 3)], dtype=T, device=dev)
lin = torch.tensor([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=T) / 4
rtab = lin.reshape(1, 9).to(dev)
s = torch.cuda.current_stream().cuda_stream
Ht = int(os.environ.get("HT", 65))
nl = int(os.environ.get("NLEV", 6))
ld = ((Ht + 16 + 15) // 16) * 16
bs = (Ht + 2) * ld
B = int(os.environ.get("B", 1))  # B samples = B workgroups, one per CU (B = 256: every CU runs a tail at once)
f = torch.randn(B * bs, dtype=T, device=dev)
v = torch.zeros(B * bs, dtype=T, device=dev)
buf = (ctypes.c_longlong * 256)()
ntab, pidl = 1, None
if os.environ.get("MULTI") == "1":  # the two-material tail: 16 stencils, per-level pattern maps (MeshCenterInterface)
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
    from feanet_amd import mesh_setup as ms
    kt = ms.stencil_table((1, 20))
    ntab = kt.shape[0]
    ktab = torch.from_numpy(kt.reshape(-1, 9).astype(np.float64)).to(dev)
    omd = torch.from_numpy(ms.omega_over_d(kt, 2 / 3., np.float64)).to(dev)
    rtab = lin.reshape(1, 9).expand(ntab, 9).contiguous().to(dev)
    pidl = torch.from_numpy(np.concatenate([ms.interface_pattern_map(((Ht - 1) >> k) + 1).reshape(-1)
                                            for k in range(nl)])).to(dev)
for rep in range(3):
    rc = L.fea_mg_coarse_tail_f64(f.data_ptr(), v.data_ptr(), Ht, Ht, nl, ld, bs,
                                  None if pidl is None else pidl.data_ptr(), ktab.data_ptr(),
                                  omd.data_ptr(), ntab, rtab.data_ptr(), rtab.data_ptr(), 1.0, 1.0, 1, 1, 0, B, s)
    assert rc == 0, rc
    torch.cuda.synchronize()
L.fea_tail_trace_read(buf)
t0 = buf[255]
prev = t0
out = []
for i in range(255):
    if buf[i] == 0 or buf[i] < t0:
        break
    out.append(buf[i] - prev)
    prev = buf[i]
print(f"multi={ntab > 1} B={B} Ht={Ht} nlev={nl}: total {prev - t0} cycles over {len(out)} phases")
print(" ".join(str(x) for x in out))
