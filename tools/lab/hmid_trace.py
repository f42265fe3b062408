"""Per-workgroup start/end and per-phase times (s_memrealtime, 100 MHz) of the HJac two-level launches
(fea_mg_hmid_down / _up) of the 4097^2 fp64 MG-HJac cycle: builds the library with -DFEA_HMID_TRACE into
tools/lab/hmid_trace.so, replays each hmid launch of the solver's plan and prints workgroup 0's phase times.
Usage: python tools/lab/hmid_trace.py build  (here)  /  python tools/lab/hmid_trace.py  (GPU box)"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
SO = os.path.join(HERE, "hmid_trace.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from feanet_amd import build
    build.build(out=SO, defines=["FEA_HMID_TRACE"])
    sys.exit(0)
import torch  # noqa: E402
from feanet_amd import _lib  # noqa: E402
_lib.LIB = SO
from feanet_amd.solver import MultigridSolver  # noqa: E402

n = int(os.environ.get("N", 4096))
T = torch.float32 if os.environ.get("DT") == "f32" else torch.float64
w = np.load(os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
hnet = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
s = MultigridSolver(n, dtype=T, smoother="hjac", hnet=hnet)
if "MINT" in os.environ:
    s.HMID_MIN_TILES = int(os.environ["MINT"])
s.set_rhs(f=torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=T))
s.load()
s.vcycle(2)
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
buf = (ctypes.c_longlong * 4096)()
for name, args in s._plan("a")[0]:
    if name not in ("mg_hmid_down", "mg_hmid_up"):
        continue
    for _ in range(5):
        _lib.call(name, T, *args, stream)
    torch.cuda.synchronize()
    _lib.lib().fea_hmid_trace_read(buf)
    T_ = args[-1]
    H = args[4] if name == "mg_hmid_down" else args[6]
    Ht = H if name == "mg_hmid_up" else ((H + 1) // 2 + 1) // 2
    nwg = (-(-(Ht - 2) // T_)) ** 2
    st = [buf[2 * i] for i in range(nwg)]
    en = [buf[2 * i + 1] for i in range(nwg)]
    t0 = min(st)
    ph = [buf[2048 + i] for i in range(16) if buf[2048 + i] >= st[0]]
    print(f"{name} H={H} T={T_} wgs={nwg}: WG start spread {(max(st) - t0) * 10} ns, first end "
          f"{(min(en) - t0) * 10} ns, last end {(max(en) - t0) * 10} ns; WG0 phases (ns from its start): "
          + " ".join(str((p - st[0]) * 10) for p in ph) + f" end {(en[0] - st[0]) * 10}", flush=True)
