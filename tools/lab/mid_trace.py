"""Per-workgroup start/end and per-phase times (s_memrealtime, 100 MHz) of the multi-level launches:
builds the whole library with -DFEA_MID_TRACE into tools/lab/mid_trace.so, runs mid_down / mid_up at
513^2 (k = 3) and prints the workgroup start/end spread and workgroup 0's phase times.
Usage: python tools/lab/mid_trace.py build  (here)  /  python tools/lab/mid_trace.py  (GPU box)"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
SO = os.path.join(HERE, "mid_trace.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
if len(sys.argv) > 1 and sys.argv[1] == "build":
    from feanet_amd import build
    build.build(out=SO, defines=["FEA_MID_TRACE"])
    sys.exit(0)
import torch  # noqa: E402
from feanet_amd import _lib  # noqa: E402
_lib.LIB = SO
from test_gpu_mg import Frame, tables  # noqa: E402

T = torch.float64
ktab, omd, R, P, kt, om, rt, pt = tables("poisson", T)
n, k = int(os.environ.get("N", 512)), int(os.environ.get("K", 3))
Td, Tu = int(os.environ.get("TD", 4)), int(os.environ.get("TU", 32))
lv = [Frame(n >> j, 1, T, "poisson") for j in range(k + 1)]
for x in lv:
    x.L.f.normal_()
    x.L.a.normal_()
fs = _lib.PtrArray([x.L.f.data_ptr() for x in lv])
fu = _lib.PtrArray([x.L.f.data_ptr() for x in lv[:k]])
buf = (ctypes.c_longlong * 4096)()
for name, call in (("down", lambda: _lib.call("mg_mid_down", T, fs, None, k, 1, lv[0].H, lv[0].W, kt.data_ptr(),
                                               om.data_ptr(), 1, rt.data_ptr(), 1, 1.0, Td, Td, None)),
                   ("up", lambda: _lib.call("mg_mid_up", T, fu, lv[k].L.a.data_ptr(), lv[0].L.b.data_ptr(), None, k, 1,
                                             lv[0].H, lv[0].W, kt.data_ptr(), om.data_ptr(), 1, pt.data_ptr(), 1, 1.0,
                                             Tu, Tu, None))):
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    _lib.lib().fea_mid_trace_read(buf)
    nwg = 256
    st = [buf[2 * i] for i in range(nwg)]
    en = [buf[2 * i + 1] for i in range(nwg)]
    t0 = min(st)
    ph = [buf[2048 + i] for i in range(9)]
    print(f"{name}: WG start spread {(max(st) - t0) * 10} ns, first end {(min(en) - t0) * 10} ns, "
          f"last end {(max(en) - t0) * 10} ns; WG0 phases (ns from its start): "
          + " ".join(str((p - st[0]) * 10) for p in ph), flush=True)
    if name == "up":
        for slot in range(2):
            print(f"  up WG0 wave marks {slot}: " + " ".join(str((buf[3072 + slot * 16 + w] - st[0]) * 10)
                                                       for w in range(16)))
