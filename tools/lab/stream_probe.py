"""What limits the fine-level kernels at sizes beyond the Infinity Cache (8193^2 fp64, ~540 MB per field)?
  1. tools/lab/stream_probe.hip: the same bytes (2 reads + 1 write per 1 KiB piece) in three visiting orders
     (linear / the product's strip march / strip march over a strip-blocked layout), task heights, row pitches;
  2. the product sweep and cycle join at 8193^2 with padded row pitches (the C ABI takes any ld >= mg_ld).
Every product-kernel variant is checked bitwise against the default-pitch result.
GPU box: python tools/lab/stream_probe.py [quick]"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
from feanet_amd import _lib
from feanet_amd.solver import MultigridSolver

QUICK = len(sys.argv) > 1 and sys.argv[1] == "quick"
lab = ctypes.CDLL(os.path.join(HERE, "stream_probe.so"))
P, I = ctypes.c_void_p, ctypes.c_int
lab.lab_stream_probe.argtypes = [I, P, P, P, I, I, I, I, I, P]
st = torch.cuda.current_stream()


def ev_time(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        fn()
        e1.record(st)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return t[len(t) // 2] * 1e-3


# ---- 0. torch device copy (1 read + 1 write)
a = torch.randn(540 * 2 ** 20 // 8, dtype=torch.float64, device="cuda")
b = torch.empty_like(a)
t = ev_time(lambda: b.copy_(a))
print(f"torch copy 540 MiB: {t * 1e6:.1f} us  {2 * a.numel() * 8 / t / 1e12:.2f} TB/s", flush=True)
del a, b

# ---- 1. probe orders
rows, nstrips = 8192, 64
LDMAX = 8704
nb = rows * LDMAX + 4096
u = torch.randn(nb, dtype=torch.float64, device="cuda")
f = torch.randn(nb, dtype=torch.float64, device="cuda")
o = torch.empty_like(u)
by = 3 * rows * nstrips * 1024
res = []
for mode, name in ((0, "linear"), (1, "strip"), (2, "tile")):
    for rb in ((32,) if QUICK else (8, 32, 128)):
        for remap in (0, 1):
            lds = (8192, 8224, 8256, 8448) if mode == 1 else (8192,)
            if QUICK and mode == 1:
                lds = (8192, 8224)
            for ld in lds:
                fn = lambda: lab.lab_stream_probe(mode, u.data_ptr(), f.data_ptr(), o.data_ptr(), rows, nstrips, ld,
                                                  rb, remap, st.cuda_stream)
                assert fn() == 0
                t = ev_time(fn)
                line = f"probe {name:6s} rb {rb:3d} remap {remap} ld {ld}: {t * 1e6:7.1f} us  {by / t / 1e12:.2f} TB/s"
                print(line, flush=True)
del u, f, o
torch.cuda.empty_cache()

# ---- 2. product sweep / join at 8193^2 with padded pitches
n = 8192
N = n + 1
s = MultigridSolver(n, dtype=torch.float64, levels=3)
L0, L1 = s.levels[0], s.levels[1]
g = torch.Generator(device="cuda")
g.manual_seed(0)
fin = torch.randn(1, 1, N, N, dtype=torch.float64, device="cuda", generator=g)
uin = torch.randn(1, 1, N, N, dtype=torch.float64, device="cuda", generator=g)
ecin = torch.randn(1, 1, L1.H, L1.W, dtype=torch.float64, device="cuda", generator=g)


def framed(x, H, W, ld):
    off = 15
    buf = torch.zeros((H + 2) * ld + 256, dtype=torch.float64, device="cuda")
    buf[: (H + 2) * ld].view(H + 2, ld)[1:H + 1, off:off + W] = x.reshape(H, W)
    return buf


def unframe(buf, H, W, ld):
    return buf[: (H + 2) * ld].view(H + 2, ld)[1:H + 1, 15:15 + W].clone()


ref_sweep = ref_join = None
for ld in ((L0.ld, L0.ld + 32) if QUICK else (L0.ld, L0.ld + 16, L0.ld + 32, L0.ld + 96, L0.ld + 224, L0.ld + 480)):
    bs = (N + 2) * ld
    ub, fb, ob = framed(uin, N, N, ld), framed(fin, N, N, ld), framed(uin, N, N, ld)
    sw = lambda: _lib.call("mg_sweep", s.dtype, ub.data_ptr(), fb.data_ptr(), ob.data_ptr(), None, s.ktab.data_ptr(),
                           s.omd.data_ptr(), 1, 1, N, N, ld, bs, st.cuda_stream)
    sw()
    torch.cuda.synchronize()
    r = unframe(ob, N, N, ld)
    if ref_sweep is None:
        ref_sweep = r
    ok = torch.equal(r, ref_sweep)
    t = ev_time(sw)
    print(f"product sweep 8193^2 ld {ld} (+{(ld - L0.ld) * 8} B): {t * 1e6:7.1f} us  "
          f"{24 * (N - 2) ** 2 / t / 1e12:.2f} TB/s  bitwise {'ok' if ok else 'MISMATCH'}", flush=True)
    for ldc in (L1.ld,) if QUICK else (L1.ld, L1.ld + 16 * ((ld - L0.ld) // 32)):
        ecb = framed(ecin, L1.H, L1.W, ldc)
        fcb = torch.zeros_like(ecb)
        jn = lambda: _lib.call("mg_cycle_join", s.dtype, ub.data_ptr(), ecb.data_ptr(), fb.data_ptr(), ob.data_ptr(),
                               fcb.data_ptr(), None, None, s.ktab.data_ptr(), s.omd.data_ptr(), 1, s.ptab.data_ptr(), 1,
                               s.rtab.data_ptr(), 1, s.w[1], s.w[0], 1, N, N, ld, bs, ldc, (L1.H + 2) * ldc,
                               None, None, None, st.cuda_stream)
        jn()
        torch.cuda.synchronize()
        r = (unframe(ob, N, N, ld), unframe(fcb, L1.H, L1.W, ldc))
        if ref_join is None:
            ref_join = r
        ok = torch.equal(r[0], ref_join[0]) and torch.equal(r[1], ref_join[1])
        t = ev_time(jn)
        jb = 24 * (N - 2) ** 2 + 16 * (L1.H - 2) ** 2
        print(f"product join  8193^2 ld {ld} ldc {ldc}: {t * 1e6:7.1f} us  {jb / t / 1e12:.2f} TB/s  "
              f"bitwise {'ok' if ok else 'MISMATCH'}", flush=True)
        del ecb, fcb
    del ub, fb, ob
    torch.cuda.empty_cache()
