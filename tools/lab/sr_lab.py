"""A/B: overlapped-strip SR (tools/lab/sr_lab.hip) vs fea_mg_sweep_restrict_f64 at 4097^2; bitwise check first."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lab = ctypes.CDLL(os.path.join(HERE, "sr_lab.so"))
P, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
lab.lab_sr_f64.argtypes = [I, P, P, P, P, P, P, P, D, I, I, I, I, I, P]
s = MultigridSolver(n, dtype=torch.float64)
g = torch.Generator(device="cuda"); g.manual_seed(0)
N = n + 1
s.set_rhs(f=torch.randn(1, 1, N, N, device="cuda", dtype=torch.float64, generator=g))
s.load(torch.randn(1, 1, N, N, device="cuda", dtype=torch.float64, generator=g))
L0, L1 = s.levels[0], s.levels[1]
st = torch.cuda.current_stream()
args = (L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), L1.f.data_ptr(), None, s.ktab.data_ptr(), s.omd.data_ptr(),
        1, s.rtab.data_ptr(), 1, s.w[0]) + L0.geom() + (L1.ld, L1.bs)
prod = lambda: _lib.call("mg_sweep_restrict", s.dtype, *args, st.cuda_stream)
prod(); torch.cuda.synchronize()
ref_u, ref_f = L0.b.clone(), L1.f.clone()
uo = L0.a.clone(); fc = torch.zeros_like(L1.f)

def ev_time(fn, reps=40):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st); fn(); e1.record(st)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return t[len(t) // 2] * 1e3

nodes = (N - 2) ** 2
bytes_ = 24 * nodes + 8 * ((N + 1) // 2 - 2) ** 2
res = []
for rep in range(2):
    res.append(("product", 0, 0, ev_time(prod)))
    for nt in (11, 21, 41, 61, 40):
        for rb in (32, 64):
            fn = lambda: lab.lab_sr_f64(nt, L0.a.data_ptr(), L0.f.data_ptr(), uo.data_ptr(), fc.data_ptr(),
                                        s.ktab.data_ptr(), s.omd.data_ptr(), s.rtab.data_ptr(), s.w[0], N, N, L0.ld,
                                        L1.ld, rb, st.cuda_stream)
            if rep == 0:
                uo.copy_(L0.a); fc.zero_()
                assert fn() == 0
                torch.cuda.synchronize()
                okU = torch.equal(L0.view(uo), L0.view(ref_u))
                okF = torch.equal(L1.view(fc)[:, 1:-1, 1:-1], L1.view(ref_f)[:, 1:-1, 1:-1])
                if not (okU and okF):
                    du = (L0.view(uo) - L0.view(ref_u)).abs().max().item()
                    df = (L1.view(fc) - L1.view(ref_f))[:, 1:-1, 1:-1].abs().max().item()
                    print(f"nt {nt} rb {rb}: MISMATCH u {du:.3e} f {df:.3e}", flush=True)
            res.append(("ovl", nt, rb, ev_time(fn)))
best = {}
for k, nt, rb, t in res:
    best[(k, nt, rb)] = min(best.get((k, nt, rb), 1e9), t)
for (k, nt, rb), t in sorted(best.items(), key=lambda x: x[1]):
    print(f"{k:8s} nt {nt} rb {rb:3d}: {t:7.2f} us  {bytes_ / t / 1e3:6.0f} GB/s  frac {bytes_ / t / 1e3 / 8000:.3f}")
