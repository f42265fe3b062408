"""A/B timing of fine-sweep variants (tools/lab/sweep_lab.hip) against fea_mg_sweep_f64, 4097^2 fp64.
Each variant's output is checked bitwise against the product kernel before it is timed."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
from feanet_amd.solver import MultigridSolver
from feanet_amd import _lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lab = ctypes.CDLL(os.path.join(HERE, "sweep_lab.so"))
P, I = ctypes.c_void_p, ctypes.c_int
lab.lab_sweep_f64.argtypes = [I, P, P, P, P, P, I, I, I, P]
s = MultigridSolver(n, dtype=torch.float64)
g = torch.Generator(device="cuda"); g.manual_seed(0)
N = n + 1
s.set_rhs(f=torch.randn(1, 1, N, N, device="cuda", dtype=torch.float64, generator=g))
s.load(torch.randn(1, 1, N, N, device="cuda", dtype=torch.float64, generator=g))
L0 = s.levels[0]
st = torch.cuda.current_stream()
_lib.call("mg_sweep", s.dtype, L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), None, s.ktab.data_ptr(),
          s.omd.data_ptr(), s.ntab, *L0.geom(), st.cuda_stream)
ref = L0.b.clone()
out = L0.a.clone()

def ev_time(fn, reps=40):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st); fn(); e1.record(st)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return t[len(t) // 2] * 1e3

bytes_ = 24 * (N - 2) ** 2
prod = lambda: _lib.call("mg_sweep", s.dtype, L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), None,
                         s.ktab.data_ptr(), s.omd.data_ptr(), s.ntab, *L0.geom(), st.cuda_stream)
res = []
for rep in range(2):
    tp = ev_time(prod)
    res.append(("product", 0, tp))
    for var in (110, 111, 120, 121, 130, 131, 210, 211, 220, 221, 410, 411):
        for rb in (8, 16, 32, 64):
            fn = lambda: lab.lab_sweep_f64(var, L0.a.data_ptr(), L0.f.data_ptr(), out.data_ptr(), s.ktab.data_ptr(),
                                           s.omd.data_ptr(), N, L0.ld, rb, st.cuda_stream)
            if rep == 0:
                out.copy_(L0.a)
                assert fn() == 0
                torch.cuda.synchronize()
                if not torch.equal(out, ref):
                    print(f"variant {var} rb {rb}: MISMATCH", flush=True)
                    continue
            res.append((var, rb, ev_time(fn)))
best = {}
for var, rb, t in res:
    k = (var, rb)
    best[k] = min(best.get(k, 1e9), t)
for (var, rb), t in sorted(best.items(), key=lambda x: x[1]):
    print(f"variant {var!s:8s} rb {rb:3d}: {t:7.2f} us  {bytes_ / t / 1e3:6.0f} GB/s  frac {bytes_ / t / 1e3 / 8000:.3f}")
