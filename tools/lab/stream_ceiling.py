"""The HBM streaming ceiling on this box for fields beyond the Infinity Cache (tools/lab/stream_probe.hip
`lab_flow`): read-only, write-only, copy and 2-read + 1-write linear streams with 1..8 pieces in flight
per wave, normal / nontemporal loads and stores; then the allocation (placement) spread of one stream and
of the product sweep at 8193^2 over fresh allocations.
GPU box: python tools/lab/stream_ceiling.py [pmc]   (pmc: a short fixed set for rocprofv3 --pmc passes)"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
from feanet_amd import _lib
from feanet_amd.solver import MultigridSolver

PMC = len(sys.argv) > 1 and sys.argv[1] == "pmc"
lab = ctypes.CDLL(os.path.join(HERE, "stream_probe.so"))
P, I, LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
lab.lab_flow.argtypes = [I, P, P, P, P, LL, I, P]
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


def bufs(mib):
    n = mib * 2 ** 20 // 8
    return [torch.randn(n, dtype=torch.float64, device="cuda") for _ in range(4)], n * 8 // 1024


def flows(variants, mib=540, rb=32):
    (a, b, c, d), pieces = bufs(mib)
    pieces -= pieces % rb
    for var in variants:
        nr, nw = var // 10000, (var // 1000) % 10
        fn = lambda: lab.lab_flow(var, a.data_ptr(), b.data_ptr(), c.data_ptr(), d.data_ptr(), pieces, rb, st.cuda_stream)
        assert fn() == 0, var
        t = ev_time(fn, 10 if PMC else 20)
        by = (nr + nw) * pieces * 1024
        print(f"flow {mib} MiB rb {rb} R{nr} W{nw} depth {(var // 100) % 10} ntl {(var // 10) % 10} nts {var % 10}: "
              f"{t * 1e6:7.1f} us  {by / t / 1e12:.2f} TB/s", flush=True)
    del a, b, c, d
    torch.cuda.empty_cache()


def product(n, reps=20, tag=""):
    N = n + 1
    s = MultigridSolver(n, dtype=torch.float64, levels=3)
    L0, L1 = s.levels[0], s.levels[1]
    L0.f.normal_()
    L0.a.normal_()
    L1.a.normal_()
    sw = lambda: _lib.call("mg_sweep", s.dtype, L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), None,
                           s.ktab.data_ptr(), s.omd.data_ptr(), 1, *L0.geom(), st.cuda_stream)
    name, args = s._join_call("a", L1.a.data_ptr())
    jn = lambda: _lib.call(name, s.dtype, *args, st.cuda_stream)
    ts, tj = ev_time(sw, reps), ev_time(jn, reps)
    print(f"product {N}^2 {tag}: sweep {ts * 1e6:7.1f} us {24 * (N - 2) ** 2 / ts / 1e12:.2f} TB/s, "
          f"join {tj * 1e6:7.1f} us {(24 * (N - 2) ** 2 + 16 * (L1.H - 2) ** 2) / tj / 1e12:.2f} TB/s", flush=True)
    del s
    torch.cuda.empty_cache()


if PMC:
    flows((21201, 21101))
    product(8192, 10)
    sys.exit(0)

flows((10100, 10200, 10400, 10800, 10410, 20200, 20400))                 # read-only
flows((1100, 1101))                                                      # write-only
flows((11101, 11201, 11401, 11801, 11200, 11411))                        # copy
flows((21101, 21201, 21401, 21801, 21200, 21400, 21411, 21211))          # 2 reads + 1 write
flows((21201, 11201, 10200), mib=2048)                                    # larger fields
flows((21201, 21401), rb=8)
flows((21201, 21401), rb=128)
# placement spread: fresh allocations (the caching allocator hands back different blocks each time)
keep = []
for i in range(4):
    keep.append(torch.empty(int((i + 1) * 97e6) // 8, dtype=torch.float64, device="cuda"))  # shifts the next blocks
    flows((21201,))
    product(8192, tag=f"alloc {i}")
