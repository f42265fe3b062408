"""Lab: where the fixed cost of a synchronised vcycle(k) call goes (4097^2 fp64 solver, graph replay).
For k = 1, 2, 5, 10, 20: the wall time of [synchronize; vcycle(k); synchronize] (the bench's timed region), the
GPU time between HIP events recorded just before and after the call on the solver's stream, and the host time
of the call alone.  SPIN=1 sets hipDeviceScheduleSpin through hipSetDeviceFlags before torch touches the GPU
(the synchronize then polls instead of waiting for an interrupt)."""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
for p in (os.path.join(ROOT, "multigrid-feanet_amd"), ROOT):
    sys.path.insert(0, p)
if os.environ.get("SPIN") == "2":  # round-5 first probe: the system HIP runtime loaded BEFORE torch's own copy
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(int(os.environ.get("SPIN_FLAG", "1"))))  # 1 = hipDeviceScheduleSpin
    print("hipSetDeviceFlags (system runtime, before torch) rc", rc, flush=True)
import torch  # noqa: E402
if os.environ.get("SPIN") == "1":  # torch's own runtime, before the device context exists
    _p = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    _h = ctypes.CDLL(_p if os.path.exists(_p) else "libamdhip64.so.7")
    print("hipSetDeviceFlags(spin) rc", _h.hipSetDeviceFlags(ctypes.c_uint(1)), flush=True)

from feanet_amd.solver import MultigridSolver  # noqa: E402

s = MultigridSolver(4096, dtype=torch.float64)
g = torch.Generator(device="cuda")
g.manual_seed(1)
s.set_rhs(f=torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
s.load()
st = torch.cuda.current_stream()
for k in (1, 2, 5, 10, 20, 40):
    for _ in range(8):
        s.vcycle(k)
    torch.cuda.synchronize()
    wall, gpu, host = [], [], []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        s.vcycle(k)
        e1.record(st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        wall.append(t2 - t0)
        host.append(t1 - t0)
        gpu.append(e0.elapsed_time(e1) * 1e-3)
    med = lambda x: sorted(x)[len(x) // 2] * 1e6
    print(f"k={k:3d}: wall {med(wall):8.1f} us ({med(wall) / k:6.1f}/cycle)  gpu(events) {med(gpu):8.1f} us "
          f"({med(gpu) / k:6.1f}/cycle)  host call {med(host):6.1f} us  wall-gpu {med(wall) - med(gpu):6.1f}", flush=True)
# an empty synchronize and a trivial kernel round trip
x = torch.zeros(1, device="cuda")
ts = []
for _ in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x.add_(1)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"trivial kernel round trip {sorted(ts)[25] * 1e6:.1f} us", flush=True)
print("HIP runtimes mapped:", sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}), flush=True)
