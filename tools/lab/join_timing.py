"""How to time the cycle join inside the V-cycle with HIP events (GPU box, under rocprofv3 to compare):
(a) events around every join of an eager replay of vcycle(K); (b) events around whole eager replays
with and without the joins (difference / K); (c) back-to-back isolated joins."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch
import bench
from feanet_amd import _lib
from feanet_amd.solver import MultigridSolver

s = MultigridSolver(4096, dtype=torch.float64)
g = torch.Generator(device="cuda"); g.manual_seed(0)
s.set_rhs(f=torch.randn(1, 1, 4097, 4097, device="cuda", dtype=torch.float64, generator=g))
s.load()
s.vcycle(20)
torch.cuda.synchronize()
K = 100
st = torch.cuda.current_stream()
print("a) per-join events in cycle:", bench.time_join_in_cycle(s, K) * 1e6, "us", flush=True)


def replay(skip_join):
    prog, end = s.joined_program(K)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _, launches in prog:
        for name, args in launches:
            if skip_join and name == "mg_cycle_join":
                continue
            _lib.call(name, s.dtype, *args, st.cuda_stream)
    e1.record(st)
    e1.synchronize()
    s._state = end
    return e0.elapsed_time(e1) * 1e-3


for rep in range(2):
    w, wo = replay(False), replay(True)
    print(f"b) whole replay {w / K * 1e6:.1f} us/cycle, without joins {wo / K * 1e6:.1f}, diff "
          f"{(w - wo) / (K - 1) * 1e6:.1f} us", flush=True)
r = bench.time_fine_kernels(s, 30)
print("c) isolated back-to-back:", r["fea_mg_cycle_join"][0] * 1e6, "us", flush=True)
