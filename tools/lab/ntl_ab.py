"""Same-process A/B of library builds on the fine-level kernels (sweep, cycle join) at the sizes beyond the
Infinity Cache: two builds are loaded side by side (each CDLL keeps its own kernels) and timed on the SAME
buffers, alternating, so allocation placement cannot bias the comparison; outputs are compared bitwise.
Then (C5 only) the join's task-height knobs on the in-tree build.
GPU box:  python3 tools/lab/ntl_ab.py VARIANT.so"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multigrid-feanet_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from feanet_amd import _lib  # noqa: E402
from feanet_amd.solver import MultigridSolver  # noqa: E402

base = _lib.lib()
_lib._lib = None
_lib.LIB = os.path.abspath(sys.argv[1])
var = _lib.lib()
libs = {"in-tree": base, os.path.basename(sys.argv[1]): var}


def run(n, B, T, reps, knobs=False):
    s = MultigridSolver(n, dtype=T, batch=B, levels=3)
    L0, L1 = s.levels[0], s.levels[1]
    g = torch.Generator(device="cuda")
    g.manual_seed(n + B)
    for t in (L0.f, L0.a, L1.a):
        t.normal_(generator=g)
    res = {}
    outs = {}
    for rnd in range(2):
        for name, h in libs.items():
            _lib._lib = h
            L0.b.zero_()
            r = bench.time_fine_kernels(s, reps)
            outs[name] = L0.b.clone()  # the last kernel timed wrote L0.b (cycle join)
            for k, (t, by) in r.items():
                res.setdefault((name, k), []).append(t)
    same = all(torch.equal(o, next(iter(outs.values()))) for o in outs.values())
    for (name, k), ts in sorted(res.items(), key=lambda x: (x[0][1], x[0][0])):
        if k not in ("fea_mg_sweep", "fea_mg_cycle_join"):
            continue
        t = min(ts)
        by = r[k][1]
        print(f"{B} x {n + 1}^2 {T}: {k:18s} {name:22s} {t * 1e6:8.1f} us {by / t / 1e12:.2f} TB/s "
              f"({by / t / 8e12:.3f})  [{', '.join(f'{x * 1e6:.1f}' for x in ts)}]", flush=True)
    print(f"  outputs bitwise equal across builds: {same}", flush=True)
    if knobs:
        _lib._lib = base
        for env in ({}, {"FEANET_JOIN_RB": "16"}, {"FEANET_JOIN_RB": "32"}, {"FEANET_JOIN_RB": "128"},
                    {"FEANET_JOIN_RB": "256"}, {"FEANET_BALANCE": "0"}, {"FEANET_RB_OCC": "3"},
                    {"FEANET_RB_OCC": "2"}, {"FEANET_TARGET_WAVES": "8192"}, {}):
            for k in ("FEANET_JOIN_RB", "FEANET_BALANCE", "FEANET_RB_OCC", "FEANET_TARGET_WAVES"):
                os.environ.pop(k, None)
            os.environ.update(env)
            name, args = s._join_call("a", L1.a.data_ptr())
            t = bench.time_kernel(name, s.dtype, args, reps, torch.cuda.current_stream())
            parts = _lib.join_norm_parts(B, L0.H, L0.W, 4 if T == torch.float32 else 8)
            print(f"  join knobs {env}: {t * 1e6:8.1f} us ({r['fea_mg_cycle_join'][1] / t / 8e12:.3f}), "
                  f"{B * parts} waves", flush=True)
        for k in ("FEANET_JOIN_RB", "FEANET_BALANCE", "FEANET_RB_OCC", "FEANET_TARGET_WAVES"):
            os.environ.pop(k, None)
    del s
    torch.cuda.empty_cache()


run(8192, 1, torch.float64, 10)
run(1024, 256, torch.float32, 5, knobs=True)
run(4096, 1, torch.float64, 20)
