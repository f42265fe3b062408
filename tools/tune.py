# (historical record: its FEANET_TARGET_WAVES / FEANET_JOIN_RB knobs were removed in round 3; the values it chose are compile-time constants now)
"""Interleaved A/B timing of V-cycle variants in one process (guide §5.4 rule 24).

Each variant = solver kwargs + environment knobs (FEANET_TARGET_WAVES, FEANET_NT_BYTES) that are
in force while its launch sequence is built and captured into a graph; timings are interleaved.
usage: tune.py N variant-set   (sets: nt, tw, fuse)"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd"))
import torch
from feanet_amd.solver import MultigridSolver

SETS = {
    "nt": {"nt_off": ({}, {"FEANET_NT_BYTES": str(1 << 50)}), "nt_32M": ({}, {}),
           "nt_8M": ({}, {"FEANET_NT_BYTES": str(8 << 20)}), "nt_all": ({}, {"FEANET_NT_BYTES": "0"})},
    "tw": {f"tw{t}": ({}, {"FEANET_TARGET_WAVES": str(t)}) for t in (1024, 2048, 4096, 8192)},
    "fuse": {"fuse": ({}, {}), "nofuse": (dict(fuse=False), {}), "notail": (dict(coarse_tail=False), {})},
    "joinrb": {f"jrb{r}": ({}, {"FEANET_JOIN_RB": str(r)}) for r in (32, 64, 128, 256)},
}


def make(n, kw, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        s = MultigridSolver(n, dtype=torch.float64, **kw)
        g = torch.Generator(device="cuda"); g.manual_seed(0)
        s.set_rhs(f=torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g))
        s.load(); s.vcycle(4); s.vcycle(4); torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return s


def timeit(s, k=30):
    torch.cuda.synchronize(); t = time.perf_counter(); s.vcycle(k); torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e6


n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sets = sys.argv[2:] or ["fuse"]
for name in sets:
    ss = {k: make(n, kw, env) for k, (kw, env) in SETS[name].items()}
    res = {k: [] for k in ss}
    for r in range(7):
        for k, s in ss.items():
            res[k].append(timeit(s))
    for k, v in res.items():
        v.sort()
        print(f"[{name}] {k:8s} median {v[3]:8.1f} us  min {v[0]:8.1f} us", flush=True)
    del ss
    torch.cuda.empty_cache()
