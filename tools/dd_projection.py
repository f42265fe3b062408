"""Per-rank projection of the domain-decomposed V-cycle on ONE GPU.

For a global grid split over P ranks (Pr x Pc blocks), one rank's whole program — its distributed levels
0 .. Ld-1 with their ghost lines, the agglomeration copies and the redundant coarse sub-cycle (levels >= Ld
of the global grid) — runs on this GPU with a communicator that moves nothing (NullComm): the time per
V-cycle is that rank's kernel time, i.e. the N-GPU cycle time without communication (PackComm, the default,
runs the halo pack / unpack kernels of every exchange too; --no-pack leaves them out).  The rank with the
most ghost lines (an interior block) bounds the cycle.  Reported per Ld beside the single-GPU solver on the
same global grid, so the agglomeration level can be chosen from measurements.

GPU box:  python tools/dd_projection.py [--n 8192] [--steps 50] [--ld 3,4,5,6] [--out FILE.json]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "multigrid-feanet_amd"))
import torch  # noqa: E402

from feanet_amd.dd import DDSolver, default_grid, default_agglomeration, global_levels, halo_staging, copy_blocks  # noqa: E402
from feanet_amd.solver import MultigridSolver  # noqa: E402


class NullComm:
    """A communicator that moves nothing: exchanges and the all-gather are no-ops, the all-reduce is the
    identity.  Only for timing one rank's kernels (values are not those of a real decomposition)."""
    gpu = True
    capturable = True  # (--segments: False, the segment-wise path)

    def exchange_many(self, s, items, wait=True, packed=False):
        return None

    def exchange(self, s, l, name, d):
        return None

    def exchange_finish(self, handle):
        return None

    def allgather(self, target, source):
        return None

    def allreduce_sum(self, t):
        return t


class PackComm(NullComm):
    """NullComm plus the halo exchange's device work: the pack into the staging buffer (folded into the kernel
    segment before the exchange, as with TorchComm) and the unpack from it (dd.halo_staging: the same kernels
    and plans as TorchComm) — only the messages are missing."""

    def _staging(self, s, items):
        plans = s.__dict__.setdefault("_pack_plans", {})
        if tuple(items) not in plans:
            regs = [r for l, name, d in items for r in s.regions(l, name, d)]
            direct = all(a.is_contiguous() and b.is_contiguous() for _, _, a, b in regs)  # row slabs: in place
            st = halo_staging(regs)[:2] if regs and not direct else None
            if st is not None:
                st[1].buf.zero_()
            plans[tuple(items)] = st
        return plans[tuple(items)]

    def halo_pack(self, s, *item_lists):
        import numpy as np
        sends = [st[0] for st in (self._staging(s, items) for items in item_lists if items) if st is not None]
        if not sends:
            return None
        recs = np.concatenate([x.records for x in sends])
        return lambda stream: copy_blocks(recs, True, sends[0].esz, sends[0].buf.device, stream)

    def exchange_many(self, s, items, wait=True, packed=False):
        st = self._staging(s, items)
        if st is not None:
            if not packed:
                st[0].copy(True)
            st[1].copy(False)
        return None


def time_cycles(vcycle, steps, reps=3):
    for _ in range(4):  # eager run + graph capture of every chunk, then warm replays
        vcycle(steps)
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        vcycle(steps)
        th = (time.perf_counter() - t0) / steps  # host issue time (the GPU is host-bound when it is ~ t)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / steps
        if best is None or t < best:
            best = t
            time_cycles.host = th
    return best


def coarse_plan_time(s, reps):
    """GPU time of the replicated coarse sub-cycle as the decomposed cycle runs it: the coarse solver's launch
    plan (levels >= Ld) captured as one HIP graph, `reps` back-to-back replays timed with HIP events on the
    stream (no load(), no host issue in the measurement)."""
    from feanet_amd.dd import _launch_list
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        _launch_list(s.coarse_plan, s.dtype, st)  # eager once
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph, stream=st):
            _launch_list(s.coarse_plan, s.dtype, st)
        for _ in range(3):
            gph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            gph.replay()
        e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def interior_rank(Pr, Pc):
    """A rank with the most neighbours (ghost lines on every side it can have)."""
    ri = 1 if Pr > 2 else 0
    ci = 1 if Pc > 2 else 0
    return ri * Pc + ci


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--ld", default=None, help="agglomeration levels to try (default: default-1 .. default+2)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-pack", action="store_true", help="leave out the halo pack / unpack kernels")
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel eagerly (no HIP graphs)")
    ap.add_argument("--segments", action="store_true",
                    help="one graph per kernel segment between communication steps (the path of communicators that "
                         "cannot be captured) instead of whole captured cycles")
    ap.add_argument("--graph-min", type=int, default=None, help="DDSolver(graph_min=): shorter segments eager")
    ap.add_argument("--no-fold-gather", action="store_true",
                    help="DDSolver(fold_gather=False): the agglomeration's staging / placement as copy launches")
    ap.add_argument("--smoother", default="jac", choices=["jac", "hjac"],
                    help="hjac: the learned HRelax smoother (the bench's HNet weights) on both sides")
    ap.add_argument("--problem", default="poisson", choices=["poisson", "interface"],
                    help="interface: the two-material problem (linear transfers) on both sides")
    ap.add_argument("--split", action="store_true",
                    help="captured cycles with the border / interior split of the finest join (DDSolver split_join)")
    args = ap.parse_args()
    n = args.n
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    f = torch.randn(1, 1, n + 1, n + 1, dtype=torch.float64, device="cuda", generator=g)
    skw = {} if args.problem == "poisson" else {"problem": "interface"}
    if args.smoother == "hjac":
        import numpy as np
        w = np.load(os.path.join(HERE, "..", "multigrid-feanet_amd", "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
        skw.update(smoother="hjac", hnet=np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)]))
    single = MultigridSolver(n, dtype=torch.float64, **skw)
    single.set_rhs(f=f)
    single.load()
    t1 = time_cycles(single.vcycle, args.steps)
    print(f"single GPU {n + 1}^2: {t1 * 1e6:.1f} us per V-cycle", flush=True)
    del single
    torch.cuda.empty_cache()
    rec = {"n": n, "smoother": args.smoother, "problem": args.problem, "single_gpu_us": t1 * 1e6, "ranks": {}}
    L = global_levels(n, n)
    for P in (int(x) for x in args.ranks.split(",")):
        Pr, Pc = default_grid(P)
        r = interior_rank(Pr, Pc)
        d = default_agglomeration(n, n, Pr, L, Pc=Pc)
        lds = [int(x) for x in args.ld.split(",")] if args.ld else [x for x in range(d - 1, d + 3) if 1 <= x <= L - 2]
        rec["ranks"][P] = {"grid": f"{Pr}x{Pc}", "rank": r, "default_ld": d, "ld": {}}
        for Ld in lds:
            try:
                comm = NullComm() if args.no_pack else PackComm()
                comm.capturable = not args.segments
                s = DDSolver(n, n, r, P, comm=comm, agglomerate=Ld, grid=(Pr, Pc),
                             graph=not args.no_graph, split_join=args.split, fold_gather=not args.no_fold_gather,
                             **skw, **({} if args.graph_min is None else {"graph_min": args.graph_min}))
            except ValueError as e:
                print(f"P={P} {Pr}x{Pc} Ld={Ld}: not partitionable ({e})", flush=True)
                continue
            s.set_rhs(f)
            s.load()
            t = time_cycles(s.vcycle, args.steps)
            th = time_cycles.host
            c = s.coarse
            c.set_rhs(f=torch.randn(1, 1, c.H, c.W, dtype=torch.float64, device="cuda", generator=g))
            tc = coarse_plan_time(s, args.steps)
            p0, q0 = s.parts[0], s.cparts[0]
            info = {"us_per_cycle": t * 1e6, "host_issue_us_per_cycle": th * 1e6, "coarse_subcycle_us": tc * 1e6,
                    "local_fine": f"{p0.Hloc}x{q0.Hloc}", "ghost0": s.part.ghost(0), "depths": list(s.depths),
                    "coarse_grid": f"{c.H}x{c.W}", "projected_speedup": t1 / t}
            rec["ranks"][P]["ld"][Ld] = info
            print(f"P={P} {Pr}x{Pc} rank {r} Ld={Ld}: {t * 1e6:7.1f} us per cycle (host issue {th * 1e6:5.1f} us; coarse sub-cycle {tc * 1e6:5.1f} "
                  f"us GPU on {c.H}x{c.W}; local fine {p0.Hloc}x{q0.Hloc}, ghost {s.part.ghost(0)}), speed-up "
                  f"{t1 / t:.2f} (no communication)", flush=True)
            del s, c
            torch.cuda.empty_cache()
    if args.out:
        json.dump(rec, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
