#!/usr/bin/env python3
"""Benchmark: DoF-updates/s per V-cycle (fp64) + achieved HBM GB/s, 4097^2 Poisson (BASELINE.json).

One "step" = one full V-cycle (12 levels, V(1,1), the reference's MultiGrid.Step schedule) of the
fused HIP kernels on a 4097 x 4097 fp64 Poisson problem resident in HBM (synthetic seeded
right-hand side, zero initial guess), replayed as a HIP graph.  value = B * N^2 * ranks / t_step.

Also reported on the same JSON line:
  roofline      the DOMINANT kernel of the timed region: fea_mg_cycle_join on the finest level (every
                boundary between two V-cycles: post-sweep of cycle k + pre-sweep, residual and
                restriction of cycle k+1; 28 B per fine node, ~45 % of a V-cycle), timed INSIDE the
                cycle (HIP events around each join launch of an eager replay of vcycle(K), on the
                solver's stream); achieved = algorithmic bytes per launch / that average, vs the
                8 TB/s HBM peak; `traffic` = measured HBM bytes per launch from rocprofv3 PMC
                (profiles/pmc_traffic.json, if present)
  north_star_kernel  the fine-level Ke-stencil Jacobi sweep fea_mg_sweep on its own (24 B per node:
                read u, read f, write u'), back-to-back launches — the north star's >= 70 % target
  fine_level_kernels  the same measurement (isolated, back-to-back) for every level-0 kernel
  cpu_baseline  the reference's PyTorch-CPU formulation (oracle/torch_cpu.py: conv2d / conv_transpose2d,
                MultiGrid.Step) on the same workload with all of this job's host cores, a bounded sample
                of whole V-cycles, rank 0 at N = 1 only (the 1-thread numpy oracle beside it).

Multi-GPU (torchrun, one process per GPU): domain decomposition (feanet_amd.dd) of ONE global grid,
8193^2 by default (BASELINE config C4; strong scaling: the same grid over 2, 4, 8 GPUs), 2-D blocks
(2x1, 2x2, 4x2) with a one-phase RCCL halo exchange (up to eight neighbours) once per V-cycle and an agglomerated coarse
solve; value = global DoF / t_step.  --weak keeps 4096 x 4096 intervals per GPU instead (4097^2,
8193x4097, 8193^2, 16385x8193); --mode replicas runs independent problems.  At N = 1 the default is
the metric configuration (4097^2, one GPU, no decomposition).  Timing: barrier + synchronize on both
sides of the K steps, max over ranks.
"""
import argparse
import contextlib
import faulthandler
import json
import math
import os
import sys
import threading
import time
from datetime import timedelta

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "DoF-updates/sec per V-cycle (fp64) + achieved HBM GB/s, 4097² Poisson"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


EXIT_HANG = 3  # a bounded phase ran out of time (PhaseGuard)


def dist_init(force=False, backend="nccl", timeout_s=150.0, cuda=True):
    """One process per GPU (torchrun env).  force: create the process group even for one rank (the
    domain-decomposed path always talks through torch.distributed).  backend "gloo": rehearsal of the
    multi-rank path with several processes on one GPU (RCCL refuses two ranks on one device).  timeout_s: the
    process group's collective timeout (both backends; with RCCL async error handling on, a collective stuck
    past it aborts the communicator and ends the process instead of waiting for the 10-minute default)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if cuda:
        if backend == "gloo":  # rehearsal: more ranks than GPUs share them
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
    if ws > 1 or force:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(ws))
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        to = timedelta(seconds=timeout_s)
        if backend == "gloo":
            dist.init_process_group("gloo", timeout=to)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=to)
    return ws, rank


class PhaseGuard:
    """Bounded phases of a run, one guard per rank.  A phase that outlives its limit — a collective that a peer
    never entered, a captured RCCL block whose messages never complete — ends THIS process (os._exit, never an
    exec) instead of holding every rank until the driver's timeout: the guard's thread names the rank and the
    phase on stderr, dumps every thread's stack, runs the phase's on_expire (which may print the record so far
    and choose the exit status; default EXIT_HANG) and exits.  Collectives and graph replays release the GIL, so
    the thread runs while the main thread waits in one; faulthandler's own timer (no GIL needed) backs it up
    30 s later.  Every rank guards the same phases, so a hang in a collective ends all of them."""

    def __init__(self, rank):
        self.rank = rank
        self.cv = threading.Condition()
        self.cur = None  # (name, deadline, seconds, on_expire)
        threading.Thread(target=self._watch, daemon=True, name="bench-phase-guard").start()

    @contextlib.contextmanager
    def phase(self, name, seconds, on_expire=None):
        with self.cv:
            prev = self.cur
            self.cur = (name, time.monotonic() + seconds, seconds, on_expire)
            self.cv.notify_all()
        faulthandler.dump_traceback_later(seconds + 30, exit=True)
        try:
            yield
        finally:
            faulthandler.cancel_dump_traceback_later()
            with self.cv:
                self.cur = prev
                self.cv.notify_all()
            if prev is not None:
                faulthandler.dump_traceback_later(max(1.0, prev[1] - time.monotonic()) + 30, exit=True)

    def _watch(self):
        with self.cv:
            while True:
                if self.cur is None:
                    self.cv.wait()
                    continue
                left = self.cur[1] - time.monotonic()
                if left > 0:
                    self.cv.wait(left)
                    continue
                name, _, seconds, on_expire = self.cur
                break
        log(f"[bench] rank {self.rank}: phase '{name}' did not finish within {seconds:.0f} s (a collective or "
            f"communication step some rank never completed); exiting")
        faulthandler.dump_traceback(all_threads=True)
        code = EXIT_HANG
        if on_expire is not None:
            try:
                code = on_expire(name, seconds)
            except BaseException as e:  # the exit must happen whatever the callback does
                log(f"[bench] rank {self.rank}: on_expire failed: {e!r}")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, ws):
    if ws == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def time_kernel(name, dtype, args, reps, stream):
    """Average duration of one C-ABI kernel launch from HIP events recorded on its stream."""
    from feanet_amd import _lib
    for _ in range(3):
        _lib.call(name, dtype, *args, stream.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(stream)
        _lib.call(name, dtype, *args, stream.cuda_stream)
        e1.record(stream)
    ev[-1][1].synchronize()
    return sum(e0.elapsed_time(e1) for e0, e1 in ev) / reps * 1e-3


def time_fine_kernels(s, reps):
    """The fine-level kernels at 4097^2: the north-star sweep (fea_mg_sweep, the `roofline` kernel) and
    the fused kernels the V-cycle actually runs on level 0: sweep+residual+restriction (first cycle),
    prolongation+correction+sweep (last cycle) and the cycle join (every boundary between two
    cycles: read u, f, e_c; write u, f_c).  Returns {name: (seconds per launch, algorithmic bytes)}."""
    L0, L1 = s.levels[0], s.levels[1]
    st = torch.cuda.current_stream()
    es = torch.finfo(s.dtype).bits // 8
    nodes = L0.B * (L0.H - 2) * (L0.W - 2)
    cnodes = L1.B * (L1.H - 2) * (L1.W - 2)
    geom = L0.geom()
    kt, om, nt = s.ktab.data_ptr(), s.omd.data_ptr(), s.ntab
    p0 = None if L0.pid is None else L0.pid.data_ptr()
    p1 = None if L1.pid is None else L1.pid.data_ptr()
    nr, npt = s.rtab.shape[0], s.ptab.shape[0]
    pb = 1 if L0.pid is not None else 0  # two-material problems read a pattern byte per node
    out = {}
    args = (L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), p0, kt, om, nt) + geom
    out["fea_mg_sweep"] = (time_kernel("mg_sweep", s.dtype, args, reps, st), (3 * es + pb) * nodes)
    args = (L0.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), L1.f.data_ptr(), p0, kt, om, nt,
            s.rtab.data_ptr(), nr, s.w[0]) + geom + (L1.ld, L1.bs, None, None, None)
    out["fea_mg_sweep_restrict"] = (time_kernel("mg_sweep_restrict", s.dtype, args, reps, st),
                                    (3 * es + pb) * nodes + es * cnodes)
    args = (L0.a.data_ptr(), L1.a.data_ptr(), L0.f.data_ptr(), L0.b.data_ptr(), p0, p1, kt, om, nt,
            s.ptab.data_ptr(), npt, s.w[1]) + geom + (L1.ld, L1.bs)
    out["fea_mg_prolong_sweep"] = (time_kernel("mg_prolong_sweep", s.dtype, args, reps, st),
                                   (3 * es + pb) * nodes + (es + pb) * cnodes)
    name, args = s._join_call("a", L1.a.data_ptr())
    out["fea_mg_cycle_join"] = (time_kernel(name, s.dtype, args, reps, st),
                                (3 * es + pb) * nodes + (2 * es + pb) * cnodes)
    if s.smoother == "hjac":  # the learned smoother's fused sweep (Jacobi + 3 masked convs, one pass)
        args = (L0.a.data_ptr(), None, L0.f.data_ptr(), L0.b.data_ptr(), p0, kt, om, nt, s.hw.data_ptr(), s.nl) + geom
        out["fea_mg_hsweep"] = (time_kernel("mg_hsweep", s.dtype, args, reps, st), (3 * es + pb) * nodes)
    return out


def time_join_in_cycle(s, k):
    """The cycle-join kernel timed INSIDE the V-cycle with HIP events on the solver's stream: two eager
    replays of vcycle(k)'s launch sequence (same kernels, buffers and cache history as the graph
    replays); in the first an event pair brackets [the launch before each join, the join], in the
    second [the launch before each join] alone.  The difference of the two averages is the join's
    duration with the event pair's own dispatch overhead cancelled.  Returns seconds per join
    (None if the solver does not join cycles)."""
    from feanet_amd import _lib
    if not s._joinable() or k < 2:
        return None
    st = torch.cuda.current_stream()

    def replay(with_join):
        prog, end = s.joined_program(k)
        ev = []
        for _, launches in prog:
            for i, (name, args) in enumerate(launches):
                nxt = launches[i + 1][0] if i + 1 < len(launches) else None
                if nxt == "mg_cycle_join":  # the launch before a join opens the bracket
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    _lib.call(name, s.dtype, *args, st.cuda_stream)
                    if not with_join:
                        e1.record(st)
                    ev.append((e0, e1))
                elif name == "mg_cycle_join":
                    _lib.call(name, s.dtype, *args, st.cuda_stream)
                    if with_join:
                        ev[-1][1].record(st)
                else:
                    _lib.call(name, s.dtype, *args, st.cuda_stream)
        s._state = end
        ev[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / len(ev) * 1e-3

    with_join = replay(True)
    without = replay(False)
    return with_join - without


def time_fine_launch_in_cycle(s, reps=5):
    """Solvers whose cycles are not joined (the learned smoother's MG-HJac schedule): every launch of the V-cycle
    plan timed INSIDE the cycle — eager replays of the plan with a HIP event on the solver's stream between
    consecutive launches — and the slowest finest-level launch returned as (kernel name, seconds per launch,
    algorithmic bytes per launch).  Algorithmic bytes per fine node / coarse node: hsweep u, f -> u' (3 es);
    hsweep + restriction also writes f_c (es per coarse node); prolongation + hsweep also reads e_c (es)."""
    from feanet_amd import _lib
    st = torch.cuda.current_stream()
    L0, L1 = s.levels[0], s.levels[1]
    f0 = L0.f.data_ptr()
    es = torch.finfo(s.dtype).bits // 8
    pb = 1 if L0.pid is not None else 0
    nodes = L0.B * (L0.H - 2) * (L0.W - 2)
    cnodes = L1.B * (L1.H - 2) * (L1.W - 2)
    fslot = {"mg_hsweep": 2, "mg_hsweep_restrict": 2, "mg_prolong_hsweep": 3, "mg_sweep": 1,
             "mg_sweep_restrict": 1, "mg_prolong_sweep": 2}
    cbytes = {"mg_hsweep": 0, "mg_sweep": 0, "mg_hsweep_restrict": es, "mg_sweep_restrict": es,
              "mg_prolong_hsweep": es + pb, "mg_prolong_sweep": es + pb}
    acc = {}
    for _ in range(reps):
        plan, end = s._plan(s._state)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(plan) + 1)]
        ev[0].record(st)
        for i, (name, args) in enumerate(plan):
            _lib.call(name, s.dtype, *args, st.cuda_stream)
            ev[i + 1].record(st)
        s._state = end
        ev[-1].synchronize()
        for i, (name, args) in enumerate(plan):
            if name in fslot and args[fslot[name]] == f0:
                acc.setdefault((i, name), []).append(ev[i].elapsed_time(ev[i + 1]) * 1e-3)
    if not acc:
        return None
    (i, name), ts = max(acc.items(), key=lambda kv: sum(kv[1]))
    return "fea_" + name, sum(ts) / len(ts), (3 * es + pb) * nodes + cbytes[name] * cnodes


def load_traffic(kernel_key):
    """Measured HBM bytes per launch from a rocprofv3 PMC record (profiles/pmc_traffic.json), only if it was
    taken on the kernel source this run executes (SHA-256 stamp of csrc/framed_ops.hip); else (None, why)."""
    from tools.pmc_traffic import kernel_source_sha
    p = os.environ.get("FEANET_PMC_TRAFFIC", os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        rec = d.get(kernel_key)
        if not rec:
            return None, None
        if rec.get("kernel_source_sha256") != kernel_source_sha():
            return None, f"{os.path.relpath(p, ROOT)} was measured on other kernel source (stale), not reported"
        return rec["hbm_bytes_per_launch"], rec.get("source")
    except Exception:
        return None, None


def host_threads():
    """Host cores for the CPU baseline: the process's CPU affinity, capped by OMP_NUM_THREADS
    when the environment sets it (the GPU box gives one GPU's job a 16-core share of a larger host)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, len(os.sched_getaffinity(0))


def _time_cycles(step, v, seconds_budget, max_timed=5):
    t0 = time.perf_counter()
    v = step(v)  # warm-up cycle (page-in, allocation)
    first = time.perf_counter() - t0
    k = max(3, min(max_timed, int(seconds_budget / max(first, 1e-3)) - 1))
    times = []
    for _ in range(k):
        t0 = time.perf_counter()
        v = step(v)
        times.append(time.perf_counter() - t0)
    return float(np.median(times)), k


def cpu_baseline(n, seconds_budget=16.0):
    """The reference's PyTorch-CPU formulation (oracle/torch_cpu.py: conv2d identity split + stencil,
    f - K u, omega/d, stride-2 conv restriction, conv_transpose2d prolongation — MultiGrid.Step of
    M-FEANet-mg_test.ipynb) on the same 4097^2 fp64 Poisson workload, all host cores of this job; the
    numpy oracle (1 thread) beside it as a secondary number."""
    from oracle import feanet_oracle as orc
    from oracle.torch_cpu import TorchCPUMultigrid
    threads, affinity = host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    N = n + 1
    f = rng.standard_normal((1, 1, N, N))
    ft = torch.from_numpy(f)
    mt = TorchCPUMultigrid(n, dtype=torch.float64)
    with torch.no_grad():
        t, k = _time_cycles(lambda v: mt.step(v, ft), torch.zeros(1, 1, N, N, dtype=torch.float64), seconds_budget)
    torch.set_num_threads(prev)
    mo = orc.OracleMultigrid(n, "poisson", np.float64)
    tn, kn = _time_cycles(lambda v: mo.step(v, f[:, 0]), np.zeros((1, N, N)), 6.0, max_timed=3)
    return {"value": N * N / t, "unit": "DoF-updates/s", "cores": threads, "kind": "port",
            "sample": f"{k} timed V-cycles (median {t:.2f} s, +1 warm-up) of the {N}x{N} fp64 Poisson V(1,1) "
                      f"workload by the reference's PyTorch-CPU formulation restated op for op "
                      f"(oracle/torch_cpu.py: conv2d/conv_transpose2d, MultiGrid.Step), torch.set_num_threads({threads}) "
                      f"(process affinity {affinity} CPUs, OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}), "
                      f"host of the GPU box",
            "torch_threads": threads,
            "numpy_oracle_1thread": {"value": N * N / tn, "unit": "DoF-updates/s", "cores": 1,
                                     "sample": f"{kn} V-cycles (median {tn:.2f} s) by oracle/feanet_oracle.py"}}


def dd_problem_kw(args):
    """Solver keywords of the decomposed run's problem: Poisson, or the two-material problem with the linear or the
    learned (BASELINE C3) transfers; weighted Jacobi or the learned smoother (--smoother hjac) — the same for DDSolver
    and for the single-GPU solver it is checked against."""
    kw = {}
    if args.smoother == "hjac":  # the learned smoother (M-FEANet-mg_test.ipynb HRelax, the bench's HNet weights)
        w = np.load(os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
        kw.update(smoother="hjac", hnet=np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)]))
    if args.problem != "interface":
        return kw
    kw["problem"] = "interface"
    if args.transfer == "learned":
        w = np.load(os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "weights", "multigrid_interface_ratio.npz"))
        kw.update(R=w["R"][0], P=w["P"][:, 0], w=w["w"])
    return kw


def dd_rhs(args, m, n, T, B):
    """The decomposed run's global right-hand side (every rank draws the same one and keeps its block): seeded randn
    f for Poisson, the nodal source F = ones (FNet applied) for the two-material problem."""
    if args.problem == "interface":
        return {"F": torch.ones(B, 1, m + 1, n + 1, device="cuda", dtype=T)}
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    return {"f": torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=T, generator=g)}


def single_gpu_same_grid(args, m, n, T, B, steps, ms_dd):
    """The single-GPU MultigridSolver on the decomposed run's global grid ((m+1) x (n+1), same rhs),
    timed like the main line (warm-up calls, then one vcycle(steps) between synchronisations)."""
    from feanet_amd.solver import MultigridSolver
    s = MultigridSolver(n, rows=None if m == n else m, dtype=T, batch=B, **dd_problem_kw(args))
    s.set_rhs(**dd_rhs(args, m, n, T, B))
    s.load()
    for _ in range(6):
        s.vcycle(steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.vcycle(steps)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    del s
    torch.cuda.empty_cache()
    return {"ms_per_step": t * 1e3, "value": B * (m + 1) * (n + 1) / t, "unit": "DoF-updates/s",
            "speedup_of_this_line": t * 1e3 / ms_dd,
            "workload": f"{m + 1}x{n + 1} {args.problem} V-cycle on one GPU (MultigridSolver, no decomposition), rank 0"}


def dd_reference_block(args, owned, m, n, T, B, cycles=3):
    """The single-GPU MultigridSolver's iterate after `cycles` V-cycles from zero on the decomposed run's global grid
    and rhs, cut to this rank's owned block ((y0, y1), (x0, x1)); run on the rank's own GPU, no
    communication.  The reference point of every dd mode's parity check."""
    from feanet_amd.solver import MultigridSolver
    (y0, y1), (x0, x1) = owned
    ref = MultigridSolver(n, rows=None if m == n else m, dtype=T, batch=B, **dd_problem_kw(args))
    ref.set_rhs(**dd_rhs(args, m, n, T, B))
    ref.load()
    ref.vcycle(cycles)
    exp = ref.solution()[:, :, y0:y1, x0:x1].clone()
    del ref
    torch.cuda.empty_cache()
    return exp


def dd_parity(s, exp, m, n, ws, cycles=3, repeats=3):
    """Every rank: the decomposed solver's owned block after `cycles` V-cycles from zero against the single-GPU
    solver's (dd_reference_block), `repeats` times from a fresh load — the first run of a program is eager, the
    second captures its blocks (capturing communicators) and replays them, the third replays — so the check covers
    the path the timed cycles took.  The decomposed cycle is bitwise the single-GPU one by construction
    (tests/test_gpu_dd.py); this puts that claim on the line of every multi-GPU run, i.e. on the RCCL path itself.
    Returns the max over ranks and repeats of the largest absolute difference and of the count of differing nodes."""
    dmax, nbad = 0.0, 0.0
    for _ in range(repeats):
        s.load()
        s.vcycle(cycles)
        _, _, u = s.owned_block()
        dmax = max(dmax, (u - exp).abs().max().item())
        nbad = max(nbad, float((u != exp).sum().item()))
        del u
    gloo = ws > 1 and torch.distributed.get_backend() != "nccl"  # gloo reduces host tensors
    out = torch.tensor([dmax, nbad], dtype=torch.float64, device="cpu" if gloo else "cuda")
    if ws > 1:
        torch.distributed.all_reduce(out, op=torch.distributed.ReduceOp.MAX)
    return {"cycles": cycles, "repeats": repeats, "bitwise_equal": bool(out[1].item() == 0),
            "max_abs_diff": out[0].item(), "max_differing_nodes_per_rank": int(out[1].item()),
            "against": f"single-GPU MultigridSolver on the same {m + 1}x{n + 1} grid, V-cycles from zero, every "
                       f"rank's owned block, {repeats} runs (eager / captured / replayed)"}


def dd_domain(P, n0):
    """Weak-scaled global grid for P slabs of n0 x n0 intervals each, aspect ratio <= 2 when P is a
    power of two: 1 -> n0 x n0, 2 -> 2n0 x n0, 4 -> 2n0 x 2n0, 8 -> 4n0 x 2n0 (rows x columns)."""
    if P & (P - 1) == 0:
        k = P.bit_length() - 1
        return n0 << ((k + 1) // 2), n0 << (k // 2)
    return n0 * P, n0


def launch_ranks(n, timeout_s):
    """`bench.py --gpus N` (N > 1) started without a launcher: run the same command line under
    torch.distributed.run (one rank per GPU, rendezvous on 127.0.0.1) as a CHILD process — nothing here has
    touched the GPU, and the process is not replaced (no exec) — forward its one JSON line to stdout (anything
    else it printed there goes to stderr) and return its exit status.  The child gets timeout_s in all (the
    ranks bound their own phases well inside it, PhaseGuard); past it the launcher's process group is killed and
    the status is EXIT_HANG.  The port is picked by binding port 0 and released just before the launch (a small
    window in which another process could take it; the rendezvous then fails loudly, it does not hang)."""
    import signal
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n} without a launcher: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout_s)
        rc = p.returncode
    except subprocess.TimeoutExpired:
        log(f"[bench] the {n} ranks did not finish within {timeout_s:.0f} s: killing them")
        os.killpg(p.pid, signal.SIGKILL)
        out, _ = p.communicate()
        rc = EXIT_HANG
    lines = out.splitlines()
    recs = [ln for ln in lines if ln.startswith("{")]
    for ln in lines:
        if not ln.startswith("{"):
            log(ln)
    if recs:
        print(recs[-1], flush=True)
    if rc == 0 and len(recs) != 1:
        log(f"[bench] expected one JSON line from rank 0, got {len(recs)}")
        return 1
    return rc


def selftest_hang(args):
    """--selftest-hang S (CPU, gloo, >= 2 ranks): rank 1 never enters the barrier rank 0 waits in, under the same
    process-group timeout and PhaseGuard the GPU path uses (limit S), so the run must end non-zero within about S
    seconds with the rank and phase named on stderr (tests/test_bench_cli.py)."""
    ws, rank = dist_init(force=True, backend="gloo", timeout_s=4 * args.selftest_hang, cuda=False)
    guard = PhaseGuard(rank)
    import torch.distributed as dist
    with guard.phase("selftest: barrier that rank 1 skips", args.selftest_hang):
        if rank == 1:
            time.sleep(10 * args.selftest_hang)
        dist.barrier()
    return 0


# domain-decomposition modes timed on every N > 1 line, safest first: (name, whole-cycle capture, level-0 halo
# overlapped with the coarse levels, finest join split into border rectangles + the exchange on a side stream)
DD_MODES = [("segments", False, False, False), ("segments+overlap_l0", False, True, False),
            ("segments+split_join", False, False, True), ("captured", True, False, False),
            ("captured+overlap_l0", True, True, False), ("captured+split_join", True, False, True)]


def time_steps(s, steps, warmup, ws):
    """The contract's timing: warm-up calls of the timed call itself (vcycle(steps)), so that every graph the timed
    call replays (its blocks of joined cycles, keyed by start buffer and size; 6 calls cover every step count) has
    run once eagerly and been captured before the clock starts — at least `warmup` cycles; then barrier +
    synchronize, ONE vcycle(steps), synchronize + barrier, max over ranks.  Returns (seconds, warm-up cycles run)."""
    calls = max(6, -(-warmup // steps))
    calls += calls % 2
    for _ in range(calls):
        s.vcycle(steps)
    torch.cuda.synchronize()
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.vcycle(steps)
    torch.cuda.synchronize()
    barrier(ws)
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, ws), calls * steps


def time_to_solution(conv, ms_step, eps=1e-6):
    """Cycles (and microseconds at the measured rate) to cut the residual by `eps` from the zero guess, at the
    contraction factor measured over the first 8 cycles."""
    if not (0.0 < conv < 1.0):
        return None
    cyc = math.ceil(math.log(eps) / math.log(conv))
    return {"eps": eps, "contraction": conv, "cycles": cyc, "us": cyc * ms_step * 1e3,
            "note": "cycles = ceil(log(eps) / log(contraction)), contraction over the first 8 cycles from zero"}


def jacobi_same_grid(args, B, T, f):
    """MG-Jacobi (the default V(1,1)) on the grid and right-hand side of a --smoother hjac line: its per-cycle time
    (vcycle(K) with K = min(steps, 200), after the same warm-up) and time to 1e-6, beside the learned smoother's."""
    from feanet_amd.solver import MultigridSolver
    s = MultigridSolver(args.n, problem=args.problem, dtype=T, batch=B, levels=args.levels)
    s.set_rhs(f=f)
    s.load()
    conv = contraction(s)
    k = max(1, min(args.steps, 200))
    t, _ = time_steps(s, k, args.warmup, 1)
    ms = t / k * 1e3
    del s
    return {"ms_per_step": ms, "time_to_solution": time_to_solution(conv, ms), "steps": k}


def contraction(s):
    """Residual contraction factor per cycle over the first 8 cycles from zero (before the fp64 floor)."""
    s.load()
    r0 = s.residual_norm()
    s.vcycle(8)
    conv = float((s.residual_norm().max() / r0.max()).item()) ** (1.0 / 8)
    s.load()
    return conv


def roofline_record(fine, lvl, args, jt=None, jsrc=None, dom=None, tkey_ok=False, ws=1):
    """The `roofline` and `north_star_kernel` objects from the fine-level kernel timings (see the module doc)."""
    L0 = lvl.levels[0]
    kt, kbytes = fine["fea_mg_sweep"]
    kt = max_over_ranks(kt, ws)
    if dom is not None:
        name, r_t, r_bytes = dom
        rkern = (f"{name} (fine level {L0.H}x{L0.W} {args.dtype}; the slowest launch of the cycle, which joins no "
                 f"cycles)")
        tkey, jsrc = None, ("HIP events on the solver's stream between consecutive launches of eager replays of the "
                            "V-cycle plan")
    else:
        if jt is None and "fea_mg_cycle_join" in fine:
            jt = fine["fea_mg_cycle_join"][0]
            jsrc = "HIP events, back-to-back launches of fea_mg_cycle_join on the level-0 buffers"
        if jt is not None:
            r_bytes = fine["fea_mg_cycle_join"][1]
            r_t = max_over_ranks(jt, ws)
            rkern = f"fea_mg_cycle_join (fine level {L0.H}x{L0.W} {args.dtype}: post-sweep of cycle k + pre-sweep, " \
                    f"residual and restriction of cycle k+1 in one pass)"
            tkey = "mg_cycle_join_f64_4097"
        else:
            rkern, r_t, r_bytes, tkey, jsrc = (f"fea_mg_sweep ({L0.H}x{L0.W} {args.dtype})", kt, kbytes,
                                               "mg_sweep_f64_4097", "HIP events, back-to-back launches")
    achieved = r_bytes / r_t / 1e9
    traffic, tsrc = load_traffic(tkey) if (tkey_ok and tkey) else (None, None)
    ns_traffic, ns_src = load_traffic("mg_sweep_f64_4097") if tkey_ok else (None, None)
    roof = {"bound": "hbm", "kernel": rkern, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc, "avg_launch_us": r_t * 1e6,
            "algorithmic_bytes_per_launch": r_bytes, "timing": jsrc}
    ns = {"kernel": f"fea_mg_sweep (fine-level Ke-stencil Jacobi sweep, {L0.H}x{L0.W} {args.dtype}, 24 B/node)",
          "achieved": kbytes / kt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": kbytes / kt / 1e9 / HBM_PEAK_GBS,
          "avg_launch_us": kt * 1e6, "algorithmic_bytes_per_launch": kbytes, "traffic": ns_traffic,
          "traffic_source": ns_src, "target_frac": 0.70}
    fl = {k: {"avg_launch_us": tk * 1e6, "algorithmic_bytes": nb, "achieved_GBps": nb / tk / 1e9,
              "frac": nb / tk / 1e9 / HBM_PEAK_GBS} for k, (tk, nb) in fine.items()}
    return roof, ns, fl


def base_record(args, value, ms_step, ws, warm, workload, mode, parallelism, rhs, levels, B):
    return {
        "metric": METRIC,
        "value": value,
        "unit": "DoF-updates/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_executed_steps": warm,
        "warmup_note": ("warmup = the requested --warmup; warmup_executed_steps = the untimed cycles actually run "
                        "before the clock (>= warmup: whole calls of the timed vcycle(steps), so every HIP graph it "
                        "replays is captured before timing)"),
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if (mode == "dd" and not args.weak) else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": {"randn": "synthetic (seeded Gaussian rhs, zero initial guess)",
                 "ones": "synthetic (uniform nodal source F = ones, FNet applied, as MM_Interface_error.ipynb; zero "
                         "initial guess)",
                 "families": "synthetic (nodal sources from the six Data/RHS/generate_rhs.py families, seeded, FNet "
                             "applied; zero initial guess)"}[rhs],
        "config": {"workload": workload, "mode": mode, "batch": B, "levels": levels, "parallelism": parallelism},
    }


def run_dd(args, ws, rank, T, B, guard, emit):
    """The N > 1 line: ONE global grid domain-decomposed over the ranks (feanet_amd.dd), every DD mode of DD_MODES
    selected by --dd-modes timed in turn on the live communicator (each its own solver, warm-up and K timed cycles,
    and its own bitwise dd_parity), each under a bounded phase.  The line's headline (value, ms_per_step,
    config.dd_mode, dd_parity) is the FASTEST mode whose parity is bitwise; every mode is listed under dd_modes.
    The first mode is required (any failure ends the run non-zero); a later mode that fails is recorded and skipped,
    and one that hangs past --mode-timeout ends the run with the record so far printed (exit 0: the headline was
    measured on modes that completed; the hung one is named in dd_modes)."""
    from feanet_amd.dd import DDSolver, TorchComm, default_grid
    if args.weak:
        m, nc = dd_domain(ws, args.n)
    else:
        m = nc = args.global_n or 8192
    grid = tuple(int(x) for x in args.grid.lower().split("x")) if args.grid else default_grid(ws)
    wanted = [x.strip() for x in args.dd_modes.split(",")] if args.dd_modes != "all" else [x[0] for x in DD_MODES]
    modes = [md for md in DD_MODES if md[0] in wanted]
    if args.backend != "nccl":  # capture needs device communication (gloo stages through the host)
        modes = [md for md in modes if not md[1]]
    if not modes:
        raise SystemExit(f"bench: no dd mode selected from {args.dd_modes!r} for backend {args.backend}")
    if args.problem == "interface" and m != nc:
        raise SystemExit(f"bench: the two-material problem is defined on the square; the dd grid is {m}x{nc}")
    rhs = dd_rhs(args, m, nc, T, B)  # one global problem: every rank draws the same rhs and keeps its block
    pkw = dd_problem_kw(args)
    dof = B * (m + 1) * (nc + 1)
    rec, exp, results = None, None, []

    def expire(name, seconds):  # a mode after the first hung: print what was measured, name the hung mode
        if rec is None:
            return EXIT_HANG
        rec["dd_modes"].append({"mode": name.split(" ")[-1], "status": f"did not finish within {seconds:.0f} s on "
                                f"rank {rank} (phase '{name}'); every rank exited"})
        if rank == 0:
            emit(rec)
        return 0

    for i, (name, cap, ov, sj) in enumerate(modes):
        t0 = time.perf_counter()
        try:
            with guard.phase(f"dd mode {name}", args.mode_timeout, None if i == 0 else expire):
                s = DDSolver(nc, m, rank, ws, comm=TorchComm(capture=cap), agglomerate=args.agglomerate, dtype=T,
                             batch=B, grid=grid, overlap_l0=ov, split_join=sj, **pkw)
                s.set_rhs(**rhs)
                s.load()
                conv = contraction(s) if i == 0 else None
                t, warm = time_steps(s, args.steps, args.warmup, ws)
                captured = bool(s.comm.capturable and s._capture_ok and s.use_graph)
                par = None
                if not args.no_dd_parity:
                    if exp is None:
                        exp = dd_reference_block(args, s.owned_block()[:2], m, nc, T, B)
                    par = dd_parity(s, exp, m, nc, ws)
                    if cap:
                        captured = captured and bool(s._capture_ok)
        except Exception as e:
            if i == 0:
                raise
            log(f"[bench] rank {rank}: dd mode {name} failed: {e!r}")
            rec["dd_modes"].append({"mode": name, "status": f"error: {str(e)[:300]}"})
            torch.cuda.synchronize()
            continue
        ms = t / args.steps * 1e3
        r = {"mode": name, "status": "ok", "ms_per_step": ms, "value": dof / (t / args.steps),
             "cycle_graphs": ("captured (kernels + RCCL calls, one HIP graph per block of up to "
                              f"{s.GRAPH_CYCLES} cycles)") if captured else
                             ("segments (one HIP graph per kernel segment between communication steps)" if not cap else
                              "segments (capture requested, refused on some rank: all ranks fell back)"),
             "capture_requested": cap, "overlap_l0": ov, "split_join": sj, "backend": args.backend,
             "dd_parity": par, "mode_seconds": round(time.perf_counter() - t0, 2)}
        results.append(r)
        if i == 0:
            fine = time_fine_kernels(s.local, args.kernel_reps)
            # the learned smoother joins no cycles: its dominant kernel is the slowest finest-level launch of the
            # local cycle (timed in the rank's local V-cycle plan, which has the same finest-level launches)
            dom = time_fine_launch_in_cycle(s.local) if args.smoother == "hjac" else None
            roof, ns, fl = roofline_record(fine, s.local, args, dom=dom, ws=ws)
            p0, q0 = s.parts[0], s.cparts[0]
            workload = (f"{m + 1}x{nc + 1} {args.problem} {args.dtype} V-cycle, L={s.L}, V(1,1)"
                        f"{' (learned HRelax smoother)' if args.smoother == 'hjac' else ''}, domain-decomposed into "
                        f"{grid[0]}x{grid[1]} blocks of {p0.e - p0.s} x {q0.e - q0.s} owned nodes (+{s.part.ghost(0)} "
                        f"ghost lines per side), levels >= {s.Ld} agglomerated, batch {B}"
                        + ("" if args.weak else " (BASELINE config C4 when 8193^2 over 8 GPUs)"))
            parallelism = (f"dd{ws}: {grid[0]}x{grid[1]} 2-D blocks, RCCL halo exchange (one phase, packed, depths "
                           f"{s.depths}) once per V-cycle + all-gather of level {s.Ld}, redundant coarse solve")
            rec = base_record(args, r["value"], ms, ws, warm, workload, "dd", parallelism,
                              "ones" if args.problem == "interface" else "randn", s.L, B)
            rec.update({"roofline": roof, "north_star_kernel": ns, "fine_level_kernels": fl,
                        "vcycle_hbm_gbps_algorithmic": None, "vcycle_algorithmic_bytes": None,
                        "residual_contraction_per_cycle": conv, "dd_modes": results, "cpu_baseline": None})
            if args.problem == "interface":
                rec["config"]["transfer"] = ("learned ratio R/P/w" if "R" in pkw else "linear")
            if ws > 1:
                # the same global grid on ONE GPU (rank 0; the others wait at the barrier): the strong-scaling base
                # point of this line, so speed-up and efficiency follow from the line itself
                del s
                torch.cuda.empty_cache()
                with guard.phase("single-GPU base point (rank 0) + barrier", args.mode_timeout):
                    if rank == 0:
                        rec["single_gpu_same_grid"] = single_gpu_same_grid(args, m, nc, T, B, args.steps, ms)
                    barrier(ws)
        ok = [x for x in results if x["status"] == "ok" and (x["dd_parity"] is None or x["dd_parity"]["bitwise_equal"])]
        best = min(ok, key=lambda x: x["ms_per_step"]) if ok else results[0]
        rec["value"], rec["ms_per_step"] = best["value"], best["ms_per_step"]
        rec["headline_mode"] = best["mode"]
        rec["config"]["dd_mode"] = {k: best[k] for k in ("mode", "cycle_graphs", "capture_requested", "overlap_l0",
                                                         "split_join", "backend")}
        rec["config"]["parallelism"] = rec["config"]["parallelism"].split("; headline mode")[0] + \
            f"; headline mode {best['mode']} (fastest bitwise of {len(results)} timed)"
        if best["dd_parity"] is not None:
            rec["dd_parity"] = best["dd_parity"]
        if "single_gpu_same_grid" in rec:
            rec["single_gpu_same_grid"]["speedup_of_this_line"] = \
                rec["single_gpu_same_grid"]["ms_per_step"] / best["ms_per_step"]
        if "s" in locals():
            del s
        torch.cuda.empty_cache()
    return rec


def run_single(args, ws, rank, T, B):
    """N = 1 (or --mode replicas): the metric configuration by default — one 4097^2 fp64 Poisson problem per GPU."""
    from feanet_amd.solver import MultigridSolver
    n = args.n
    N = n + 1
    rhs = args.rhs or ("families" if B > 1 else "ones" if args.problem == "interface" else "randn")
    hnet, kw = None, {}
    wdir = os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "weights")
    if args.smoother == "hjac":
        w = np.load(os.path.join(wdir, "hnet_iso_poisson_33x33.npz"))
        hnet = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
    learned = args.problem == "interface" and args.transfer == "learned"
    if learned:  # BASELINE C3: FEANet/multigrid.py's trained ratio R / P / w (MM_Interface_error.ipynb)
        w = np.load(os.path.join(wdir, "multigrid_interface_ratio.npz"))
        kw = dict(R=w["R"][0], P=w["P"][:, 0], w=w["w"])
    s = MultigridSolver(n, problem=args.problem, dtype=T, batch=B, levels=args.levels, smoother=args.smoother,
                        hnet=hnet, **kw)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + rank)
    if rhs == "families":
        from tools import rhs_families
        s.set_rhs(F=rhs_families.batch(B, N, T, "cuda", seed=rank))
    elif rhs == "ones":
        s.set_rhs(F=torch.ones(B, 1, N, N, device="cuda", dtype=T))
    else:
        s.set_rhs(f=torch.randn(B, 1, N, N, device="cuda", dtype=T, generator=g))
    dof = B * N * N * ws
    workload = (f"{N}x{N} {args.problem} {args.dtype} V-cycle, L={s.L}, V(1,1) (MultiGrid.Step semantics"
                f"{', learned HRelax smoother' if args.smoother == 'hjac' else ''}"
                f"{', learned ratio R/P/w of FEANet/multigrid.py (BASELINE C3)' if learned else ''}), batch {B} per GPU")
    parallelism = "replicas (one independent problem per GPU)" if ws > 1 else "single GPU"
    s.load()
    conv = contraction(s)
    t, warm = time_steps(s, args.steps, args.warmup, ws)
    ms_step = t / args.steps * 1e3
    rec = base_record(args, dof / (t / args.steps), ms_step, ws, warm, workload, "single" if ws == 1 else "replicas",
                      parallelism, rhs, s.L, B)
    fine = time_fine_kernels(s, args.kernel_reps)
    L0 = s.levels[0]
    metric_cfg = (L0.H == 4097 and L0.W == 4097 and B == 1 and args.dtype == "f64" and args.problem == "poisson")
    # roofline: the DOMINANT kernel of the timed region — the finest level's cycle join (one per V-cycle
    # boundary, ~45 % of the V-cycle), timed inside the cycle with HIP events on the solver's stream
    jt = time_join_in_cycle(s, min(args.steps, 200))
    jsrc = ("HIP events in the solver's stream, eager replays of vcycle(K): [previous launch + join] minus "
            "[previous launch] per cycle")
    dom = time_fine_launch_in_cycle(s) if (jt is None and not s._joinable()) else None
    roof, ns, fl = roofline_record(fine, s, args, jt=jt, jsrc=jsrc, dom=dom, tkey_ok=(ws == 1 and metric_cfg), ws=ws)
    vbytes = s.bytes_per_vcycle(args.steps)
    rec.update({"roofline": roof, "north_star_kernel": ns, "fine_level_kernels": fl,
                "vcycle_hbm_gbps_algorithmic": vbytes / (t / args.steps) / 1e9 if (ws == 1 and vbytes) else None,
                "vcycle_algorithmic_bytes": vbytes, "residual_contraction_per_cycle": conv,
                "time_to_solution": time_to_solution(conv, ms_step)})
    if args.smoother == "hjac" and ws == 1 and B == 1:
        f = s.levels[0].view(s.levels[0].f).clone().reshape(B, 1, N, N)
        del s
        torch.cuda.empty_cache()
        rec["jacobi_same_grid"] = jacobi_same_grid(args, B, T, f)
    if args.problem == "interface":
        rec["config"]["transfer"] = ("learned ratio R/P/w (feanet_amd/weights/multigrid_interface_ratio.npz)" if learned
                                     else "linear (the reference's default RestrictionNet / ProlongationNet)")
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and args.problem == "poisson" and B == 1:
        log("[bench] timing the CPU oracle baseline ...")
        rec["cpu_baseline"] = cpu_baseline(n)
    else:
        rec["cpu_baseline"] = None
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=4096, help="intervals per edge (N = n+1 nodes); per GPU in dd mode")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--problem", default="poisson", choices=["poisson", "interface"])
    ap.add_argument("--levels", type=int, default=None, help="V-cycle levels (default int(log2 n))")
    ap.add_argument("--smoother", default="jac", choices=["jac", "hjac"],
                    help="hjac: the learned smoother of M-FEANet-mg_test.ipynb (HRelax, HNet weights "
                         "feanet_amd/weights/hnet_iso_poisson_33x33.npz), MultiGrid(mode='hjac').Step")
    ap.add_argument("--mode", default=None, choices=["single", "dd", "replicas"],
                    help="default: single at 1 GPU, dd (domain decomposition, weak scaling) at N > 1")
    ap.add_argument("--agglomerate", type=int, default=None, help="dd: level gathered for the coarse solve")
    ap.add_argument("--global-n", type=int, default=None,
                    help="dd: intervals per edge of ONE global grid split over the ranks (strong scaling; default "
                         "8192 = BASELINE config C4, 8193^2 over the GPUs)")
    ap.add_argument("--weak", action="store_true",
                    help="dd: weak scaling instead, --n x --n intervals per GPU (4097^2, 8193x4097, 8193^2, 16385x8193)")
    ap.add_argument("--grid", default=None, help="dd: rank grid PRxPC (default: 2->2x1, 4->2x2, 8->4x2)")
    ap.add_argument("--dd-modes", default="all",
                    help="dd: comma list of modes to time (" + ", ".join(x[0] for x in DD_MODES) + ") or all; the "
                         "captured ones need --backend nccl")
    ap.add_argument("--mode-timeout", type=float, default=120.0,
                    help="dd: seconds one mode (build, warm-up, timed cycles, parity) may take on a rank")
    ap.add_argument("--dist-timeout", type=float, default=150.0, help="process-group collective timeout (s)")
    ap.add_argument("--launch-timeout", type=float, default=560.0,
                    help="--gpus N without a launcher: seconds the N ranks may take in all")
    ap.add_argument("--rhs", default=None, choices=["randn", "families", "ones"],
                    help="right-hand side: seeded Gaussian assembled rhs, nodal sources from the six families of the "
                         "reference's Data/RHS/generate_rhs.py with FNet applied, or F = ones with FNet applied "
                         "(default: families for batches, the BASELINE C5 inputs; ones for the interface problem, "
                         "BASELINE C3; randn otherwise)")
    ap.add_argument("--transfer", default="learned", choices=["learned", "linear"],
                    help="interface problem: the trained ratio R/P/w of FEANet/multigrid.py (BASELINE C3, default) or "
                         "the linear transfer operators")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dd-parity", action="store_true",
                    help="dd: skip the per-rank bitwise check against a global-grid single-GPU solver (it holds the "
                         "whole global grid on every rank: ~1 GB per 8193^2 fp64 field)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend (gloo: multi-process rehearsal on one GPU, host-staged)")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--selftest-hang", type=float, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()

    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, args.launch_timeout))
    if env_ws is not None and int(env_ws) != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_ws} ranks; pass --gpus "
                 f"{env_ws} (or run without a launcher: bench.py --gpus N starts N ranks itself)")
    if args.selftest_hang is not None:
        sys.exit(selftest_hang(args))
    # stdout carries exactly ONE line, the JSON record: everything else a library writes to fd 1
    # (RCCL prints its version banner there when the communicator comes up) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    printed = []

    def emit(rec):
        if not printed:
            printed.append(True)
            print(json.dumps(rec), file=json_out, flush=True)

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    mode = args.mode or ("dd" if ws > 1 else "single")
    ws, rank = dist_init(force=(mode == "dd"), backend=args.backend, timeout_s=args.dist_timeout)
    guard = PhaseGuard(rank)
    T = torch.float64 if args.dtype == "f64" else torch.float32
    if mode == "dd":
        rec = run_dd(args, ws, rank, T, args.batch, guard, emit)
    else:
        rec = run_single(args, ws, rank, T, args.batch)
    if rank == 0:
        emit(rec)
    if torch.distributed.is_initialized():
        with guard.phase("destroy_process_group", 60, lambda *_: 0):
            torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
