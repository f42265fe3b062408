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
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multigrid-feanet_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "DoF-updates/sec per V-cycle (fp64) + achieved HBM GB/s, 4097² Poisson"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_init(force=False, backend="nccl"):
    """One process per GPU (torchrun env).  force: create the process group even for one rank (the
    domain-decomposed path always talks through torch.distributed).  backend "gloo": rehearsal of the
    multi-rank path with several processes on one GPU (RCCL refuses two ranks on one device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":  # rehearsal: more ranks than GPUs share them
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if ws > 1 or force:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(ws))
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return ws, rank


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


def single_gpu_same_grid(m, n, T, B, steps, ms_dd):
    """The single-GPU MultigridSolver on the decomposed run's global grid ((m+1) x (n+1), same seeded rhs),
    timed like the main line (warm-up calls, then one vcycle(steps) between synchronisations)."""
    from feanet_amd.solver import MultigridSolver
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    s = MultigridSolver(n, rows=None if m == n else m, dtype=T, batch=B)
    s.set_rhs(f=torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=T, generator=g))
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
            "workload": f"{m + 1}x{n + 1} poisson V-cycle on one GPU (MultigridSolver, no decomposition), rank 0"}


def dd_parity_check(s, m, n, T, B, ws, cycles=3):
    """Every rank: the decomposed solver's owned block after `cycles` V-cycles from zero against the single-GPU
    MultigridSolver's on the same global grid and seeded rhs (run on the rank's own GPU).  The decomposed
    cycle is bitwise the single-GPU one by construction (tests/test_gpu_dd.py); this puts that claim on the
    line of every multi-GPU run, i.e. on the RCCL path itself.  Returns the max over ranks of the largest
    absolute difference and of the count of differing nodes."""
    from feanet_amd.solver import MultigridSolver
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    f = torch.randn(B, 1, m + 1, n + 1, device="cuda", dtype=T, generator=g)
    s.load()
    s.vcycle(cycles)
    (y0, y1), (x0, x1), u = s.owned_block()
    ref = MultigridSolver(n, rows=None if m == n else m, dtype=T, batch=B)
    ref.set_rhs(f=f)
    del f
    ref.load()
    ref.vcycle(cycles)
    exp = ref.solution()[:, :, y0:y1, x0:x1]
    diff = (u - exp).abs()
    gloo = ws > 1 and torch.distributed.get_backend() != "nccl"  # gloo reduces host tensors (max_over_ranks)
    out = torch.tensor([diff.max().item(), float((u != exp).sum().item())], dtype=torch.float64,
                       device="cpu" if gloo else "cuda")
    del ref, exp, diff, u
    torch.cuda.empty_cache()
    if ws > 1:
        torch.distributed.all_reduce(out, op=torch.distributed.ReduceOp.MAX)
    return {"cycles": cycles, "bitwise_equal": bool(out[1].item() == 0), "max_abs_diff": out[0].item(),
            "max_differing_nodes_per_rank": int(out[1].item()),
            "against": f"single-GPU MultigridSolver on the same {m + 1}x{n + 1} grid, V-cycles from zero, every "
                       f"rank's owned block"}


def dd_domain(P, n0):
    """Weak-scaled global grid for P slabs of n0 x n0 intervals each, aspect ratio <= 2 when P is a
    power of two: 1 -> n0 x n0, 2 -> 2n0 x n0, 4 -> 2n0 x 2n0, 8 -> 4n0 x 2n0 (rows x columns)."""
    if P & (P - 1) == 0:
        k = P.bit_length() - 1
        return n0 << ((k + 1) // 2), n0 << (k // 2)
    return n0 * P, n0


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: run the same command line under
    torch.distributed.run (one rank per GPU, rendezvous on 127.0.0.1) as a CHILD process — nothing here has
    touched the GPU, and the process is not replaced (no exec) — forward its one JSON line to stdout (anything
    else it printed there goes to stderr) and return its exit status."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n} without a launcher: {' '.join(cmd)}")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = r.stdout.splitlines()
    recs = [ln for ln in lines if ln.startswith("{")]
    for ln in lines:
        if not ln.startswith("{"):
            log(ln)
    if recs:
        print(recs[-1], flush=True)
    if r.returncode == 0 and len(recs) != 1:
        log(f"[bench] expected one JSON line from rank 0, got {len(recs)}")
        return 1
    return r.returncode


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
    ap.add_argument("--rhs", default=None, choices=["randn", "families"],
                    help="right-hand side: seeded Gaussian assembled rhs, or nodal sources from the six "
                         "families of the reference's Data/RHS/generate_rhs.py with FNet applied (default: "
                         "families for batches, the BASELINE C5 inputs; randn otherwise)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dd-parity", action="store_true",
                    help="dd: skip the per-rank bitwise check against a global-grid single-GPU solver (it holds the "
                         "whole global grid on every rank: ~1 GB per 8193^2 fp64 field)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend (gloo: multi-process rehearsal on one GPU, host-staged)")
    ap.add_argument("--kernel-reps", type=int, default=50)
    args = ap.parse_args()

    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_ws is not None and int(env_ws) != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_ws} ranks; pass --gpus "
                 f"{env_ws} (or run without a launcher: bench.py --gpus N starts N ranks itself)")
    # stdout carries exactly ONE line, the JSON record: everything else a library writes to fd 1
    # (RCCL prints its version banner there when the communicator comes up) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    mode = args.mode or ("dd" if ws > 1 else "single")
    ws, rank = dist_init(force=(mode == "dd"), backend=args.backend)
    from feanet_amd.solver import MultigridSolver
    T = torch.float64 if args.dtype == "f64" else torch.float32
    n, B = args.n, args.batch
    rhs = args.rhs or ("families" if B > 1 else "randn")
    g = torch.Generator(device="cuda")
    if mode == "dd":
        if args.problem != "poisson":
            raise SystemExit("bench: the domain-decomposed path runs the Poisson problem")
        from feanet_amd.dd import DDSolver, TorchComm, default_grid
        if args.weak:
            m, nc = dd_domain(ws, n)
        else:
            m = nc = args.global_n or 8192
        grid = tuple(int(x) for x in args.grid.lower().split("x")) if args.grid else default_grid(ws)
        s = DDSolver(nc, m, rank, ws, comm=TorchComm(), agglomerate=args.agglomerate, dtype=T, batch=B, grid=grid)
        g.manual_seed(1234)  # one global problem: every rank draws the same rhs and keeps its rows
        f = torch.randn(B, 1, m + 1, nc + 1, device="cuda", dtype=T, generator=g)
        s.set_rhs(f)
        del f
        torch.cuda.empty_cache()
        dof = B * (m + 1) * (nc + 1)
        lvl = s.local
        p0, q0 = s.parts[0], s.cparts[0]
        workload = (f"{m + 1}x{nc + 1} poisson {args.dtype} V-cycle, L={s.L}, V(1,1), domain-decomposed into "
                    f"{grid[0]}x{grid[1]} blocks of {p0.e - p0.s} x {q0.e - q0.s} owned nodes (+{s.part.ghost(0)} "
                    f"ghost lines per side), levels >= {s.Ld} agglomerated, batch {B}"
                    + ("" if args.weak else " (BASELINE config C4 when 8193^2 over 8 GPUs)"))
        parallelism = (f"dd{ws}: {grid[0]}x{grid[1]} 2-D blocks, RCCL halo exchange (one phase, packed, depths "
                       f"{s.depths}) once per V-cycle + all-gather of level {s.Ld}, redundant coarse solve")
    else:
        N = n + 1
        hnet = None
        if args.smoother == "hjac":
            w = np.load(os.path.join(ROOT, "multigrid-feanet_amd", "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
            hnet = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
        s = MultigridSolver(n, problem=args.problem, dtype=T, batch=B, levels=args.levels, smoother=args.smoother,
                            hnet=hnet)
        g.manual_seed(1234 + rank)
        if rhs == "families":
            from tools import rhs_families
            s.set_rhs(F=rhs_families.batch(B, N, T, "cuda", seed=rank))
        else:
            s.set_rhs(f=torch.randn(B, 1, N, N, device="cuda", dtype=T, generator=g))
        dof = B * N * N * ws
        lvl = s
        workload = (f"{N}x{N} {args.problem} {args.dtype} V-cycle, L={s.L}, V(1,1) (MultiGrid.Step semantics"
                    f"{', learned HRelax smoother' if args.smoother == 'hjac' else ''}), batch {B} per GPU")
        parallelism = "replicas (one independent problem per GPU)" if ws > 1 else "single GPU"
    s.load()
    # contraction factor over the first 8 cycles (before the fp64 floor), then restart from zero
    r0 = s.residual_norm()
    s.vcycle(8)
    conv = float((s.residual_norm().max() / r0.max()).item()) ** (1.0 / 8)
    s.load()

    # warm-up: the timed call itself (vcycle(steps)), repeated so that every graph the timed call
    # replays (its blocks of joined cycles, keyed by start buffer and size; 5 calls cover every step
    # count) has run once eagerly and been captured before the clock starts.  At least --warmup cycles.
    calls = max(6, -(-args.warmup // args.steps))
    calls += calls % 2
    warm = 0
    for _ in range(calls):
        s.vcycle(args.steps)
        warm += args.steps
    torch.cuda.synchronize()
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.vcycle(args.steps)
    torch.cuda.synchronize()
    barrier(ws)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    t = max_over_ranks(t, ws)
    ms_step = t / args.steps * 1e3
    value = dof / (t / args.steps)

    fine = time_fine_kernels(lvl, args.kernel_reps)
    L0 = lvl.levels[0]
    metric_cfg = (L0.H == 4097 and L0.W == 4097 and B == 1 and args.dtype == "f64" and args.problem == "poisson")
    # north-star kernel: the fine-level Ke-stencil Jacobi sweep on its own (back-to-back launches)
    kt, kbytes = fine["fea_mg_sweep"]
    kt = max_over_ranks(kt, ws)
    # roofline: the DOMINANT kernel of the timed region — the finest level's cycle join (one per V-cycle
    # boundary, ~45 % of the V-cycle), timed inside the cycle with HIP events on the solver's stream
    jt = time_join_in_cycle(s, min(args.steps, 200)) if mode == "single" else None
    jsrc = ("HIP events in the solver's stream, eager replays of vcycle(K): [previous launch + join] minus "
            "[previous launch] per cycle")
    dom = None
    if jt is None and mode == "single" and not s._joinable():
        dom = time_fine_launch_in_cycle(s)  # no join in this schedule: its own slowest fine-level launch
    if dom is not None:
        name, r_t, r_bytes = dom
        rkern = (f"{name} (fine level {L0.H}x{L0.W} {args.dtype}; the slowest launch of the cycle, which joins no "
                 f"cycles)")
        tkey, jsrc = None, ("HIP events on the solver's stream between consecutive launches of eager replays of the "
                            "V-cycle plan")
    elif jt is None and "fea_mg_cycle_join" in fine:
        jt = fine["fea_mg_cycle_join"][0]
        jsrc = "HIP events, back-to-back launches of fea_mg_cycle_join on the level-0 buffers"
    if dom is None and jt is not None:
        jbytes = fine["fea_mg_cycle_join"][1] if "fea_mg_cycle_join" in fine else None
        jt = max_over_ranks(jt, ws)
        rkern = f"fea_mg_cycle_join (fine level {L0.H}x{L0.W} {args.dtype}: post-sweep of cycle k + pre-sweep, " \
                f"residual and restriction of cycle k+1 in one pass)"
        r_t, r_bytes, tkey = jt, jbytes, "mg_cycle_join_f64_4097"
    elif dom is None:
        rkern, r_t, r_bytes, tkey, jsrc = (f"fea_mg_sweep ({L0.H}x{L0.W} {args.dtype})", kt, kbytes,
                                           "mg_sweep_f64_4097", "HIP events, back-to-back launches")
    achieved = r_bytes / r_t / 1e9
    traffic, tsrc = load_traffic(tkey) if (mode == "single" and metric_cfg) else (None, None)
    ns_traffic, ns_src = load_traffic("mg_sweep_f64_4097") if (mode == "single" and metric_cfg) else (None, None)
    vbytes = s.bytes_per_vcycle(args.steps) if mode == "single" else None
    dd_mode = None
    if mode == "dd":  # the path the timed cycles actually took (a refused capture falls back on every rank)
        captured = bool(getattr(s.comm, "capturable", False) and s._capture_ok and s.use_graph)
        dd_mode = {"cycle_graphs": "captured (kernels + RCCL calls, one HIP graph per block of up to "
                                   f"{s.GRAPH_CYCLES} cycles)" if captured else "segments (one HIP graph per kernel "
                                   "segment between communication steps)",
                   "split_join": bool(s.split_join and captured), "overlap_l0": bool(s.overlap_l0),
                   "backend": args.backend}
        parallelism += (f"; cycles {'captured whole' if captured else 'in kernel segments'}, split_join "
                        f"{dd_mode['split_join']}, overlap_l0 {dd_mode['overlap_l0']}")

    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "DoF-updates/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": warm,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if (mode == "dd" and not args.weak) else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": ("synthetic (seeded Gaussian rhs, zero initial guess)" if rhs == "randn" else
                 "synthetic (nodal sources from the six Data/RHS/generate_rhs.py families, seeded, FNet applied; "
                 "zero initial guess)"),
        "config": {"workload": workload, "mode": mode, "batch": B, "levels": s.L, "parallelism": parallelism,
                   **({"dd_mode": dd_mode} if dd_mode else {})},
        "roofline": {"bound": "hbm", "kernel": rkern,
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": tsrc, "avg_launch_us": r_t * 1e6,
                     "algorithmic_bytes_per_launch": r_bytes, "timing": jsrc},
        "north_star_kernel": {"kernel": f"fea_mg_sweep (fine-level Ke-stencil Jacobi sweep, {L0.H}x{L0.W} "
                                        f"{args.dtype}, 24 B/node)",
                              "achieved": kbytes / kt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": kbytes / kt / 1e9 / HBM_PEAK_GBS, "avg_launch_us": kt * 1e6,
                              "algorithmic_bytes_per_launch": kbytes, "traffic": ns_traffic,
                              "traffic_source": ns_src, "target_frac": 0.70},
        "fine_level_kernels": {k: {"avg_launch_us": tk * 1e6, "algorithmic_bytes": nb,
                                   "achieved_GBps": nb / tk / 1e9, "frac": nb / tk / 1e9 / HBM_PEAK_GBS}
                               for k, (tk, nb) in fine.items()},
        "vcycle_hbm_gbps_algorithmic": vbytes / (t / args.steps) / 1e9 if (ws == 1 and vbytes) else None,
        "vcycle_algorithmic_bytes": vbytes,
        "residual_contraction_per_cycle": conv,
    }
    if mode == "dd" and ws > 1:
        # the same global grid on ONE GPU (rank 0; the others wait at the barrier): the strong-scaling base
        # point of this line, so speed-up and efficiency follow from the line itself
        if rank == 0:
            rec["single_gpu_same_grid"] = single_gpu_same_grid(m, nc, T, B, args.steps, ms_step)
        barrier(ws)
    if mode == "dd" and not args.no_dd_parity:
        rec["dd_parity"] = dd_parity_check(s, m, nc, T, B, ws)
    if rank == 0 and ws == 1 and mode == "single" and not args.no_cpu_baseline and args.problem == "poisson" \
            and B == 1:
        log("[bench] timing the CPU oracle baseline ...")
        rec["cpu_baseline"] = cpu_baseline(n)
    elif rank == 0:
        rec["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(rec), file=json_out, flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
