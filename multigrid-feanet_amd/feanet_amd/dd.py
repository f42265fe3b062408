"""Domain-decomposed V-cycle over several MI355X GPUs: 2-D blocks + halo exchange.

The fine grid ((m+1) x (n+1) nodes; Poisson, or the two-material problem on the square; weighted Jacobi or the
learned HRelax smoother) is cut into a Pr x Pc grid of blocks, one per rank (one
process per GPU, torch.distributed over RCCL/xGMI; rank r = ri * Pc + ci).  Row slabs are the Pc = 1
case.  Levels 0 .. Ld-1 are distributed; the level-Ld restriction is all-gathered and the rest of the
V-cycle (levels >= Ld of the global grid) is solved redundantly on every rank by a single-GPU
MultigridSolver, whose correction each rank copies back for its block.  The result is bitwise the
single-GPU V-cycle on the global grid (same kernels, same per-node arithmetic, same coarse schedule),
which the tests check.

Layout (class Partition, one per axis).  Interior row offsets t_r = r * m / Pr split level 0; level l
uses t_r / 2^l, so fine rows (2I-1, 2I) and coarse row I always live on the same rank.  Rank row ri
owns global rows [s, e) = [1 + t_ri, 1 + t_ri+1) (the last one up to H-1) and stores rows
[gr0, gr0 + Hloc) with gr0 = t_ri - G_l (0 on the first): G_l = G * 2^(Ld-l) ghost rows per side, the
doubling keeping gr0_l = 2 gr0_{l+1} so the unmodified level kernels pair fine and coarse rows exactly
as on one grid.  Columns are split the same way (same G).  The level kernels compute every local
interior node (a block is just a smaller rectangular grid to them); ghost rows and columns near the
block edge are refreshed by exchanges, deeper ones are redundant work.

Communication (communication-avoiding).  Every level kernel already computes the ghost nodes it
stores, so ghost values stay correct to a depth that shrinks by one per sweep and halves per
restriction — the same in both directions, so one scalar depth describes a block's valid region and
the validity simulation of the slab case (exchange_depths) applies unchanged; an exchange is needed
only where that depth would run out.  Per V-cycle:
  after the finest pre-smoothing (or the cycle join):  D1 of f_1 (and D0 of the pre-smoothed finest
                                                       iterate, joined cycles)
  at level Ld:  all-gather of the owned blocks of f_Ld -> the replicated coarse solve -> local copy
  after the finest post-smoothing (unjoined cycles):   D0 of the finest iterate
An exchange of depth d is ONE round of messages with up to eight neighbours (DDSolver.regions): d ghost
rows of the owned columns from the neighbours above / below, d ghost columns of the owned rows from the
left / right, and the d x d corner regions the 9-point stencil needs from the diagonal neighbours; all
regions of one exchange are packed into one staging buffer by one kernel (fea_dd_copy_blocks), sent as one
message per neighbour and unpacked by one kernel (row slabs: contiguous rows, sent in place).  D0 and D1 are the
smallest depths for which the validity simulation keeps every owned node exact.
"""
import os

import torch

from . import _lib, mesh_setup as ms, ops
from .schedule import hjac_schedule, pair_prolongations, pair_restrictions, vcycle_schedule
from .solver import MultigridSolver


def global_levels(m, n):
    """Levels of the global grid (MultigridSolver's default for a rectangle)."""
    L = 1
    while n % (1 << L) == 0 and m % (1 << L) == 0 and (n >> L) >= 2 and (m >> L) >= 2:
        L += 1
    return L


def default_agglomeration(m, n, P, L, max_nodes=None, Pc=1):
    """Smallest Ld whose global level has <= max_nodes nodes (default 2^18), within what the partition allows (P
    row blocks, Pc column blocks).  At 8193^2 (BASELINE C4) that is Ld = 5 (257^2) at 2, 4 and 8 ranks: the per-rank
    projection (one rank's whole captured program on one GPU, tools/dd_projection.py, profiles/r06_dd) runs 257.2 /
    156.6 / 109.1 us at Ld = 5 against 279.5 / 161.1 / 111.5 at Ld = 4 and 278.2 / 168.5 / 118.3 at Ld = 6 on 2 / 4 / 8
    ranks (round 5, before the round-6 task heights, had Ld = 4 ahead at 8 ranks).  Scope of that evidence: ONE grid
    and single-GPU projections whose communicator moves nothing, so message and all-gather costs are not modelled;
    for other grids the rule is only "stop coarsening the distributed levels once the global level is this small",
    pinned by tests/test_dd.py for several sizes, not a measured optimum."""
    if max_nodes is None:
        max_nodes = 1 << 18
    Ld = 1
    while Ld < L - 1 and ((m >> Ld) + 1) * ((n >> Ld) + 1) > max_nodes and m % (P << (Ld + 1)) == 0 \
            and m // (P << (Ld + 1)) >= 4 and n % (Pc << (Ld + 1)) == 0 and (Pc == 1 or n // (Pc << (Ld + 1)) >= 4):
        Ld += 1
    return Ld


class LevelPart:
    """Rank r's rows of one level: owned global rows [s, e), stored rows [gr0, gr0 + Hloc),
    owned local rows [lo, hi)."""

    def __init__(self, H, s, e, gr0, gend):
        self.H, self.s, self.e, self.gr0 = H, s, e, gr0
        self.Hloc = gend - gr0
        self.lo, self.hi = s - gr0, e - gr0

    def __repr__(self):
        return f"LevelPart(H={self.H}, own=[{self.s},{self.e}), rows=[{self.gr0},{self.gr0 + self.Hloc}))"


class Partition:
    """One axis of the decomposition: m intervals split over P ranks for Ld distributed levels with G
    ghost lines per side at level Ld (doubling per finer level); n: the other axis' intervals (checked
    to coarsen Ld times).  Rows of the slab layout; the column axis of a 2-D grid is Partition(n, m, Pc)."""

    def __init__(self, m, n, P, Ld, G=4):
        if P < 1 or Ld < 1:
            raise ValueError("Partition: need P >= 1 and Ld >= 1")
        if m % (P << Ld) or m // (P << Ld) < G:
            raise ValueError(f"Partition: {m} rows do not split into {P} slabs over {Ld} levels "
                             f"(need m divisible by P*2^Ld with >= {G} coarse rows per rank)")
        if n % (1 << Ld) or (n >> Ld) < 2:
            raise ValueError(f"Partition: {n} columns do not coarsen {Ld} times")
        self.m, self.n, self.P, self.Ld, self.G = m, n, P, Ld, G

    def ghost(self, l):
        return self.G << (self.Ld - l)

    def rows_per_rank(self, l):
        return (self.m // self.P) >> l

    def level(self, l, r):
        H = (self.m >> l) + 1
        c = self.rows_per_rank(l)
        g = self.ghost(l)
        t = r * c
        s = 1 + t
        e = 1 + t + c if r < self.P - 1 else H - 1
        gr0 = 0 if r == 0 else t - g
        gend = H if r == self.P - 1 else e + g
        return LevelPart(H, s, e, gr0, gend)


class Partition2D:
    """Pr x Pc blocks (rank r = ri * Pc + ci): a row Partition and a column Partition with the same G and
    Ld.  level(l, r) / clevel(l, r): rank r's row / column LevelPart of level l."""

    def __init__(self, m, n, Pr, Pc, Ld, G=4):
        self.rows = Partition(m, n, Pr, Ld, G)
        self.cols = Partition(n, m, Pc, Ld, G) if Pc > 1 else None
        self.m, self.n, self.Pr, self.Pc, self.Ld, self.G = m, n, Pr, Pc, Ld, G
        self.P = Pr * Pc

    def ghost(self, l):
        return self.rows.ghost(l)

    def rows_per_rank(self, l):
        return self.rows.rows_per_rank(l)

    def cols_per_rank(self, l):
        return (self.n // self.Pc) >> l

    def level(self, l, r):
        return self.rows.level(l, r // self.Pc)

    def clevel(self, l, r):
        if self.cols is None:  # one column block: all columns, no ghosts
            W = (self.n >> l) + 1
            return LevelPart(W, 1, W - 1, 0, W)
        return self.cols.level(l, r % self.Pc)


def default_grid(P):
    """Pr x Pc for P ranks: rows split at least as finely as columns (a row halo is one contiguous run
    of the framed layout, a column halo a packed strip), as square as possible: 2 -> 2x1, 4 -> 2x2,
    8 -> 4x2."""
    best = (P, 1)
    for Pc in range(1, P + 1):
        if P % Pc == 0 and P // Pc >= Pc:
            best = (P // Pc, Pc)
    return best


def dd_schedule(Ld, nu1=1, nu2=1, fuse=True, start="a", depths=(4, 4), smoother="jac"):
    """The distributed part of one (unjoined) V-cycle: kernel steps of feanet_amd.schedule plus
    ("exchange", l, buf, depth), ("gather",), ("coarse",), ("scatter", dst).  depths = (D0, D1).
    smoother="hjac": the learned smoother's V-cycle (hjac_schedule), its levels >= Ld agglomerated the same way."""
    D0, D1 = depths
    if smoother == "hjac":
        steps, end = hjac_schedule(Ld + 1, nu1, nu2, start, tail_from=Ld, fuse=fuse)
    else:
        steps, end = vcycle_schedule(Ld + 1, nu1, nu2, None, start, tail_from=Ld, fuse=fuse)
    out = []
    for i, st in enumerate(steps):
        kind, l = st[0], st[1]
        if kind in ("coarse_tail", "hjac_tail"):
            out += [("gather",), ("coarse",), ("scatter", st[2])]
            continue
        out.append(st)
        if kind in ("resid_restrict", "sweep_restrict", "hsweep_restrict") and l == 0 and Ld >= 2:
            out.append(("exchange", 1, "f", D1))
    out.append(("exchange", 0, end, D0))
    return out, end


def _restricted(r):
    """Ghost depth of a restriction whose fine input is valid to depth r (fine rows 2I-1..2I+1)."""
    return (r - 1) // 2 if r >= 1 else -1


def simulate_validity(program, Ld, ghost, init=None, nl=0):
    """Row validity along a list of dd steps: for every (level, buffer) the number of ghost rows past
    the owned rows that hold the single-grid values (owned rows exact iff >= 0).  Buffers start as in
    `init` (default: fully valid, as after load()); f_0 is static (fully valid).  Returns False as soon
    as a kernel would write a wrong owned row, else the final validity map.  Steps may also be
    ("join", pre, ec_name).  nl: HNet conv layers of the learned smoother's steps (HRelax: the Jacobi
    sweep j = J(u) loses one line, each of the nl 3x3 convolutions of (j - u) * g one more)."""
    INF = 1 << 30
    v = dict(init or {})
    g = [ghost(l) for l in range(Ld + 1)]

    def get(l, name):
        if name is None or name == "zero":
            return INF
        if name == "omdf":  # omd*f recomputed pointwise: valid where f is
            return get(l, "f")
        if name == "f" and l == 0:
            return g[0]
        return v.get((l, name), g[l])

    def put(l, name, val):
        val = min(val, g[l])
        v[(l, name)] = val
        return val >= 0

    for st in program:
        k = st[0]
        if k == "exchange":
            l, name, d = st[1], st[2], st[3]
            if get(l, name) < 0 or d > g[l]:
                return False
            v[(l, name)] = max(get(l, name), d)
        elif k in ("gather", "coarse"):
            if k == "gather" and get(Ld, "f") < 0:
                return False
        elif k == "scatter":
            v[(Ld, st[1])] = g[Ld]
        elif k == "sweep":
            l = st[1]
            if not put(l, st[3], min(get(l, st[2]) - 1, get(l, "f"))):
                return False
        elif k in ("hsweep", "hsweep_restrict"):
            l, src, dst = st[1], st[2], st[3]
            it = min(get(l, src) - 1, get(l, "f")) - nl
            if not put(l, dst, it):
                return False
            if k == "hsweep_restrict" and not put(l + 1, "f", _restricted(min(it - 1, get(l, "f")))):
                return False
        elif k == "prolong_hsweep":
            l, src, ec, dst = st[1:5]
            x = min(get(l, src), 2 * get(l + 1, ec) - 1)
            if not put(l, dst, min(x - 1, get(l, "f")) - nl):
                return False
        elif k in ("resid_restrict", "sweep_restrict"):
            l, src, dst = st[1], st[2], st[3]
            if k == "sweep_restrict" or src is None:
                it = min(get(l, src) - 1 if src is not None else INF, get(l, "f"))
                if not put(l, dst, it):
                    return False
            else:
                it = get(l, src)
            if not put(l + 1, "f", _restricted(min(it - 1, get(l, "f")))):
                return False
        elif k in ("prolong_sweep", "prolong_add"):
            l, src, ec, dst = st[1:5]
            x = min(get(l, src), 2 * get(l + 1, ec) - 1)
            if not put(l, dst, (min(x - 1, get(l, "f")) if k == "prolong_sweep" else x)):
                return False
        elif k == "join":
            pre, ec = st[1], st[2]
            other = "b" if pre == "a" else "a"
            x = min(get(0, pre), 2 * get(1, ec) - 1)
            post = min(x - 1, get(0, "f"))
            nxt = min(post - 1, get(0, "f"))
            if post < 0 or not put(0, other, nxt) or not put(1, "f", _restricted(min(nxt - 1, get(0, "f")))):
                return False
        else:
            raise ValueError(f"simulate_validity: unknown step {st!r}")
    return v


def exchange_depths(Ld, ghost, nu1=1, nu2=1, fuse=True, joined=True, smoother="jac", nl=0):
    """Smallest (D0, D1) (by bytes: D1 rows are half as wide) keeping the owned rows exact in every
    program DDSolver runs.  Across program boundaries only the finest iterate carries over, and every
    program ends by exchanging it (D0 rows): so checking each program once from the weakest start
    state (finest iterates valid to exactly D0) covers any sequence of them (induction)."""
    def programs(D):
        out = [dd_schedule(Ld, nu1, nu2, fuse, "a", D, smoother)[0]]
        if joined:
            for njoin in (0, 1, 2):
                seq, s = [], "a"
                for kind in ["head"] + ["join"] * njoin + ["tail"]:
                    st, s = _joined_chunk_steps(Ld, nu1, nu2, fuse, kind, s, D)
                    seq += st
                out.append(seq)
        return out

    def ok(D0, D1):
        init = {(0, "a"): D0, (0, "b"): D0}
        return all(simulate_validity(p, Ld, ghost, init, nl) for p in programs((D0, D1)))

    best = None
    top1 = ghost(1) if Ld >= 2 else 1
    for D0 in range(1, min(ghost(0), 32) + 1):
        if not ok(D0, top1):
            continue
        lo, hi = 1, top1
        while lo < hi:
            mid = (lo + hi) // 2
            if ok(D0, mid):
                hi = mid
            else:
                lo = mid + 1
        cost = 2 * D0 + (lo if Ld >= 2 else 0)
        if best is None or cost < best[0]:
            best = (cost, (D0, lo))
    if best is None:
        raise ValueError(f"exchange_depths: no exchange depths keep the slabs exact (Ld={Ld}); "
                         "more ghost rows are needed")
    return best[1]


def _joined_chunk_steps(Ld, nu1, nu2, fuse, kind, s, D):
    """Steps of one chunk of a joined program (see DDSolver.chunk): ("head", start) = SR(0) and its
    exchanges; ("join", pre) = levels >= 1 of the cycle, then the cycle join; ("tail", pre) = levels
    >= 1, then the last PS(0).  Returns (steps, state after the chunk) with the cycle join as
    ("join", pre, ec) (ec = the level-1 correction buffer)."""
    D0, D1 = D
    other = lambda x: "b" if x == "a" else "a"
    s0 = s if kind == "head" else other(s)  # the start buffer of the cycle the chunk belongs to
    steps, _ = dd_schedule(Ld, nu1, nu2, fuse, s0, D)
    ps0 = max(i for i, st in enumerate(steps) if st[0] == "prolong_sweep" and st[1] == 0)
    body = [st for st in steps[1:ps0] if st[0] != "exchange" or st[1] != 0]
    i_mid = 0
    while i_mid < len(body) and body[i_mid][0] == "exchange":
        i_mid += 1
    if kind == "head":
        ex = [("exchange", 0, other(s), D0)] + body[:i_mid]
        return [steps[0]] + ex, other(s)
    mid = body[i_mid:]
    if kind == "join":
        ec = steps[ps0][3]
        last = [("join", s, ec), ("exchange", 0, other(s), D0)]
        if Ld >= 2:
            last.append(("exchange", 1, "f", D1))
        return mid + last, other(s)
    ps = steps[ps0]
    return mid + [ps, ("exchange", 0, ps[4], D0)], other(s)


def _joined(nu1, nu2, fuse, smoother="jac"):
    """Whether the local solver joins consecutive cycles (MultigridSolver._joinable for a DD slab)."""
    return nu1 == 1 and nu2 == 1 and fuse and smoother == "jac"


def _partition_for(m, n, P, Ld, nu1=1, nu2=1, fuse=True, grid=None, smoother="jac", nl=0):
    """The Pr x Pc partition (default P x 1: row slabs) with the fewest ghost lines (G at level Ld,
    doubling per finer level) for which exchange depths exist, and those depths.  Ghost lines are
    redundant work."""
    Pr, Pc = grid if grid is not None else (P, 1)
    if Pr * Pc != P:
        raise ValueError(f"DD: grid {Pr} x {Pc} does not hold {P} ranks")
    err = None
    for G in (2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
        try:
            part = Partition2D(m, n, Pr, Pc, Ld, G)
        except ValueError as e:
            err = e
            break
        try:
            return part, exchange_depths(Ld, part.ghost, nu1, nu2, fuse, joined=_joined(nu1, nu2, fuse, smoother),
                                         smoother=smoother, nl=nl)
        except ValueError as e:
            err = e
    raise ValueError(f"DD: no {Pr} x {Pc} partition of a {m} x {n} grid with Ld = {Ld}: {err}")


def _launch_list(launches, dtype, stream):
    """C-ABI calls, ("copy", (dst, src)) device copies, ("rects", (records, elem_size)) strided rectangle copies
    (fea_dd_copy_rects) and ("fn", f) device steps f(stream), in order, on `stream`."""
    for name, args in launches:
        if name == "copy":
            with torch.cuda.stream(stream):
                args[0].copy_(args[1])
        elif name == "rects":
            _lib.call_raw("dd_copy_rects", args[0].ctypes.data, len(args[0]), args[1], stream.cuda_stream)
        elif name == "fn":  # a communicator's device step (halo pack), launched on `stream`
            args(stream)
        else:
            _lib.call(name, dtype, *args, stream.cuda_stream)


_DD_RECT_WORDS = 6  # fea_dd_copy_rects record: int64 dst, src, dst_ld, src_ld, rows, cols


def _rect_records(dst, src):
    """A device copy dst <- src between two equal-shape strided views as fea_dd_copy_rects records (host int64
    [n, 6]): the columns are the dimension of unit stride in both, the rows the largest other dimension, one
    rectangle per index of the remaining ones.  None when the views do not decompose so (no unit-stride
    dimension in common, a row pitch below the row length, different dtypes or devices)."""
    import itertools
    import numpy as np
    if dst.shape != src.shape or dst.dtype != src.dtype or dst.device != src.device or dst.numel() == 0:
        return None
    dims = [k for k in range(dst.dim()) if dst.shape[k] > 1]
    cols = [k for k in dims if dst.stride(k) == 1 and src.stride(k) == 1]
    if not cols:
        if dims:
            return None
        cols = [dst.dim() - 1] if dst.dim() else []
    if not cols:
        return None
    k = cols[0]
    rest = [d for d in dims if d != k]
    r = max(rest, key=lambda d: dst.shape[d]) if rest else None
    nrows = dst.shape[r] if r is not None else 1
    ncols = dst.shape[k]
    dld = dst.stride(r) if r is not None else ncols
    sld = src.stride(r) if r is not None else ncols
    if dld < ncols or sld < ncols:
        return None
    esz = dst.element_size()
    outer = [d for d in rest if d != r]
    recs = []
    for idx in itertools.product(*[range(dst.shape[d]) for d in outer]):
        do = sum(i * dst.stride(d) for i, d in zip(idx, outer))
        so = sum(i * src.stride(d) for i, d in zip(idx, outer))
        recs.append((dst.data_ptr() + do * esz, src.data_ptr() + so * esz, dld, sld, nrows, ncols))
    return np.array(recs, dtype=np.int64).reshape(-1, _DD_RECT_WORDS)


def _as_rect_copies(launches):
    """("copy", (dst, src)) launches -> ("rects", (records, elem_size)) where the views decompose (one
    fea_dd_copy_rects launch instead of a generic strided-copy kernel)."""
    out = []
    for name, args in launches:
        if name == "copy":
            recs = _rect_records(*args)
            if recs is not None:
                out.append(("rects", (recs, args[0].element_size())))
                continue
        out.append((name, args))
    return out


def _split_exchanges(items, overlap_l0=False):
    """An exchange batch as (now, later): later = its finest-level items when overlap_l0 (not waited for until
    a level-0 kernel runs), else nothing (one message batch and one unpack for all of it)."""
    if not overlap_l0:
        return list(items), []
    return [it for it in items if it[0] != 0], [it for it in items if it[0] == 0]


def _rows(t, B, bs, ld, y0, y1):
    """[B, (y1-y0)*ld] view of local rows y0..y1-1 of a framed buffer."""
    return t.as_strided((B, (y1 - y0) * ld), (bs, 1), t.storage_offset() + (y0 + 1) * ld)


def _block(t, B, bs, ld, y0, y1, x0, x1):
    """[B, y1-y0, x1-x0] (strided) view of local rows y0..y1-1, columns x0..x1-1 of a framed buffer."""
    off = 128 // t.element_size() - 1
    return t.as_strided((B, y1 - y0, x1 - x0), (bs, ld, 1), t.storage_offset() + (y0 + 1) * ld + off + x0)


class DDSolver:
    """One rank of the domain-decomposed V-cycle.

    Args: n, rows: global intervals (columns, rows) of the fine grid; rank, world: this rank and the
    number of ranks; grid: (Pr, Pc) blocks, Pr * Pc = world (default (world, 1): row slabs; see
    default_grid for the 2-D choice); comm: a TorchComm (one process per GPU) or None when driven by a
    LocalGroup; agglomerate: Ld (default: see default_agglomeration); overlap_l0: send the finest level's halo
    as a second message batch that completes only before the next level-0 kernel (overlapping levels 1 .. and
    the coarse solve) instead of with the coarse-level halo in one batch — one more message group and one
    more unpack launch per cycle; graph_min: kernel segments of fewer launches run eagerly instead of as HIP
    graphs (on this chip a graph launch between two communication steps costs ~8 us of GPU time, a short
    eager segment less); split_join: the finest join as border rectangles + the halo exchange on a side stream
    beside the interior rectangle (captured cycles: inside the block's graph; segment-wise: eager launches for that
    segment) — off by default: on one GPU (8-rank projection,
    8193^2, 4x2) the split costs 142 instead of 117 us per cycle (thin border rectangles are mostly pipeline
    fill, the interior shares the CUs with them), more than an exchange of this size takes; overlap_l0
    overlaps the level-0 halo with the coarse levels instead; problem / prop / shape / size / R / P / w (the
    two-material problem on the square: each rank's levels carry their window of the global pattern maps) and
    smoother / hnet (the learned HRelax smoother, unjoined cycles) as MultigridSolver; other args as MultigridSolver.
    """

    def __init__(self, n, rows, rank, world, comm=None, agglomerate=None, dtype=torch.float64, device=None,
                 batch=1, nu1=1, nu2=1, fuse=True, graph=True, grid=None, overlap_l0=False, graph_min=5,
                 split_join=False, fold_gather=True, problem="poisson", prop=(1, 20), shape=0, size=2.0, R=None,
                 P=None, w=(1.0, 1.0), smoother="jac", hnet=None):
        self.n, self.m = n, rows
        self.overlap_l0 = overlap_l0
        self.graph_min = graph_min
        self.rank, self.P = rank, world
        self.Pr, self.Pc = grid if grid is not None else (world, 1)
        self.ri, self.ci = divmod(rank, self.Pc)
        self.comm = comm
        self.L = global_levels(rows, n)
        # the learned smoother stops coarsening the distributed levels earlier: its coarse levels cost more per node
        # (the replicated coarse sub-cycle on 257^2 takes 74 us against Jacobi's 24) while its ghost lines grow with
        # 1 + nl lines per sweep — at 8193^2 the projection's best Ld is 3 (1025^2) at 2, 4 and 8 ranks
        # (profiles/r06_dd_hjac/dd_projection_hjac.txt: 8 ranks 334.7 us at Ld = 3 against 382.7 at Ld = 5)
        self.Ld = (default_agglomeration(rows, n, self.Pr, self.L, Pc=self.Pc,
                                         max_nodes=(1 << 21) if smoother == "hjac" else None)
                   if agglomerate is None else int(agglomerate))
        if not 1 <= self.Ld <= self.L - 1:
            raise ValueError(f"DDSolver: agglomeration level {self.Ld} outside [1, {self.L - 1}]")
        if smoother not in ("jac", "hjac"):
            raise ValueError(f"DDSolver: unknown smoother {smoother!r}")
        if smoother == "hjac" and hnet is None:
            raise ValueError("DDSolver: smoother='hjac' needs the HNet weights (hnet=[nl, 3, 3])")
        self.smoother = smoother
        nl = 0 if hnet is None else int(torch.as_tensor(hnet).reshape(-1, 3, 3).shape[0])
        self.part, self.depths = _partition_for(rows, n, world, self.Ld, nu1, nu2, fuse, grid=(self.Pr, self.Pc),
                                                smoother=smoother, nl=nl)
        self.parts = [self.part.level(l, rank) for l in range(self.Ld + 1)]    # rows
        self.cparts = [self.part.clevel(l, rank) for l in range(self.Ld + 1)]  # columns
        self.dtype, self.B = dtype, batch
        self.device = torch.device(device if device is not None else "cuda")
        self.nu1, self.nu2, self.fuse = nu1, nu2, fuse
        p0, q0 = self.parts[0], self.cparts[0]
        self.problem = problem
        self.mass = ms.mass_stencil(size / n)  # FNet of the global grid (the local solvers' own mesh size differs)
        kw = {}
        local_maps = None
        if problem == "interface":
            # MeshCenterInterface (FEANet/mesh.py:4-120) on the global square: every rank's levels take their window
            # of the global level's pattern map; the agglomerated coarse solver builds the global maps of its levels
            if rows != n:
                raise ValueError("DDSolver: the two-material problem is defined on the square only")
            kw = dict(problem="interface", prop=prop, shape=shape, size=size, R=R, P=P, w=w)
            local_maps = []
            for l, (lp, lq) in enumerate(zip(self.parts, self.cparts)):
                gmap = ms.interface_pattern_map((n >> l) + 1, shape, size)
                local_maps.append(gmap[lp.gr0:lp.gr0 + lp.Hloc, lq.gr0:lq.gr0 + lq.Hloc])
        elif problem != "poisson":
            raise ValueError(f"DDSolver: unknown problem {problem!r}")
        if smoother == "hjac":  # MultiGrid(mode='hjac').Step: every relaxation one HRelax sweep
            kw.update(smoother="hjac", hnet=hnet)
        self.local = MultigridSolver(q0.Hloc - 1, rows=p0.Hloc - 1, levels=self.Ld + 1, dtype=dtype,
                                     device=self.device, batch=batch, nu1=nu1, nu2=nu2, fuse=fuse, coarse_tail=False,
                                     graph=False, pid_maps=local_maps, **kw)
        self.coarse = MultigridSolver(n >> self.Ld, rows=rows >> self.Ld, levels=self.L - self.Ld, dtype=dtype,
                                      device=self.device, batch=batch, nu1=nu1, nu2=nu2, fuse=fuse,
                                      coarse_tail=True, graph=False, zero_start=True, **kw)
        for l, (lp, lq) in enumerate(zip(self.parts, self.cparts)):
            Lv = self.local.levels[l]
            assert Lv.H == lp.Hloc and Lv.W == lq.Hloc, (l, Lv.H, Lv.W, lp, lq)
        self.coarse_plan, self.coarse_end = self.coarse._build("a")
        assert self.joinable() == _joined(nu1, nu2, fuse, smoother)
        self.use_graph = graph
        self._capture_ok = True
        # captured cycles: the finest join split into border rectangles (run with the halo exchange on a side
        # stream) and the interior (split_join; DDSolver.join_rects)
        self.split_join = split_join
        # fold_gather (2-D blocks, communicators with a device pack): the agglomeration's staging and placement copies
        # run inside the restriction that computes f_Ld and the coarse plan's first launch (DDSolver._send_form /
        # _gathered_form) instead of as copy launches of their own
        self.fold_gather = fold_gather
        self._segs = {}
        self._graphs = {}
        self._state = "a"
        self._raw = None  # smoother="hjac": the un-reset initial iterate the first cycle after load() reads
        self._hjac_first = False
        self.norm_sq = torch.zeros(batch, dtype=torch.float64, device=self.device)

    # ------------------------------------------------------------------ data
    @property
    def H(self):
        return self.m + 1

    @property
    def W(self):
        return self.n + 1

    def _local_rows(self, x):
        """This rank's stored block (rows [gr0, gr0 + Hloc), columns [gc0, gc0 + Wloc)) of a global
        [B, 1, H, W] tensor, contiguous."""
        p0, q0 = self.parts[0], self.cparts[0]
        x = x.to(self.device, self.dtype).reshape(-1, 1, self.H, self.W)
        if x.shape[0] == 1 and self.B > 1:
            x = x.expand(self.B, 1, self.H, self.W)
        return x[:, :, p0.gr0:p0.gr0 + p0.Hloc, q0.gr0:q0.gr0 + q0.Hloc].contiguous()

    def set_rhs(self, f=None, F=None):
        """Assembled right-hand side of the GLOBAL problem f, [B, 1, H, W] (any device), or its nodal source F
        (FNet applied to the global field first, as MultigridSolver.set_rhs(F=...))."""
        if (f is None) == (F is None):
            raise ValueError("DDSolver.set_rhs: give exactly one of f (assembled) or F (source)")
        if F is not None:
            F = F.to(self.device, self.dtype).reshape(-1, 1, self.H, self.W)
            f = ops.conv3x3(F, torch.from_numpy(self.mass))
        self.local._pack(self._local_rows(f), self.local.levels[0].f, reset=False)

    def load(self, u0=None, bc=None):
        """Global initial iterate (zero by default), reset_boundary applied: u0 * geo + bc
        (jacobi.py:27-29; square geometry, bc = Dirichlet data, zero inside)."""
        H, W = self.H, self.W
        u = torch.zeros((self.B, 1, H, W), dtype=self.dtype, device=self.device) if u0 is None else \
            u0.to(self.device, self.dtype).reshape(-1, 1, H, W).expand(self.B, 1, H, W)
        u = u * (1 - _boundary_mask(H, W, u))
        if bc is not None:
            u = u + bc.to(self.device, self.dtype).reshape(-1, 1, H, W)
        x = self._local_rows(u)
        L0 = self.local.levels[0]
        self.local._pack(x, L0.a, reset=False)
        self.local._pack(x, L0.b, reset=False)
        self._state = "a"
        if self.smoother == "hjac":
            # HRelax forms J(u) - u with the iterate the driver passed, before reset_boundary (as
            # MultigridSolver.load): the first cycle's first level-0 sweep reads it (chunk ("first", s)); one buffer
            # for the solver's life, so captured segments keep its address
            raw = torch.zeros((self.B, 1, H, W), dtype=self.dtype, device=self.device) if u0 is None else \
                u0.to(self.device, self.dtype).reshape(-1, 1, H, W).expand(self.B, 1, H, W)
            if self._raw is None:
                self._raw = torch.zeros_like(L0.a)
            self.local._pack(self._local_rows(raw), self._raw, reset=False)
            self._hjac_first = True

    def owned_block(self):
        """((y0, y1), (x0, x1), u[B, 1, y1-y0, x1-x0]): the current iterate on the global nodes this rank
        owns — its interior block plus the global boundary lines on the edges of the domain it touches,
        so the ranks' blocks tile the whole grid."""
        p0, q0 = self.parts[0], self.cparts[0]
        L0 = self.local.levels[0]
        v = L0.view(L0.buf(self._state))
        ly0 = 0 if self.ri == 0 else p0.lo
        ly1 = p0.Hloc if self.ri == self.Pr - 1 else p0.hi
        lx0 = 0 if self.ci == 0 else q0.lo
        lx1 = q0.Hloc if self.ci == self.Pc - 1 else q0.hi
        return ((p0.gr0 + ly0, p0.gr0 + ly1), (q0.gr0 + lx0, q0.gr0 + lx1),
                v[:, ly0:ly1, lx0:lx1].unsqueeze(1).clone())

    def owned_solution(self):
        """(s, e, u[B, 1, e-s, W]): the current iterate on the interior rows this rank owns (row slabs)."""
        if self.Pc != 1:
            raise RuntimeError("DDSolver.owned_solution: row slabs only; use owned_block()")
        p0 = self.parts[0]
        L0 = self.local.levels[0]
        v = L0.view(L0.buf(self._state))
        return p0.s, p0.e, v[:, p0.lo:p0.hi].unsqueeze(1).clone()

    def residual_norm_sq_local(self):
        """Sum over owned interior nodes of (f - K u)^2 per sample (float64 device tensor [B])."""
        L0 = self.local.levels[0]
        p0, q0 = self.parts[0], self.cparts[0]
        loc = self.local
        _lib.call("mg_residual_norm", self.dtype, L0.buf(self._state).data_ptr(), L0.f.data_ptr(),
                  None if L0.pid is None else L0.pid.data_ptr(), loc.ktab.data_ptr(), loc.ntab, loc.norm_out.data_ptr(), loc.ws.data_ptr(), *L0.geom(),
                  p0.lo, p0.hi, q0.lo, q0.hi, torch.cuda.current_stream(self.device).cuda_stream)
        return loc.norm_out * loc.norm_out

    # ------------------------------------------------------------------ plan
    def _segs_of(self, steps):
        """Kernel steps -> [("k", launches, touches_level0) | ("c", comm step, False)], consecutive
        kernels merged into one segment (one graph launch); segments that touch level 0 are flagged, so
        the level-0 halo exchange completes only before them (vcycle) — behind the coarse-level
        segments and the all-gather in front of them."""
        segs = []
        fold = self.comm is not None and hasattr(self.comm, "halo_pack")
        place = None  # the gathered blocks' placement, folded into the next kernel segment
        if self.local.pair_levels:
            # two-level launches on the distributed levels between the communication steps (same per-level
            # computations on the same local nodes, so the ghost validity of every step is unchanged)
            ok = lambda l: l >= 1 and l + 2 <= self.Ld
            steps = pair_prolongations(pair_restrictions(steps, ok), ok, finest_first=False)
        direct = None  # ("scatter", dst) folded into the next launch: it reads the coarse solution in place
        for si, st in enumerate(steps):
            if st[0] == "scatter" and self._scatter_direct(st, steps[si + 1] if si + 1 < len(steps) else None):
                direct = st
                continue
            if st[0] == "exchange":  # consecutive exchanges go out as one batch of P2P ops
                if self.P == 1:
                    continue  # no neighbours
                if segs and segs[-1][0] == "c" and segs[-1][1][0] == "exchanges":
                    segs[-1][1][1].append(st[1:])
                else:
                    segs.append(("c", ("exchanges", [st[1:]]), False))
                continue
            if st[0] == "gather" and self.P > 1:
                if fold and self.Pc > 1 and segs and segs[-1][0] == "k":
                    # 2-D blocks: the owned block goes to the all-gather's send buffer and the gathered blocks into
                    # the coarse f.  Both fold into the launches around the all-gather where those are the zero-
                    # guess restriction that computes f_Ld (its _send form stores the block too) and the coarse
                    # plan's mid_down (its _gathered form reads the blocks and places them); otherwise a staging
                    # copy ends the kernel segment before the all-gather and a placement copy starts the one after.
                    tgt = self.gather_target()
                    sent = self._send_form(segs[-1][1][-1]) if self.fold_gather else None
                    if sent is not None:
                        segs[-1][1][-1] = sent
                    else:
                        segs[-1][1].append(("copy", (self._gsend, self.gather_source())))
                    place = ("place", self.gather_place_views(tgt))
                    segs.append(("c", ("gather", True), False))
                else:
                    segs.append(("c", st, False))
                continue
            lvl0 = st[0] == "join" or (st[0] not in ("gather", "scatter", "coarse") and st[1] == 0)
            if st[0] == "gather":  # one rank: the all-gather is a device copy
                launches = [("copy", (self.gather_target(), self.gather_source()))]
            elif st[0] == "scatter":  # a device copy, captured with the kernels around it
                launches = [("copy", self.scatter_views(st[1]))]
            elif st[0] == "coarse":
                launches = list(self.coarse_plan)
            elif st[0] == "join":
                launches = [self.local._join_call(st[1], self.local._ptr(1, st[2]))]
            else:
                launches = [self.local.bind_step(st)]
                if direct is not None:
                    launches, direct = [self._read_coarse_in_place(launches[0])], None
            if place is not None:
                gath = self._gathered_form(launches[0]) if self.fold_gather else None
                if gath is not None:
                    launches = [gath] + launches[1:]
                else:
                    launches = [("copy", place[1])] + launches
                place = None
            if segs and segs[-1][0] == "k":
                segs[-1][1].extend(launches)
                if lvl0:
                    segs[-1] = ("k", segs[-1][1], True)
            else:
                segs.append(("k", launches, lvl0))
        if fold:
            # each exchange batch's pack (TorchComm.halo_pack: one kernel) ends the kernel segment before it
            for i, (kind, st, _) in enumerate(segs):
                if kind == "c" and st[0] == "exchanges" and i > 0 and segs[i - 1][0] == "k":
                    f = self.comm.halo_pack(self, *_split_exchanges(st[1], self.overlap_l0))
                    if f is not None:
                        segs[i - 1][1].append(("fn", f))
                    segs[i] = ("c", ("exchanges", st[1], True), False)
        return [(kind, _as_rect_copies(st), lvl0) if kind == "k" else (kind, st, lvl0) for kind, st, lvl0 in segs]

    def _send_form(self, launch):
        """The _send form of the zero-guess restriction `launch` when it computes f_Ld (2-D blocks: it then also
        stores this rank's block of f_Ld into the all-gather's send buffer, fea_mg_zero_restrict2_send /
        fea_mg_zero_restrict_send), else None."""
        name, args = launch
        f_ld = self.local.levels[self.Ld].f.data_ptr()
        pl, ql = self.parts[self.Ld], self.cparts[self.Ld]
        blk = (self._gsend.data_ptr(), pl.lo, pl.lo + self.part.rows_per_rank(self.Ld), ql.lo,
               ql.lo + self.part.cols_per_rank(self.Ld))
        if name == "mg_zero_restrict2" and args[2] == f_ld:
            return ("mg_zero_restrict2_send", tuple(args) + blk)
        if name == "mg_residual_restrict" and args[3] == f_ld and args[0] is None and args[2] is None:
            # (u, f, v_out, fc, pid, ktab, omd, ntab, rtab, nrtab, w0, geometry ...) -> (f, fc, pid, ..., geometry ...)
            return ("mg_zero_restrict_send", (args[1], args[3]) + tuple(args[4:]) + blk)
        return None

    def _gathered_form(self, launch):
        """The coarse plan's first launch in its _gathered form when it is the mid_down over the coarse top level (it
        then reads f_Ld's blocks from the all-gather's buffer and places them, fea_mg_mid_down_gathered), else None."""
        name, args = launch
        if name != "mg_mid_down" or args[0].arr[0] != self.coarse.levels[0].f.data_ptr():
            return None
        c, cc = self.part.rows_per_rank(self.Ld), self.part.cols_per_rank(self.Ld)
        return ("mg_mid_down_gathered", tuple(args) + (self._gstage.data_ptr(), self.Pr, self.Pc, c, cc))

    def _scatter_direct(self, st, nxt):
        """Can the scatter step `st` (coarse solution -> level Ld's buffer st[1]) be dropped, the next step reading
        the coarse solver's buffer in place?  Only for a level-pair prolongation ("prolong_sweep2" at Ld - 2, whose
        kernel reads the level-Ld values element by element: any row pitch and alignment) on pattern-free levels.
        Local level Ld's frame is a window of the coarse field (local row / column 0 = global gr0 / gc0), so
        every node the step's valid outputs use holds the same value; only the window's outer frame line (rows
        / columns -1 and H) then shows the global neighbours instead of the local frame's padding, which reaches
        ghost nodes the exchange depths already treat as invalid."""
        if nxt is None or nxt[0] != "prolong_sweep2" or nxt[1] + 2 != self.Ld or nxt[2] != st[1]:
            return False
        return self.local.levels[self.Ld].pid is None and self.coarse.levels[0].pid is None

    def _read_coarse_in_place(self, launch):
        """mg_prolong2's launch with its level-(l+2) correction (argument 1; row pitch and sample stride: the last
        two arguments) taken from the coarse solver's solution window of this rank instead of level Ld."""
        name, args = launch
        assert name == "mg_prolong2", name
        Lc = self.coarse.levels[0]
        pl = self.parts[self.Ld]
        gc0 = self.cparts[self.Ld].gr0 if self.Pc > 1 else 0
        buf = Lc.buf(self.coarse_end)
        win = buf.data_ptr() + (pl.gr0 * Lc.ld + gc0) * buf.element_size()
        args = list(args)
        args[1] = win
        args[-2], args[-1] = Lc.ld, Lc.bs
        return (name, tuple(args))

    def joinable(self):
        return self.local._joinable()

    def chunk(self, key):
        """Cached launch/communication segments of one program chunk:
        ("cycle", s): a whole V-cycle from buffer s;  ("head", s): its first step (SR(0)) and exchanges;
        ("join", pre): the rest of a cycle whose pre-smoothed iterate is in `pre`, ending in the cycle
        join into the other buffer;  ("tail", pre): the same ending in the last PS(0)."""
        if key in self._segs:
            return self._segs[key]
        kind, b = key
        if kind in ("cycle", "first"):
            steps, end = dd_schedule(self.Ld, self.nu1, self.nu2, self.fuse, b, self.depths, self.smoother)
        else:
            steps, end = _joined_chunk_steps(self.Ld, self.nu1, self.nu2, self.fuse, kind, b, self.depths)
        segs = self._segs_of(steps)
        if kind == "first":  # the first finest-level HRelax sweep reads the un-reset iterate (load())
            segs = self._first_sweep_raw(segs)
        res = (segs, end)
        self._segs[key] = res
        return res

    def _first_sweep_raw(self, segs):
        """The segments with the cycle's first level-0 HRelax sweep given the un-reset iterate (its u_raw slot,
        argument 1), as MultigridSolver._vcycles_plain does for the first cycle after load()."""
        f0 = self.local.levels[0].f.data_ptr()
        out, done = [], False
        for kind, launches, lvl0 in segs:
            if kind == "k" and not done:
                launches = list(launches)
                for i, (name, args) in enumerate(launches):
                    fi = {"mg_hsweep": 2, "mg_hsweep_restrict": 2, "mg_prolong_hsweep": 3}.get(name)
                    if fi is not None and args[fi] == f0:
                        launches[i] = (name, (args[0], self._raw.data_ptr()) + tuple(args[2:]))
                        done = True
                        break
            out.append((kind, launches, lvl0))
        return out

    def program(self, k):
        """The chunks of vcycle(k) from the current state, and the end state."""
        s = self._state
        if self._hjac_first and k >= 1:  # learned smoother, first cycle after load(): never joined
            s1 = self.chunk(("first", s))[1]
            keys, end = self._program_from(s1, k - 1)
            return [("first", s)] + keys, end
        return self._program_from(s, k)

    def _program_from(self, s, k):
        if k < 1:
            return [], s
        if k >= 2 and self.joinable():
            keys = [("head", s)]
            pre = "b" if s == "a" else "a"
            for _ in range(k - 1):
                keys.append(("join", pre))
                pre = "b" if pre == "a" else "a"
            keys.append(("tail", pre))
            return keys, ("b" if pre == "a" else "a")
        keys = []
        for _ in range(k):
            keys.append(("cycle", s))
            s = self.chunk(("cycle", s))[1]
        return keys, s

    def segments(self, start):
        """One unjoined V-cycle (kept for callers/tests): (segments, end buffer)."""
        return self.chunk(("cycle", start))

    def run_kernels(self, key, i):
        """Kernel segment i of chunk `key` (graph-replayed after its first run)."""
        segs, _ = self.chunk(key)
        launches = segs[i][1]
        gkey = (key, i)
        stream = torch.cuda.current_stream(self.device)
        if len(launches) < self.graph_min:  # a graph launch costs more GPU time than a few eager launches
            _launch_list(launches, self.dtype, stream)
            return
        if not self.use_graph or gkey not in self._graphs:
            if self.use_graph:
                self._graphs[gkey] = None  # eager once, capture on the second use
            _launch_list(launches, self.dtype, stream)
            return
        g = self._graphs[gkey]
        if g is None:
            # thread-local capture: the communicator's own threads (the NCCL watchdog) keep running
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(self.device)
            s.wait_stream(stream)
            try:
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    _launch_list(launches, self.dtype, s)
            except RuntimeError:  # capture refused: this rank keeps launching eagerly
                torch.cuda.synchronize(self.device)
                self.use_graph = False
                _launch_list(launches, self.dtype, stream)
                return
            stream.wait_stream(s)
            self._graphs[gkey] = g
        g.replay()

    # buffers the communication steps touch
    def level_rows(self, l, name, y0, y1):
        Lv = self.local.levels[l]
        return _rows(Lv.buf(name), Lv.B, Lv.bs, Lv.ld, y0, y1)

    def level_block(self, l, name, y0, y1, x0, x1):
        Lv = self.local.levels[l]
        return _block(Lv.buf(name), Lv.B, Lv.bs, Lv.ld, y0, y1, x0, x1)

    def gather_source(self):
        """Owned block of f_Ld padded to rows_per_rank x cols_per_rank (ranks on the last row / column
        add the zero boundary line).  Row slabs: whole framed rows (a contiguous run)."""
        pl, ql = self.parts[self.Ld], self.cparts[self.Ld]
        c = self.part.rows_per_rank(self.Ld)
        if self.Pc == 1:
            return self.level_rows(self.Ld, "f", pl.lo, pl.lo + c)
        return self.level_block(self.Ld, "f", pl.lo, pl.lo + c, ql.lo, ql.lo + self.part.cols_per_rank(self.Ld))

    def gather_target(self):
        """Row slabs: rows [1, 1 + P*c) of the coarse solver's top-level f (the P chunks in rank order).
        2-D blocks: a [P, B, c_r, c_c] staging buffer, placed by gather_place()."""
        Lc = self.coarse.levels[0]
        c = self.part.rows_per_rank(self.Ld)
        if self.Pc == 1:
            return _rows(Lc.f, Lc.B, Lc.bs, Lc.ld, 1, 1 + self.P * c)
        if getattr(self, "_gstage", None) is None:
            cc = self.part.cols_per_rank(self.Ld)
            # zero-filled once: a communicator that moves nothing (the projection's PackComm) then leaves a
            # deterministic coarse right-hand side instead of whatever the allocator handed back
            self._gstage = torch.zeros((self.P, self.B, c, cc), dtype=self.dtype, device=self.device)
            self._gsend = torch.zeros((self.B, c, cc), dtype=self.dtype, device=self.device)
        return self._gstage

    def gather_place_views(self, blocks):
        """(destination, source) of the placement of the gathered blocks ([P, B, c_r, c_c], rank order) into
        the coarse f: two strided [B, Pr, c_r, Pc, c_c] views, of the framed field and of the staging buffer."""
        Lc = self.coarse.levels[0]
        c, cc = self.part.rows_per_rank(self.Ld), self.part.cols_per_rank(self.Ld)
        Pr, Pc, B = self.Pr, self.Pc, Lc.B
        off = 128 // Lc.f.element_size() - 1
        dst = Lc.f.as_strided((B, Pr, c, Pc, cc), (Lc.bs, c * Lc.ld, Lc.ld, cc, 1),
                              Lc.f.storage_offset() + 2 * Lc.ld + off + 1)
        return dst, blocks.view(Pr, Pc, B, c, cc).permute(2, 0, 3, 1, 4)

    def gather_place(self, blocks):
        """2-D blocks: copy the gathered blocks into the coarse f — ONE copy between two strided views."""
        dst, src = self.gather_place_views(blocks)
        dst.copy_(src)

    def gather(self, folded=False):
        """The level-Ld all-gather over the communicator (the coarse solver's f on every rank).  folded: the
        staging copy and the placement run inside the kernel segments around it (_segs_of)."""
        if self.Pc == 1:
            self.comm.allgather(self.gather_target(), self.gather_source())
            return
        tgt = self.gather_target()
        if not folded:
            self._gsend.copy_(self.gather_source())
        self.comm.allgather(tgt, self._gsend)
        if not folded:
            self.gather_place(tgt)

    def scatter_views(self, dst):
        """(destination, source): this rank's stored block of the coarse solution -> level Ld's `dst`."""
        pl, ql = self.parts[self.Ld], self.cparts[self.Ld]
        Lc = self.coarse.levels[0]
        if self.Pc == 1:
            src = _rows(Lc.buf(self.coarse_end), Lc.B, Lc.bs, Lc.ld, pl.gr0, pl.gr0 + pl.Hloc)
            return self.level_rows(self.Ld, dst, 0, pl.Hloc), src
        src = _block(Lc.buf(self.coarse_end), Lc.B, Lc.bs, Lc.ld, pl.gr0, pl.gr0 + pl.Hloc, ql.gr0, ql.gr0 + ql.Hloc)
        return self.level_block(self.Ld, dst, 0, pl.Hloc, 0, ql.Hloc), src

    def scatter(self, dst):
        """Copy this rank's block of the coarse solution into level Ld's buffer `dst`."""
        d, s = self.scatter_views(dst)
        d.copy_(s)

    def regions(self, l, name, d):
        """The halo of depth d on level l's buffer `name`, ONE phase: [(peer, (dy, dx), send view, receive
        view)] for every neighbour, diagonal ones included — up/down: d rows of the owned columns; left/right:
        the owned rows of d columns; corners: d x d.  Every send view lies in the sender's OWNED nodes, so all
        messages can be in flight at once (the two-phase x-then-y form carried the corners through the ghost
        columns instead, two dependent message rounds).  Row slabs (Pc = 1): whole framed rows (contiguous
        runs, sent in place)."""
        lp, lq = self.parts[l], self.cparts[l]
        out = []
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                ri, ci = self.ri + dy, self.ci + dx
                if (dy, dx) == (0, 0) or not (0 <= ri < self.Pr and 0 <= ci < self.Pc):
                    continue
                sr, rr = {-1: ((lp.lo, lp.lo + d), (lp.lo - d, lp.lo)), 0: ((lp.lo, lp.hi), (lp.lo, lp.hi)),
                          1: ((lp.hi - d, lp.hi), (lp.hi, lp.hi + d))}[dy]
                sc, rc = {-1: ((lq.lo, lq.lo + d), (lq.lo - d, lq.lo)), 0: ((lq.lo, lq.hi), (lq.lo, lq.hi)),
                          1: ((lq.hi - d, lq.hi), (lq.hi, lq.hi + d))}[dx]
                if self.Pc == 1:
                    send, recv = self.level_rows(l, name, *sr), self.level_rows(l, name, *rr)
                else:
                    send, recv = self.level_block(l, name, *sr, *sc), self.level_block(l, name, *rr, *rc)
                out.append((ri * self.Pc + ci, (dy, dx), send, recv))
        return out

    # ------------------------------------------------------------------ driver (one process per rank)
    GRAPH_CYCLES = 16  # joined cycles per captured graph (capturable communicators)

    def vcycle(self, k=1):
        if self.comm is None:
            raise RuntimeError("DDSolver.vcycle: no communicator (use LocalGroup for in-process ranks)")
        keys, end = self.program(k)
        if self.use_graph and getattr(self.comm, "capturable", False) and self._capture_ok:
            self._vcycle_captured(keys)
        else:
            self._run_chunks(keys, captured=False)
        self._state = end
        if k >= 1:
            self._hjac_first = False

    def _vcycle_captured(self, keys):
        """vcycle with every chunk's kernels AND communication steps captured in one HIP graph per block of up to
        GRAPH_CYCLES consecutive cycle joins (head and tail chunks: one graph each): a cycle costs no graph-launch
        gaps between its kernel segments and ~one host graph launch per block.  Each block runs eagerly once
        (plans, communicator set-up), is captured the second time and replayed after that.  A communicator whose
        operations cannot be captured (capture raises) turns this off for the solver; it then runs the
        segment-wise path.

        The decision is collective: a capture records the communicator's calls without running them, so after
        every capture the ranks agree (one all-reduce, outside the graph) whether ALL of them captured; if any
        refused, every rank discards its graphs and runs the segment-wise path from that block on — the same
        calls in the same order on every rank, so no message is left unmatched.  Only capture failures count as
        a refusal (_is_capture_error); any other error inside the capture (e.g. an invalid kernel argument) is
        reported through the same all-reduce as an error and then raised on EVERY rank (the failing rank re-raises
        its own exception, its peers a RuntimeError naming the failure count), so no rank is left waiting in a
        collective its failed peer never enters."""
        i = 0
        while i < len(keys):
            key = keys[i]
            n = 1
            if key[0] == "join":
                while i + n < len(keys) and keys[i + n][0] == "join" and n < self.GRAPH_CYCLES:
                    n += 1
            block = keys[i:i + n]
            gkey = ("cap",) + tuple(block)
            g = self._graphs.get(gkey)
            if g is None and gkey not in self._graphs:
                self._graphs[gkey] = None  # eager once
                self._run_chunks(block, captured=False)
            elif g is None:
                stream = torch.cuda.current_stream(self.device)
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream(self.device)
                s.wait_stream(stream)
                refused, error = False, None
                try:
                    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                        self._run_chunks(block, captured=True)
                except RuntimeError as e:
                    if _is_capture_error(e):
                        refused = True
                    else:
                        error = e
                    g = None
                    torch.cuda.synchronize(self.device)
                stream.wait_stream(s)
                n_refused, n_errors = self._agree(refused, error is not None)
                if n_errors:  # every rank raises: the failing one its own error, the others name it
                    if error is not None:
                        raise error
                    raise RuntimeError(f"DDSolver: {n_errors} peer rank(s) failed inside a captured block of "
                                       f"cycles {block[0]}..{block[-1]} (rank {self.rank} aborts with them)")
                if n_refused:  # some rank refused: every rank leaves the captured path
                    self._capture_ok = False
                    self._graphs = {k: v for k, v in self._graphs.items() if k[0] != "cap"}
                    self._run_chunks(keys[i:], captured=False)
                    return
                self._graphs[gkey] = g
                g.replay()
            else:
                g.replay()
            i += n

    def _agree(self, refused, failed):
        """(ranks that refused the capture, ranks that failed with another error): one all-reduce of the two
        counts through the communicator (this rank's own flags when it is alone)."""
        if getattr(self.comm, "world", 1) <= 1:
            return int(refused), int(failed)
        t = torch.tensor([float(refused), float(failed)], dtype=torch.float64, device=self.device)
        t = self.comm.allreduce_sum(t)
        return int(t[0].item()), int(t[1].item())

    def _run_chunks(self, keys, captured=False):
        """Issue the chunks' kernel segments and communication steps in order on the current stream; captured:
        inside a graph capture (kernel segments launched directly, the level-0 halo completed within the block)."""
        pending = None  # level-0 halo exchange in flight (overlaps the coarse levels' kernels)
        for key in keys:
            segs, _ = self.chunk(key)
            skip = -1
            for i, (kind, st, lvl0) in enumerate(segs):
                if i == skip:
                    continue
                if kind == "k":
                    if lvl0 and pending is not None:
                        self.comm.exchange_finish(pending)
                        pending = None
                    if self.split_join and self._split_join(segs, i):
                        skip = i + 1  # the exchange ran beside the interior join (eager launches off capture)
                    elif captured:
                        _launch_list(segs[i][1], self.dtype, torch.cuda.current_stream(self.device))
                    else:
                        self.run_kernels(key, i)
                elif st[0] == "exchanges":
                    # coarse-level halos first (the next kernel needs them), the finest iterate's
                    # halo after, not waited for until a level-0 kernel runs: on RCCL both go out on
                    # the communicator's stream in this order, so the compute stream only waits for
                    # the first batch and level 1 .. Ld-1 run while the finest rows are in flight
                    now, later = _split_exchanges(st[1], self.overlap_l0)
                    packed = len(st) > 2 and st[2]
                    if pending is not None:
                        self.comm.exchange_finish(pending)
                        pending = None
                    if now:
                        self.comm.exchange_many(self, now, packed=packed)
                    if later:
                        pending = self.comm.exchange_many(self, later, wait=False, packed=packed)
                elif st[0] == "gather":
                    self.gather(folded=len(st) > 1 and st[1] is True)
                elif st[0] == "scatter":
                    self.scatter(st[1])
        if pending is not None:
            self.comm.exchange_finish(pending)

    def join_rects(self):
        """(border rectangles, interior rectangle) of the finest level's cycle join, as fea_mg_cycle_join_rects takes
        them ({I0, I1, c0, c1}: coarse rows, odd fine-column bounds): the border holds every node the cycle's halo
        exchange sends (owned nodes within D0 fine / D1 coarse lines of an edge with a neighbour) or receives (the
        ghost lines), so the interior join can run while the messages are in flight."""
        if getattr(self, "_rects", None) is not None:
            return self._rects
        D0, D1 = self.depths
        p0, q0, p1, q1 = self.parts[0], self.cparts[0], self.parts[1], self.cparts[1]
        Hc, W = self.local.levels[1].H, self.local.levels[0].W
        up, down = self.ri > 0, self.ri < self.Pr - 1
        left, right = self.ci > 0, self.ci < self.Pc - 1
        odd_up = lambda x: x if x & 1 else x + 1
        odd_down = lambda x: x if x & 1 else x - 1
        Ia = max(p1.lo + D1, (p0.lo + D0 + 2) // 2) if up else 1
        Ib = min(p1.hi - D1, (p0.hi - D0 + 1) // 2) if down else Hc - 1
        ca = max(2 * (q1.lo + D1) - 1, odd_up(q0.lo + D0)) if left else 1
        cb = min(2 * (q1.hi - D1) - 1, odd_down(q0.hi - D0)) if right else W - 1
        if not (1 <= Ia < Ib <= Hc - 1 and 1 <= ca < cb <= W - 1):
            self._rects = ([], None)
            return self._rects
        border = [r for r in ((1, Ia, 1, W - 1), (Ib, Hc - 1, 1, W - 1), (Ia, Ib, 1, ca), (Ia, Ib, cb, W - 1))
                  if r[0] < r[1] and r[2] < r[3]]
        self._rects = (border, (Ia, Ib, ca, cb))
        return self._rects

    def _split_join(self, segs, i):
        """Captured cycles: a kernel segment that ends in the cycle join (+ the halo pack) followed by its halo
        exchange runs as [the segment's other kernels] -> the border rectangles' join, the pack, the exchange and
        the unpack on a side stream BESIDE the interior rectangle's join on the compute stream -> rejoin.  Returns
        False (nothing issued) where the pattern or the rectangles do not apply."""
        launches = segs[i][1]
        if i + 1 >= len(segs) or segs[i + 1][0] != "c" or segs[i + 1][1][0] != "exchanges" or self.P == 1:
            return False
        nj = [k for k, (name, _) in enumerate(launches) if name == "mg_cycle_join"]
        if len(nj) != 1 or any(name not in ("fn",) for name, _ in launches[nj[0] + 1:]):
            return False
        border, inner = self.join_rects()
        if inner is None or not border:
            return False
        j = nj[0]
        jargs = launches[j][1][:23]  # mg_cycle_join's arguments up to bsc (no norm)
        rects = self.__dict__.setdefault("_rect_arrays", {})
        arrs = []
        for key, rs in (("border", border), ("inner", [inner])):
            if key not in rects:
                import ctypes
                rects[key] = (ctypes.c_int * (4 * len(rs)))(*[x for r in rs for x in r])
            arrs.append((len(rs), ctypes_addr(rects[key])))
        main = torch.cuda.current_stream(self.device)
        side = self.__dict__.get("_side")
        if side is None:
            side = self._side = torch.cuda.Stream(self.device)
        _launch_list(launches[:j], self.dtype, main)
        side.wait_stream(main)
        st = segs[i + 1][1]
        with torch.cuda.stream(side):
            _launch_list([("mg_cycle_join_rects", jargs + arrs[0])] + launches[j + 1:], self.dtype, side)
            now, later = _split_exchanges(st[1], self.overlap_l0)
            items = list(now) + list(later)
            self.comm.exchange_many(self, items, packed=len(st) > 2 and st[2])
        _launch_list([("mg_cycle_join_rects", jargs + arrs[1])], self.dtype, main)
        main.wait_stream(side)
        return True

    def residual_norm(self):
        n2 = self.residual_norm_sq_local()
        if self.comm is not None:
            n2 = self.comm.allreduce_sum(n2)
        return torch.sqrt(n2)


_CAPTURE_WORDS = ("operation not permitted when stream is capturing", "stream is capturing",
                  "hiperrorstreamcapture", "cudaerrorstreamcapture", "hiperrorcapturedevent", "cudaerrorcapturedevent",
                  "operation not permitted on an event last recorded in a capturing stream",
                  "capture was invalidated", "capture sequence", "stream capture")


def _is_capture_error(e):
    """Does this exception say that stream capture was refused (rather than that a call was wrong)?  HIP's
    stream-capture error codes 900-908 (hipErrorStreamCapture*, hipErrorCapturedEvent) by number or name, and the
    wording torch and RCCL use for a call made while a stream captures.  Nothing else: the C ABI's FEA_EINVAL
    ('invalid arguments'), autograd's 'backward through the graph' or a fault during a graph replay propagate."""
    msg = str(e)
    if "invalid arguments" in msg:
        return False
    if any(f"hipError_t {c})" in msg or f"error {c}" in msg for c in range(900, 909)):
        return True
    low = msg.lower()
    return any(w in low for w in _CAPTURE_WORDS)


def ctypes_addr(arr):
    import ctypes
    return ctypes.addressof(arr)


def _boundary_mask(H, W, like):
    m = torch.zeros((H, W), dtype=like.dtype, device=like.device)
    m[0, :] = 1
    m[-1, :] = 1
    m[:, 0] = 1
    m[:, -1] = 1
    return m


_DD_BLOCK_WORDS = 4  # fea_dd_copy_blocks record: int64 base, int64 stage, int64 ld, int32 rows + int32 cols


class _Staging:
    """Pack / unpack of a list of [B, rows, cols] (or [B, run]) framed-buffer views to / from one contiguous
    staging buffer (fea_dd_copy_blocks: one launch for all of them).  Views are concatenated in order.
    `records`: the block table (host int64 [nblocks, 4]); copy_blocks() launches any concatenation of them."""

    def __init__(self, views, device, dtype):
        import numpy as np
        sizes = []
        for v in views:
            if v.dim() == 2:  # [B, run]: whole framed rows of a row slab
                (B, cols), (bs, one), rows, ld = v.shape, v.stride(), 1, v.shape[1]
            else:
                (B, rows, cols), (bs, ld, one) = v.shape, v.stride()
            assert one == 1
            sizes.append((B, rows, cols, bs, ld))
        self.n = sum(B * rows * cols for B, rows, cols, _, _ in sizes)
        self.buf = torch.empty(max(self.n, 1), dtype=dtype, device=device)
        self.esz = self.buf.element_size()
        recs, off = [], 0
        for v, (B, rows, cols, bs, ld) in zip(views, sizes):
            for b in range(B):
                recs.append((v.data_ptr() + b * bs * self.esz, self.buf.data_ptr() + off * self.esz, ld,
                             rows | (cols << 32)))
                off += rows * cols
        self.records = np.array(recs, dtype=np.int64).reshape(-1, _DD_BLOCK_WORDS)

    def copy(self, to_stage, stream=None):
        copy_blocks(self.records, to_stage, self.esz, self.buf.device, stream)


def copy_blocks(records, to_stage, esz, device, stream=None):
    """One fea_dd_copy_blocks launch (per 48 blocks) over a block table (host int64 [nblocks, 4])."""
    import numpy as np
    recs = np.ascontiguousarray(records, dtype=np.int64)
    stream = torch.cuda.current_stream(device) if stream is None else stream
    _lib.call_raw("dd_copy_blocks", recs.ctypes.data, len(recs), esz, int(to_stage), stream.cuda_stream)


def halo_staging(regs):
    """Staging of one exchange's regions (DDSolver.regions of all its items): the send views grouped per
    neighbour (in item order, the order the neighbour unpacks them in) in one buffer, the receive views
    likewise in another; seg_s / seg_r: (peer, element offset, element count) of each neighbour's message."""
    peers = sorted({p for p, _, _, _ in regs})
    by_send = [[a for p, _, a, _ in regs if p == q] for q in peers]
    by_recv = [[b for p, _, _, b in regs if p == q] for q in peers]
    dev, dt = regs[0][2].device, regs[0][2].dtype
    send = _Staging([v for vs in by_send for v in vs], dev, dt)
    recv = _Staging([v for vs in by_recv for v in vs], dev, dt)
    seg_s, seg_r, i_s, i_r = [], [], 0, 0
    for q, vs, vr in zip(peers, by_send, by_recv):
        ns, nr = sum(v.numel() for v in vs), sum(v.numel() for v in vr)
        seg_s.append((q, i_s, ns))
        seg_r.append((q, i_r, nr))
        i_s += ns
        i_r += nr
    return send, recv, seg_s, seg_r


class TorchComm:
    """Halo exchange / all-gather / all-reduce over torch.distributed.  With the nccl backend (RCCL
    on ROCm) device buffers are sent directly; with gloo they are staged through host memory."""

    def __init__(self, group=None, dist=None, capture=None):
        if dist is None:  # (tests pass an in-process stand-in with the same interface)
            import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.gpu = dist.get_backend(group) == "nccl"
        # Whole-cycle capture (kernels + RCCL calls in one HIP graph per block of cycles; host issue 4-5 us per cycle
        # instead of 42-52) is OPT-IN (capture=True or FEANET_DD_CAPTURE=1): it has run against stand-in
        # communicators only, never on a multi-rank RCCL job, so the default is the segment-wise path (one graph per
        # kernel segment between communication steps).  bench.py times both on every N > 1 line (dd_modes) under a
        # bounded phase.  If any rank's capture is refused, all ranks fall back together (_vcycle_captured).
        self.capturable = self.gpu and capture if capture is not None else (
            self.gpu and os.environ.get("FEANET_DD_CAPTURE", "0") == "1")

    def exchange(self, s, l, name, d):
        self.exchange_many(s, [(l, name, d)])

    def _plan(self, s, items):
        """One round of P2P messages for every (level, buffer, depth) in `items` (DDSolver.regions, diagonal
        neighbours included).  Row slabs with RCCL: each region is a contiguous run of the framed layout and
        is sent / received in place.  Otherwise: every region of all items is packed into one staging buffer
        with one kernel, ONE message per neighbour (its regions in item order — the peer unpacks in the same
        order), and unpacked with one kernel; gloo moves the staging buffers through host memory."""
        dist = self.dist
        regs = [r for l, name, d in items for r in s.regions(l, name, d)]
        if not regs:
            return {"ops": [], "direct": True}
        direct = self.gpu and all(a.is_contiguous() and b.is_contiguous() for _, _, a, b in regs)
        if direct:
            ops = [dist.P2POp(dist.isend, a, p, self.group) for p, _, a, _ in regs]
            ops += [dist.P2POp(dist.irecv, b, p, self.group) for p, _, _, b in regs]
            return {"ops": ops, "direct": True}
        send, recv, seg_s, seg_r = halo_staging(regs)
        dt = send.buf.dtype
        if self.gpu:
            sb, rb = send.buf, recv.buf
        else:
            sb, rb = torch.empty(send.buf.shape, dtype=dt), torch.empty(recv.buf.shape, dtype=dt)
        ops = [dist.P2POp(dist.isend, sb[o:o + n], q, self.group) for q, o, n in seg_s]
        ops += [dist.P2POp(dist.irecv, rb[o:o + n], q, self.group) for q, o, n in seg_r]
        return {"ops": ops, "direct": False, "send": send, "recv": recv, "sb": sb, "rb": rb}

    def _cached_plan(self, s, items):
        # plans hold views of s's buffers: cached on s itself (keyed by this communicator), never on
        # the communicator under id(s), which a later solver could reuse
        plans = s.__dict__.setdefault("_comm_plans", {})
        key = (id(self), tuple(items))
        plan = plans.get(key)
        if plan is None:
            plan = self._plan(s, items)
            plans[key] = plan
        return plan

    def halo_pack(self, s, *item_lists):
        """The device step that packs the send regions of exchange_many(s, items) for every items in
        item_lists — ONE launch, f(stream) — or None when all regions go out in place.  The solver launches it
        inside its kernel segment (captured in the segment's graph) and then calls
        exchange_many(..., packed=True)."""
        import numpy as np
        sends = [p["send"] for p in (self._cached_plan(s, items) for items in item_lists if items)
                 if p["ops"] and not p["direct"]]
        if not sends:
            return None
        recs = np.concatenate([st.records for st in sends])
        esz, dev = sends[0].esz, sends[0].buf.device
        return lambda stream: copy_blocks(recs, True, esz, dev, stream)

    def exchange_many(self, s, items, wait=True, packed=False):
        """Refresh d ghost lines around rank s's block for every (level, buffer, d) in `items`: pack, ONE
        batch of P2P ops with every neighbour (diagonal ones included), unpack.  The plans are built once per
        item list and reused (fixed device views).  packed: the pack already ran (halo_pack).  wait=False: return a handle for exchange_finish instead of
        completing the batch (with RCCL its ops run on the communicator's stream meanwhile; finishing makes
        the current stream wait for them and unpacks, the host does not block)."""
        plan = self._cached_plan(s, items)
        if not plan["ops"]:
            return None
        if not plan["direct"]:
            if not packed:
                plan["send"].copy(True)
            if not self.gpu:
                plan["sb"].copy_(plan["send"].buf)
        handle = (self.dist.batch_isend_irecv(plan["ops"]), plan)
        if wait:
            self.exchange_finish(handle)
            return None
        return handle

    def exchange_finish(self, handle):
        if handle is None:
            return
        works, plan = handle
        for w in works:
            w.wait()
        if not plan["direct"]:
            if not self.gpu:
                plan["recv"].buf.copy_(plan["rb"])
            plan["recv"].copy(False)

    def allgather(self, target, source):
        dist = self.dist
        if self.gpu and target.is_contiguous() and source.is_contiguous():
            dist.all_gather_into_tensor(target.reshape(-1), source.reshape(-1), group=self.group)
            return
        src = source.contiguous() if self.gpu else source.cpu()
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        if target.dim() == 4:  # 2-D blocks: [P, B, c_r, c_c] staging, rank order
            target.copy_(torch.stack(parts, 0))
            return
        B = source.shape[0]
        full = torch.stack([p.reshape(B, -1) for p in parts], 1).reshape(B, -1)
        target.copy_(full)

    def allreduce_sum(self, t):
        if self.gpu:
            self.dist.all_reduce(t, group=self.group)
            return t
        c = t.cpu()
        self.dist.all_reduce(c, group=self.group)
        return c.to(t.device)


class LocalGroup:
    """All P ranks in one process (one device): the same schedule executed in lockstep with the
    exchanges done as device copies.  Used to test the decomposition on a single GPU."""

    def __init__(self, n, rows, world, **kw):
        self.ranks = [DDSolver(n, rows, r, world, comm=None, **kw) for r in range(world)]  # kw: grid=(Pr, Pc), ...

    def set_rhs(self, f=None, F=None):
        for s in self.ranks:
            s.set_rhs(f, F)

    def load(self, u0=None, bc=None):
        for s in self.ranks:
            s.load(u0, bc)

    def vcycle(self, k=1):
        r0 = self.ranks[0]
        keys, end = r0.program(k)
        for key in keys:
            segs, _ = r0.chunk(key)
            for i, (kind, st, _) in enumerate(segs):
                if kind == "k":
                    for s in self.ranks:
                        s.chunk(key)
                        s.run_kernels(key, i)
                elif st[0] == "exchanges":
                    for l, name, d in st[1]:
                        self._exchange(l, name, d)
                elif st[0] == "gather":
                    chunks = [s.gather_source() for s in self.ranks]
                    for s in self.ranks:
                        tgt = s.gather_target()
                        if s.Pc == 1:
                            c = chunks[0].shape[1]
                            for r, ch in enumerate(chunks):
                                tgt[:, r * c:(r + 1) * c].copy_(ch)
                        else:
                            for r, ch in enumerate(chunks):
                                tgt[r].copy_(ch)
                            s.gather_place(tgt)
                elif st[0] == "scatter":
                    for s in self.ranks:
                        s.scatter(st[1])
        for s in self.ranks:
            s._state = end
            if k >= 1:
                s._hjac_first = False

    def _exchange(self, l, name, d):
        """TorchComm.exchange_many as device copies: every receive region from its peer's matching send
        region (the one facing the receiver).  Sends read owned nodes only, so the order does not matter."""
        for q in self.ranks:
            for peer, (dy, dx), _, recv in q.regions(l, name, d):
                p = self.ranks[peer]
                send = [sv for pr, dr, sv, _ in p.regions(l, name, d) if pr == q.rank and dr == (-dy, -dx)]
                recv.copy_(send[0])

    def solution(self):
        """Global iterate assembled from the ranks' owned blocks (they tile the grid)."""
        s0 = self.ranks[0]
        out = torch.zeros((s0.B, 1, s0.H, s0.W), dtype=s0.dtype, device=s0.device)
        for s in self.ranks:
            (y0, y1), (x0, x1), u = s.owned_block()
            out[:, :, y0:y1, x0:x1] = u
        return out

    def residual_norm(self):
        return torch.sqrt(sum(s.residual_norm_sq_local() for s in self.ranks))
