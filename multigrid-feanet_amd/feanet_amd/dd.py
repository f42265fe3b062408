"""Domain-decomposed V-cycle over several MI355X GPUs: row slabs + halo exchange.

The fine grid ((m+1) x (n+1) nodes, Poisson) is cut into P row slabs, one per rank (one process
per GPU, torch.distributed over RCCL/xGMI).  Levels 0 .. Ld-1 are distributed; the level-Ld
restriction is all-gathered and the rest of the V-cycle (levels >= Ld of the global grid) is solved
redundantly on every rank by a single-GPU MultigridSolver, whose correction each rank copies back
for its slab.  The result is bitwise the single-GPU V-cycle on the global grid (same kernels, same
per-node arithmetic, same coarse schedule), which the tests check.

Layout (class Partition).  Interior row offsets t_r = r * m / P split level 0; level l uses
t_r / 2^l, so fine rows (2I-1, 2I) and coarse row I always live on the same rank.  Rank r owns
global rows [s, e) = [1 + t_r, 1 + t_{r+1}) (the last rank up to H-1) and stores rows
[gr0, gr0 + Hloc) with gr0 = t_r - G_l (0 on rank 0): G_l = G * 2^(Ld-l) ghost rows per side, the
doubling keeping gr0_l = 2 gr0_{l+1} so the unmodified level kernels pair fine and coarse rows
exactly as on one grid.  The level kernels compute every local interior row; ghost rows near the
slab edge are refreshed by exchanges, deeper ones are redundant work (G_0 rows per side, a few %).

Communication (communication-avoiding).  Every level kernel already computes the ghost rows it
stores, so ghost rows stay correct to a depth that shrinks by one row per sweep and halves per
restriction; an exchange is needed only where that depth would run out.  Per V-cycle:
  after the finest pre-smoothing (or the cycle join):  D1 rows of f_1 (and D0 rows of the
                                                       pre-smoothed finest iterate, joined cycles)
  at level Ld:  all-gather of the owned rows of f_Ld -> the replicated coarse solve -> local copy
  after the finest post-smoothing (unjoined cycles):   D0 rows of the finest iterate
i.e. ONE batch of neighbour messages and one all-gather per V-cycle, whatever Ld.  D0 and D1 are the
smallest depths for which a row-validity simulation of the schedule (exchange_depths) keeps every
owned row exact; the result stays bitwise the single-GPU V-cycle.
"""
import torch

from . import _lib
from .schedule import vcycle_schedule
from .solver import MultigridSolver



def global_levels(m, n):
    """Levels of the global grid (MultigridSolver's default for a rectangle)."""
    L = 1
    while n % (1 << L) == 0 and m % (1 << L) == 0 and (n >> L) >= 2 and (m >> L) >= 2:
        L += 1
    return L


def default_agglomeration(m, n, P, L, max_nodes=1 << 20):
    """Smallest Ld whose global level has <= max_nodes nodes, within what the partition allows."""
    Ld = 1
    while Ld < L - 1 and ((m >> Ld) + 1) * ((n >> Ld) + 1) > max_nodes and m % (P << (Ld + 1)) == 0 \
            and m // (P << (Ld + 1)) >= 4:
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


def dd_schedule(Ld, nu1=1, nu2=1, fuse=True, start="a", depths=(4, 4)):
    """The distributed part of one (unjoined) V-cycle: kernel steps of feanet_amd.schedule plus
    ("exchange", l, buf, depth), ("gather",), ("coarse",), ("scatter", dst).  depths = (D0, D1)."""
    D0, D1 = depths
    steps, end = vcycle_schedule(Ld + 1, nu1, nu2, None, start, tail_from=Ld, fuse=fuse)
    out = []
    for i, st in enumerate(steps):
        kind, l = st[0], st[1]
        if kind == "coarse_tail":
            out += [("gather",), ("coarse",), ("scatter", st[2])]
            continue
        out.append(st)
        if kind in ("resid_restrict", "sweep_restrict") and l == 0 and Ld >= 2:
            out.append(("exchange", 1, "f", D1))
    out.append(("exchange", 0, end, D0))
    return out, end


def _restricted(r):
    """Ghost depth of a restriction whose fine input is valid to depth r (fine rows 2I-1..2I+1)."""
    return (r - 1) // 2 if r >= 1 else -1


def simulate_validity(program, Ld, ghost, init=None):
    """Row validity along a list of dd steps: for every (level, buffer) the number of ghost rows past
    the owned rows that hold the single-grid values (owned rows exact iff >= 0).  Buffers start as in
    `init` (default: fully valid, as after load()); f_0 is static (fully valid).  Returns False as soon
    as a kernel would write a wrong owned row, else the final validity map.  Steps may also be
    ("join", pre, ec_name)."""
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


def exchange_depths(Ld, ghost, nu1=1, nu2=1, fuse=True, joined=True):
    """Smallest (D0, D1) (by bytes: D1 rows are half as wide) keeping the owned rows exact in every
    program DDSolver runs.  Across program boundaries only the finest iterate carries over, and every
    program ends by exchanging it (D0 rows): so checking each program once from the weakest start
    state (finest iterates valid to exactly D0) covers any sequence of them (induction)."""
    def programs(D):
        out = [dd_schedule(Ld, nu1, nu2, fuse, "a", D)[0]]
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
        return all(simulate_validity(p, Ld, ghost, init) for p in programs((D0, D1)))

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


def _joined(nu1, nu2, fuse):
    """Whether the local solver joins consecutive cycles (MultigridSolver._joinable for a DD slab)."""
    return nu1 == 1 and nu2 == 1 and fuse


def _partition_for(m, n, P, Ld, nu1=1, nu2=1, fuse=True):
    """The slab partition with the fewest ghost rows (G ghost rows at level Ld, doubling per finer
    level) for which exchange depths exist, and those depths.  Ghost rows are redundant work."""
    err = None
    for G in (2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
        try:
            part = Partition(m, n, P, Ld, G)
        except ValueError as e:
            err = e
            break
        try:
            return part, exchange_depths(Ld, part.ghost, nu1, nu2, fuse, joined=_joined(nu1, nu2, fuse))
        except ValueError as e:
            err = e
    raise ValueError(f"DD: no slab partition of {m} rows over {P} ranks with Ld = {Ld}: {err}")


def _launch_list(launches, dtype, stream):
    """C-ABI calls and ("copy", (dst, src)) device copies, in order, on `stream`."""
    for name, args in launches:
        if name == "copy":
            with torch.cuda.stream(stream):
                args[0].copy_(args[1])
        else:
            _lib.call(name, dtype, *args, stream.cuda_stream)


def _rows(t, B, bs, ld, y0, y1):
    """[B, (y1-y0)*ld] view of local rows y0..y1-1 of a framed buffer."""
    return t.as_strided((B, (y1 - y0) * ld), (bs, 1), t.storage_offset() + (y0 + 1) * ld)


class DDSolver:
    """One rank of the domain-decomposed V-cycle.

    Args: n, rows: global intervals (columns, rows) of the fine grid; rank, world: this rank and the
    number of slabs; comm: a TorchComm (one process per GPU) or None when driven by a LocalGroup;
    agglomerate: Ld (default: see default_agglomeration); other args as MultigridSolver (Poisson).
    """

    def __init__(self, n, rows, rank, world, comm=None, agglomerate=None, dtype=torch.float64, device=None,
                 batch=1, nu1=1, nu2=1, fuse=True, graph=True):
        self.n, self.m = n, rows
        self.rank, self.P = rank, world
        self.comm = comm
        self.L = global_levels(rows, n)
        self.Ld = default_agglomeration(rows, n, world, self.L) if agglomerate is None else int(agglomerate)
        if not 1 <= self.Ld <= self.L - 1:
            raise ValueError(f"DDSolver: agglomeration level {self.Ld} outside [1, {self.L - 1}]")
        self.part, self.depths = _partition_for(rows, n, world, self.Ld, nu1, nu2, fuse)
        self.parts = [self.part.level(l, rank) for l in range(self.Ld + 1)]
        self.dtype, self.B = dtype, batch
        self.device = torch.device(device if device is not None else "cuda")
        self.nu1, self.nu2, self.fuse = nu1, nu2, fuse
        p0 = self.parts[0]
        self.local = MultigridSolver(n, rows=p0.Hloc - 1, levels=self.Ld + 1, dtype=dtype, device=self.device,
                                     batch=batch, nu1=nu1, nu2=nu2, fuse=fuse, coarse_tail=False, graph=False)
        self.coarse = MultigridSolver(n >> self.Ld, rows=rows >> self.Ld, levels=self.L - self.Ld, dtype=dtype,
                                      device=self.device, batch=batch, nu1=nu1, nu2=nu2, fuse=fuse,
                                      coarse_tail=True, graph=False, zero_start=True)
        for l, lp in enumerate(self.parts):
            Lv = self.local.levels[l]
            assert Lv.H == lp.Hloc and Lv.W == (n >> l) + 1, (l, Lv.H, lp)
        self.coarse_plan, self.coarse_end = self.coarse._build("a")
        assert self.joinable() == _joined(nu1, nu2, fuse)
        self.use_graph = graph
        self._segs = {}
        self._graphs = {}
        self._state = "a"
        self.norm_sq = torch.zeros(batch, dtype=torch.float64, device=self.device)

    # ------------------------------------------------------------------ data
    @property
    def H(self):
        return self.m + 1

    @property
    def W(self):
        return self.n + 1

    def _local_rows(self, x):
        """Rows [gr0, gr0 + Hloc) of a global [B, 1, H, W] tensor, contiguous."""
        p0 = self.parts[0]
        x = x.to(self.device, self.dtype).reshape(-1, 1, self.H, self.W)
        if x.shape[0] == 1 and self.B > 1:
            x = x.expand(self.B, 1, self.H, self.W)
        return x[:, :, p0.gr0:p0.gr0 + p0.Hloc].contiguous()

    def set_rhs(self, f):
        """Assembled right-hand side of the GLOBAL problem, [B, 1, H, W] (any device)."""
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

    def owned_solution(self):
        """(s, e, u[B, 1, e-s, W]): the current iterate on the rows this rank owns."""
        p0 = self.parts[0]
        L0 = self.local.levels[0]
        v = L0.view(L0.buf(self._state))
        return p0.s, p0.e, v[:, p0.lo:p0.hi].unsqueeze(1).clone()

    def residual_norm_sq_local(self):
        """Sum over owned rows of (f - K u)^2 per sample (float64 device tensor [B])."""
        L0 = self.local.levels[0]
        p0 = self.parts[0]
        loc = self.local
        _lib.call("mg_residual_norm", self.dtype, L0.buf(self._state).data_ptr(), L0.f.data_ptr(), None,
                  loc.ktab.data_ptr(), loc.ntab, loc.norm_out.data_ptr(), loc.ws.data_ptr(), *L0.geom(),
                  p0.lo, p0.hi, torch.cuda.current_stream(self.device).cuda_stream)
        return loc.norm_out * loc.norm_out

    # ------------------------------------------------------------------ plan
    def _segs_of(self, steps):
        """Kernel steps -> [("k", launches, touches_level0) | ("c", comm step, False)], consecutive
        kernels merged into one segment (one graph launch); segments that touch level 0 are flagged, so
        the level-0 halo exchange completes only before them (vcycle) — behind the coarse-level
        segments and the all-gather in front of them."""
        segs = []
        for st in steps:
            if st[0] == "exchange":  # consecutive exchanges go out as one batch of P2P ops
                if self.P == 1:
                    continue  # no neighbours
                if segs and segs[-1][0] == "c" and segs[-1][1][0] == "exchanges":
                    segs[-1][1][1].append(st[1:])
                else:
                    segs.append(("c", ("exchanges", [st[1:]]), False))
                continue
            if st[0] == "gather" and self.P > 1:
                segs.append(("c", st, False))
                continue
            lvl0 = st[0] == "join" or (st[0] not in ("gather", "scatter", "coarse") and st[1] == 0)
            if st[0] == "gather":  # one rank: the all-gather is a device copy
                launches = [("copy", (self.gather_target(), self.gather_source()))]
            elif st[0] == "scatter":  # a device copy, captured with the kernels around it
                pl = self.parts[self.Ld]
                Lc = self.coarse.levels[0]
                src = _rows(Lc.buf(self.coarse_end), Lc.B, Lc.bs, Lc.ld, pl.gr0, pl.gr0 + pl.Hloc)
                launches = [("copy", (self.level_rows(self.Ld, st[1], 0, pl.Hloc), src))]
            elif st[0] == "coarse":
                launches = list(self.coarse_plan)
            elif st[0] == "join":
                launches = [self.local._join_call(st[1], self.local._ptr(1, st[2]))]
            else:
                launches = [self.local.bind_step(st)]
            if segs and segs[-1][0] == "k":
                segs[-1][1].extend(launches)
                if lvl0:
                    segs[-1] = ("k", segs[-1][1], True)
            else:
                segs.append(("k", launches, lvl0))
        return segs

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
        if kind == "cycle":
            steps, end = dd_schedule(self.Ld, self.nu1, self.nu2, self.fuse, b, self.depths)
        else:
            steps, end = _joined_chunk_steps(self.Ld, self.nu1, self.nu2, self.fuse, kind, b, self.depths)
        res = (self._segs_of(steps), end)
        self._segs[key] = res
        return res

    def program(self, k):
        """The chunks of vcycle(k) from the current state, and the end state."""
        s = self._state
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

    def gather_source(self):
        """Owned rows of f_Ld, padded to rows_per_rank (the last rank adds the zero boundary row)."""
        pl = self.parts[self.Ld]
        c = self.part.rows_per_rank(self.Ld)
        return self.level_rows(self.Ld, "f", pl.lo, pl.lo + c)

    def gather_target(self):
        """Rows [1, 1 + P*c) of the coarse solver's top-level f: the P gathered chunks in rank order."""
        Lc = self.coarse.levels[0]
        c = self.part.rows_per_rank(self.Ld)
        return _rows(Lc.f, Lc.B, Lc.bs, Lc.ld, 1, 1 + self.P * c)

    def scatter(self, dst):
        """Copy this rank's rows of the coarse solution into level Ld's buffer `dst`."""
        pl = self.parts[self.Ld]
        Lc = self.coarse.levels[0]
        src = _rows(Lc.buf(self.coarse_end), Lc.B, Lc.bs, Lc.ld, pl.gr0, pl.gr0 + pl.Hloc)
        self.level_rows(self.Ld, dst, 0, pl.Hloc).copy_(src)

    # ------------------------------------------------------------------ driver (one process per rank)
    def vcycle(self, k=1):
        if self.comm is None:
            raise RuntimeError("DDSolver.vcycle: no communicator (use LocalGroup for in-process ranks)")
        keys, end = self.program(k)
        pending = None  # level-0 halo exchange in flight (overlaps the coarse levels' kernels)
        for key in keys:
            segs, _ = self.chunk(key)
            for i, (kind, st, lvl0) in enumerate(segs):
                if kind == "k":
                    if lvl0 and pending is not None:
                        self.comm.exchange_finish(pending)
                        pending = None
                    self.run_kernels(key, i)
                elif st[0] == "exchanges":
                    # coarse-level halos first (the next kernel needs them), the finest iterate's
                    # halo after, not waited for until a level-0 kernel runs: on RCCL both go out on
                    # the communicator's stream in this order, so the compute stream only waits for
                    # the first batch and level 1 .. Ld-1 run while the finest rows are in flight
                    now = [it for it in st[1] if it[0] != 0]
                    later = [it for it in st[1] if it[0] == 0]
                    if pending is not None:
                        self.comm.exchange_finish(pending)
                        pending = None
                    if now:
                        self.comm.exchange_many(self, now)
                    if later:
                        pending = self.comm.exchange_many(self, later, wait=False)
                elif st[0] == "gather":
                    self.comm.allgather(self.gather_target(), self.gather_source())
                elif st[0] == "scatter":
                    self.scatter(st[1])
        if pending is not None:
            self.comm.exchange_finish(pending)
        self._state = end

    def residual_norm(self):
        n2 = self.residual_norm_sq_local()
        if self.comm is not None:
            n2 = self.comm.allreduce_sum(n2)
        return torch.sqrt(n2)


def _boundary_mask(H, W, like):
    m = torch.zeros((H, W), dtype=like.dtype, device=like.device)
    m[0, :] = 1
    m[-1, :] = 1
    m[:, 0] = 1
    m[:, -1] = 1
    return m


class TorchComm:
    """Halo exchange / all-gather / all-reduce over torch.distributed.  With the nccl backend (RCCL
    on ROCm) device buffers are sent directly; with gloo they are staged through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.gpu = dist.get_backend(group) == "nccl"

    def _stage(self, t):
        return t.contiguous() if self.gpu else t.cpu()

    def exchange(self, s, l, name, d):
        self.exchange_many(s, [(l, name, d)])

    def exchange_many(self, s, items, wait=True):
        """Refresh d ghost rows on both sides of rank s's slab for every (level, buffer, d) in `items`,
        as ONE batch of P2P ops.  The op lists are built once per item list and reused (fixed device
        views).  wait=False: return a handle for exchange_finish instead of completing the batch (with
        RCCL the ops run on the communicator's stream meanwhile; finishing makes the current stream
        wait for them, the host does not block)."""
        dist = self.dist
        # plans hold views of s's buffers: cached on s itself (keyed by this communicator), never on
        # the communicator under id(s), which a later solver could reuse
        plans = s.__dict__.setdefault("_comm_plans", {})
        key = (id(self), tuple(items))
        plan = plans.get(key)
        if plan is None:
            sends, recvs = [], []
            for l, name, d in items:
                lp = s.parts[l]
                if s.rank > 0:
                    sends.append((s.level_rows(l, name, lp.lo, lp.lo + d), s.rank - 1))
                    recvs.append((s.level_rows(l, name, lp.lo - d, lp.lo), s.rank - 1))
                if s.rank < s.P - 1:
                    sends.append((s.level_rows(l, name, lp.hi - d, lp.hi), s.rank + 1))
                    recvs.append((s.level_rows(l, name, lp.hi, lp.hi + d), s.rank + 1))
            direct = self.gpu and all(t.is_contiguous() for t, _ in sends + recvs)
            if direct:
                sb = [t for t, _ in sends]
                rb = [t for t, _ in recvs]
            else:
                dev = sends[0][0].device if (sends and self.gpu) else "cpu"
                sb = [torch.empty(t.shape, dtype=t.dtype, device=dev) for t, _ in sends]
                rb = [torch.empty(t.shape, dtype=t.dtype, device=dev) for t, _ in recvs]
            ops = [dist.P2POp(dist.isend, b, peer, self.group) for b, (_, peer) in zip(sb, sends)]
            ops += [dist.P2POp(dist.irecv, b, peer, self.group) for b, (_, peer) in zip(rb, recvs)]
            plan = (ops, direct, list(zip(sb, [t for t, _ in sends])), list(zip(rb, [t for t, _ in recvs])))
            plans[key] = plan
        ops, direct, spairs, rpairs = plan
        if not ops:
            return None
        if not direct:
            for b, t in spairs:
                b.copy_(t)
        handle = (dist.batch_isend_irecv(ops), direct, rpairs)
        if not wait:
            return handle
        self.exchange_finish(handle)
        return None

    def exchange_finish(self, handle):
        if handle is None:
            return
        works, direct, rpairs = handle
        for w in works:
            w.wait()
        if not direct:
            for b, t in rpairs:
                t.copy_(b)

    def allgather(self, target, source):
        dist = self.dist
        if self.gpu and target.is_contiguous() and source.is_contiguous():
            dist.all_gather_into_tensor(target.reshape(-1), source.reshape(-1), group=self.group)
            return
        src = self._stage(source)
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
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
        self.ranks = [DDSolver(n, rows, r, world, comm=None, **kw) for r in range(world)]

    def set_rhs(self, f):
        for s in self.ranks:
            s.set_rhs(f)

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
                        c = chunks[0].shape[1]
                        for r, ch in enumerate(chunks):
                            tgt[:, r * c:(r + 1) * c].copy_(ch)
                elif st[0] == "scatter":
                    for s in self.ranks:
                        s.scatter(st[1])
        for s in self.ranks:
            s._state = end

    def _exchange(self, l, name, d):
        for r, s in enumerate(self.ranks):
            lp = s.parts[l]
            if r > 0:
                q = self.ranks[r - 1]
                qp = q.parts[l]
                s.level_rows(l, name, lp.lo - d, lp.lo).copy_(q.level_rows(l, name, qp.hi - d, qp.hi))
            if r < len(self.ranks) - 1:
                q = self.ranks[r + 1]
                qp = q.parts[l]
                s.level_rows(l, name, lp.hi, lp.hi + d).copy_(q.level_rows(l, name, qp.lo, qp.lo + d))

    def solution(self):
        """Global iterate assembled from the owned rows (boundary rows from ranks 0 / P-1)."""
        s0 = self.ranks[0]
        out = torch.zeros((s0.B, 1, s0.H, s0.W), dtype=s0.dtype, device=s0.device)
        for s in self.ranks:
            a, b, u = s.owned_solution()
            out[:, :, a:b] = u
            L0 = s.local.levels[0]
            v = L0.view(L0.buf(s._state))
            p0 = s.parts[0]
            if s.rank == 0:
                out[:, 0, 0] = v[:, 0]
            if s.rank == s.P - 1:
                out[:, 0, -1] = v[:, p0.Hloc - 1]
        return out

    def residual_norm(self):
        return torch.sqrt(sum(s.residual_norm_sq_local() for s in self.ranks))
