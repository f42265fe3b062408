"""CPU restatement of one rank of the domain-decomposed V-cycle (feanet_amd.dd) with the oracle's
operators on numpy slabs and torch.distributed (gloo) for the exchanges: checks the partition,
the communication schedule and the coarse agglomeration without a GPU.  Test infrastructure."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "multigrid-feanet_amd"))

from oracle import feanet_oracle as orc  # noqa: E402


def problem(m, n, B, seed=0):
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((B, m + 1, n + 1))
    u0 = rng.standard_normal((B, m + 1, n + 1))
    geo, _ = orc.square_geometry((m + 1, n + 1), np.float64)
    bc = rng.random((B, m + 1, n + 1)) * (1 - geo)
    return f, u0 * geo + bc


class OracleRank:
    """Rank r's local levels as numpy arrays, kernel steps executed with oracle operators (local
    boundary rows are kept, the framed kernels' semantics)."""

    def __init__(self, m, n, P, r, Ld, f, u, nu=(1, 1)):
        from feanet_amd.dd import _partition_for, global_levels
        self.m, self.n, self.P, self.r, self.Ld = m, n, P, r, Ld
        self.L = global_levels(m, n)
        # the partition and exchange depths DDSolver uses (the oracle runs its unjoined cycles)
        self.part, self.depths = _partition_for(m, n, P, Ld, nu[0], nu[1], fuse=True)
        self.parts = [self.part.level(l, r) for l in range(Ld + 1)]
        self.lv = [orc.Level(n >> l, "poisson", np.float64, m=p.Hloc - 1) for l, p in enumerate(self.parts)]
        B = f.shape[0]
        self.B = B
        p0 = self.parts[0]
        self.bufs = [dict() for _ in range(Ld + 1)]
        for l, p in enumerate(self.parts):
            z = np.zeros((B, p.Hloc, (n >> l) + 1))
            self.bufs[l] = {"f": z.copy(), "a": z.copy(), "b": z.copy(), "zero": z.copy()}
        self.bufs[0]["f"] = f[:, p0.gr0:p0.gr0 + p0.Hloc].copy()
        self.bufs[0]["a"] = u[:, p0.gr0:p0.gr0 + p0.Hloc].copy()
        self.bufs[0]["b"] = u[:, p0.gr0:p0.gr0 + p0.Hloc].copy()
        self.R = (orc.np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32) / 4)[None]
        self.nu = nu
        self.coarse = orc.OracleMultigrid(n >> Ld, "poisson", np.float64, levels=self.L - Ld, rows=m >> Ld)

    def sweep(self, l, src, f):
        lv = self.lv[l]
        return orc.jacobi_sweep(src, f, lv.pid, lv.ktab, lv.geo, src * (1 - lv.geo))

    def kernel(self, st):
        kind, l = st[0], st[1]
        b = self.bufs
        lv = self.lv
        if kind == "sweep":
            src = b[l]["zero"] if st[2] is None else b[l][st[2]]
            b[l][st[3]] = self.sweep(l, src, b[l]["f"])
        elif kind in ("resid_restrict", "sweep_restrict"):
            if kind == "sweep_restrict":
                v = self.sweep(l, b[l][st[2]], b[l]["f"])
                b[l][st[3]] = v
            elif st[2] is None:
                v = self.sweep(l, b[l]["zero"], b[l]["f"])
                if st[3] is not None:
                    b[l][st[3]] = v
            else:
                v = b[l][st[2]]
            r = b[l]["f"] - lv[l].K(v)
            fc = orc.restrict(r, lv[l].pid, self.R)
            keep = b[l + 1]["f"].copy()
            keep[:, 1:-1, 1:-1] = fc[:, 1:-1, 1:-1]
            b[l + 1]["f"] = keep
        elif kind == "prolong_sweep":
            # the kernel's semantics: the corrected field x enters the stencil on every row (also the
            # slab's local edge rows), interior nodes are swept, edge rows keep the source values
            src = self.sweep(l, b[l]["zero"], b[l]["f"]) if st[2] == "omdf" else b[l][st[2]]
            x = src + orc.prolong(b[l + 1][st[3]], lv[l + 1].pid, self.R)
            omd = orc.omega_over_d(lv[l].ktab, 2. / 3., np.float64)[0]
            swept = omd * (b[l]["f"] - lv[l].K(x)) + x
            b[l][st[4]] = np.where(lv[l].geo > 0, swept, src)
        else:
            raise AssertionError(kind)

    def rows(self, l, name, y0, y1):
        return self.bufs[l][name][:, y0:y1]

    def coarse_solve(self, fglob):
        """The replicated coarse sub-cycle: the oracle V-cycle of levels >= Ld from a zero guess."""
        from feanet_amd.schedule import vcycle_schedule
        from test_schedule import interpret
        steps, end = vcycle_schedule(self.L - self.Ld, 1, 1, None, "a", None, True, top_zero=True)
        mg = self.coarse
        mg.w = (1.0, 1.0)
        bufs = interpret(mg, steps, np.zeros_like(fglob), fglob)
        return bufs[0][end]


def run_rank(rank, world, m, n, Ld, port, outdir, cycles=2):
    """Process entry: one rank of the oracle DD V-cycle over gloo; saves its owned rows."""
    import torch
    import torch.distributed as dist
    from feanet_amd.dd import dd_schedule
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    B = 2
    f, u = problem(m, n, B)
    R = OracleRank(m, n, world, rank, Ld, f, u)
    state = "a"
    for _ in range(cycles):
        steps, end = dd_schedule(Ld, 1, 1, True, state, R.depths)
        for st in steps:
            if st[0] == "exchange":
                l, name, DEPTH = st[1], st[2], st[3]
                lp = R.parts[l]
                ops, recv = [], []
                if rank > 0:
                    ops.append(dist.P2POp(dist.isend, torch.from_numpy(R.rows(l, name, lp.lo, lp.lo + DEPTH).copy()),
                                          rank - 1))
                    t = torch.empty((B, DEPTH, (n >> l) + 1), dtype=torch.float64)
                    ops.append(dist.P2POp(dist.irecv, t, rank - 1))
                    recv.append((t, lp.lo - DEPTH))
                if rank < world - 1:
                    ops.append(dist.P2POp(dist.isend, torch.from_numpy(R.rows(l, name, lp.hi - DEPTH, lp.hi).copy()),
                                          rank + 1))
                    t = torch.empty((B, DEPTH, (n >> l) + 1), dtype=torch.float64)
                    ops.append(dist.P2POp(dist.irecv, t, rank + 1))
                    recv.append((t, lp.hi))
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
                for t, y0 in recv:
                    R.bufs[l][name][:, y0:y0 + DEPTH] = t.numpy()
            elif st[0] == "gather":
                pl = R.parts[Ld]
                c = R.part.rows_per_rank(Ld)
                chunk = torch.from_numpy(R.rows(Ld, "f", pl.lo, pl.lo + c).copy())
                parts = [torch.empty_like(chunk) for _ in range(world)]
                dist.all_gather(parts, chunk)
                fglob = np.zeros((B, (m >> Ld) + 1, (n >> Ld) + 1))
                fglob[:, 1:1 + world * c] = np.concatenate([p.numpy() for p in parts], axis=1)
            elif st[0] == "coarse":
                eglob = R.coarse_solve(fglob)
            elif st[0] == "scatter":
                pl = R.parts[Ld]
                R.bufs[Ld][st[1]] = eglob[:, pl.gr0:pl.gr0 + pl.Hloc].copy()
            else:
                R.kernel(st)
        state = end
    p0 = R.parts[0]
    np.save(os.path.join(outdir, f"rank{rank}.npy"), R.bufs[0][state][:, p0.lo:p0.hi])
    dist.destroy_process_group()
