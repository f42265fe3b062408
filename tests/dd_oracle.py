"""CPU restatement of one rank of the domain-decomposed V-cycle (feanet_amd.dd) with the oracle's
operators on numpy blocks and torch.distributed (gloo) for the exchanges: checks the 2-D partition
(row slabs = 1 column block), the two-phase halo exchange, the communication schedule and the coarse
agglomeration without a GPU — for the Poisson and the two-material problem (each rank's levels carry their window
of the global pattern maps) and for weighted Jacobi and the learned HRelax smoother.  Test infrastructure."""
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
    """Rank r's local levels as numpy arrays (its stored block: rows [gr0, gr0 + Hloc) x columns
    [gc0, gc0 + Wloc)), kernel steps executed with oracle operators (the block's edge lines are kept,
    the framed kernels' semantics)."""

    def __init__(self, m, n, P, r, Ld, f, u, nu=(1, 1), grid=None, problem="poisson", hw=None):
        from feanet_amd.dd import _partition_for, global_levels
        self.m, self.n, self.P, self.r, self.Ld = m, n, P, r, Ld
        self.Pr, self.Pc = grid if grid is not None else (P, 1)
        self.ri, self.ci = divmod(r, self.Pc)
        self.L = global_levels(m, n)
        # the partition and exchange depths DDSolver uses (the oracle runs its unjoined cycles)
        self.hw = hw
        self.smoother = "jac" if hw is None else "hjac"
        self.part, self.depths = _partition_for(m, n, P, Ld, nu[0], nu[1], fuse=True, grid=(self.Pr, self.Pc),
                                                smoother=self.smoother, nl=0 if hw is None else len(hw))
        self.parts = [self.part.level(l, r) for l in range(Ld + 1)]
        self.cparts = [self.part.clevel(l, r) for l in range(Ld + 1)]
        self.lv = [orc.Level(q.Hloc - 1, "poisson", np.float64, m=p.Hloc - 1)
                   for p, q in zip(self.parts, self.cparts)]
        if problem == "interface":  # the window of the global level's MeshCenterInterface map (oracle mesh loops)
            for l, (p, q, lv) in enumerate(zip(self.parts, self.cparts, self.lv)):
                ktab, pid = orc.interface_mesh((n >> l) + 1)
                lv.ktab, lv.pid = ktab, np.asarray(pid)[p.gr0:p.gr0 + p.Hloc, q.gr0:q.gr0 + q.Hloc]
        B = f.shape[0]
        self.B = B
        p0, q0 = self.parts[0], self.cparts[0]
        self.bufs = [dict() for _ in range(Ld + 1)]
        for l, (p, q) in enumerate(zip(self.parts, self.cparts)):
            z = np.zeros((B, p.Hloc, q.Hloc))
            self.bufs[l] = {"f": z.copy(), "a": z.copy(), "b": z.copy(), "zero": z.copy()}
        blk = (slice(None), slice(p0.gr0, p0.gr0 + p0.Hloc), slice(q0.gr0, q0.gr0 + q0.Hloc))
        self.bufs[0]["f"] = f[blk].copy()
        self.bufs[0]["a"] = u[blk].copy()
        self.bufs[0]["b"] = u[blk].copy()
        self.R = (orc.np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32) / 4)[None]
        if problem == "interface":
            self.R = np.broadcast_to(self.R, (16, 3, 3))
        self.nu = nu
        self.coarse = orc.OracleMultigrid(n >> Ld, problem, np.float64, levels=self.L - Ld, rows=m >> Ld)
        self.coarse.hw = hw

    def sweep(self, l, src, f):
        lv = self.lv[l]
        return orc.jacobi_sweep(src, f, lv.pid, lv.ktab, lv.geo, src * (1 - lv.geo))

    def hrelax(self, l, src, f):
        """HRelax on the block (M-FEANet-mg_test.ipynb:147-155) with the framed kernels' semantics: the block's
        edge lines keep their values (J keeps them, the masked HNet correction is zero there)."""
        j = self.sweep(l, src, f)
        return j + orc.hnet(j - src, self.lv[l].geo, self.hw)

    def restrict_into(self, l, v):
        b, lv = self.bufs, self.lv
        fc = orc.restrict(b[l]["f"] - lv[l].K(v), lv[l].pid, self.R)
        keep = b[l + 1]["f"].copy()
        keep[:, 1:-1, 1:-1] = fc[:, 1:-1, 1:-1]
        b[l + 1]["f"] = keep

    def kernel(self, st):
        kind, l = st[0], st[1]
        b = self.bufs
        lv = self.lv
        if kind in ("hsweep", "hsweep_restrict"):
            src = b[l]["zero"] if st[2] is None else b[l][st[2]]
            v = self.hrelax(l, src, b[l]["f"])
            b[l][st[3]] = v
            if kind == "hsweep_restrict":
                self.restrict_into(l, v)
        elif kind == "prolong_hsweep":
            x = b[l][st[2]] + orc.prolong(b[l + 1][st[3]], lv[l + 1].pid, self.R)
            b[l][st[4]] = self.hrelax(l, x, b[l]["f"])
        elif kind == "sweep":
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
            self.restrict_into(l, v)
        elif kind == "prolong_sweep":
            # the kernel's semantics: the corrected field x enters the stencil on every node (also the
            # block's local edge lines), interior nodes are swept, edge lines keep the source values
            src = self.sweep(l, b[l]["zero"], b[l]["f"]) if st[2] == "omdf" else b[l][st[2]]
            x = src + orc.prolong(b[l + 1][st[3]], lv[l + 1].pid, self.R)
            omd = orc.omega_over_d(lv[l].ktab, 2. / 3., np.float64)
            omd = omd[0] if len(omd) == 1 else omd[np.asarray(lv[l].pid, np.int64)]
            swept = omd * (b[l]["f"] - lv[l].K(x)) + x
            b[l][st[4]] = np.where(lv[l].geo > 0, swept, src)
        else:
            raise AssertionError(kind)

    def halo(self, l, name, d, phase):
        """[(send array, peer, (row slice, column slice) to receive into)] — DDSolver.halo's regions."""
        p, q = self.parts[l], self.cparts[l]
        a = self.bufs[l][name]
        out = []
        if phase == "x":
            rows = slice(p.lo, p.hi)
            if self.ci > 0:
                out.append((a[:, rows, q.lo:q.lo + d].copy(), self.r - 1, (rows, slice(q.lo - d, q.lo))))
            if self.ci < self.Pc - 1:
                out.append((a[:, rows, q.hi - d:q.hi].copy(), self.r + 1, (rows, slice(q.hi, q.hi + d))))
        else:
            cols = slice(None)
            if self.ri > 0:
                out.append((a[:, p.lo:p.lo + d].copy(), self.r - self.Pc, (slice(p.lo - d, p.lo), cols)))
            if self.ri < self.Pr - 1:
                out.append((a[:, p.hi - d:p.hi].copy(), self.r + self.Pc, (slice(p.hi, p.hi + d), cols)))
        return out

    def coarse_solve(self, fglob):
        """The replicated coarse sub-cycle: the oracle V-cycle of levels >= Ld from a zero guess."""
        from feanet_amd.schedule import hjac_schedule, vcycle_schedule
        from test_schedule import interpret
        if self.hw is not None:
            steps, end = hjac_schedule(self.L - self.Ld, 1, 1, "zero", None, True)
        else:
            steps, end = vcycle_schedule(self.L - self.Ld, 1, 1, None, "a", None, True, top_zero=True)
        mg = self.coarse
        mg.w = (1.0, 1.0)
        bufs = interpret(mg, steps, np.zeros_like(fglob), fglob)
        return bufs[0][end]


def run_rank(rank, world, m, n, Ld, port, outdir, cycles=2, grid=None, kind="poisson", hw=None):
    """Process entry: one rank of the oracle DD V-cycle over gloo; saves its owned block."""
    import torch
    import torch.distributed as dist
    from feanet_amd.dd import dd_schedule
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    B = 2
    f, u = problem(m, n, B)
    R = OracleRank(m, n, world, rank, Ld, f, u, grid=grid, problem=kind, hw=hw)
    state = "a"
    for _ in range(cycles):
        steps, end = dd_schedule(Ld, 1, 1, True, state, R.depths, R.smoother)
        for st in steps:
            if st[0] == "exchange":
                l, name, DEPTH = st[1], st[2], st[3]
                for phase, cnt in (("x", R.Pc), ("y", R.Pr)):
                    if cnt == 1:
                        continue
                    ops, recv = [], []
                    for arr, peer, where in R.halo(l, name, DEPTH, phase):
                        ops.append(dist.P2POp(dist.isend, torch.from_numpy(arr), peer))
                        t = torch.empty(arr.shape, dtype=torch.float64)
                        ops.append(dist.P2POp(dist.irecv, t, peer))
                        recv.append((t, where))
                    for w in dist.batch_isend_irecv(ops):
                        w.wait()
                    for t, (rs, cs) in recv:
                        R.bufs[l][name][:, rs, cs] = t.numpy()
            elif st[0] == "gather":
                pl, ql = R.parts[Ld], R.cparts[Ld]
                c, cc = R.part.rows_per_rank(Ld), R.part.cols_per_rank(Ld)
                chunk = torch.from_numpy(R.bufs[Ld]["f"][:, pl.lo:pl.lo + c, ql.lo:ql.lo + cc].copy())
                parts = [torch.empty_like(chunk) for _ in range(world)]
                dist.all_gather(parts, chunk)
                fglob = np.zeros((B, (m >> Ld) + 1, (n >> Ld) + 1))
                for q, pt in enumerate(parts):
                    qi, qj = divmod(q, R.Pc)
                    fglob[:, 1 + qi * c:1 + (qi + 1) * c, 1 + qj * cc:1 + (qj + 1) * cc] = pt.numpy()
            elif st[0] == "coarse":
                eglob = R.coarse_solve(fglob)
            elif st[0] == "scatter":
                pl, ql = R.parts[Ld], R.cparts[Ld]
                R.bufs[Ld][st[1]] = eglob[:, pl.gr0:pl.gr0 + pl.Hloc, ql.gr0:ql.gr0 + ql.Hloc].copy()
            else:
                R.kernel(st)
        state = end
    p0, q0 = R.parts[0], R.cparts[0]
    np.save(os.path.join(outdir, f"rank{rank}.npy"), R.bufs[0][state][:, p0.lo:p0.hi, q0.lo:q0.hi])
    with open(os.path.join(outdir, f"rank{rank}.idx"), "w") as fh:
        fh.write(f"{p0.s} {p0.e} {q0.s} {q0.e}\n")
    dist.destroy_process_group()
