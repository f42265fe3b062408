"""Periodic weighted-Jacobi sweeps on a domain-decomposed grid (multi-GPU case).

The reference's periodic smoother `JacobiBlockPBC` (FEANet/jacobi.py:50-97) extends the iterate
circularly (`pbc_boundary`, :72-79), applies K, crops and adds `reset_boundary(u)` (:81-84):

    u'(a, b) = omd (f(a+1, b+1) - sum_d W[d] u((a+dy) mod n, (b+dx) mod n)) + u(a mod n, b mod n)

on the N x N nodes (period n = N - 1; f is the (N+2)^2 forcing term of its drivers).  On one GPU that is
`fea_jacobi_sweep_pbc`.  Here the n x n period is cut into a Pr x Pc grid of blocks, one per rank; the
circular extension becomes a PERIODIC halo exchange (the left neighbour of the first block column is
the last one, and so on, wrapping in both axes):

- each rank stores its owned block plus G ghost lines per side; one exchange refreshes all G of them
  and is followed by G sweeps without communication (every sweep leaves one ghost line less valid, the
  owned block stays exact) — communication-avoiding, as the decomposed V-cycle (`dd.py`);
- an exchange is an x phase (G owned columns to the left / right neighbours) then a y phase (G rows over
  the whole local width, ghost columns included), so the corner ghosts travel through the two phases;
  a rank that is its own neighbour along an axis (Pr or Pc = 1) copies locally, two ranks that are each
  other's left AND right neighbour (P = 2) match their two messages by posting order;
- the sweep itself is the generic HIP sweep `fea_jacobi_sweep` on the local (h + 2G) x (w + 2G) array
  with the reset mask set to one and zero boundary values, i.e. u' = omd (f - K u) + u at every local
  node — per node the same expression, in the same order, as `fea_jacobi_sweep_pbc` (values on the
  outermost ghost ring use zero padding and are never used), so the owned blocks are BITWISE the
  single-GPU periodic sweep's (tests/test_gpu_pbc_dd.py).

Host side only; the product path has no CPU fallback (the local sweep is the HIP kernel).  The CPU test
suite drives the same exchange logic over gloo with an oracle local sweep (tests/test_pbc_dd.py).
"""
import numpy as np
import torch


def _split(n, P, i):
    return i * n // P, (i + 1) * n // P


class PeriodicJacobiDD:
    """Rank `rank` of a Pr x Pc block decomposition (rank = ri * Pc + ci) of the n x n period of an
    N x N (N = n + 1) periodic problem, batch B.  comm: a PeriodicComm (torch.distributed) or None for
    a single rank.  ghost: G, sweeps per exchange.  ktab: the single 3 x 3 stencil; omd: omega / d."""

    def __init__(self, n, rank, grid, ktab, omd, comm=None, ghost=2, batch=1, dtype=torch.float64, device=None,
                 local_sweep=None):
        Pr, Pc = grid
        if rank < 0 or rank >= Pr * Pc:
            raise ValueError(f"PeriodicJacobiDD: rank {rank} outside a {Pr}x{Pc} grid")
        if n < max(Pr, Pc) * ghost:
            raise ValueError(f"PeriodicJacobiDD: blocks of a period {n} over {Pr}x{Pc} ranks are thinner than "
                             f"the {ghost} ghost lines")
        self.n, self.N, self.B, self.G = n, n + 1, batch, ghost
        self.Pr, self.Pc, self.rank = Pr, Pc, rank
        self.ri, self.ci = divmod(rank, Pc)
        self.r0, self.r1 = _split(n, Pr, self.ri)
        self.c0, self.c1 = _split(n, Pc, self.ci)
        self.h, self.w = self.r1 - self.r0, self.c1 - self.c0
        if min(self.h, self.w) < ghost:
            raise ValueError("PeriodicJacobiDD: a block is thinner than the ghost depth")
        self.comm = comm
        self.dtype = dtype
        self.device = torch.device("cuda" if device is None else device)
        self.H, self.W = self.h + 2 * ghost, self.w + 2 * ghost
        shape = (batch, 1, self.H, self.W)
        self.u = torch.zeros(shape, dtype=dtype, device=self.device)
        self.v = torch.zeros_like(self.u)
        self.f = torch.zeros_like(self.u)
        self.ktab = torch.as_tensor(np.asarray(ktab, np.float64).reshape(1, 9), dtype=dtype).to(self.device)
        self.omd = torch.as_tensor(np.asarray(omd, np.float64).reshape(1), dtype=dtype).to(self.device)
        self.ones = torch.ones((self.H, self.W), dtype=dtype, device=self.device)
        self._sweep = local_sweep or self._hip_sweep
        self._fresh = 0  # sweeps left before the next exchange

    # ------------------------------------------------------------------ data
    def _rows(self):  # global period rows / columns of the local array (ghosts wrap)
        return (np.arange(self.r0 - self.G, self.r1 + self.G) % self.n,
                np.arange(self.c0 - self.G, self.c1 + self.G) % self.n)

    def set_rhs(self, f_ext):
        """f_ext: the global (N+2)^2 forcing term [B, 1, N+2, N+2] (any device); this rank keeps f(a+1, b+1)
        of its local nodes (ghosts: their periodic images; only owned values reach owned results)."""
        rr, cc = self._rows()
        f = torch.as_tensor(f_ext)
        sub = f[..., torch.as_tensor(rr + 1)[:, None], torch.as_tensor(cc + 1)[None, :]]
        self.f.copy_(sub.reshape(self.B, 1, self.H, self.W))

    def load(self, u=None):
        """u: the global N x N iterate [B, 1, N, N] (its periodic part is used), or None for zero."""
        if u is None:
            self.u.zero_()
        else:
            rr, cc = self._rows()
            sub = torch.as_tensor(u)[..., torch.as_tensor(rr)[:, None], torch.as_tensor(cc)[None, :]]
            self.u.copy_(sub.reshape(self.B, 1, self.H, self.W))
        self._fresh = self.G  # the ghosts were loaded from the global field: valid to depth G

    def owned(self):
        g = self.G
        return self.u[..., g:g + self.h, g:g + self.w]

    # ------------------------------------------------------------------ sweeps
    def _hip_sweep(self, u, f, out):
        from . import _lib
        st = torch.cuda.current_stream(self.device).cuda_stream
        _lib.call("jacobi_sweep", self.dtype, u.data_ptr(), f.data_ptr(), out.data_ptr(), None, self.ktab.data_ptr(),
                  self.omd.data_ptr(), 1, self.ones.data_ptr(), 0, None, 0, self.B, self.H, self.W, st)

    def sweep(self, k=1):
        """k periodic Jacobi sweeps (JacobiBlockPBC.jacobi_convolution + reset, k times)."""
        for _ in range(k):
            if self._fresh == 0:
                self.exchange()
            self._sweep(self.u, self.f, self.v)
            self.u, self.v = self.v, self.u
            self._fresh -= 1

    def exchange(self):
        """Refresh the G ghost lines around the owned block from the periodic neighbours."""
        g, h, w = self.G, self.h, self.w
        u = self.u
        # x phase: owned rows, G columns each way
        rows = slice(g, g + h)
        self._phase(
            peer_lo=self.ri * self.Pc + (self.ci - 1) % self.Pc, peer_hi=self.ri * self.Pc + (self.ci + 1) % self.Pc,
            send_lo=u[..., rows, g:2 * g], send_hi=u[..., rows, w:w + g],
            recv_lo=u[..., rows, 0:g], recv_hi=u[..., rows, w + g:w + 2 * g])
        # y phase: G rows over the whole local width (the ghost columns just received ride along)
        self._phase(
            peer_lo=((self.ri - 1) % self.Pr) * self.Pc + self.ci, peer_hi=((self.ri + 1) % self.Pr) * self.Pc + self.ci,
            send_lo=u[..., g:2 * g, :], send_hi=u[..., h:h + g, :],
            recv_lo=u[..., 0:g, :], recv_hi=u[..., h + g:h + 2 * g, :])
        self._fresh = g

    def _phase(self, peer_lo, peer_hi, send_lo, send_hi, recv_lo, recv_hi):
        """send_lo goes to the lower neighbour, where it fills that rank's UPPER ghost (recv_hi); send_hi
        to the upper neighbour's lower ghost.  Messages are posted in the order (to lower, to upper) and
        received in the order (from upper, from lower), so a rank that is both neighbours (two ranks along
        the axis) matches them by order; a rank that is its own neighbour copies."""
        if peer_lo == self.rank and peer_hi == self.rank:
            recv_hi.copy_(send_lo)
            recv_lo.copy_(send_hi)
            return
        if self.comm is None:
            raise RuntimeError("PeriodicJacobiDD: more than one rank needs a communicator")
        self.comm.exchange([(send_lo, peer_lo), (send_hi, peer_hi)], [(recv_hi, peer_hi), (recv_lo, peer_lo)])

    # ------------------------------------------------------------------ results
    def gather(self):
        """The global N x N iterate [B, 1, N, N] on every rank (blocks all-gathered, periodic copies in the
        last row / column).  Equal to the single-GPU sweep's output whenever the forcing term is periodic —
        as the reference's drivers build it (FNet of the periodic extension); the sweeps themselves only
        ever read the periodic part of the iterate."""
        blocks = self.comm.allgather_blocks(self.owned().contiguous(), self.Pr * self.Pc) if self.comm else \
            [self.owned().contiguous()]
        out = torch.empty((self.B, 1, self.N, self.N), dtype=self.dtype, device=self.u.device)
        for q, blk in enumerate(blocks):
            qi, qj = divmod(q, self.Pc)
            a0, a1 = _split(self.n, self.Pr, qi)
            b0, b1 = _split(self.n, self.Pc, qj)
            out[..., a0:a1, b0:b1] = blk.to(out.device)
        out[..., self.n, :self.n] = out[..., 0, :self.n]
        out[..., :, self.n] = out[..., :, 0]
        return out


class PeriodicComm:
    """Point-to-point strips and block all-gather over torch.distributed.  nccl (RCCL): device buffers;
    gloo: host buffers.  Strips are packed into contiguous buffers (columns are strided)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.gpu = dist.get_backend(group) == "nccl"

    def _buf(self, t):
        return t.contiguous() if self.gpu else t.detach().cpu().contiguous()

    def exchange(self, sends, recvs):
        dist = self.dist
        sb = [self._buf(t) for t, _ in sends]
        rb = [torch.empty(t.shape, dtype=t.dtype, device=(t.device if self.gpu else "cpu")) for t, _ in recvs]
        ops = [dist.P2POp(dist.isend, b, p, self.group) for b, (_, p) in zip(sb, sends)]
        ops += [dist.P2POp(dist.irecv, b, p, self.group) for b, (_, p) in zip(rb, recvs)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for b, (t, _) in zip(rb, recvs):
            t.copy_(b)

    def allgather_blocks(self, blk, world):
        """Every rank's block (blocks may differ in shape by one line): padded to the largest, gathered."""
        dist = self.dist
        shp = torch.tensor(list(blk.shape[-2:]), dtype=torch.int64, device=(blk.device if self.gpu else "cpu"))
        shapes = [torch.empty_like(shp) for _ in range(world)]
        dist.all_gather(shapes, shp, group=self.group)
        hmax = max(int(s[0]) for s in shapes)
        wmax = max(int(s[1]) for s in shapes)
        pad = torch.zeros(blk.shape[:-2] + (hmax, wmax), dtype=blk.dtype, device=blk.device)
        pad[..., :blk.shape[-2], :blk.shape[-1]] = blk
        pad = self._buf(pad)
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=self.group)
        return [p[..., :int(s[0]), :int(s[1])] for p, s in zip(parts, shapes)]
