"""MultigridSolver: the MI355X V-cycle over solver-owned framed level buffers.

`MultigridSolver` is the facade named by BASELINE.json's north star; it executes the reference's
V-cycle (FEANet/multigrid.py MultiGrid.iterate :159-185 == M-FEANet-mg_test.ipynb MultiGrid.Step
:27346-27372 == MM_Model_convergence.ipynb rec_V_cycle :132-148 for nu1 = nu2 = 1) with the fused
HIP level kernels of framed_ops.hip:

  down, level 0 :  nu1 sweeps               (fea_mg_sweep)
                   residual + restriction    (fea_mg_residual_restrict)
  down, level l :  zero-guess sweep + residual + restriction in one pass
                   (fea_mg_residual_restrict with u = NULL)
  coarsest      :  nu1 + nu2 sweeps from zero (no exact solve, as the reference)
  up, level l   :  prolongation + correction + post-sweep in one pass (fea_mg_prolong_sweep)

The launch sequence of one V-cycle is built once (a list of C-ABI calls with fixed device
pointers) and replayed as a HIP graph.  Everything stays on the device; the only host syncs
are the ones a caller asks for (e.g. `.item()` on the residual norm, as the reference drivers do).
"""
import itertools
import math
import time
import weakref

import numpy as np
import torch

from . import _lib, mesh_setup as ms, ops
from .schedule import (OMDF, extend_tail, group_hmid, group_mid, hjac_schedule, pair_prolongations, pair_restrictions,
                       vcycle_schedule)


_SOLVERS = weakref.WeakValueDictionary()  # handle -> live MultigridSolver (torch.ops.feanet.mg_step)
_HANDLES = itertools.count(1)


def solver_by_handle(h):
    s = _SOLVERS.get(int(h))
    if s is None:
        raise RuntimeError(f"feanet: no live MultigridSolver with handle {h}")
    return s


class _Level:
    """Framed buffers of one level: H x W nodes (H = rows, W = columns)."""

    def __init__(self, m, n, B, dtype, device, pid_np=None, pid_shape=None):
        self.m, self.n = m, n
        self.H, self.W = m + 1, n + 1
        self.N = self.W
        esz = 4 if dtype == torch.float32 else 8
        self.ld, self.bs = _lib.mg_layout(self.H, self.W, esz)
        self.B = B
        self.dtype = dtype
        self.device = device
        numel = B * self.bs + 256
        self.f = torch.zeros(numel, dtype=dtype, device=device)
        self.a = torch.zeros(numel, dtype=dtype, device=device)
        self.b = torch.zeros(numel, dtype=dtype, device=device)
        self.zero = None
        self.c = None  # third iterate buffer of the finest level (solve(): the block's start state)
        self.pid = None
        if pid_np is not None:
            off = 128 // esz - 1
            p = np.zeros((self.H + 2, self.ld), np.uint8)
            p[1:self.H + 1, off:off + self.W] = pid_np
            self.pid = torch.from_numpy(p.reshape(-1)).to(device)
            self.pid = torch.cat([self.pid, torch.zeros(256, dtype=torch.uint8, device=device)])
        elif pid_shape is not None:  # (shape, size): built on the device straight into the frame
            off = 128 // esz - 1
            self.pid = torch.zeros((self.H + 2) * self.ld + 256, dtype=torch.uint8, device=device)
            ms.interface_pattern_map_device(self.N, pid_shape[0], pid_shape[1], device=device,
                                            out=self.pid.data_ptr() + self.ld + off, ld=self.ld)

    def buf(self, name):
        if name in ("zero", "c") and getattr(self, name) is None:
            setattr(self, name, torch.zeros_like(self.a))
        return getattr(self, name)

    def view(self, t):
        """[B, H, W] view of the interior+boundary nodes of a framed buffer (plumbing / tests)."""
        off = 128 // t.element_size() - 1
        return t[:self.B * self.bs].view(self.B, self.H + 2, self.ld)[:, 1:self.H + 1, off:off + self.W]

    def geom(self):
        return (self.B, self.H, self.W, self.ld, self.bs)


class MultigridSolver:
    """Geometric-multigrid V-cycle for FEANet's structured-quad FE problems on one MI355X.

    Args:
        n: fine-grid intervals per edge (N = n + 1 nodes), a power of two >= 2.
        rows: intervals in the row direction when the domain is a rectangle (Poisson, or the two-material
            problem with explicit pid_maps; default n, the reference's square).  n and rows must be divisible by 2^(L-1).
        levels: number of levels L (default int(log2 n), the reference's choice; coarsest n/2^(L-1);
            for a rectangle, the most levels whose coarsest grid has >= 2 intervals each way).
        problem: "poisson" (MeshSquare, one stencil) or "interface" (MeshCenterInterface, 16
            stencils; `prop` coefficients, `shape` 0 circle / 1 rectangle inclusion).
        dtype: torch.float32 or torch.float64.  batch: number of right-hand sides B.
        R, P: restriction / prolongation kernels, [C, 3, 3] with C = 1 or 16 (per-pattern, the
            learned 16-channel operators of FEANet/multigrid.py); default the bilinear kernel
            [[1,2,1],[2,4,2],[1,2,1]]/4 for both (mg_test; == MM's 4 x full-weighting/16).
        w: ratios (w_R, w_P) multiplying restriction/prolongation (FEANet/multigrid.py:170,178).
        nu1, nu2: pre/post sweeps per level; the coarsest level gets nu1 + nu2 sweeps.
        compat: None, or "mm_interface_q2" to reproduce MM_Interface_error.ipynb:141 (pre-smoothing
            applied to the finest grid at every depth).
        graph: replay the V-cycle as a HIP graph (default True).
        coarse_tail: run every level with N <= 65 (below the finest) as one LDS-resident launch
            (fea_mg_coarse_tail); False keeps one launch per level op.
        fuse: run the last pre-sweep of a level fused with its residual + restriction
            (fea_mg_sweep_restrict, one read of u and f); False issues them separately.
        zero_start: every V-cycle starts the finest level from a zero guess too (the replicated coarse
            sub-solve of the domain-decomposed path, feanet_amd.dd).
        smoother: "jac" (weighted Jacobi) or "hjac" (the learned smoother of M-FEANet-mg_test.ipynb,
            HJacIterator.HRelax: Jacobi + HNet correction; `hnet` = its [nl, 3, 3] conv weights, e.g.
            feanet_amd/weights/hnet_iso_poisson_33x33.npz).  "hjac" runs fea_mg_hsweep for every
            relaxation (MultiGrid(mode='hjac').Step semantics); with coarse_tail its levels of <= 65^2 nodes
            that fit in LDS run as one fea_mg_hjac_tail launch.
        join_cycles: vcycle(k) with k >= 2 runs the finest level's post-smooth of each cycle and the
            pre-smooth + residual + restriction of the next as one pass (fea_mg_cycle_join; bitwise
            the same result, 28 instead of 52 B per node between two cycles).  V(1,1) Jacobi only.
        mid: run latency-bound coarse levels (B*H*W <= MID_NODES) up to four per launch
            (fea_mg_mid_down / fea_mg_mid_up, bitwise the per-level kernels); with smoother="hjac", two per
            launch (fea_mg_hmid_down / fea_mg_hmid_up, bitwise the fused per-level HJac kernels).
        pair_levels: two consecutive zero-guess restrictions, and two recomputed-iterate prolongations, left
            to single-level launches run as one each (fea_mg_zero_restrict2 / fea_mg_prolong2, bitwise the two).
        pid_maps: two-material problem only — explicit per-level pattern maps ([H_l, W_l] uint8, one per level)
            instead of the MeshCenterInterface maps of the square: a domain-decomposed rank's window of the
            global level maps (feanet_amd.dd.DDSolver(problem="interface")); allows a rectangular window.
    """

    MID_NODES = 20000     # levels with <= this many nodes (B*H*W) may go to the LDS-tile multi-level launches (groups
    #                       of >= 2 consecutive levels above the coarse tail).  Round 6: 20000 (<= 129^2, which forms no
    #                       group above the 65^2 tail, so the standard plans run the streaming two-level kernels on
    #                       every level above it) — metric V-cycle 132.6 -> 128.8 us, C2 35.9 -> 33.6, C4 grid 528 ->
    #                       519, C3 92.0 -> 90.0, C5 level, DD 8-rank projection 108.9 -> 104.6 against 300000 (<= 513^2,
    #                       rounds 2-5), once this round's task heights had sped the two-level kernels up
    #                       (profiles/r06_ab/mid_nodes.txt).  Larger values still select the multi-level launches (bitwise).
    MID_NODES_DOWN = None  # per-direction overrides of MID_NODES (None: MID_NODES)
    MID_NODES_UP = None
    MID_MIN_TILES = 200   # workgroups a multi-level launch should give the 256 CUs
    MID_MAX_REDUNDANCY = 3.0  # staged top-level region / owned nodes (down pass)
    HMID_NODES = 300000   # learned-smoother levels paired into the HJac two-level launches: <= 513^2 nodes
    HMID_MIN_TILES = 64   # workgroups an HJac two-level launch should give the CUs (one per CU: LDS)
    TAIL_MAX_N = 65       # the coarse tail (one LDS-resident launch) covers the levels of at most this many rows / columns
    TAIL_EXT = True       # the single-level restriction / prolongation right above the coarse tail run inside the
    TAIL_EXT_MIN_BATCH = 64  # tail's launch (fea_mg_coarse_tail_ext: single pattern, V(1,1)) for batches of at least
    #                       this many samples: one workgroup per sample moves the level's traffic through one CU, which
    #                       only pays when the samples fill the chip (C5, 256 x 1025^2 fp32: 1142 -> 1125 us; at B = 1
    #                       the metric cycle 130.1 -> 134.1 us, C2 33.8 -> 37.6; profiles/r06_ab/tail_ext.txt)

    def __init__(self, n, levels=None, problem="poisson", dtype=torch.float64, device=None, batch=1,
                 omega=2.0 / 3.0, size=2.0, prop=(1, 20), shape=0, R=None, P=None, w=(1.0, 1.0),
                 nu1=1, nu2=1, compat=None, graph=True, coarse_tail=True, fuse=True, rows=None, zero_start=False,
                 smoother="jac", hnet=None, join_cycles=True, mid=True, pair_levels=True, pid_maps=None):
        m = n if rows is None else int(rows)
        if rows is None and (n < 2 or (n & (n - 1)) != 0):
            raise ValueError(f"MultigridSolver: n={n} must be a power of two >= 2")
        if m < 2 or n < 2:
            raise ValueError(f"MultigridSolver: need >= 2 intervals each way (got {m} x {n})")
        if dtype not in (torch.float32, torch.float64):
            raise TypeError("MultigridSolver: dtype must be torch.float32 or torch.float64")
        self.device = torch.device(device if device is not None else "cuda")
        ops.require_hip(torch.empty(0, device=self.device), "solver device")
        self.n, self.m = n, m
        if levels is None:
            L = 1
            while (n % (1 << L) == 0 and m % (1 << L) == 0 and (n >> L) >= 2 and (m >> L) >= 2):
                L += 1
            self.L = L if rows is not None else int(math.log2(n))
        else:
            self.L = int(levels)
        s_ = 1 << (self.L - 1)
        if self.L < 1 or n % s_ or m % s_ or n // s_ < 2 or m // s_ < 2:
            raise ValueError(f"MultigridSolver: {self.L} levels do not fit a {m} x {n} grid")
        self.dtype = dtype
        self.B = int(batch)
        self.omega = omega
        self.size = size
        self.problem = problem
        self.nu1, self.nu2 = int(nu1), int(nu2)
        self.compat = compat
        self.use_graph = graph
        self.fuse = fuse
        self.zero_start = zero_start
        self.join_cycles = join_cycles
        self.mid = bool(mid)
        self.pair_levels = bool(pair_levels)
        if smoother not in ("jac", "hjac"):
            raise ValueError(f"MultigridSolver: unknown smoother {smoother!r}")
        self.smoother = smoother
        if smoother == "hjac":
            if hnet is None:
                raise ValueError("MultigridSolver: smoother='hjac' needs the HNet weights (hnet=[nl, 3, 3])")
            if compat is not None:
                raise ValueError("MultigridSolver: smoother='hjac' follows MultiGrid(mode='hjac').Step only")
            hw = np.asarray(torch.as_tensor(hnet).detach().cpu().float().numpy(), np.float32).reshape(-1, 3, 3)
            if not 1 <= hw.shape[0] <= 3:
                raise ValueError("MultigridSolver: HNet with 1..3 conv layers supported")
        hjac_tail = coarse_tail and smoother == "hjac"
        if smoother == "hjac":
            coarse_tail = False
        npdt = np.float32 if dtype == torch.float32 else np.float64
        multi = problem == "interface"
        if problem not in ("poisson", "interface"):
            raise ValueError(f"MultigridSolver: unknown problem {problem!r}")
        if multi and m != n and pid_maps is None:
            raise ValueError("MultigridSolver: the two-material problem is defined on the square only")
        if pid_maps is not None:  # explicit per-level maps (a domain-decomposed rank's window of the global maps)
            if not multi:
                raise ValueError("MultigridSolver: pid_maps is for the two-material problem")
            pid_maps = [np.ascontiguousarray(p, np.uint8) for p in pid_maps]
        ktab = ms.stencil_table(prop if multi else None)
        self.ntab = ktab.shape[0]
        lin = ms.linear_transfer_kernel() / np.float32(4.0)
        R = lin[None] if R is None else np.asarray(torch.as_tensor(R).detach().cpu().float().numpy(), np.float32)
        P = lin[None] if P is None else np.asarray(torch.as_tensor(P).detach().cpu().float().numpy(), np.float32)
        R = R.reshape(-1, 3, 3)
        P = P.reshape(-1, 3, 3)
        if multi:  # per-pattern tables cover every pattern id
            R = np.broadcast_to(R, (self.ntab, 3, 3)) if R.shape[0] == 1 else R
            P = np.broadcast_to(P, (self.ntab, 3, 3)) if P.shape[0] == 1 else P
        elif R.shape[0] != 1 or P.shape[0] != 1:
            raise ValueError("MultigridSolver: the Poisson problem has one pattern; R/P must be [1, 3, 3]")
        w = [float(x) for x in (w.detach().cpu().tolist() if torch.is_tensor(w) else w)]
        self.w = (w[0], w[1])
        dev = self.device
        self.ktab_np = ktab
        self.hw = None
        self.nl = 0
        if smoother == "hjac":
            self.hw = torch.from_numpy(hw.reshape(-1).astype(npdt)).to(dev)
            self.nl = hw.shape[0]
        self.ktab = torch.from_numpy(ktab.reshape(-1, 9).astype(npdt)).to(dev)
        self.omd = torch.from_numpy(ms.omega_over_d(ktab, omega, npdt)).to(dev)
        self.rtab = torch.from_numpy(np.ascontiguousarray(R).reshape(-1, 9).astype(npdt)).to(dev)
        self.ptab = torch.from_numpy(np.ascontiguousarray(P).reshape(-1, 9).astype(npdt)).to(dev)
        self.levels = []
        for l in range(self.L):
            nl, ml = n >> l, m >> l
            if pid_maps is not None:
                if pid_maps[l].shape != (ml + 1, nl + 1):
                    raise ValueError(f"MultigridSolver: pid_maps[{l}] is {pid_maps[l].shape}, level {l} is "
                                     f"{(ml + 1, nl + 1)}")
                self.levels.append(_Level(ml, nl, self.B, dtype, dev, pid_np=pid_maps[l]))
                continue
            # two-material pattern maps: built on the device (setup_ops.hip), bit-identical to the host
            self.levels.append(_Level(ml, nl, self.B, dtype, dev, pid_shape=(shape, size) if multi else None))
        if pid_maps is not None:
            self.fine_pid = torch.from_numpy(pid_maps[0]).to(dev)
        else:
            self.fine_pid = ms.interface_pattern_map_device(n + 1, shape, size, device=dev) if multi else None
        if multi:  # the framed kernels read each node's stiffness row from its own pattern (K symmetric; checked)
            for Lv in self.levels:
                off = 128 // (4 if dtype == torch.float32 else 8) - 1
                pv = Lv.pid[:(Lv.H + 2) * Lv.ld].view(Lv.H + 2, Lv.ld)[1:Lv.H + 1, off:off + Lv.W]
                if ms.stencil_mirror_mismatches(ktab, pv):
                    raise ValueError("MultigridSolver: the stiffness table is not symmetric on this pattern map "
                                     "(the framed two-material kernels need K_ij == K_ji bit for bit)")
        self.tail_from = None
        if coarse_tail:
            esz = 4 if dtype == torch.float32 else 8
            for l in range(1, self.L):
                Lv = self.levels[l]
                if (Lv.H <= self.TAIL_MAX_N and Lv.W <= self.TAIL_MAX_N
                        and 0 < _lib.coarse_tail_lds_bytes(Lv.H, Lv.W, self.L - l, esz, multi) <= _lib.TAIL_LDS_LIMIT):
                    self.tail_from = l
                    break
        # learned smoother: the levels of <= 65^2 nodes whose f, u and two scratch fields fit in LDS
        self.hjac_tail_from = None
        if hjac_tail:
            esz = 4 if dtype == torch.float32 else 8
            for l in range(1, self.L):
                Lv = self.levels[l]
                if (Lv.H <= 65 and Lv.W <= 65
                        and 0 < _lib.hjac_tail_lds_bytes(Lv.H, Lv.W, self.L - l, esz, multi) <= _lib.TAIL_LDS_LIMIT):
                    self.hjac_tail_from = l
                    break
        t_from = self.tail_from if self.tail_from is not None else self.hjac_tail_from
        if t_from is not None and multi:
            maps = [pid_maps[l].reshape(-1) if pid_maps is not None else
                    ms.interface_pattern_map(self.levels[l].N, shape, size).reshape(-1) for l in range(t_from, self.L)]
            self.tail_pid = torch.from_numpy(np.concatenate(maps)).to(dev)
        else:
            self.tail_pid = None
        self.ws = torch.zeros(max(1, _lib.norm_workspace_bytes(self.B, m + 1, n + 1) // 8), dtype=torch.float64,
                              device=dev)
        self.norm_out = torch.zeros(self.B, dtype=torch.float64, device=dev)
        self._state = "a"
        # joinable solvers rest BETWEEN cycles in a pipelined ("mid-cycle") state after vcycle(k): see
        # _vcycles_pipelined; None = the iterate is materialised in buffer self._state
        self._mid = None
        self._hist = None  # solve(): fused residual-norm history + counters (_ensure_hist)
        self._cnt = None
        self._hist_gen = 0
        self._f1_snap = None
        self._sws = None  # solve(): per-cycle partial norm sets of a graph block
        self._bc_version = object()  # identity changes with every set_boundary (third-buffer packing)
        self._c_bc = None
        # Dirichlet data the finest iterate buffers a/b carry: set_boundary takes effect at the next load(),
        # and the third buffer c (a materialised end iterate) is packed with the same data as a/b
        self._ab_bc, self._ab_version = None, self._bc_version
        self._plans = {}
        self._graphs = {}
        self._eager_runs = {}
        self.mass = ms.mass_stencil(size / n)
        self.handle = next(_HANDLES)  # torch.ops.feanet.mg_step(u, f, handle, cycles)
        _SOLVERS[self.handle] = self

    # ------------------------------------------------------------------ problem data
    @property
    def N(self):
        return self.n + 1

    @property
    def H(self):
        return self.m + 1

    @property
    def W(self):
        return self.n + 1

    def _check_field(self, x, name):
        ops.require_hip(x, name)
        x = x.to(self.dtype)
        H, W = self.H, self.W
        if x.numel() == H * W:
            x = x.reshape(1, 1, H, W).expand(self.B, 1, H, W)
        if tuple(x.shape[-2:]) != (H, W) or x.numel() != self.B * H * W:
            raise ValueError(f"MultigridSolver: {name} must be [{self.B}, 1, {H}, {W}]")
        return x.reshape(self.B, 1, H, W).contiguous()

    def set_rhs(self, f=None, F=None):
        """Set the assembled right-hand side f (= FNet(F), the `forcing_term` of the reference) or
        the nodal source F (FNet applied on the device, FEANet/model.py:49-61)."""
        if (f is None) == (F is None):
            raise ValueError("MultigridSolver.set_rhs: give exactly one of f (assembled) or F (source)")
        if F is not None:
            F = self._check_field(F, "F")
            f = ops.conv3x3(F, torch.from_numpy(self.mass))
        f = self._check_field(f, "f")
        L0 = self.levels[0]
        self._collapse()  # a pipelined next pre-smooth was made with the old right-hand side
        self._pack(f, L0.f, geo=None, bc=None, reset=False)

    def set_boundary(self, bc_value=None, geometry_idx=None):
        """Dirichlet data of the fine level (the `boundary_value` / `geometry_idx` of JacobiBlock).
        The framed kernels implement the square geometry (geo.py:13-30); other geometries go through
        FEANet.jacobi.JacobiBlock's generic operator."""
        if geometry_idx is not None:
            g = self._check_field(geometry_idx, "geometry_idx")
            sq = torch.ones_like(g)
            sq[..., 0, :] = 0
            sq[..., -1, :] = 0
            sq[..., :, 0] = 0
            sq[..., :, -1] = 0
            if not torch.equal(g, sq):
                raise NotImplementedError("MultigridSolver: only the square geometry (geo.py:13-30) is fused")
        self._bc = None if bc_value is None else self._check_field(bc_value, "boundary_value")
        self._bc_version = object()

    def _pack(self, x, dst, geo=None, bc=None, reset=True):
        """x (None: zeros) -> framed dst; reset: x*geo + bc (square geometry), else a raw copy."""
        Lv = self.levels[0]
        bp, bs = (None, 0)
        if bc is not None:
            bp, bs = bc.data_ptr(), self.H * self.W
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.call("mg_pack", self.dtype, None if x is None else x.data_ptr(), dst.data_ptr(), None,
                  0 if reset else -1, bp, bs, *Lv.geom(), stream)

    def load(self, u0=None):
        """Set the fine-grid iterate (reset_boundary applied: u*geo + bc, jacobi.py:27-29)."""
        L0 = self.levels[0]
        bc = getattr(self, "_bc", None)
        if u0 is not None:
            u0 = self._check_field(u0, "u0")
        self._pack(u0, L0.a, bc=bc)
        self._pack(u0, L0.b, bc=bc)  # both ping-pong buffers carry the boundary values
        self._mid = None
        self._ab_bc, self._ab_version = bc, self._bc_version
        if L0.c is not None and self._c_bc is not self._ab_version:
            self._pack(u0, L0.c, bc=bc)  # c only needs the Dirichlet values on its boundary nodes
            self._c_bc = self._ab_version
        self._state = "a"
        if self.smoother == "hjac":
            # HRelax forms J(u) - u with the iterate the driver passed, before reset_boundary
            # (M-FEANet-mg_test.ipynb:151-153; the drivers pass un-reset zeros, :27478-27489): the
            # first sweep of the next V-cycle sees bc - u0 on the boundary nodes
            self._raw = torch.zeros_like(L0.a)
            self._pack(u0, self._raw, reset=False)  # u0 None: zeros
            self._hjac_first = True

    def solution(self):
        """Current fine iterate as a contiguous [B, 1, H, W] tensor."""
        L0 = self.levels[0]
        out = torch.empty((self.B, 1, self.H, self.W), dtype=self.dtype, device=self.device)
        _lib.call("mg_unpack", self.dtype, L0.buf(self._iterate()).data_ptr(), out.data_ptr(), *L0.geom(),
                  ops._stream(out))
        return out

    def residual_norm(self):
        """Per-sample ||(f - K u)[1:-1, 1:-1]||_2 of the current iterate (float64 device tensor [B])."""
        L0 = self.levels[0]
        _lib.call("mg_residual_norm", self.dtype, L0.buf(self._iterate()).data_ptr(), L0.f.data_ptr(),
                  None if L0.pid is None else L0.pid.data_ptr(), self.ktab.data_ptr(), self.ntab,
                  self.norm_out.data_ptr(), self.ws.data_ptr(), *L0.geom(), 0, 0, 0, 0,
                  torch.cuda.current_stream(self.device).cuda_stream)
        return self.norm_out.clone()

    def set_transfer(self, R=None, P=None, w=None):
        """Replace the restriction / prolongation kernels (and the ratios w) of a built solver, for training
        loops that update them between V-cycles (FEANet/multigrid.py:132-157 under an optimizer).

        R / P ([npat or 1, 3, 3], any device) are rounded to float32 like the constructor's and copied into the
        resident tables IN PLACE on the current stream: the launch plans and captured HIP graphs hold the tables'
        addresses, so they stay valid and nothing is reallocated or recaptured.  The ratios are passed by value
        into the launches, so new ratios (w != the current ones) drop the plans and graphs instead; the level
        buffers are kept either way.

        A solver resting in the pipelined state (after vcycle) has not stored its last cycle's end iterate: it
        is recomputed from the pre-smoothed iterate and the level-1 correction with the CURRENT P (_collapse).
        So that state is collapsed first, with the old tables, before any of them changes."""
        if R is not None or P is not None or w is not None:
            self._collapse()
        for src, dst, name in ((R, self.rtab, "R"), (P, self.ptab, "P")):
            if src is None:
                continue
            t = torch.as_tensor(src).detach().to(device=self.device, dtype=torch.float32).reshape(-1, 9)
            if t.shape[0] not in (1, dst.shape[0]):
                raise ValueError(f"MultigridSolver.set_transfer: {name} has {t.shape[0]} patterns, the solver "
                                 f"{dst.shape[0]}")
            dst.copy_(t.to(self.dtype).expand(dst.shape[0], 9))
        if w is not None:
            w = [float(x) for x in (w.detach().cpu().tolist() if torch.is_tensor(w) else w)]
            if (w[0], w[1]) != self.w:
                self.w = (w[0], w[1])
                self._plans.clear()
                self._graphs.clear()
                self._eager_runs.clear()

    # ------------------------------------------------------------------ schedule
    def _ptr(self, lvl, name):
        if name == OMDF:  # recomputed in the kernel (u = NULL)
            return None
        return self.levels[lvl].buf(name).data_ptr()

    def _build(self, start):
        """Bind the symbolic schedule (feanet_amd.schedule) to C-ABI calls with device pointers:
        list of (name, args-without-stream) for one V-cycle from buffer `start`, and the end buffer."""
        if self.smoother == "hjac":
            steps, end = hjac_schedule(self.L, self.nu1, self.nu2, "zero" if self.zero_start else start,
                                       tail_from=self.hjac_tail_from, fuse=self.fuse)
            if self.mid and self.fuse:
                steps = group_hmid(steps, self._pick_hmid())
        else:
            steps, end = vcycle_schedule(self.L, self.nu1, self.nu2, self.compat, start, self.tail_from, self.fuse,
                                         top_zero=self.zero_start)
            if self.mid:
                steps = group_mid(steps, lambda lv: self._pick_mid(lv, False), lambda lv: self._pick_mid(lv, True))
            if self.pair_levels:
                ok = lambda l: l + 2 < self.L and self.levels[l + 2].H >= 3 and self.levels[l + 2].W >= 3
                steps = pair_prolongations(pair_restrictions(steps, ok), ok)
            if self._tail_ext_ok():
                steps = extend_tail(steps)
        return [self.bind_step(st) for st in steps], end

    def _tail_ext_ok(self):
        """fea_mg_coarse_tail_ext's scope: the single-pattern V(1,1) tail, the level above it at most 129 wide."""
        t = self.tail_from
        return (self.TAIL_EXT and t is not None and self.B >= self.TAIL_EXT_MIN_BATCH and self.ntab == 1
                and self.nu1 == 1 and self.nu2 == 1 and self.compat is None and self.levels[t - 1].W <= 129 and self.levels[t - 1].H <= 129)

    def _mid_tile(self, up, a, k):
        """Tile size for a multi-level launch over levels a..a+k-1 (down: tile of level a+k; up: of
        level a), or None: the largest power of two whose LDS footprint fits, that gives the chip
        >= MID_MIN_TILES workgroups (or the most it can) and, going down, stages <= MID_MAX_REDUNDANCY
        times the top level's nodes."""
        esz = 4 if self.dtype == torch.float32 else 8
        multi = self.ntab > 1
        tl = self.levels[a if up else a + k]
        top = self.levels[a]
        best = None
        for T in ((128, 64, 32, 16, 8) if up else (32, 16, 8, 4, 2)):
            if _lib.mid_lds_bytes(up, k, T, T, esz, multi) <= 0:
                continue
            tiles = self.B * -(-(tl.H - 2) // T) * -(-(tl.W - 2) // T)
            if not up:
                reg = (T << k) + 3 * ((1 << k) - 1)
                if reg * reg * tiles > self.MID_MAX_REDUNDANCY * self.B * top.H * top.W:
                    continue
            best = T
            if tiles >= self.MID_MIN_TILES:
                return T
        return best

    def _hmid_tile(self, up, a):
        """Tile size of an HJac two-level launch over levels a, a+1 (down: tile of level a+2; up: of level a):
        the largest whose LDS footprint fits and that gives >= HMID_MIN_TILES workgroups, else the smallest that
        fits (None: none does)."""
        esz = 4 if self.dtype == torch.float32 else 8
        tl = self.levels[a if up else a + 2]
        fit = [T for T in ((64, 32, 16, 8) if up else (16, 8, 4, 2))
               if _lib.hmid_lds_bytes(up, T, self.nl, esz, self.ntab > 1) > 0]
        for T in fit:
            if self.B * -(-(tl.H - 2) // T) * -(-(tl.W - 2) // T) >= self.HMID_MIN_TILES:
                return T
        return fit[-1] if fit else None

    def _pick_hmid(self):
        """(a, T_down, T_up) for the HJac levels paired into two-level launches: streamed coarse levels (a >= 1,
        above the HJac tail) of <= HMID_NODES nodes, paired from the coarse end upward."""
        top = self.hjac_tail_from if self.hjac_tail_from is not None else self.L - 1
        el = [l for l in range(1, top) if self.B * self.levels[l].H * self.levels[l].W <= self.HMID_NODES]
        pairs = []
        hi = len(el)
        while hi >= 2:
            a = el[hi - 2]
            if el[hi - 1] == a + 1 and a + 2 < self.L:
                td, tu = self._hmid_tile(False, a), self._hmid_tile(True, a)
                if td and tu:
                    pairs.append((a, td, tu))
                    hi -= 2
                    continue
            hi -= 1
        return pairs

    def _pick_mid(self, levels, up):
        """Groups (a, k, T) of consecutive latency-bound levels, formed from the coarse end upward."""
        cap = self.MID_NODES_UP if up else self.MID_NODES_DOWN
        cap = self.MID_NODES if cap is None else cap
        el = sorted(l for l in levels
                    if self.B * self.levels[l].H * self.levels[l].W <= cap and l + 1 < self.L)
        groups = []
        hi = len(el)
        while hi >= 2:
            for k in range(min(4, hi), 1, -1):
                a = el[hi - k]
                if el[hi - 1] - a != k - 1:
                    continue
                T = self._mid_tile(up, a, k)
                if T:
                    groups.append((a, k, T))
                    hi -= k
                    break
            else:
                hi -= 1
        return groups

    def bind_step(self, st):
        """One schedule step -> (C-ABI function base name, args without the stream)."""
        lv = self.levels
        kt, om, nt = self.ktab.data_ptr(), self.omd.data_ptr(), self.ntab
        rt, pt = self.rtab.data_ptr(), self.ptab.data_ptr()
        nr, npt = self.rtab.shape[0], self.ptab.shape[0]

        def pid(l):
            return None if lv[l].pid is None else lv[l].pid.data_ptr()

        def ptr(l, name):
            return None if name is None else self._ptr(l, name)

        def geom(l):
            return lv[l].geom()

        def cgeom(l):
            return (lv[l + 1].ld, lv[l + 1].bs)

        kind, l = st[0], st[1]
        f = lv[l].f.data_ptr()
        if kind == "sweep":
            return ("mg_sweep", (ptr(l, st[2]), f, ptr(l, st[3]), pid(l), kt, om, nt) + geom(l))
        if kind == "hsweep":
            return ("mg_hsweep", (ptr(l, st[2]), None, f, ptr(l, st[3]), pid(l), kt, om, nt, self.hw.data_ptr(),
                                  self.nl) + geom(l))
        if kind == "resid_restrict":
            return ("mg_residual_restrict", (ptr(l, st[2]), f, ptr(l, st[3]), lv[l + 1].f.data_ptr(), pid(l),
                                             kt, om, nt, rt, nr, self.w[0]) + geom(l) + cgeom(l))
        if kind == "resid_restrict2":
            return ("mg_zero_restrict2", (f, lv[l + 1].f.data_ptr(), lv[l + 2].f.data_ptr(), pid(l), pid(l + 1),
                                          kt, om, nt, rt, nr, self.w[0]) + geom(l) + cgeom(l) + cgeom(l + 1))
        if kind == "sweep_restrict":
            return ("mg_sweep_restrict", (ptr(l, st[2]), f, ptr(l, st[3]), lv[l + 1].f.data_ptr(), pid(l),
                                          kt, om, nt, rt, nr, self.w[0]) + geom(l) + cgeom(l) + (None, None, None))
        if kind == "prolong_sweep":
            return ("mg_prolong_sweep", (ptr(l, st[2]), ptr(l + 1, st[3]), f, ptr(l, st[4]), pid(l),
                                         pid(l + 1), kt, om, nt, pt, npt, self.w[1]) + geom(l) + cgeom(l))
        if kind == "prolong_sweep2":
            return ("mg_prolong2", (lv[l + 1].f.data_ptr(), ptr(l + 2, st[2]), f, ptr(l, st[3]), pid(l), pid(l + 1),
                                    pid(l + 2), kt, om, nt, pt, npt, self.w[1]) + geom(l) + cgeom(l) + cgeom(l + 1))
        if kind == "prolong_add":
            return ("mg_prolong_add", (ptr(l, st[2]), ptr(l + 1, st[3]), ptr(l, st[4]), pid(l + 1), pt, npt,
                                       self.w[1]) + geom(l) + cgeom(l))
        if kind == "mid_down":
            a, k, T = st[1], st[2], st[3]
            fs = _lib.PtrArray([lv[j].f.data_ptr() for j in range(a, a + k + 1)])
            pids = _lib.PtrArray([pid(j) for j in range(a, a + k + 1)]) if nt > 1 else None
            TR, TC = T if isinstance(T, tuple) else (T, T)
            return ("mg_mid_down", (fs, pids, k, self.B, lv[a].H, lv[a].W, kt, om, nt, rt, nr, self.w[0], TR, TC))
        if kind == "mid_up":
            a, k, csrc, dst, T = st[1:6]
            fs = _lib.PtrArray([lv[j].f.data_ptr() for j in range(a, a + k)])
            pids = _lib.PtrArray([pid(j) for j in range(a, a + k + 1)]) if nt > 1 else None
            TR, TC = T if isinstance(T, tuple) else (T, T)
            return ("mg_mid_up", (fs, ptr(a + k, csrc), ptr(a, dst), pids, k, self.B, lv[a].H, lv[a].W, kt, om, nt,
                                  pt, npt, self.w[1], TR, TC))
        if kind == "coarse_tail":
            t = l
            return ("mg_coarse_tail", (lv[t].f.data_ptr(), ptr(t, st[2]), lv[t].H, lv[t].W, self.L - t, lv[t].ld,
                                       lv[t].bs, None if self.tail_pid is None else self.tail_pid.data_ptr(),
                                       kt, om, nt, rt, pt, self.w[0], self.w[1], self.nu1, self.nu2,
                                       int(self.compat == "mm_interface_q2"), lv[t].B))
        if kind == "coarse_tail_ext":
            x, t = l, l + 1
            return ("mg_coarse_tail_ext", (f, ptr(x, st[2]), lv[x].H, lv[x].W, lv[x].ld, lv[x].bs, self.L - t, kt, om,
                                           nt, rt, pt, self.w[0], self.w[1], lv[x].B))
        if kind == "hsweep_restrict":
            return ("mg_hsweep_restrict", (ptr(l, st[2]), None, f, ptr(l, st[3]), lv[l + 1].f.data_ptr(), pid(l), kt,
                                           om, nt, self.hw.data_ptr(), self.nl, rt, nr, self.w[0]) + geom(l) +
                    cgeom(l))
        if kind == "prolong_hsweep":
            return ("mg_prolong_hsweep", (ptr(l, st[2]), None, ptr(l + 1, st[3]), f, ptr(l, st[4]), pid(l), pid(l + 1), kt,
                                          om, nt, self.hw.data_ptr(), self.nl, pt, npt, self.w[1]) + geom(l) +
                    cgeom(l))
        if kind == "hmid_down":
            a, da, da1, T = st[1:5]
            fs = _lib.PtrArray([lv[j].f.data_ptr() for j in range(a, a + 3)])
            us = _lib.PtrArray([ptr(a, da), ptr(a + 1, da1)])
            pids = _lib.PtrArray([pid(j) for j in range(a, a + 3)]) if nt > 1 else None
            return ("mg_hmid_down", (fs, us, pids, self.B, lv[a].H, lv[a].W, kt, om, nt, self.hw.data_ptr(), self.nl,
                                     rt, nr, self.w[0], T))
        if kind == "hmid_up":
            a, u0, u1, esrc, dst, T = st[1:7]
            fs = _lib.PtrArray([lv[a].f.data_ptr(), lv[a + 1].f.data_ptr()])
            us = _lib.PtrArray([ptr(a, u0), ptr(a + 1, u1)])
            pids = _lib.PtrArray([pid(j) for j in range(a, a + 3)]) if nt > 1 else None
            return ("mg_hmid_up", (fs, us, ptr(a + 2, esrc), ptr(a, dst), pids, self.B, lv[a].H, lv[a].W, kt, om, nt,
                                   self.hw.data_ptr(), self.nl, pt, npt, self.w[1], T))
        if kind == "hjac_tail":
            t = l
            return ("mg_hjac_tail", (lv[t].f.data_ptr(), ptr(t, st[2]), lv[t].H, lv[t].W, self.L - t, lv[t].ld,
                                     lv[t].bs, None if self.tail_pid is None else self.tail_pid.data_ptr(),
                                     kt, om, nt, rt, pt, self.hw.data_ptr(), self.nl, self.w[0], self.w[1],
                                     self.nu1, self.nu2, lv[t].B))
        raise ValueError(f"MultigridSolver: unknown schedule step {kind!r}")

    def _plan(self, start):
        if start not in self._plans:
            self._plans[start] = self._build(start)
        return self._plans[start]

    def _launch(self, plan):
        stream = torch.cuda.current_stream(self.device).cuda_stream
        for name, args in plan:
            if name == "norm_append":  # dtype-free entry point
                _lib.call_raw(name, *args, stream)
            else:
                _lib.call(name, self.dtype, *args, stream)

    def _joinable(self):
        return (self.join_cycles and self.smoother == "jac" and self.nu1 == 1 and self.nu2 == 1 and
                self.compat is None and not self.zero_start and self.fuse and self.L >= 2)

    def _join_call(self, pre, ec_ptr, norm=False, out=None, norm_ws=None):
        """fea_mg_cycle_join: PS(0) of the cycle whose pre-smoothed iterate is in `pre`, fused with the
        next cycle's SR(0); the new pre-smoothed iterate lands in the other buffer.  norm: also append the
        residual norm of the cycle's end iterate to the solve history (solve())."""
        lv = self.levels
        L0, L1 = lv[0], lv[1]
        pid = None if L0.pid is None else L0.pid.data_ptr()
        pidc = None if L1.pid is None else L1.pid.data_ptr()
        out = out or ("b" if pre == "a" else "a")
        return ("mg_cycle_join", (self._ptr(0, pre), ec_ptr, L0.f.data_ptr(), self._ptr(0, out),
                                  L1.f.data_ptr(), pid, pidc, self.ktab.data_ptr(), self.omd.data_ptr(), self.ntab,
                                  self.ptab.data_ptr(), self.ptab.shape[0], self.rtab.data_ptr(),
                                  self.rtab.shape[0], self.w[1], self.w[0]) + L0.geom() + (L1.ld, L1.bs) +
                ((norm_ws, None, None) if norm_ws is not None else
                 (self.ws.data_ptr(), self._hist.data_ptr(), self._cnt.data_ptr()) if norm else (None, None, None)))

    def _run_segment(self, key, launches):
        """Launch a fixed list of calls: eager the first time, then as a captured HIP graph."""
        if not self.use_graph or self._eager_runs.get(key, 0) == 0:
            self._eager_runs[key] = self._eager_runs.get(key, 0) + 1
            self._launch(launches)
            return
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.graph(g, stream=s):
                self._launch(launches)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._graphs[key] = g
        g.replay()

    def joined_program(self, k):
        """vcycle(k) with joined cycle boundaries as [(segment key, launches)] plus the end buffer:
        the first cycle's SR(0), k-1 segments (coarse part + cycle join) and the last coarse part +
        PS(0).  (Also used by bench.py to time the join kernel inside the cycle.)"""
        other = lambda b: "b" if b == "a" else "a"
        s0 = self._state
        plan, _ = self._plan(s0)
        head, mid = plan[0], plan[1:-1]
        ec_ptr = plan[-1][1][1]  # level-1 correction the finest prolongation reads (same every cycle)
        prog = [(("head", s0), [head])]
        pre = other(s0)
        for _ in range(k - 1):
            prog.append((("join", pre), mid + [self._join_call(pre, ec_ptr)]))
            pre = other(pre)
        tail = self._plan(other(pre))[0][-1]  # PS(0): pre -> other(pre)
        prog.append((("tail", pre), mid + [tail]))
        return prog, other(pre)

    GRAPH_CYCLES = 32  # max joined cycles per HIP graph

    @staticmethod
    def graph_blocks(njoin, G):
        """Block sizes the njoin cycle joins of vcycle(njoin + 1) are replayed in: as many blocks of G
        (a power of two) as fit, then the binary decomposition of the remainder, largest first."""
        blocks = [G] * (njoin // G)
        r = njoin % G
        b = G
        while r:
            b //= 2
            if r >= b:
                blocks.append(b)
                r -= b
        return blocks

    @staticmethod
    def pipe_blocks(njoin, G):
        """Block sizes of vcycle(njoin): as many blocks of G as fit, then the remainder as ONE block (one graph
        per remainder size, at most G of them): a call of k <= G cycles is a single graph launch, so its fixed
        cost (the submission of the first graph, the gap in front of every further graph) is paid once."""
        return [G] * (njoin // G) + ([njoin % G] if njoin % G else [])

    def _ensure_c(self):
        """The finest level's third buffer with the Dirichlet values of the iterate buffers a/b on its boundary
        nodes (its interior is always written before it is read; a set_boundary() not yet followed by a load()
        does not show, as in the unjoined solver)."""
        L0 = self.levels[0]
        if L0.c is None or self._c_bc is not self._ab_version:
            L0.buf("c")
            self._pack(None, L0.c, bc=self._ab_bc)
            self._c_bc = self._ab_version

    def _collapse(self):
        """Leave the pipelined state: the last cycle's end iterate recomputed (PS(0) from the join's
        inputs) into the buffer of the now-discarded next pre-smooth, which becomes the resting state."""
        m = self._mid
        if m is None:
            return
        name, args = self._plan("a")[0][-1]
        args = (self._ptr(0, m["last"]), args[1], args[2], self._ptr(0, m["pre"])) + args[4:]
        self._launch([(name, args)])
        self._state = m["pre"]
        self._mid = None

    def _iterate(self):
        """Name of the finest-level buffer holding the current iterate.  In the pipelined state the
        last cycle's end iterate v is not stored (the cycle join went on to the next pre-smooth): it is
        recomputed once by the last post-smooth PS(0) from the join's inputs, still intact — the
        pre-smoothed iterate `last` and the level-1 correction — into buffer c (bitwise the unjoined
        cycle's result)."""
        m = self._mid
        if m is None:
            return self._state
        if not m["mat"]:
            self._ensure_c()
            name, args = self._plan("a")[0][-1]  # PS(0): (u, ec, f, out, ...)
            args = (self._ptr(0, m["last"]), args[1], args[2], self._ptr(0, "c")) + args[4:]
            self._launch([(name, args)])
            m["mat"] = True
        return "c"

    def _vcycles_pipelined(self, k):
        """k V-cycles as k x [levels >= 1 of a cycle + the cycle join] (fea_mg_cycle_join: post-smooth of
        the cycle and pre-smooth + residual + restriction of the next, 28 instead of 52 B per fine node).
        The solver rests between calls in the pipelined state the join leaves — the NEXT cycle's
        pre-smoothed iterate in `pre`, its restricted residual in f_1 — so consecutive calls pay neither a
        separate first pre-smooth nor a last post-smooth: every call, whatever k, runs exactly k cycles'
        work at the steady-state rate.  From a loaded iterate the first call opens the pipeline with that
        pre-smooth (fea_mg_sweep_restrict).  The end iterate is materialised only when asked for
        (_iterate).  Replayed as few HIP graphs: blocks of GRAPH_CYCLES joins plus one block of the rest
        (pipe_blocks), keyed by (pipeline opened?, buffer, size)."""
        other = lambda b: "b" if b == "a" else "a"
        plan, _ = self._plan("a")
        mid = plan[1:-1]  # levels >= 1 (they never touch the finest level's iterate buffers)
        ec_ptr = plan[-1][1][1]  # level-1 correction the finest prolongation reads (same every cycle)
        if self._mid is None:
            s0 = self._state
            head = [self._plan(s0)[0][0]]
            pre = other(s0)
        else:
            head, pre = [], self._mid["pre"]
        G = max(1, self.GRAPH_CYCLES)
        G = 1 << (G.bit_length() - 1)
        for nb in self.pipe_blocks(k, G):
            key = ("pipe", bool(head), pre, nb)
            g = self._graphs.get(key)
            if g is not None:
                g.replay()
                if nb % 2:
                    pre = other(pre)
            else:
                launches = list(head)
                for _ in range(nb):
                    launches += mid + [self._join_call(pre, ec_ptr)]
                    pre = other(pre)
                self._run_segment(key, launches)
            head = []
        self._mid = {"pre": pre, "last": other(pre), "mat": False}

    def vcycle(self, k=1):
        """Run k V-cycles on the resident iterate (asynchronous; no host sync)."""
        if k < 1:
            return
        if self._joinable() and not getattr(self, "_hjac_first", False):
            self._vcycles_pipelined(k)
            return
        self._vcycles_plain(k)

    def _vcycles_plain(self, k):
        """k unjoined V-cycles (one replay of the whole-cycle plan each) from the materialised iterate."""
        self._collapse()
        for _ in range(k):
            plan, end = self._plan(self._state)
            if getattr(self, "_hjac_first", False):
                self._hjac_first = False
                first = list(plan)
                # the first finest-level sweep of the cycle (its f is level 0's), whatever precedes it
                f0 = self.levels[0].f.data_ptr()
                for i, (name, args) in enumerate(first):
                    fi = {"mg_hsweep": 2, "mg_hsweep_restrict": 2, "mg_prolong_hsweep": 3}.get(name)  # f's slot
                    if fi is not None and args[fi] == f0:
                        first[i] = (name, (args[0], self._raw.data_ptr()) + args[2:])
                        break
                self._launch(first)
                self._state = end
                continue
            if not self.use_graph or self._eager_runs.get(self._state, 0) == 0:
                self._eager_runs[self._state] = self._eager_runs.get(self._state, 0) + 1
                self._launch(plan)
            else:
                g = self._graphs.get(self._state)
                if g is None:
                    g = torch.cuda.CUDAGraph()
                    s = torch.cuda.Stream(self.device)
                    s.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.graph(g, stream=s):
                        self._launch(plan)
                    torch.cuda.current_stream(self.device).wait_stream(s)
                    self._graphs[self._state] = g
                g.replay()
            self._state = end

    def step(self, u, f, cycles=1):
        """Functional form of MultiGrid.Step / MultiGrid.iterate: `cycles` V-cycles from u with rhs f,
        returns the new fine iterate — through the custom op torch.ops.feanet.mg_step (MultiGrid.iterate's
        fused path takes the same op)."""
        from . import torch_ops  # noqa: F401  (registers torch.ops.feanet.mg_step)
        return torch.ops.feanet.mg_step(u, f, self.handle, int(cycles))

    def _step(self, u, f, cycles=1):
        """Body of feanet::mg_step.  One cycle from a freshly loaded iterate, read at once, runs the unjoined
        plan (SR(0) + coarse levels + PS(0), 52 B per fine node): the pipelined form would add a cycle join's
        next pre-smooth and a recomputed post-smooth that nothing reads.  More cycles run joined."""
        if cycles < 1:
            raise ValueError("MultigridSolver.step: cycles must be >= 1")
        self._mid = None  # whatever a previous call left in flight is replaced by u below
        self.set_rhs(f=f)
        self.load(u)
        if cycles == 1:
            self._vcycles_plain(1)
        else:
            self.vcycle(cycles)
        return self.solution()

    def solve(self, u0=None, f=None, F=None, eps=1e-6, max_cycles=100, bc_value=None):
        """Driver loop of the reference notebooks (M-FEANet-mg_test.ipynb:27426-27436,
        MM_Model_convergence.ipynb:196-203): V-cycles until max_b ||r_b|| <= eps (at most max_cycles;
        stops after a non-finite norm, :27434-27436).  Returns (u [B,1,N,N], residual history: list of
        per-sample numpy arrays, first entry = the initial residual).

        Joinable solvers (V(1,1) Jacobi) run the device-resident loop of _solve_joined: the residual
        norm of every cycle comes out of the cycle join (fused, no extra pass) and the host looks at the
        history once per block of cycles.  The result — iterate and history — is that of the per-cycle
        loop (bitwise the same iterate; norms summed in another fixed order)."""
        if bc_value is not None:
            self.set_boundary(bc_value)
        if f is not None or F is not None:
            self.set_rhs(f=f, F=F)
        self.load(u0)
        if self._joinable() and not getattr(self, "_hjac_first", False) and self.use_graph:
            return self._solve_joined(eps, max_cycles, u0)
        hist = [self.residual_norm().cpu().numpy()]
        while hist[-1].max() > eps and len(hist) <= max_cycles:
            self.vcycle()
            hist.append(self.residual_norm().cpu().numpy())
            if not np.all(np.isfinite(hist[-1])):
                break
        return self.solution(), hist

    SOLVE_BLOCK_MAX = 64  # cycles per host check of the solve loop

    def _ensure_hist(self, rows):
        """Device history of fused residual norms (rows of B) and the join's counters; captured solve
        graphs hold these pointers, so a reallocation retires them (new generation in their keys)."""
        if self._hist is None or self._hist.shape[0] < rows:
            self._hist = torch.zeros((max(1024, rows), self.B), dtype=torch.float64, device=self.device)
            self._cnt = torch.zeros(2, dtype=torch.int32, device=self.device)
            self._hist_gen += 1

    def _read_hist(self, r0, r1):
        """History rows r0..r1-1 to the host: one async copy into pinned memory, then a stream sync."""
        n = (r1 - r0) * self.B
        if getattr(self, "_hist_host", None) is None or self._hist_host.numel() < self._hist.numel():
            self._hist_host = torch.empty(self._hist.numel(), dtype=torch.float64, pin_memory=True)
        out = self._hist_host[:n]
        out.copy_(self._hist[r0:r1].reshape(-1), non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return out.numpy().reshape(r1 - r0, self.B).copy()

    def _set_cnt(self, row):
        """Join counters for the next norm-fused launch: arrival count 0, history row `row` (device-side
        fills, no host synchronisation)."""
        self._cnt[0].fill_(0)
        self._cnt[1].fill_(row)

    def _solve_joined(self, eps, max_cycles, u0=None):
        """The solve loop on the device.  State between blocks ("mid-cycle"): the pre-smoothed iterate of
        the next cycle in a finest-level buffer S, its restricted residual in f_1 — what a cycle join
        leaves.  A block runs nb x [levels >= 1 of a cycle + the norm-fused cycle join] (graph blocks of
        graph_blocks(nb)), its joins ping-ponging between the two finest-level buffers other than S (a
        third buffer, so S survives the block untouched); join i appends ||r|| of the iterate at the end
        of cycle i to the device history.  The host reads the block's norms once and
          * stops at the first cycle j with max_b ||r_b|| <= eps (or a non-finite norm), as the reference;
          * if j is the block's last cycle, its end iterate v_j (never stored by the join) is recomputed by
            the last post-smooth PS(0) from the join's inputs, still intact: bitwise the unjoined result;
          * if j is earlier (the contraction beat the prediction), the block is re-run from S to j (f_1 of
            S from a copy taken at the block's start).
        The initial norm comes from the first pre-smooth (fea_mg_sweep_restrict with the fused norm).
        Block sizes: 3 cycles, then the predicted count to eps from the last contraction ratio plus its
        last increase (V-cycle contraction grows towards its asymptotic rate; the extrapolation is bounded
        so the prediction errs short: another block costs one host round trip, an overshoot a re-run)."""
        self._ensure_hist(max_cycles + 2)
        L0, L1 = self.levels[0], self.levels[1]
        self._ensure_c()

        def stop(h):
            return (not np.all(np.isfinite(h))) or h.max() <= eps

        if max_cycles < 1:
            return self.solution(), [self.residual_norm().cpu().numpy()]
        s0 = self._state
        plan, _ = self._plan(s0)
        head, mid = plan[0], plan[1:-1]
        ec_ptr = plan[-1][1][1]
        gen = self._hist_gen
        assert head[0] == "mg_sweep_restrict", head[0]
        hargs = head[1][:-3] + (self.ws.data_ptr(), self._hist.data_ptr(), self._cnt.data_ptr())
        head_launch = (head[0], hargs)  # pre-smooth + initial norm (row 0): opens the first block's graph
        self._set_cnt(0)
        S = "b" if s0 == "a" else "a"
        # deferred norms: each joined cycle of a graph block writes its partial sums to its own set, one
        # reduction launch per graph block appends the block's rows
        esz = 4 if self.dtype == torch.float32 else 8
        per = _lib.join_norm_parts(self.B, L0.H, L0.W, esz)
        stride = per * self.B
        Gmax = self.SOLVE_BLOCK_MAX
        if self._sws is None or self._sws.numel() < Gmax * stride:
            self._sws = torch.zeros(Gmax * stride, dtype=torch.float64, device=self.device)
            self._hist_gen += 1  # captured solve graphs hold the old workspace pointer
            gen = self._hist_gen
        log = self._solve_log = []
        trace = getattr(self, "_trace", False)  # diagnostics: synchronise and time every phase

        def mark(what):
            if trace:
                torch.cuda.synchronize(self.device)
                log.append((what, time.perf_counter()))
        mark("head")

        def run_joins(S, nb, with_head=False):
            """nb norm-fused cycles from start buffer S (after the first pre-smooth if with_head), one graph
            per block of up to SOLVE_BLOCK_MAX cycles; returns (last read buffer, last written)."""
            X, Y = [x for x in "abc" if x != S]
            p, t, last = S, X, None
            for blk in ([nb] if nb <= Gmax else self.graph_blocks(nb, Gmax)):
                # (first read, first write, second write) fixes the whole buffer sequence of the block
                key = ("sblock", with_head, p, t, Y if t == X else X, blk, gen)
                g = self._graphs.get(key)
                if g is not None:  # captured: replay without rebuilding the launch list
                    for _ in range(blk):
                        last, p, t = p, t, (Y if t == X else X)
                    g.replay()
                    with_head = False
                    continue
                launches = [head_launch] if with_head else []
                with_head = False
                for i in range(blk):  # cycle i of the graph block: partial sums into set i
                    launches += mid + [self._join_call(p, ec_ptr, out=t, norm_ws=self._sws.data_ptr() + 8 * i * stride)]
                    last, p, t = p, t, (Y if t == X else X)
                launches.append(("norm_append", (self._sws.data_ptr(), stride, per, self.B, blk, self._hist.data_ptr(),
                                                 self._cnt.data_ptr())))
                self._run_segment(key, launches)
            return last, p

        hist = None
        c = 0
        q = None
        while True:
            h = float(hist[-1].max()) if hist is not None else float("inf")
            if eps <= 0.0 or (q is not None and not 0.0 < q < 1.0):
                nb = self.SOLVE_BLOCK_MAX
            elif q is None:
                nb = 3
            else:
                nb = int(math.ceil(math.log(eps / h) / math.log(q))) if h > eps else 1
            nb = max(1, min(nb, self.SOLVE_BLOCK_MAX, max_cycles - c))
            if nb > 1 and hist is not None:  # f_1 of the start state: the joins overwrite it, a re-run
                if self._f1_snap is None:      # needs it back (the first block re-runs from u0 instead)
                    self._f1_snap = torch.empty_like(L1.f)
                self._f1_snap.copy_(L1.f)
            last_read, end = run_joins(S, nb, with_head=hist is None)
            mark("joins")
            log.append(("block", c, nb))
            if hist is None:
                rows = self._read_hist(0, 1 + nb)
                hist = [rows[0]]
                if stop(hist[0]):  # the loaded guess already meets eps: no cycle at all
                    self.load(u0)
                    return self.solution(), hist
                new = rows[1:]
            else:
                new = self._read_hist(c + 1, c + 1 + nb)
            mark("read")
            j = next((i for i in range(nb) if stop(new[i])), None)
            if j is not None and j < nb - 1:  # converged inside the block: re-run S -> cycle c + j + 1
                if c == 0:
                    self.load(u0)
                    self._set_cnt(0)
                else:
                    L1.f.copy_(self._f1_snap)
                    self._set_cnt(c + 1)
                last_read, end = run_joins(S, j + 1, with_head=c == 0)
                log.append(("rerun", c, j + 1))
                mark("rerun")
            keep = nb if j is None else j + 1
            hist += [new[i] for i in range(keep)]
            c += keep
            S = end
            if j is not None or c >= max_cycles:
                break
            rs = [float(hist[i + 1].max() / hist[i].max()) for i in (len(hist) - 3, len(hist) - 2)
                  if i >= 0 and hist[i].max() > 0]
            q = rs[-1] if rs else None
            if len(rs) == 2 and q is not None:
                # V-cycle contraction grows towards its asymptote: extrapolate the last step (bounded), so
                # the prediction is not systematically one cycle short
                q = min(q + max(0.0, rs[1] - rs[0]), 1.15 * q)
        # v of the last cycle: PS(0) from the last join's inputs (its pre-smoothed iterate `last_read`, the
        # level-1 correction untouched since), into a ping-pong buffer of the unjoined plans
        D = "b" if last_read == "a" else "a"
        name, args = self._plan("a")[0][-1]
        args = (self._ptr(0, last_read), args[1], args[2], self._ptr(0, D)) + args[4:]
        self._run_segment(("tail", last_read, D), [(name, args)])
        self._state = D
        mark("tail")
        u = self.solution()
        mark("solution")
        return u, hist

    # ------------------------------------------------------------------ accounting
    def bytes_per_vcycle(self, k=1):
        """Algorithmic HBM bytes per V-cycle as executed (DESIGN.md §3 accounting).  Joinable solvers run
        every cycle as [levels >= 1 + one fea_mg_cycle_join] (pipelined, _vcycles_pipelined)."""
        esz = 4 if self.dtype == torch.float32 else 8
        plan = self._plan("a")[0]
        if not self._joinable():
            return self._plan_bytes(plan)
        L0, L1 = self.levels[0], self.levels[1]
        nodes = L0.B * (L0.H - 2) * (L0.W - 2)
        coarse = L1.B * (L1.H - 2) * (L1.W - 2)
        pb = 1 if self.problem == "interface" else 0
        join = nodes * (3 * esz + pb) + coarse * (2 * esz + pb)
        return self._plan_bytes(plan[1:-1]) + join

    def _plan_bytes(self, plan):
        esz = 4 if self.dtype == torch.float32 else 8
        pb = 1 if self.problem == "interface" else 0
        total = 0
        for name, args in plan:
            if name in ("mg_coarse_tail", "mg_hjac_tail"):
                continue
            if name == "mg_coarse_tail_ext":  # read f_X twice (down, up), write v_X (the tail itself: LDS)
                H, W, B = args[2], args[3], args[-1]
                total += 3 * esz * B * (H - 2) * (W - 2)
                continue
            if name == "mg_hsweep":  # read u (NULL: zero guess) and f (+ pattern), write out
                B, H, W = args[-5:-2]
                total += B * (H - 2) * (W - 2) * (esz * (3 if args[0] is not None else 2) + pb)
                continue
            if name in ("mg_hsweep_restrict", "mg_prolong_hsweep"):  # (..., B, H, W, ld, bs, ldc, bsc)
                B, H, W = args[-7:-4]
                nodes = B * (H - 2) * (W - 2)
                coarse = B * ((H + 1) // 2 - 2) * ((W + 1) // 2 - 2)
                if name == "mg_hsweep_restrict":  # read u (or not), f; write out, f_c
                    total += nodes * (esz * (3 if args[0] is not None else 2) + pb) + coarse * esz
                else:  # read u, f, e; write out
                    total += nodes * (3 * esz + pb) + coarse * (esz + pb)
                continue
            if name in ("mg_hmid_down", "mg_hmid_up"):
                B, H, W = args[3:6] if name == "mg_hmid_down" else args[5:8]
                n = []
                for _ in range(3):
                    n.append(B * (H - 2) * (W - 2))
                    H, W = (H + 1) // 2, (W + 1) // 2
                if name == "mg_hmid_down":  # read f_a; write u_a, f_(a+1), u_(a+1), f_(a+2)
                    total += esz * (2 * n[0] + 2 * n[1] + n[2]) + pb * (n[0] + n[1])
                else:  # read u_a, f_a, u_(a+1), f_(a+1), e; write u_a
                    total += esz * (3 * n[0] + 2 * n[1] + n[2]) + pb * (n[0] + n[1] + n[2])
                continue
            if name in ("mg_mid_down", "mg_mid_up"):
                k, B, H, W = args[4:8] if name == "mg_mid_up" else args[2:6]
                sizes = []
                for _ in range(k + 1):
                    sizes.append(B * (H - 2) * (W - 2))
                    H, W = (H + 1) // 2, (W + 1) // 2
                if name == "mg_mid_down":  # read f_a, write f_{a+1..a+k}
                    total += esz * sum(sizes) + pb * sum(sizes[:-1])
                else:  # read f_a..f_{a+k-1}, u_{a+k}; write u_a
                    total += esz * (sum(sizes) + sizes[0]) + pb * sum(sizes)
                continue
            if name == "mg_zero_restrict2":  # read f_l (+ pattern), write f_{l+1}, f_{l+2}
                B, H, W = args[-9:-6]
                n0 = B * (H - 2) * (W - 2)
                H, W = (H + 1) // 2, (W + 1) // 2
                n1 = B * (H - 2) * (W - 2)
                n2 = B * ((H + 1) // 2 - 2) * ((W + 1) // 2 - 2)
                total += n0 * (esz + pb) + (n1 + n2) * esz
                continue
            if name == "mg_prolong2":  # read f_l, f_{l+1} (+ patterns), e_{l+2}; write u_l
                B, H, W = args[-9:-6]
                n0 = B * (H - 2) * (W - 2)
                H, W = (H + 1) // 2, (W + 1) // 2
                n1 = B * (H - 2) * (W - 2)
                n2 = B * ((H + 1) // 2 - 2) * ((W + 1) // 2 - 2)
                total += n0 * (2 * esz + pb) + n1 * (esz + pb) + n2 * (esz + pb)
                continue
            if name == "mg_sweep_restrict":  # (..., B, H, W, ld, bs, ldc, bsc, norm_ws, norm_hist, norm_cnt)
                B, H, W = args[-10:-7]
            else:
                B, H, W = (args[-7:-4] if name in ("mg_residual_restrict", "mg_prolong_sweep", "mg_prolong_add")
                           else args[-5:-2])
            nodes = B * (H - 2) * (W - 2)
            coarse = B * ((H + 1) // 2 - 2) * ((W + 1) // 2 - 2)
            if name == "mg_sweep":
                total += nodes * (esz * (3 if args[0] is not None else 2) + pb)
            elif name == "mg_residual_restrict":
                total += nodes * (esz * (2 if args[0] is not None else 1) + pb) + coarse * esz
                if args[0] is None and args[2] is not None:
                    total += nodes * esz  # v written
            elif name == "mg_sweep_restrict":
                total += nodes * (3 * esz + pb) + coarse * esz
            elif name == "mg_prolong_sweep":  # u = NULL: the iterate is recomputed from f
                total += nodes * ((3 if args[0] is not None else 2) * esz + pb) + coarse * (esz + pb)
            elif name == "mg_prolong_add":
                total += nodes * 2 * esz + coarse * (esz + pb)
        return total
