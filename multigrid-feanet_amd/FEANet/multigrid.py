"""Two-material multigrid with learned inter-grid operators (reference: FEANet/multigrid.py:12-185).

Same classes and methods as the reference (SingleGrid, RestrictionNet, ProlongationNet,
MultiGrid with Restrict / Interpolate / qm / random_sampling / forward / iterate) and the same
state_dict keys (`w`, `conv.net.weight`, `deconv.net.weight`), with every operator a HIP kernel.
Reference bugs fixed here: SingleGrid.Relax loops single sweeps instead of passing
an `n_iter=` argument jacobi_convolution does not accept.  Buffers are allocated on the input's
device/dtype instead of hard-coded CPU float32.

`MultiGrid.iterate` always runs the fused MultigridSolver V-cycle forward (the custom op
torch.ops.feanet.mg_step).  When autograd is recording and an input or the R/P weights need a gradient,
the call is wrapped in `_FusedIterate`: its backward recomputes the cycle from the module-level HIP
operators (each with a registered HIP adjoint) and back-propagates through that, so the detached
iterations of `forward` (the first m-1 of m, multigrid.py:147-150) never pay for the per-op path.
Both paths compute the reference's schedule.
"""
import numpy as np
import torch
import torch.nn as nn

from FEANet.geo import Geometry
from FEANet.jacobi import JacobiBlock
from FEANet.mesh import MeshCenterInterface
from FEANet.model import FNet, KNet
from feanet_amd import ops


class SingleGrid:
    """One level: two-material mesh, KNet/FNet, JacobiBlock (multigrid.py:12-47)."""

    def __init__(self, size, n, device=None):
        self.size = size
        self.n = n
        self.omega = 2 / 3.
        self.property = [1, 20]
        self.plate = Geometry(nnode_edge=n + 1)
        self.grid = MeshCenterInterface(size, prop=self.property, nnode_edge=n + 1)
        dev = self.plate.geometry_idx.device if device is None else device
        self.v = torch.zeros((1, 1, n + 1, n + 1), dtype=torch.float32, device=dev)
        self.f = torch.zeros((1, 1, n + 1, n + 1), dtype=torch.float32, device=dev)
        self.InstantiateFEANet()
        self.jac = JacobiBlock(self.Knet, self.grid, self.omega, self.plate.geometry_idx, self.plate.boundary_value)

    def IsCoarsest(self):
        return self.n == 2

    def InstantiateFEANet(self):
        self.Knet = KNet(self.grid)
        self.fnet = FNet(self.size / self.n)
        for param in self.Knet.parameters():
            param.requires_grad = False
        for param in self.fnet.parameters():
            param.requires_grad = False

    def Relax(self, v, f, num_sweeps_down):
        for _ in range(num_sweeps_down):
            v = self.jac.jacobi_convolution(v, f)
        return v


class RestrictionNet(nn.Module):
    """16-channel stride-2 restriction, one 3x3 kernel per node pattern (multigrid.py:50-60)."""

    def __init__(self, linear_tensor_R):
        super().__init__()
        self.n_channel = 16
        self.net = nn.Conv2d(self.n_channel, 1, kernel_size=3, stride=2, bias=False)
        with torch.no_grad():
            for i in range(self.n_channel):
                self.net.weight[0, i] = torch.as_tensor(linear_tensor_R).to(self.net.weight)

    def forward(self, x_split):
        """x_split [B, 16, H, W] (already cropped) -> [B, 1, (H-3)/2+1, ...] (valid stride-2 conv)."""
        # the HIP restriction works on the full (uncropped) field and pads; rebuild that frame
        B, C, H, W = x_split.shape
        full = torch.zeros((B, C, H + 2, W + 2), dtype=x_split.dtype, device=x_split.device)
        full[:, :, 1:-1, 1:-1] = x_split
        return ops.restrict(full, self.net.weight[0], 1.0)[:, :, 1:-1, 1:-1]


class ProlongationNet(nn.Module):
    """16-channel stride-2 transposed conv, one kernel per coarse-node pattern (multigrid.py:62-73)."""

    def __init__(self, linear_tensor_P):
        super().__init__()
        self.n_channel = 16
        self.net = nn.ConvTranspose2d(self.n_channel, 1, kernel_size=3, stride=2, padding=1, bias=False)
        with torch.no_grad():
            for i in range(self.n_channel):
                self.net.weight[i, 0] = torch.as_tensor(linear_tensor_P).to(self.net.weight)

    def forward(self, x_split):
        return ops.prolong(x_split, self.net.weight[:, 0], 1.0)


class _FusedIterate(torch.autograd.Function):
    """Forward: the fused V-cycle.  Backward: gradients of the same cycle as composed from the module-level
    operators (`iterate_modules`), recomputed from the saved inputs — the fused forward keeps no per-level
    intermediates, so the adjoint cycle needs them rebuilt once, only when a gradient is actually asked for."""

    @staticmethod
    def forward(ctx, x, f, wr, wp, w, mg):
        ctx.mg = mg
        ctx.save_for_backward(x, f)
        return mg._fused(x).step(x, f)

    @staticmethod
    def backward(ctx, g):
        x, f = ctx.saved_tensors
        mg = ctx.mg
        params = (mg.conv.net.weight, mg.deconv.net.weight, mg.w)
        # the recompute writes the per-level fields of mg.grids; put the forward's back afterwards so the
        # module keeps no backward-time tensors (nor the autograd graph they would hold alive)
        saved = {j: (gr.v, gr.f) for j, gr in mg.grids.items()}
        try:
            with torch.enable_grad():
                xd = x.detach().requires_grad_(ctx.needs_input_grad[0])
                fd = f.detach().requires_grad_(ctx.needs_input_grad[1])
                out = mg.iterate_modules(xd, fd)
                wanted = [t for t, need in zip((xd, fd) + params, ctx.needs_input_grad[:5]) if need]
                got = iter(torch.autograd.grad(out, wanted, g, allow_unused=True))
        finally:
            for j, (v, fj) in saved.items():
                mg.grids[j].v, mg.grids[j].f = v, fj
        return tuple(next(got) if need else None for need in ctx.needs_input_grad[:5]) + (None,)


class MultiGrid(nn.Module):
    """V-cycle with learned R/P and ratios w on the two-material problem (multigrid.py:75-185)."""

    def __init__(self, n, linear_tensor_R, linear_tensor_P, linear_ratio):
        super().__init__()
        self.m0 = 2
        self.m = 6
        self.size = 2
        self.n = n
        self.L = int(np.log2(n))
        self.solution = []
        self.n_arr = self.SizeArray()
        self.grids = self.GridDict()
        self.conv = RestrictionNet(linear_tensor_R)
        self.deconv = ProlongationNet(linear_tensor_P)
        self.w = nn.Parameter(torch.as_tensor(linear_ratio).to(self.conv.net.weight))
        self.conv.requires_grad_(True)
        self.deconv.requires_grad_(True)
        self.w.requires_grad_(False)
        self._solver = None
        self._solver_key = None
        self._solver_ver = None

    def GridDict(self):
        return {i: SingleGrid(self.size, int(self.n_arr[i])) for i in range(self.L)}

    def SizeArray(self):
        return np.array([int(self.n / (2. ** i)) for i in range(self.L)])

    def Restrict(self, rF):
        """rF already split [B,16,N,N] -> conv over the interior, zero-padded (multigrid.py:115-122)."""
        return ops.restrict(rF, self.conv.net.weight[0], 1.0)

    def Interpolate(self, eFC):
        """eFC already split [B,16,Nc,Nc] -> transposed conv (multigrid.py:124-130)."""
        return ops.prolong(eFC, self.deconv.net.weight[:, 0], 1.0)

    def qm(self, x):
        res1 = self.f - self.grids[0].Knet(x)
        res0 = self.f - self.grids[0].Knet(self.v_m0)
        return torch.mean(torch.pow(torch.norm(res1[:, :, 1:-1, 1:-1], dim=(2, 3)) /
                                    torch.norm(res0[:, :, 1:-1, 1:-1], dim=(2, 3)).detach(),
                                    1.0 / (self.m - self.m0 + 1)))

    def random_sampling(self, v):
        d1, d2, d3, d4 = v.shape
        for i in range(d1):
            for j in range(d2):
                coef = 10 * np.random.rand(2) - 5
                v[i, j, :, :] = torch.from_numpy(coef[0] * np.random.random((d3, d4)) + coef[1]).to(v)

    def forward(self, F):
        self.f = self.grids[0].fnet(F)
        self.v = torch.zeros_like(F)
        self.random_sampling(self.v)
        U = torch.clone(self.v)
        for i in range(self.m - 1):
            U = self.iterate(U, self.f).detach()
            if i == self.m0 - 1:
                self.v_m0 = U.detach().clone()
        return self.iterate(U, self.f)

    # ------------------------------------------------------------------ V-cycle
    def _transfer_version(self):
        return tuple((t.data_ptr(), t._version) for t in (self.conv.net.weight, self.deconv.net.weight, self.w))

    def _fused(self, x):
        """The MultigridSolver of this batch shape, built once.  An optimizer step changes R / P in place
        (their _version moves): the new values are copied into the solver's resident tables
        (MultigridSolver.set_transfer) instead of rebuilding it, so level buffers, pattern maps and captured
        graphs are reused across training steps; the ratios w are read back to the host only when they change.

        Changes are detected by (data_ptr, _version) of R, P and w: in-place updates must go through tracked
        tensor ops (optimizer steps, `with torch.no_grad(): w.copy_(...)`) or reassign the parameter.  Writes
        through `.data` (e.g. `mg.w.data.fill_(...)`) do not move `_version` and are NOT seen: call
        `self._solver_ver = None` after such a write (the next iterate then copies all three)."""
        from feanet_amd.solver import MultigridSolver
        key = (x.shape[0], x.dtype, x.device)
        ver = self._transfer_version()
        if self._solver is None or self._solver_key != key:
            self._solver = MultigridSolver(self.n, levels=self.L, problem="interface", dtype=x.dtype,
                                           device=x.device, batch=x.shape[0], size=self.size,
                                           R=self.conv.net.weight[0], P=self.deconv.net.weight[:, 0],
                                           w=(float(self.w[0]), float(self.w[1])))
            self._solver_key = key
        elif ver != self._solver_ver:
            old = self._solver_ver or (None, None, None)
            self._solver.set_transfer(R=self.conv.net.weight[0] if ver[0] != old[0] else None,
                                      P=self.deconv.net.weight[:, 0] if ver[1] != old[1] else None,
                                      w=self.w if ver[2] != old[2] else None)
        self._solver_ver = ver
        return self._solver

    def iterate(self, x, f):
        """One V-cycle (multigrid.py:159-185): the fused solver forward; differentiable through _FusedIterate
        when autograd records (recomputed module-level cycle in backward)."""
        params = (self.conv.net.weight, self.deconv.net.weight, self.w)
        needs_grad = torch.is_grad_enabled() and (x.requires_grad or f.requires_grad or any(
            p.requires_grad for p in params))
        if needs_grad:
            v = _FusedIterate.apply(x, f, *params, self)
        else:
            v = self._fused(x).step(x, f)
        self.grids[0].v, self.grids[0].f = v, f
        return v

    def iterate_modules(self, x, f):
        """The same V-cycle composed from the module-level HIP operators (autograd-free forward)."""
        n_batches = x.shape[0]
        g = self.grids
        g[0].v = g[0].Relax(x, f, 1)
        g[0].f = f
        for j in range(self.L - 1):
            rF = g[j].f - g[j].Knet(g[j].v)
            rF = g[j].Knet.split_x(rF)
            g[j + 1].f = self.w[0] * self.Restrict(rF)
            z = torch.zeros((n_batches, 1, self.n_arr[j + 1] + 1, self.n_arr[j + 1] + 1), dtype=x.dtype,
                            device=x.device)
            g[j + 1].v = g[j + 1].Relax(z, g[j + 1].f, 1)
        g[self.L - 1].v = g[self.L - 1].Relax(g[self.L - 1].v, g[self.L - 1].f, 1)
        for j in range(self.L - 2, -1, -1):
            eFC = g[j + 1].Knet.split_x(g[j + 1].v)
            g[j].v = g[j].v + self.w[1] * self.Interpolate(eFC)
            g[j].v = g[j].Relax(g[j].v, g[j].f, 1)
            g[j + 1].v = torch.zeros_like(g[j + 1].v)
        return g[0].v
