"""The generic HIP operators as PyTorch custom ops: `torch.ops.feanet.<name>`.

BASELINE.json's north star asks for the kernels to be "surfaced to the Python host as PyTorch-ROCm
custom ops".  Each op below is registered with torch.library for the HIP ('cuda') device only; its
implementation is the ctypes call of feanet_amd.ops (one HIP kernel, the caller's current stream), a
fake implementation gives output shapes for tracing / meta tensors, and the differentiable ones carry
their HIP adjoints (feanet_amd.autograd) through register_autograd.  CPU tensors find no kernel and
raise — there is no CPU fallback.  These ops ARE the product path of the generic operators: the
FEANet drop-in modules and feanet_amd.ops' public functions call torch.ops.feanet.*.

  feanet::knet_apply(u, ktab, pid?)                   KNet.forward        FEANet/model.py:22-30
  feanet::split_x(x, pid?, C)                         KNet.split_x        FEANet/model.py:37-47
  feanet::residual(u, f, ktab, pid?)                  f - K u             FEANet/multigrid.py:168
  feanet::jacobi_sweep(u, f, ktab, omd, pid?, geo?, bc?)  jacobi_convolution  FEANet/jacobi.py:39-47
  feanet::restrict(x, rtab, w0, pid?)                 MultiGrid.Restrict  FEANet/multigrid.py:115-122
  feanet::prolong(e, ptab, w1, pidc?, add?)           MultiGrid.Interpolate FEANet/multigrid.py:124-130
  feanet::residual_norm(u, f?, ktab?, pid?)           driver residual norm M-FEANet-mg_test.ipynb:27428
  feanet::pbc_pad(u, lo, hi)                          JacobiBlockPBC.pbc_boundary / reset_boundary
  feanet::jacobi_sweep_pbc(u, f, ktab, omd)           JacobiBlockPBC.jacobi_convolution FEANet/jacobi.py:86-97
  feanet::mg_step(u, f, solver, cycles)               MultiGrid.Step / iterate (fused V-cycles of a
                                                      MultigridSolver)  M-FEANet-mg_test.ipynb:27346-27372,
                                                      FEANet/multigrid.py:159-185
"""
from typing import Optional

import torch
from torch import Tensor

from . import autograd as _ag
from . import ops

_DEV = "cuda"


def _full(bwd, n):
    """A backward over all n schema inputs: the dispatcher drops trailing arguments equal to their
    defaults (None pattern maps, geometry, ...) from what autograd tracks, so needs_input_grad is
    padded for the shared backward bodies and the result trimmed back."""
    def backward(ctx, g):
        nig = tuple(ctx.needs_input_grad)
        ctx.needs_input_grad = nig + (False,) * (n - len(nig))
        try:
            out = bwd(ctx, g)
        finally:
            ctx.needs_input_grad = nig
        return tuple(out)[:len(nig)]
    return backward


@torch.library.custom_op("feanet::knet_apply", mutates_args=(), device_types=_DEV)
def knet_apply(u: Tensor, ktab: Tensor, pid: Optional[Tensor] = None) -> Tensor:
    return ops._knet_apply(u, ktab, pid)


@knet_apply.register_fake
def _(u, ktab, pid=None):
    return torch.empty_like(u, memory_format=torch.contiguous_format)


def _knet_setup(ctx, inputs, output):
    u, ktab, pid = inputs
    ctx.save_for_backward(u, ktab, pid)


knet_apply.register_autograd(_full(_ag.knet_backward, 3), setup_context=_knet_setup)


@torch.library.custom_op("feanet::residual", mutates_args=(), device_types=_DEV)
def residual(u: Tensor, f: Tensor, ktab: Tensor, pid: Optional[Tensor] = None) -> Tensor:
    return ops._residual(u, f, ktab, pid)


@residual.register_fake
def _(u, f, ktab, pid=None):
    return torch.empty_like(u, memory_format=torch.contiguous_format)


def _res_setup(ctx, inputs, output):
    u, f, ktab, pid = inputs
    ctx.save_for_backward(u, ktab, pid)


residual.register_autograd(_full(_ag.residual_backward, 4), setup_context=_res_setup)


@torch.library.custom_op("feanet::jacobi_sweep", mutates_args=(), device_types=_DEV)
def jacobi_sweep(u: Tensor, f: Tensor, ktab: Tensor, omd: Tensor, pid: Optional[Tensor] = None,
                 geo: Optional[Tensor] = None, bc: Optional[Tensor] = None) -> Tensor:
    return ops._jacobi_sweep(u, f, ktab, omd, pid, geo, bc)


@jacobi_sweep.register_fake
def _(u, f, ktab, omd, pid=None, geo=None, bc=None):
    return torch.empty_like(u, memory_format=torch.contiguous_format)


def _js_setup(ctx, inputs, output):
    u, f, ktab, omd, pid, geo, bc = inputs
    ctx.save_for_backward(u, ktab, omd, pid, geo, bc)


jacobi_sweep.register_autograd(_full(_ag.jacobi_backward, 7), setup_context=_js_setup)


@torch.library.custom_op("feanet::split_x", mutates_args=(), device_types=_DEV)
def split_x(x: Tensor, pid: Optional[Tensor], C: int) -> Tensor:
    return ops._split_x(x, pid, C)


@split_x.register_fake
def _(x, pid, C):
    B, _, H, W = x.shape
    return x.new_empty((B, C, H, W))


def _split_setup(ctx, inputs, output):
    x, pid, C = inputs
    ctx.save_for_backward(pid)
    ctx.xshape = x.shape


split_x.register_autograd(_full(_ag.split_backward, 3), setup_context=_split_setup)


@torch.library.custom_op("feanet::restrict", mutates_args=(), device_types=_DEV)
def restrict(x: Tensor, rtab: Tensor, w0: float = 1.0, pid: Optional[Tensor] = None) -> Tensor:
    return ops._restrict(x, rtab, w0, pid)


@restrict.register_fake
def _(x, rtab, w0=1.0, pid=None):
    B, _, H, W = x.shape
    return x.new_empty((B, 1, (H + 1) // 2, (W + 1) // 2))


def _restrict_setup(ctx, inputs, output):
    x, rtab, w0, pid = inputs
    ctx.save_for_backward(x, rtab, pid)
    ctx.w0 = float(w0)


restrict.register_autograd(_full(_ag.restrict_backward, 4), setup_context=_restrict_setup)


@torch.library.custom_op("feanet::prolong", mutates_args=(), device_types=_DEV)
def prolong(e: Tensor, ptab: Tensor, w1: float = 1.0, pidc: Optional[Tensor] = None,
            add: Optional[Tensor] = None) -> Tensor:
    return ops._prolong(e, ptab, w1, pidc, add)


@prolong.register_fake
def _(e, ptab, w1=1.0, pidc=None, add=None):
    B, _, Hc, Wc = e.shape
    return e.new_empty((B, 1, 2 * Hc - 1, 2 * Wc - 1))


def _prolong_setup(ctx, inputs, output):
    e, ptab, w1, pidc, add = inputs
    ctx.save_for_backward(e, ptab, pidc)
    ctx.w1 = float(w1)


prolong.register_autograd(_full(_ag.prolong_backward, 5), setup_context=_prolong_setup)


@torch.library.custom_op("feanet::residual_norm", mutates_args=(), device_types=_DEV)
def residual_norm(u: Tensor, f: Optional[Tensor] = None, ktab: Optional[Tensor] = None,
                  pid: Optional[Tensor] = None) -> Tensor:
    return ops.residual_norm(u, f, ktab, pid)


@residual_norm.register_fake
def _(u, f=None, ktab=None, pid=None):
    H, W = u.shape[-2:]
    return u.new_empty((u.numel() // (H * W),), dtype=torch.float64)


@torch.library.custom_op("feanet::pbc_pad", mutates_args=(), device_types=_DEV)
def pbc_pad(u: Tensor, lo: int, hi: int) -> Tensor:
    return ops.pbc_pad(u, lo, hi)


@pbc_pad.register_fake
def _(u, lo, hi):
    M = u.shape[-1] - 1 + lo + hi
    return u.new_empty(u.shape[:-2] + (M, M))


@torch.library.custom_op("feanet::jacobi_sweep_pbc", mutates_args=(), device_types=_DEV)
def jacobi_sweep_pbc(u: Tensor, f: Tensor, ktab: Tensor, omd: Tensor) -> Tensor:
    return ops.jacobi_sweep_pbc(u, f, ktab, omd)


@jacobi_sweep_pbc.register_fake
def _(u, f, ktab, omd):
    return torch.empty_like(u, memory_format=torch.contiguous_format)


@torch.library.custom_op("feanet::mg_step", mutates_args=(), device_types=_DEV)
def mg_step(u: Tensor, f: Tensor, solver: int, cycles: int = 1) -> Tensor:
    """`cycles` fused V-cycles of the MultigridSolver with handle `solver` (MultigridSolver.handle) from
    the fine iterate u with right-hand side f; returns the new iterate [B, 1, H, W].  The solver's level
    buffers, HIP graphs and schedule stay resident between calls: this op is the whole-cycle form of
    MultiGrid.Step(v, f) (one pass per fused level kernel) that a notebook loop can call as
    `u = torch.ops.feanet.mg_step(u, f, solver.handle)`.

    Contract: only the returned tensor is defined.  The op is registered functional (mutates_args=()), so
    under torch.compile an op whose result is unused may be dropped, and ops may be reordered against direct
    calls of the solver's methods: what solver.solution() / residual_norm() return after it is not part of
    the op's meaning (read the returned tensor instead)."""
    from .solver import solver_by_handle
    return solver_by_handle(solver)._step(u, f, cycles)


@mg_step.register_fake
def _(u, f, solver, cycles=1):
    from .solver import solver_by_handle
    s = solver_by_handle(solver)
    return u.new_empty((s.B, 1, s.H, s.W))
