"""torch.autograd Functions over the generic HIP operators and their HIP adjoints.

The reference trains its inter-grid operators by back-propagating through a V-cycle
(MultiGrid.forward + qm, FEANet/multigrid.py:132-157: `conv.net.weight` / `deconv.net.weight`
require grad, everything upstream of them does not); torch's conv2d / conv_transpose2d backward
supplies its gradients.  Here every forward op and every adjoint is a HIP kernel
(generic_ops.hip: k_knet_adj, k_jacobi_adj, k_restrict_adj, k_prolong_adj, k_tapgrad_*), so a
training step through `FEANet.multigrid.MultiGrid` never leaves the device and never touches a
CPU fallback.  `feanet_amd.ops` routes to these Functions whenever autograd needs a graph.

Gradients provided:
  knet_apply    d/du, d/d(stencils)        (KNet net2 weights; conv3x3 = FNet / HNet layers)
  jacobi_sweep  d/du, d/df, d/d(stencils)  (omega/d, geometry and boundary values are constants)
  residual      d/du, d/df, d/d(stencils)
  split_x       d/dx
  restrict      d/dx, d/d(kernels)         (RestrictionNet.net.weight, multigrid.py:50-60)
  prolong       d/de, d/d(kernels), d/dadd (ProlongationNet.net.weight, multigrid.py:62-73)
Kernel gradients are for split inputs (C > 1, one kernel per channel) or a single kernel; the
per-pattern (pid) kernel mode has no weight gradient and raises if one is requested.
"""
import torch

from . import _lib, ops


def _frozen(ctx, name, *idx):
    if any(ctx.needs_input_grad[i] for i in idx):
        raise NotImplementedError(f"feanet_amd: no gradient w.r.t. the {name} (constants of the operator, "
                                  "FEANet/jacobi.py:17-37); set requires_grad=False on it")


def _like(g, ref):
    return g.contiguous() if g.dtype == ref.dtype else g.to(ref.dtype).contiguous()


def _knet_adj(g, ktab, pid):
    g = g.contiguous()
    B, H, W = ops._bhw(g)
    tab = ops._table(ktab, g.dtype, g.device)
    out = torch.empty_like(g)
    _lib.call("knet_apply_adj", g.dtype, g.data_ptr(), out.data_ptr(), ops._ptr(pid), tab.data_ptr(),
              tab.shape[0], B, H, W, ops._stream(g))
    return out


def _stencil_grad(g, u, ktab, pid, scale=1.0):
    """d/dW of sum(g . K u) in ktab's shape/dtype (fea_stencil_weight_grad)."""
    g, u = g.contiguous(), u.contiguous()
    B, H, W = ops._bhw(g)
    ntab = ktab.numel() // 9
    gw = torch.empty((ntab, 9), dtype=g.dtype, device=g.device)
    ws = torch.empty(max(1, _lib.stencil_grad_ws_bytes(ntab, B, H, W) // 8), dtype=torch.float64, device=g.device)
    _lib.call("stencil_weight_grad", g.dtype, g.data_ptr(), u.data_ptr(), ops._ptr(pid if ntab > 1 else None), ntab,
              float(scale), gw.data_ptr(), ws.data_ptr(), B, H, W, ops._stream(g))
    return gw.reshape(ktab.shape).to(ktab.dtype)


# Backward bodies shared by the torch.library registrations of torch_ops.py (the product path) and
# the autograd.Function classes below (kept as a reference path for the tests).  Each reads what its
# forward saved (ctx.saved_tensors, scalars on ctx) and returns one gradient per op input.

def knet_backward(ctx, g):  # saved (u, ktab, pid)
    u, ktab, pid = ctx.saved_tensors
    gu = _knet_adj(g, ktab, pid) if ctx.needs_input_grad[0] else None
    gk = _stencil_grad(g, u, ktab, pid) if ctx.needs_input_grad[1] else None
    return gu, gk, None


def residual_backward(ctx, g):  # saved (u, ktab, pid)
    u, ktab, pid = ctx.saved_tensors
    gu = -_knet_adj(g, ktab, pid) if ctx.needs_input_grad[0] else None
    gk = _stencil_grad(g, u, ktab, pid, -1.0) if ctx.needs_input_grad[2] else None
    return gu, (g if ctx.needs_input_grad[1] else None), gk, None


class KNetApply(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, ktab, pid):
        ctx.save_for_backward(u if ctx.needs_input_grad[1] else None, ktab, pid)
        return ops._knet_apply(u, ktab, pid)

    @staticmethod
    def backward(ctx, g):
        return knet_backward(ctx, g)


class Residual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, f, ktab, pid):
        ctx.save_for_backward(u if ctx.needs_input_grad[2] else None, ktab, pid)
        return ops._residual(u, f, ktab, pid)

    @staticmethod
    def backward(ctx, g):
        return residual_backward(ctx, g)


class JacobiSweep(torch.autograd.Function):
    """out = R(u0 + omd (f - K u0)), u0 = R(u), R(v) = geo v + bc.  Gradients in u, f and the stencils
    (omega/d, geometry and boundary values are constants of the block, jacobi.py:17-37)."""

    @staticmethod
    def forward(ctx, u, f, ktab, omd, pid, geo, bc):
        ctx.save_for_backward(u if ctx.needs_input_grad[2] else None, ktab, omd, pid, geo, bc)
        return ops._jacobi_sweep(u, f, ktab, omd, pid, geo, bc)

    @staticmethod
    def backward(ctx, g):
        return jacobi_backward(ctx, g)


def jacobi_backward(ctx, g):  # saved (u, ktab, omd, pid, geo, bc)
    _frozen(ctx, "omega-over-d / geometry / boundary values", 3, 5, 6)
    u, ktab, omd, pid, geo, bc = ctx.saved_tensors
    g = g.contiguous()
    B, H, W = ops._bhw(g)
    tab = ops._table(ktab, g.dtype, g.device)
    om = torch.as_tensor(omd).to(device=g.device, dtype=g.dtype).reshape(-1).contiguous()
    geo_t, gs = ops._bcast_stride(geo, B, H, W, "geometry_idx", g.dtype, g.device)
    gu = torch.empty_like(g)
    need_gf = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
    gf = torch.empty_like(g) if need_gf else None
    _lib.call("jacobi_sweep_adj", g.dtype, g.data_ptr(), gu.data_ptr(), ops._ptr(gf), ops._ptr(pid),
              tab.data_ptr(), om.data_ptr(), tab.shape[0], ops._ptr(geo_t), gs, B, H, W, ops._stream(g))
    gk = None
    if ctx.needs_input_grad[2]:  # d/dW of -sum(gf . K u0)
        if geo is None:
            u0 = u * _interior_mask(H, W, u)
        else:
            u0 = u * geo
        if bc is not None:
            u0 = u0 + bc
        gk = _stencil_grad(gf, u0.to(g.dtype).expand(g.shape), ktab, pid, -1.0)
    return (gu if ctx.needs_input_grad[0] else None), (gf if ctx.needs_input_grad[1] else None), gk, \
        None, None, None, None


def _interior_mask(H, W, like):
    m = torch.zeros((H, W), dtype=like.dtype, device=like.device)
    m[1:-1, 1:-1] = 1
    return m


class SplitX(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pid, C):
        ctx.save_for_backward(pid)
        ctx.xshape = x.shape
        return ops._split_x(x, pid, C)

    @staticmethod
    def backward(ctx, g):
        return split_backward(ctx, g)


def split_backward(ctx, g):  # saved (pid,), ctx.xshape
    (pid,) = ctx.saved_tensors
    B, C, H, W = g.shape
    if pid is None:
        gx = g[:, :1]
    else:  # the masks partition the nodes: d x_i = g[pid(i)]_i
        idx = pid.to(torch.int64).reshape(1, 1, H, W).expand(B, 1, H, W)
        gx = torch.gather(g, 1, idx)
    return gx.reshape(ctx.xshape).contiguous(), None, None


def _weight_grad(cf, c_split, ff, f_split, C, interior, scale, Hc, Wc):
    B = cf.shape[0]
    gw = torch.empty((C, 9), dtype=cf.dtype, device=cf.device)
    ws = torch.empty(max(1, _lib.weight_grad_ws_bytes(C, B, Hc, Wc) // 8), dtype=torch.float64, device=cf.device)
    _lib.call("transfer_weight_grad", cf.dtype, cf.data_ptr(), int(c_split), ff.data_ptr(), int(f_split), C,
              int(interior), float(scale), gw.data_ptr(), ws.data_ptr(), B, Hc, Wc, ops._stream(cf))
    return gw


class Restrict(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rtab, w0, pid):
        ctx.save_for_backward(x, rtab, pid)
        ctx.w0 = float(w0)
        return ops._restrict(x, rtab, w0, pid)

    @staticmethod
    def backward(ctx, g):
        return restrict_backward(ctx, g)


def restrict_backward(ctx, g):  # saved (x, rtab, pid), ctx.w0
    x, rtab, pid = ctx.saved_tensors
    x = x.contiguous()
    g = _like(g, x)
    B, C, H, W = x.shape
    Hc, Wc = (H + 1) // 2, (W + 1) // 2
    tab = ops._table(rtab, x.dtype, x.device)
    gx = gr = None
    if ctx.needs_input_grad[0]:
        gx = torch.empty_like(x)
        pp = pid if C == 1 else None
        _lib.call("restrict_adj", x.dtype, g.data_ptr(), C, gx.data_ptr(), ops._ptr(pp), tab.data_ptr(),
                  tab.shape[0], ctx.w0, B, H, W, ops._stream(x))
    if ctx.needs_input_grad[1]:
        if C == 1 and tab.shape[0] > 1:
            raise NotImplementedError("feanet_amd: no kernel gradient in per-pattern (pid) restriction mode")
        gr = _weight_grad(g, False, x, True, C, True, ctx.w0, Hc, Wc)
        gr = gr.reshape(rtab.shape).to(rtab.dtype)
    return gx, gr, None, None



class Prolong(torch.autograd.Function):
    @staticmethod
    def forward(ctx, e, ptab, w1, pidc, add):
        ctx.save_for_backward(e, ptab, pidc)
        ctx.w1 = float(w1)
        return ops._prolong(e, ptab, w1, pidc, add)

    @staticmethod
    def backward(ctx, g):
        return prolong_backward(ctx, g)


def prolong_backward(ctx, g):  # saved (e, ptab, pidc), ctx.w1
    e, ptab, pidc = ctx.saved_tensors
    e = e.contiguous()
    g = _like(g, e)
    B, C, Hc, Wc = e.shape
    tab = ops._table(ptab, e.dtype, e.device)
    ge = gp = None
    if ctx.needs_input_grad[0]:
        ge = torch.empty_like(e)
        pp = pidc if C == 1 else None
        _lib.call("prolong_adj", e.dtype, g.data_ptr(), C, ge.data_ptr(), ops._ptr(pp), tab.data_ptr(),
                  tab.shape[0], ctx.w1, B, Hc, Wc, ops._stream(e))
    if ctx.needs_input_grad[1]:
        if C == 1 and tab.shape[0] > 1:
            raise NotImplementedError("feanet_amd: no kernel gradient in per-pattern (pid) prolongation mode")
        gp = _weight_grad(e, True, g, False, C, False, ctx.w1, Hc, Wc)
        gp = gp.reshape(ptab.shape).to(ptab.dtype)
    gadd = g if ctx.needs_input_grad[4] else None
    return ge, gp, None, None, gadd
