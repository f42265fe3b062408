"""Tensor-level wrappers of the generic HIP operators (C ABI family (1) of include/feanet_hip.h).

Every function requires HIP (torch 'cuda') tensors and launches on torch's current stream of
that device.  There is no CPU path: a CPU tensor raises, so a silent fallback cannot happen.
Tables (stencils, omega/d, R/P kernels) are device tensors of the field dtype, shape [C, 3, 3]
(or [C, 9]); pattern maps are uint8 [H, W].
"""
import torch

from . import _lib


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


def require_hip(t, name="tensor"):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"feanet_amd: {name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"feanet_amd: {name} is on {t.device}; the FEANet HIP operators run on the "
                           "MI355X only (move the tensor to 'cuda', e.g. torch.set_default_device('cuda'))")


def _field(t, name, dtype=None):
    require_hip(t, name)
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"feanet_amd: {name} has dtype {t.dtype}, expected {dtype} "
                           "(call .double() on the module for fp64, as with the reference)")
    if t.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"feanet_amd: {name} must be float32 or float64, got {t.dtype}")
    return t.contiguous()


def _table(t, dtype, device, rows=None):
    t = torch.as_tensor(t)
    if t.device != device or t.dtype != dtype:
        t = t.to(device=device, dtype=dtype)
    t = t.reshape(-1, 9).contiguous()
    if rows is not None and t.shape[0] != rows:
        raise ValueError(f"feanet_amd: table has {t.shape[0]} rows, expected {rows}")
    if t.shape[0] > 16:
        raise ValueError("feanet_amd: at most 16 stencil patterns are supported")
    return t


def _pid(pid, H, W, device):
    if pid is None:
        return None
    require_hip(pid, "pattern map")
    if pid.dtype != torch.uint8 or tuple(pid.shape[-2:]) != (H, W):
        raise ValueError(f"feanet_amd: pattern map must be uint8 [{H}, {W}]")
    return pid.contiguous()


def _bhw(x):
    if x.dim() < 2:
        raise ValueError("feanet_amd: field needs at least 2 dims (..., H, W)")
    H, W = x.shape[-2:]
    B = x.numel() // (H * W) if H * W else 0
    return B, H, W


def _knet_apply(u, ktab, pid=None):
    """y = K u with per-node-pattern stencils (KNet.forward, FEANet/model.py:22-30)."""
    u = _field(u, "u")
    B, H, W = _bhw(u)
    tab = _table(ktab, u.dtype, u.device)
    pid = _pid(pid, H, W, u.device)
    y = torch.empty_like(u)
    _lib.call("knet_apply", u.dtype, u.data_ptr(), y.data_ptr(), _ptr(pid), tab.data_ptr(), tab.shape[0],
              B, H, W, _stream(u))
    return y




def _split_x(x, pid, C):
    """x_split[:, p] = mask_p * x (KNet.split_x, FEANet/model.py:37-47); x is [B, 1, H, W]."""
    x = _field(x, "x")
    B, H, W = _bhw(x)
    pid = _pid(pid, H, W, x.device)
    out = torch.empty((B, C, H, W), dtype=x.dtype, device=x.device)
    _lib.call("split_x", x.dtype, x.data_ptr(), out.data_ptr(), _ptr(pid), C, B, H, W, _stream(x))
    return out


def _bcast_stride(t, B, H, W, name, dtype, device):
    if t is None:
        return None, 0
    t = _field(t, name, dtype)
    nb = t.numel() // (H * W)
    if tuple(t.shape[-2:]) != (H, W) or nb not in (1, B):
        raise ValueError(f"feanet_amd: {name} must be [1|B, 1, {H}, {W}]")
    return t, (0 if nb == 1 else H * W)


def _jacobi_sweep(u, f, ktab, omd, pid=None, geo=None, bc=None):
    """One weighted-Jacobi sweep with Dirichlet reset (JacobiBlock.jacobi_convolution,
    FEANet/jacobi.py:39-47).  geo/bc None = square domain / zero boundary values."""
    u = _field(u, "u")
    f = _field(f, "forcing_term", u.dtype)
    B, H, W = _bhw(u)
    if f.shape != u.shape:
        raise ValueError(f"feanet_amd: forcing term shape {tuple(f.shape)} != u shape {tuple(u.shape)}")
    tab = _table(ktab, u.dtype, u.device)
    om = torch.as_tensor(omd).to(device=u.device, dtype=u.dtype).reshape(-1).contiguous()
    if om.numel() != tab.shape[0]:
        raise ValueError("feanet_amd: omega/d table must have one entry per stencil pattern")
    pid = _pid(pid, H, W, u.device)
    geo, gs = _bcast_stride(geo, B, H, W, "geometry_idx", u.dtype, u.device)
    bc, bs = _bcast_stride(bc, B, H, W, "boundary_value", u.dtype, u.device)
    out = torch.empty_like(u)
    _lib.call("jacobi_sweep", u.dtype, u.data_ptr(), f.data_ptr(), out.data_ptr(), _ptr(pid), tab.data_ptr(),
              om.data_ptr(), tab.shape[0], _ptr(geo), gs, _ptr(bc), bs, B, H, W, _stream(u))
    return out


def _residual(u, f, ktab, pid=None):
    """r = f - K u."""
    u = _field(u, "u")
    f = _field(f, "f", u.dtype)
    B, H, W = _bhw(u)
    tab = _table(ktab, u.dtype, u.device)
    pid = _pid(pid, H, W, u.device)
    r = torch.empty_like(u)
    _lib.call("residual", u.dtype, u.data_ptr(), f.data_ptr(), r.data_ptr(), _ptr(pid), tab.data_ptr(),
              tab.shape[0], B, H, W, _stream(u))
    return r


def _restrict(x, rtab, w0=1.0, pid=None):
    """Restriction (RestrictionNet + MultiGrid.Restrict, FEANet/multigrid.py:50-60,115-122):
    x [B, C, H, W]; C > 1 means x is already split (one kernel per channel); C == 1 uses
    the kernel of each fine node's pattern (pid) or rtab[0]."""
    x = _field(x, "x")
    if x.dim() != 4:
        raise ValueError("feanet_amd: restrict expects [B, C, H, W]")
    B, C, H, W = x.shape
    tab = _table(rtab, x.dtype, x.device)
    if C > 1 and tab.shape[0] != C:
        raise ValueError(f"feanet_amd: split input has {C} channels but {tab.shape[0]} kernels")
    pid = _pid(pid, H, W, x.device) if C == 1 else None
    Hc, Wc = (H + 1) // 2, (W + 1) // 2
    out = torch.empty((B, 1, Hc, Wc), dtype=x.dtype, device=x.device)
    _lib.call("restrict", x.dtype, x.data_ptr(), C, out.data_ptr(), _ptr(pid), tab.data_ptr(), tab.shape[0],
              float(w0), B, H, W, _stream(x))
    return out


def _prolong(e, ptab, w1=1.0, pidc=None, add=None):
    """Prolongation (ProlongationNet + MultiGrid.Interpolate, FEANet/multigrid.py:62-73,124-130):
    out = add + w1 * conv_transpose2d(e, P, stride 2, pad 1); e [B, C, Hc, Wc]."""
    e = _field(e, "e")
    if e.dim() != 4:
        raise ValueError("feanet_amd: prolong expects [B, C, Hc, Wc]")
    B, C, Hc, Wc = e.shape
    tab = _table(ptab, e.dtype, e.device)
    if C > 1 and tab.shape[0] != C:
        raise ValueError(f"feanet_amd: split input has {C} channels but {tab.shape[0]} kernels")
    pidc = _pid(pidc, Hc, Wc, e.device) if C == 1 else None
    H, W = 2 * Hc - 1, 2 * Wc - 1
    if add is not None:
        add = _field(add, "add", e.dtype)
        if tuple(add.shape) != (B, 1, H, W):
            raise ValueError("feanet_amd: add must be [B, 1, 2Hc-1, 2Wc-1]")
    out = torch.empty((B, 1, H, W), dtype=e.dtype, device=e.device)
    _lib.call("prolong", e.dtype, e.data_ptr(), C, out.data_ptr(), _ptr(add), _ptr(pidc), tab.data_ptr(),
              tab.shape[0], float(w1), B, Hc, Wc, _stream(e))
    return out


def residual_norm(u, f=None, ktab=None, pid=None):
    """Per-sample ||(f - K u)[..., 1:-1, 1:-1]||_2 (or ||u[..., 1:-1, 1:-1]|| when f is None),
    float64 [B], deterministic."""
    u = _field(u, "u")
    B, H, W = _bhw(u)
    tab = None
    if f is not None:
        f = _field(f, "f", u.dtype)
        tab = _table(ktab, u.dtype, u.device)
        pid = _pid(pid, H, W, u.device)
    ws = torch.empty(max(1, _lib.norm_workspace_bytes(B, H, W) // 8), dtype=torch.float64, device=u.device)
    out = torch.empty(B, dtype=torch.float64, device=u.device)
    _lib.call("residual_norm", u.dtype, u.data_ptr(), _ptr(f), _ptr(pid) if f is not None else None,
              _ptr(tab), 0 if tab is None else tab.shape[0], out.data_ptr(), ws.data_ptr(), B, H, W, _stream(u))
    return out


# ---------------------------------------------------------------------------- public entry points
# The differentiable operators go through their PyTorch custom ops (torch.ops.feanet.*, torch_ops.py):
# the registered implementation is the HIP kernel call above, the registered autograd its HIP adjoint.

def _T():
    from . import torch_ops  # noqa: F401  (registers torch.ops.feanet.*)
    return torch.ops.feanet


def knet_apply(u, ktab, pid=None):
    """y = K u with per-node-pattern stencils (KNet.forward, FEANet/model.py:22-30)."""
    require_hip(u, "u")
    return _T().knet_apply(u, ktab, pid)


def conv3x3(x, w):
    """Single-channel 3x3 cross-correlation, zero padding (FNet.forward, HNet layers)."""
    return knet_apply(x, w, None)


def split_x(x, pid, C):
    """x_split[:, p] = mask_p * x (KNet.split_x, FEANet/model.py:37-47); x is [B, 1, H, W]."""
    require_hip(x, "x")
    return _T().split_x(x, pid, int(C))


def jacobi_sweep(u, f, ktab, omd, pid=None, geo=None, bc=None):
    """One weighted-Jacobi sweep with Dirichlet reset (JacobiBlock.jacobi_convolution,
    FEANet/jacobi.py:39-47).  geo/bc None = square domain / zero boundary values."""
    require_hip(u, "u")
    omd = torch.as_tensor(omd, device=u.device)
    return _T().jacobi_sweep(u, f, ktab, omd, pid, geo, bc)


def pbc_pad(u, lo, hi):
    """Circular extension of the periodic part u[..., :-1, :-1] (period N-1) to (N-1+lo+hi)^2:
    JacobiBlockPBC.pbc_boundary (FEANet/jacobi.py:72-79) is (1, 2), reset_boundary (:81-84) (0, 1)."""
    u = _field(u, "u")
    B, H, W = _bhw(u)
    if H != W:
        raise ValueError("feanet_amd: periodic fields are square")
    M = H - 1 + lo + hi
    out = torch.empty(u.shape[:-2] + (M, M), dtype=u.dtype, device=u.device)
    _lib.call("pbc_pad", u.dtype, u.data_ptr(), out.data_ptr(), B, H, lo, hi, _stream(u))
    return out


def jacobi_sweep_pbc(u, f, ktab, omd):
    """Periodic weighted-Jacobi sweep (JacobiBlockPBC.jacobi_convolution, FEANet/jacobi.py:86-97):
    u [.., N, N]; f the (N+2)^2 forcing term of the reference's drivers (FNet of the periodic
    extension); single-pattern stencil ktab; omd = omega/d."""
    u = _field(u, "u")
    f = _field(f, "forcing_term", u.dtype)
    B, H, W = _bhw(u)
    if H != W or f.shape[-2:] != (H + 2, W + 2) or f.numel() != B * (H + 2) * (W + 2):
        raise ValueError(f"feanet_amd: periodic sweep needs u [B,1,N,N] and f [B,1,N+2,N+2] "
                         f"(got {tuple(u.shape)}, {tuple(f.shape)})")
    tab = _table(ktab, u.dtype, u.device)
    if tab.shape[0] != 1:
        raise ValueError("feanet_amd: the periodic sweep is defined for homogeneous meshes (one stencil)")
    om = torch.as_tensor(omd).to(device=u.device, dtype=u.dtype).reshape(-1)[:1].contiguous()
    out = torch.empty_like(u)
    _lib.call("jacobi_sweep_pbc", u.dtype, u.data_ptr(), f.data_ptr(), out.data_ptr(), tab.data_ptr(),
              om.data_ptr(), B, H, _stream(u))
    return out


def residual(u, f, ktab, pid=None):
    """r = f - K u."""
    require_hip(u, "u")
    return _T().residual(u, f, ktab, pid)


def restrict(x, rtab, w0=1.0, pid=None):
    """Restriction (RestrictionNet + MultiGrid.Restrict, FEANet/multigrid.py:50-60,115-122):
    x [B, C, H, W]; C > 1 means x is already split (one kernel per channel); C == 1 uses
    the kernel of each fine node's pattern (pid) or rtab[0].  Differentiable in x and rtab."""
    require_hip(x, "x")
    return _T().restrict(x, rtab, float(w0), pid)


def prolong(e, ptab, w1=1.0, pidc=None, add=None):
    """Prolongation (ProlongationNet + MultiGrid.Interpolate, FEANet/multigrid.py:62-73,124-130):
    out = add + w1 * conv_transpose2d(e, P, stride 2, pad 1); e [B, C, Hc, Wc].
    Differentiable in e, ptab and add."""
    require_hip(e, "e")
    return _T().prolong(e, ptab, float(w1), pidc, add)
