"""torch.ops.feanet.* on the MI355X: each custom op returns exactly what the feanet_amd.ops kernel
call returns (same HIP kernel), torch.library.opcheck passes, and the registered autograd of
knet_apply / residual equals the autograd.Function path (HIP adjoints)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _data(T=torch.float64, B=2, N=33, seed=0):
    from oracle import feanet_oracle as orc
    rng = np.random.default_rng(seed)
    u = torch.from_numpy(rng.standard_normal((B, 1, N, N))).cuda().to(T)
    f = torch.from_numpy(rng.standard_normal((B, 1, N, N))).cuda().to(T)
    ktab, _ = orc.square_mesh(N)
    k = torch.from_numpy(np.asarray(ktab)).reshape(1, 9).cuda().to(T)
    return u, f, k


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
def test_custom_ops_equal_kernel_calls(T):
    import feanet_amd.torch_ops  # noqa: F401
    from feanet_amd import ops
    F = torch.ops.feanet
    u, f, k = _data(T)
    omd = torch.tensor([0.25], dtype=T, device="cuda")
    assert torch.equal(F.knet_apply(u, k), ops._knet_apply(u, k))
    assert torch.equal(F.residual(u, f, k), ops._residual(u, f, k))
    assert torch.equal(F.jacobi_sweep(u, f, k, omd), ops._jacobi_sweep(u, f, k, omd))
    r = F.restrict(u, k, 0.5)
    assert torch.equal(r, ops._restrict(u, k, 0.5))
    assert torch.equal(F.prolong(r, k, 2.0), ops._prolong(r, k, 2.0))
    assert torch.equal(F.residual_norm(u, f, k), ops.residual_norm(u, f, k))
    up = u[..., :17, :17].contiguous()
    assert torch.equal(F.pbc_pad(up, 1, 2), ops.pbc_pad(up, 1, 2))
    fp = ops.pbc_pad(up, 1, 2)
    assert torch.equal(F.jacobi_sweep_pbc(up, fp, k, omd), ops.jacobi_sweep_pbc(up, fp, k, omd))


def test_opcheck():
    import feanet_amd.torch_ops  # noqa: F401
    u, f, k = _data(torch.float64, N=17)
    F = torch.ops.feanet
    omd = torch.tensor([0.25], dtype=torch.float64, device="cuda")
    torch.library.opcheck(F.knet_apply.default, (u, k))
    torch.library.opcheck(F.residual.default, (u, f, k))
    torch.library.opcheck(F.restrict.default, (u, k, 1.0))
    torch.library.opcheck(F.jacobi_sweep.default, (u, f, k, omd))
    torch.library.opcheck(F.prolong.default, (F.restrict(u, k, 1.0), k, 1.0))
    pid = (torch.arange(17 * 17, device="cuda") % 3).to(torch.uint8).reshape(17, 17)
    torch.library.opcheck(F.split_x.default, (u, pid, 3))


def test_all_differentiable_ops_match_functions():
    """Every op with registered autograd (the product path of feanet_amd.ops and the FEANet modules) gives
    the gradients of the autograd.Function reference path, bitwise."""
    import feanet_amd.torch_ops  # noqa: F401
    from feanet_amd import autograd as ag
    u, f, k = _data(torch.float64, N=17, seed=4)
    F = torch.ops.feanet
    omd = torch.tensor([0.25], dtype=torch.float64, device="cuda")
    pid = (torch.arange(17 * 17, device="cuda") % 3).to(torch.uint8).reshape(17, 17)
    for which in ("jacobi", "split", "restrict", "prolong"):
        grads = []
        for path in ("custom", "function"):
            uu, kk, ff = u.clone().requires_grad_(), k.clone().requires_grad_(), f.clone().requires_grad_()
            if which == "jacobi":
                y = F.jacobi_sweep(uu, ff, kk, omd) if path == "custom" else \
                    ag.JacobiSweep.apply(uu, ff, kk, omd, None, None, None)
            elif which == "split":
                y = F.split_x(uu, pid, 3) if path == "custom" else ag.SplitX.apply(uu, pid, 3)
            elif which == "restrict":
                y = F.restrict(uu, kk, 0.5) if path == "custom" else ag.Restrict.apply(uu, kk, 0.5, None)
            else:
                e = uu[..., :9, :9]
                y = F.prolong(e, kk, 1.5) if path == "custom" else ag.Prolong.apply(e, kk, 1.5, None, None)
            y.backward(torch.ones_like(y))
            grads.append([t.grad for t in (uu, kk, ff)])
        for a, b in zip(*grads):
            assert (a is None and b is None) or torch.equal(a, b), which


def test_registered_autograd_matches_function():
    import feanet_amd.torch_ops  # noqa: F401
    from feanet_amd import ops
    u, f, k = _data(torch.float64, N=17, seed=3)
    g = torch.randn_like(u)
    grads = []
    for path in ("custom", "function"):
        uu, kk, ff = u.clone().requires_grad_(), k.clone().requires_grad_(), f.clone().requires_grad_()
        if path == "custom":
            y = torch.ops.feanet.knet_apply(uu, kk) + torch.ops.feanet.residual(uu, ff, kk)
        else:
            y = ops.knet_apply(uu, kk) + ops.residual(uu, ff, kk)
        y.backward(g)
        grads.append((uu.grad, kk.grad, ff.grad))
    for a, b in zip(*grads):
        assert torch.equal(a, b)
