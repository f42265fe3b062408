"""torch.ops.feanet.* registration (feanet_amd.torch_ops): the ops exist, their fake (meta)
implementations give the reference's output shapes, and a CPU tensor finds no kernel (no fallback)."""
import pytest
import torch


def test_ops_registered_and_meta_shapes():
    import feanet_amd.torch_ops  # noqa: F401
    F = torch.ops.feanet
    m = dict(device="meta", dtype=torch.float64)
    u = torch.empty(2, 1, 9, 9, **m)
    k = torch.empty(1, 9, **m)
    assert F.knet_apply(u, k).shape == u.shape
    assert F.residual(u, u, k).shape == u.shape
    assert F.jacobi_sweep(u, u, k, torch.empty(1, **m)).shape == u.shape
    assert F.restrict(u, k, 1.0).shape == (2, 1, 5, 5)
    assert F.prolong(torch.empty(2, 1, 5, 5, **m), k, 1.0).shape == (2, 1, 9, 9)
    assert F.residual_norm(u).shape == (2,)
    assert F.pbc_pad(u, 1, 2).shape == (2, 1, 11, 11)
    assert F.jacobi_sweep_pbc(u, torch.empty(2, 1, 11, 11, **m), k, torch.empty(1, **m)).shape == u.shape


def test_cpu_tensor_has_no_kernel():
    import feanet_amd.torch_ops  # noqa: F401
    u = torch.zeros(1, 1, 5, 5, dtype=torch.float64)
    with pytest.raises(Exception):
        torch.ops.feanet.knet_apply(u, torch.zeros(1, 9, dtype=torch.float64))
