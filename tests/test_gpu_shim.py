"""The drop-in `FEANet` package (multigrid-feanet_amd/FEANet) used exactly as the reference's code
uses it — MeshSquare / MeshCenterInterface -> KNet / FNet / Geometry / JacobiBlock, and
FEANet/multigrid.py's MultiGrid — against the golden outputs of the reference run on the CPU
(tests/golden/ops_*.npz, multigrid_py_iface65.npz).  Tolerances as in test_gpu_ops.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = {"f32": 2e-6, "f64": 1e-13}


@pytest.fixture
def on_gpu():
    torch.set_default_device("cuda")
    yield
    torch.set_default_device("cpu")
    torch.set_default_dtype(torch.float32)


def close(out, ref, dt, what):
    out = out.detach().cpu().numpy().astype(np.float64)
    ref = np.asarray(ref, np.float64)
    assert out.shape == ref.shape, what
    err = np.abs(out - ref).max() / max(1.0, np.abs(ref).max())
    assert err <= TOL[dt], f"{what}: {err:.3e}"


@pytest.mark.parametrize("case", ["poisson", "iface0", "iface1"])
@pytest.mark.parametrize("dt", ["f32", "f64"])
@pytest.mark.parametrize("n", [16, 32])
def test_modules_vs_reference(gold, on_gpu, case, dt, n):
    from FEANet.geo import Geometry
    from FEANet.jacobi import JacobiBlock
    from FEANet.mesh import MeshCenterInterface, MeshSquare
    from FEANet.model import FNet, KNet
    g = gold(f"ops_{case}_{dt}_n{n}.npz")
    T = torch.float64 if dt == "f64" else torch.float32
    torch.set_default_dtype(T)
    N = n + 1
    mesh = MeshSquare(2, N) if case == "poisson" else MeshCenterInterface(2, [1, 20], N, 0 if case == "iface0" else 1)
    knet, fnet = KNet(mesh), FNet(2 / n)
    if dt == "f64":
        knet, fnet = knet.double(), fnet.double()
    geo = Geometry(N)
    bc = torch.from_numpy(g["bc"]).cuda()
    jac = JacobiBlock(knet, mesh, 2 / 3., geo.geometry_idx, bc)
    np.testing.assert_array_equal(jac.d_mat.cpu().numpy(), g["d_mat"])
    u, f, F = (torch.from_numpy(g[k]).cuda() for k in ("u", "f", "F"))
    close(knet(u), g["knet"], dt, "KNet")
    np.testing.assert_array_equal(knet.split_x(u).cpu().numpy(), g["split"])
    close(fnet(F), g["fnet"], dt, "FNet")
    j1 = jac.jacobi_convolution(u, f)
    close(j1, g["jacobi"], dt, "jacobi")
    close(jac.jacobi_convolution(j1, f), g["jacobi2"], dt, "jacobi2")
    # CPU tensors are refused, never silently computed on the host
    with pytest.raises(RuntimeError, match="MI355X"):
        knet(u.cpu())


@pytest.mark.parametrize("tag,ncyc", [("linear", 13), ("learned", 12)])
@pytest.mark.parametrize("path", ["fused", "modules"])
def test_multigrid_py_iterate(gold, on_gpu, tag, ncyc, path):
    """FEANet/multigrid.py MultiGrid.iterate at 65^2 (BASELINE config 3 operators): the fused solver
    path (no grad) and the module-level path (what autograd records) both follow the reference's
    residual history and cycle count."""
    import FEANet.multigrid as mgm
    g = gold("multigrid_py_iface65.npz")
    lin = torch.asarray([[1, 2, 1], [2, 4, 2], [1, 2, 1]], dtype=torch.float32)
    mg = mgm.MultiGrid(64, lin / 16.0, lin / 4.0, torch.tensor([4.0, 1.0]))
    with torch.no_grad():
        mg.conv.net.weight[0] = torch.from_numpy(g[f"{tag}_rtab"])
        mg.deconv.net.weight[:, 0] = torch.from_numpy(g[f"{tag}_ptab"])
        mg.w.copy_(torch.from_numpy(g[f"{tag}_w"]))
    f = torch.from_numpy(g["f"]).cuda()
    u = torch.zeros_like(f)
    knet = mg.grids[0].Knet
    hist = [float(torch.norm((f - knet(u))[:, :, 1:-1, 1:-1]))]
    with torch.no_grad() if path == "fused" else torch.enable_grad():
        while hist[-1] > 5e-5 and len(hist) < 40:
            u = mg.iterate(u, f) if path == "fused" else mg.iterate_modules(u, f).detach()
            hist.append(float(torch.norm((f - knet(u))[:, :, 1:-1, 1:-1])))
    assert len(hist) - 1 == ncyc
    np.testing.assert_allclose(hist[:8], g[f"{tag}_hist"][:8], rtol=3e-3, atol=1e-5 * hist[0])
    np.testing.assert_allclose(u.cpu().numpy(), g[f"{tag}_u"], atol=2e-4 * np.abs(g[f"{tag}_u"]).max())


@pytest.mark.parametrize("shape", [0, 1])
@pytest.mark.parametrize("T", [torch.float64, torch.float32])
def test_knet_padded_multi_pattern(shape, T):
    """KNet.forward / split_x on an (N+2)^2 input of a 16-pattern mesh: the reference pads every mask
    with 1 (FEANet/model.py:26-28, 42-46).  Against that formulation in CPU PyTorch (conv2d identity
    split, padded one-hot masks, conv2d stencils)."""
    import torch.nn.functional as Fn
    from FEANet.mesh import MeshCenterInterface
    from FEANet.model import KNet
    N = 17
    mesh = MeshCenterInterface(2, [1, 20], N, shape)
    kn = KNet(mesh).to(device="cuda", dtype=T)
    u = torch.randn(2, 1, N + 2, N + 2, dtype=T, generator=torch.Generator().manual_seed(shape))
    C = kn.n_channel
    w1 = kn.net1.weight.detach().cpu()
    w2 = kn.net2.weight.detach().cpu()
    gp = Fn.pad(kn.global_pattern.cpu().to(T), (1, 1, 1, 1), "constant", 1)
    split_ref = Fn.conv2d(u, w1, padding=1) * gp
    y_ref = Fn.conv2d(split_ref, w2, padding=1)
    tol = 1e-12 if T == torch.float64 else 2e-5
    y = kn(u.cuda())
    assert (y.cpu() - y_ref).abs().max() / y_ref.abs().max() < tol
    sx = kn.split_x(u.cuda())
    assert sx.shape == (2, C, N + 2, N + 2)
    assert torch.equal(sx.cpu(), split_ref)
