"""GPU parity of the fused learned-smoother sweep (fea_mg_hsweep) and of
the MG-HJac V-cycle (MultigridSolver(smoother="hjac"), M-FEANet-mg_test.ipynb MultiGrid mode='hjac').
The sweep is compared with the oracle's HRelax (pinned by the reference's golden HRelax outputs in
test_oracle_golden.py); the V-cycle with the reference's own recorded hjac residual histories."""
import numpy as np
import pytest
import torch

from oracle import feanet_oracle as orc

pytestmark = pytest.mark.gpu
TOL = {torch.float32: 2e-5, torch.float64: 1e-12}


def npdt(T):
    return np.float32 if T == torch.float32 else np.float64


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("m,n,B", [(32, 32, 2), (64, 64, 1), (16, 256, 1), (300, 130, 2), (128, 128, 3)])
@pytest.mark.parametrize("zero", [False, True])
def test_hsweep_vs_oracle(T, problem, m, n, B, zero):
    from feanet_amd import _lib, mesh_setup as ms
    from feanet_amd.solver import _Level
    if problem == "interface" and m != n:
        pytest.skip("two-material problem is square")
    rng = np.random.default_rng(m * 7 + n + B)
    H, W = m + 1, n + 1
    pid = ms.interface_pattern_map(H) if problem == "interface" else np.zeros((H, W), np.uint8)
    L = _Level(m, n, B, T, torch.device("cuda"), pid if problem == "interface" else None)
    ktab = ms.stencil_table((1, 20) if problem == "interface" else None)
    omd = ms.omega_over_d(ktab, 2 / 3., npdt(T))
    hw = (0.3 * rng.standard_normal((3, 3, 3))).astype(np.float32)
    geo, _ = orc.square_geometry((H, W), npdt(T))
    u = rng.standard_normal((B, H, W)).astype(npdt(T))
    if zero:
        u[:] = 0
    f = rng.standard_normal((B, H, W)).astype(npdt(T))
    L.view(L.a).copy_(torch.from_numpy(u))
    L.view(L.f).copy_(torch.from_numpy(f))
    L.view(L.b).fill_(7.0)
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda().to(T)
    kt, om, hwt = cu(ktab.reshape(-1, 9)), cu(omd), cu(hw.reshape(-1))
    _lib.call("mg_hsweep", T, None if zero else L.a.data_ptr(), None, L.f.data_ptr(), L.b.data_ptr(),
              None if L.pid is None else L.pid.data_ptr(), kt.data_ptr(), om.data_ptr(), ktab.shape[0],
              hwt.data_ptr(), 3, *L.geom(), None)
    out = L.view(L.b).cpu().numpy()
    lvl = orc.Level(n, problem, npdt(T), m=m)
    lvl.bc = u * (1 - geo)  # the framed invariant: boundary nodes hold the Dirichlet values
    ref = orc.hnet_relax(u, f, lvl, hw, 1)
    err = np.abs(out[:, 1:-1, 1:-1] - ref[:, 1:-1, 1:-1]).max() / max(1.0, np.abs(ref).max())
    assert err < TOL[T], err
    assert (out[:, 0] == 7).all() and (out[:, -1] == 7).all() and (out[:, :, 0] == 7).all()


def test_hsweep_golden_hrelax(gold):
    """The reference's own HRelax outputs (HJacIterator.HRelax on a random, un-reset u, zero Dirichlet
    data, 33^2, fp32): one fused sweep with u_raw = the caller's u, then two more sweeps."""
    from feanet_amd import _lib, mesh_setup as ms
    from feanet_amd.solver import _Level
    g = gold("mg_test_isopoisson33.npz")
    u, f = g["hrelax_u"][:, 0], g["hrelax_f"][:, 0]
    B = u.shape[0]
    L = _Level(32, 32, B, torch.float32, torch.device("cuda"))
    geo, _ = orc.square_geometry(33)
    L.view(L.a).copy_(torch.from_numpy(u * geo))     # reset_boundary (zero bc)
    L.view(L.buf("zero")).copy_(torch.from_numpy(u))  # the caller's un-reset u
    L.view(L.f).copy_(torch.from_numpy(f))
    ktab = ms.stencil_table(None)
    kt = torch.from_numpy(ktab.reshape(-1, 9)).cuda()
    om = torch.from_numpy(ms.omega_over_d(ktab, 2 / 3., np.float32)).cuda()
    hw = torch.from_numpy(g["hnet_w"].reshape(-1).astype(np.float32)).cuda()
    args = (kt.data_ptr(), om.data_ptr(), 1, hw.data_ptr(), 3, *L.geom(), None)
    _lib.call("mg_hsweep", torch.float32, L.a.data_ptr(), L.buf("zero").data_ptr(), L.f.data_ptr(), L.b.data_ptr(),
              None, *args)
    np.testing.assert_allclose(L.view(L.b).cpu().numpy()[:, 1:-1, 1:-1], g["hrelax_out1"][:, 0, 1:-1, 1:-1],
                               rtol=1e-4, atol=1e-5)
    _lib.call("mg_hsweep", torch.float32, L.b.data_ptr(), None, L.f.data_ptr(), L.a.data_ptr(), None, *args)
    _lib.call("mg_hsweep", torch.float32, L.a.data_ptr(), None, L.f.data_ptr(), L.b.data_ptr(), None, *args)
    np.testing.assert_allclose(L.view(L.b).cpu().numpy()[:, 1:-1, 1:-1], g["hrelax_out3"][:, 0, 1:-1, 1:-1],
                               rtol=1e-4, atol=1e-5)


def test_hjac_vcycle_golden(gold):
    """MG-HJac on the reference's IsoPoisson 33^2 samples: the reference's cycle count and residual
    history (fp32 tolerance as the oracle's own golden test)."""
    from feanet_amd.solver import MultigridSolver
    g = gold("mg_test_isopoisson33.npz")
    w = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "multigrid-feanet_amd",
                                             "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
    hw = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
    assert np.abs(hw - g["hnet_w"]).max() == 0
    for k in range(3):
        s = MultigridSolver(32, dtype=torch.float32, smoother="hjac", hnet=hw)
        s.set_boundary(torch.from_numpy(g["boundary_value"][k]).float().cuda())
        u, hist = s.solve(F=torch.from_numpy(g["rhs"][k]).float().cuda(), eps=5e-5, max_cycles=60)
        hist = np.array([h[0] for h in hist])
        ref = g[f"hjac_hist_{k}"]
        assert len(hist) == len(ref), (hist, ref)
        np.testing.assert_allclose(hist[:5], ref[:5], rtol=5e-4, atol=1e-6 * ref[0])


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
def test_hjac_vcycle_vs_oracle(T):
    """The hjac schedule against the oracle's Step with every sweep replaced by HRelax (129^2, B=2)."""
    from feanet_amd.solver import MultigridSolver
    n, B = 128, 2
    rng = np.random.default_rng(11)
    hw = (0.2 * rng.standard_normal((3, 3, 3))).astype(np.float32)
    mg = orc.OracleMultigrid(n, "poisson", npdt(T))
    for l in mg.levels:
        l.sweep = (lambda ll, o: (lambda v, ff: (lambda j: j + orc.hnet(j - v, ll.geo, hw))(o(v, ff))))(l, l.sweep)
    f = rng.standard_normal((B, n + 1, n + 1)).astype(npdt(T))
    s = MultigridSolver(n, dtype=T, batch=B, smoother="hjac", hnet=hw)
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(B, 1, n + 1, n + 1))
    s.load()
    v = np.zeros((B, n + 1, n + 1), npdt(T))
    for k in range(3):
        s.vcycle()
        v = mg.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        if T == torch.float64 or k == 0:
            err = np.abs(got - v).max() / max(1.0, np.abs(v).max())
            assert err < (1e-10 if T == torch.float64 else 5e-5), (k, err)
