"""oracle/torch_cpu.py — the reference's PyTorch-CPU formulation timed as bench.py's cpu_baseline —
against the numpy oracle and the reference-generated golden fixtures (CPU only)."""
import numpy as np
import pytest
import torch

from oracle import feanet_oracle as orc
from oracle.torch_cpu import TorchCPUMultigrid, TorchLevel


@pytest.mark.parametrize("case", ["poisson", "iface0"])
@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_ops_vs_golden(gold, case, dt):
    g = gold(f"ops_{case}_{dt}_n32.npz")
    T = torch.float32 if dt == "f32" else torch.float64
    lv = TorchLevel(g["ktab"], g["pid"], T, geo=torch.from_numpy(g["geo"]), bc=torch.from_numpy(g["bc"]))
    u = torch.from_numpy(g["u"])
    f = torch.from_numpy(g["f"])
    tol = dict(rtol=1e-5, atol=1e-5) if dt == "f32" else dict(rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(lv.knet(u).numpy(), g["knet"], **tol)
    np.testing.assert_allclose(lv.jacobi(u, f).numpy(), g["jacobi"], **tol)
    np.testing.assert_allclose(lv.d_mat.numpy()[0, 0], g["d_mat"][0, 0], rtol=0, atol=0)


@pytest.mark.parametrize("n,L", [(64, None), (256, None), (64, 3)])
def test_step_vs_oracle_f64(n, L):
    rng = np.random.default_rng(n)
    N = n + 1
    f = rng.standard_normal((1, 1, N, N))
    v0 = rng.standard_normal((1, 1, N, N))
    geo, _ = orc.square_geometry(N, np.float64)
    bc = rng.random((1, 1, N, N)) * (1 - geo)
    mt = TorchCPUMultigrid(n, levels=L)
    mt.set_boundary(geo, bc)
    mo = orc.OracleMultigrid(n, "poisson", np.float64, levels=L)
    mo.set_boundary(geo, bc[0, 0])
    a, b = torch.from_numpy(v0), v0
    for _ in range(3):
        a = mt.step(a, torch.from_numpy(f))
        b = mo.step(b, f)
    assert np.abs(a.numpy() - b).max() / np.abs(b).max() < 1e-12
    np.testing.assert_allclose(mt.residual_norm(a, torch.from_numpy(f)).numpy(), mo.residual_norm(b, f), rtol=1e-9)


def test_interface_step_vs_oracle():
    n = 64
    rng = np.random.default_rng(9)
    f = rng.standard_normal((2, 1, n + 1, n + 1))
    mt = TorchCPUMultigrid(n, problem="interface")
    mo = orc.OracleMultigrid(n, "interface", np.float64)
    a = mt.step(torch.zeros(2, 1, n + 1, n + 1, dtype=torch.float64), torch.from_numpy(f))
    b = mo.step(np.zeros_like(f), f)
    assert np.abs(a.numpy() - b).max() / np.abs(b).max() < 1e-12


@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_mg_test_synth65_history(gold, dt):
    """The reference's own mg_test Step history (golden, 65^2, L = 6) reproduced by the restatement."""
    g = gold("mg_test_synth65.npz")
    T = torch.float32 if dt == "f32" else torch.float64
    mt = TorchCPUMultigrid(64, dtype=T, levels=6)
    mt.set_boundary(g[f"{dt}_geo"], g[f"{dt}_bc"])
    f = torch.from_numpy(g[f"{dt}_fnet_f"])
    u = torch.zeros(1, 1, 65, 65, dtype=T)
    ref = g[f"{dt}_L6_hist"]
    hist = [float(mt.residual_norm(mt.levels[0].reset_boundary(u), f)[0])]
    for _ in range(len(ref) - 1):
        u = mt.step(u, f)
        hist.append(float(mt.residual_norm(u, f)[0]))
    n = 10
    np.testing.assert_allclose(hist[:n], ref[:n], rtol=1e-9 if dt == "f64" else 5e-4,
                               atol=(1e-12 if dt == "f64" else 1e-6) * ref[0])
