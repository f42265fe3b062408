"""GPU parity of the generic C-ABI operators (fea_knet_apply, fea_split_x, fea_jacobi_sweep,
fea_residual, fea_restrict, fea_prolong, fea_residual_norm) against the golden vectors produced
by the reference and against the CPU oracle.

Tolerances (north star: results match the reference PyTorch CPU path): fp64 1e-13 and fp32 2e-6,
both relative to max(1, max|expected|), i.e. summation-order rounding only."""
import numpy as np
import pytest
import torch

from oracle import feanet_oracle as orc

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "f64": torch.float64}
TOL = {"f32": 2e-6, "f64": 1e-13}


def dev(x, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    return t.to(dt) if dt is not None else t


def close(out, ref, dt, what):
    out = out.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(out) else np.asarray(out, np.float64)
    ref = np.asarray(ref, np.float64)
    assert out.shape == ref.shape, f"{what}: shape {out.shape} vs {ref.shape}"
    err = np.abs(out - ref).max() / max(1.0, np.abs(ref).max())
    assert err <= TOL[dt], f"{what}: scaled max err {err:.3e} > {TOL[dt]}"


CASES = [(c, dt, n) for c in ("poisson", "iface0", "iface1") for dt in ("f32", "f64") for n in (16, 32)]


@pytest.mark.parametrize("case,dt,n", CASES)
def test_ops_vs_reference_golden(gold, case, dt, n):
    from feanet_amd import ops
    g = gold(f"ops_{case}_{dt}_n{n}.npz")
    T = DT[dt]
    u, f, F = dev(g["u"], T), dev(g["f"], T), dev(g["F"], T)
    ktab = dev(g["ktab"], T)
    multi = case != "poisson"
    pid = dev(g["pid"]) if multi else None
    close(ops.knet_apply(u, ktab, pid), g["knet"], dt, "knet")
    np.testing.assert_array_equal(ops.split_x(u, pid, len(g["ktab"])).cpu().numpy(), g["split"])
    close(ops.conv3x3(F, dev(orc.fnet_stencil(2 / n), T)), g["fnet"], dt, "fnet")
    omd = dev(orc.omega_over_d(g["ktab"], 2 / 3., np.float32 if dt == "f32" else np.float64), T)
    geo, bc = dev(g["geo"], T), dev(g["bc"], T)
    j1 = ops.jacobi_sweep(u, f, ktab, omd, pid, geo, bc)
    close(j1, g["jacobi"], dt, "jacobi")
    close(ops.jacobi_sweep(j1, f, ktab, omd, pid, geo, bc), g["jacobi2"], dt, "jacobi2")
    close(ops.residual(u, f, ktab, pid), g["residual"], dt, "residual")
    r = dev(g["residual"], T)
    e_c = dev(g["e_c"], T)
    lin = np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32)
    if not multi:
        close(ops.restrict(r, dev(lin / 4, T)), g["restrict_mgtest"], dt, "restrict mg_test")
        close(ops.prolong(e_c, dev(lin / 4, T)), g["prolong_mgtest"], dt, "prolong mg_test")
    else:
        w = g["w"]
        split = ops.split_x(r, pid, 16)
        close(ops.restrict(split, dev(g["rtab"], T), float(w[0])), g["restrict_learned"], dt, "restrict learned")
        close(ops.restrict(r, dev(g["rtab"], T), float(w[0]), pid), g["restrict_learned"], dt, "restrict by pid")
        pidc = dev(g["pid_c"])
        close(ops.prolong(ops.split_x(e_c, pidc, 16), dev(g["ptab"], T), float(w[1])), g["prolong_learned"], dt,
              "prolong learned")
        close(ops.prolong(e_c, dev(g["ptab"], T), float(w[1]), pidc), g["prolong_learned"], dt, "prolong by pid")
    nr = ops.residual_norm(u, f, ktab, pid).cpu().numpy()
    np.testing.assert_allclose(nr, orc.interior_norm(g["residual"]), rtol=1e-5 if dt == "f32" else 1e-12)


@pytest.mark.parametrize("dt", ["f32", "f64"])
@pytest.mark.parametrize("N,B", [(3, 1), (5, 2), (65, 3), (257, 2), (1025, 1)])
def test_ops_vs_oracle_sizes(dt, N, B):
    """Odd sizes around the 64-wide block edges, batches, both problem kinds."""
    from feanet_amd import ops
    T = DT[dt]
    npdt = np.float32 if dt == "f32" else np.float64
    rng = np.random.default_rng(N * 7 + B)
    u = rng.standard_normal((B, 1, N, N)).astype(npdt)
    f = rng.standard_normal((B, 1, N, N)).astype(npdt)
    for problem in ("poisson", "interface"):
        if problem == "poisson":
            ktab, pid = orc.square_mesh(N)
        else:
            ktab, pid = orc.interface_mesh(N) if N <= 257 else (None, None)
            if ktab is None:
                continue
        pt = dev(pid) if problem == "interface" else None
        kt = dev(ktab, T)
        close(ops.knet_apply(dev(u), kt, pt), orc.knet_apply(u, pid, ktab), dt, f"knet {problem} N={N}")
        geo, bc = orc.square_geometry(N, npdt)
        bc[0, :] = 0.5
        omd = orc.omega_over_d(ktab, 2 / 3., npdt)
        close(ops.jacobi_sweep(dev(u), dev(f), kt, dev(omd), pt, dev(geo), dev(bc)),
              orc.jacobi_sweep(u, f, pid, ktab, geo, bc), dt, f"jacobi {problem} N={N}")
        close(ops.jacobi_sweep(dev(u), dev(f), kt, dev(omd), pt), orc.jacobi_sweep(u, f, pid, ktab, geo, 0 * bc), dt,
              f"jacobi square/zero {problem} N={N}")
        if N >= 5:
            lin = np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32) / 4
            close(ops.restrict(dev(u), dev(lin, T), 1.5), orc.restrict(u, pid, lin[None], 1.5), dt, "restrict")
            Nc = (N + 1) // 2
            e = rng.standard_normal((B, 1, Nc, Nc)).astype(npdt)
            close(ops.prolong(dev(e), dev(lin, T), 0.75, add=dev(u)), u + orc.prolong(e, np.zeros((Nc, Nc), np.uint8),
                                                                                     lin[None], 0.75), dt, "prolong")


def test_cpu_tensor_raises():
    from feanet_amd import ops
    with pytest.raises(RuntimeError):
        ops.knet_apply(torch.zeros(1, 1, 5, 5), torch.zeros(1, 9).cuda())
