"""Pin the CPU oracle (oracle/feanet_oracle.py) against golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import feanet_oracle as orc

TOL = {"f32": dict(rtol=2e-5, atol=2e-5), "f64": dict(rtol=1e-12, atol=1e-12)}


def _scale_close(a, b, dt, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, np.abs(b).max())
    tol = 2e-6 if dt == "f32" else 1e-13
    err = np.abs(a - b).max() / scale
    assert err <= tol, f"{what}: max err {err:.3e} (scaled) > {tol}"


def test_tables(gold):
    t = gold("tables.npz")
    ktab, pid = orc.square_mesh(9)
    np.testing.assert_array_equal(ktab, t["square_kernel"])
    for shape in (0, 1):
        for n in (5, 9, 17, 33, 65, 129):
            ktab, pid = orc.interface_mesh(n, (1, 20), shape)
            np.testing.assert_array_equal(ktab, t[f"iface{shape}_kernel_{n}"])
            np.testing.assert_array_equal(pid, t[f"iface{shape}_pid_{n}"], err_msg=f"shape {shape} N {n}")
    ktab, _ = orc.interface_mesh(17, (3, 7), 0)
    np.testing.assert_array_equal(ktab, t["iface0_prop3_7_kernel"])
    for n in (2, 4, 16, 32, 64, 128, 4096):
        np.testing.assert_array_equal(orc.fnet_stencil(2 / n), t[f"fnet_{n}"])
    geo, bc = orc.square_geometry(17)
    np.testing.assert_array_equal(geo, t["geo_17"][0, 0])
    np.testing.assert_array_equal(bc, t["bc_17"][0, 0])


CASES = [(c, dt, n) for c in ("poisson", "iface0", "iface1") for dt in ("f32", "f64") for n in (16, 32)]


@pytest.mark.parametrize("case,dt,n", CASES)
def test_ops(gold, case, dt, n):
    g = gold(f"ops_{case}_{dt}_n{n}.npz")
    u, f, F = g["u"], g["f"], g["F"]
    pid, ktab = g["pid"], g["ktab"]
    _scale_close(orc.knet_apply(u, pid, ktab), g["knet"], dt, "knet")
    np.testing.assert_array_equal(orc.split_x(u, pid, len(ktab)), g["split"])
    _scale_close(orc.conv3x3(F, orc.fnet_stencil(2 / n)), g["fnet"], dt, "fnet")
    geo, bc = g["geo"], g["bc"]
    _scale_close(orc.jacobi_sweep(u, f, pid, ktab, geo, bc), g["jacobi"], dt, "jacobi")
    j1 = orc.jacobi_sweep(u, f, pid, ktab, geo, bc)
    _scale_close(orc.jacobi_sweep(j1, f, pid, ktab, geo, bc), g["jacobi2"], dt, "jacobi2")
    _scale_close(orc.residual(u, f, pid, ktab), g["residual"], dt, "residual")
    r = g["residual"]
    if case == "poisson":
        lin = np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32)
        _scale_close(orc.restrict(r, pid, (lin / 4)[None]), g["restrict_mgtest"], dt, "restrict mg_test")
        _scale_close(orc.prolong(g["e_c"], np.zeros(g["e_c"].shape[-2:], np.uint8), (lin / 4)[None]),
                     g["prolong_mgtest"], dt, "prolong mg_test")
        if dt == "f32":
            _scale_close(orc.restrict(r, pid, (lin / 16)[None], 4.0), g["restrict_mm"], dt, "restrict MM")
            up = orc.bilinear_upsample(g["e_c"]) * geo  # MM levels use zero bc
            _scale_close(up, g["interp_mm"], dt, "interp MM")
    else:
        w = g["w"]
        _scale_close(orc.restrict(r, pid, g["rtab"], w[0]), g["restrict_learned"], dt, "restrict learned")
        _scale_close(orc.prolong(g["e_c"], g["pid_c"], g["ptab"], w[1]), g["prolong_learned"], dt,
                     "prolong learned")


def _hist_close(ours, ref, ncmp, rtol, floor=1e-6):
    """Residual histories: relative agreement, plus an absolute floor tied to the first residual
    (fp32 summation-order noise does not shrink with the residual)."""
    ours = np.asarray(ours)
    ref = np.asarray(ref)
    k = min(ncmp, len(ref), len(ours))
    np.testing.assert_allclose(ours[:k], ref[:k], rtol=rtol, atol=floor * abs(ref[0]))


def run_step_hist(mg, u, f, eps, maxc):
    hist = [float(mg.residual_norm(mg_reset(mg, u), f)[0])]
    while hist[-1] > eps and len(hist) < maxc:
        u = mg.step(u, f)
        hist.append(float(mg.residual_norm(u, f)[0]))
    return np.array(hist), u


def mg_reset(mg, u):
    lv = mg.levels[0]
    return u * lv.geo + lv.bc


def test_mg_test_isopoisson(gold):
    g = gold("mg_test_isopoisson33.npz")
    for k in range(3):
        mg = orc.OracleMultigrid(32, "poisson", np.float32)
        geo = g["boundary_index"][k].astype(np.float32)
        bc = g["boundary_value"][k].astype(np.float32)
        mg.set_boundary(geo, bc)
        F = g["rhs"][k].astype(np.float32)[None, None]
        f = orc.conv3x3(F, orc.fnet_stencil(2 / 32))
        np.testing.assert_allclose(f, g[f"jac_fnet_f_{k}"], rtol=1e-5, atol=1e-7)
        u0 = np.zeros((1, 1, 33, 33), np.float32)
        hist, u = run_step_hist(mg, u0, f, 5e-5, 60)
        ref = g[f"jac_hist_{k}"]
        assert len(hist) == len(ref)
        _hist_close(hist, ref, 6, 2e-4)
        np.testing.assert_allclose(mg.step(u0, f), g[f"jac_u_first_{k}"], rtol=1e-4, atol=1e-6)
        # MG solution reaches the dataset's direct solve (1e-6 .. 8e-6)
        assert np.abs(u[0, 0] - g["u"][k]).max() < 2e-5
        # hjac: learned smoother on every level
        hw = g["hnet_w"]
        lv = mg.levels
        orig = [l.sweep for l in lv]
        for l in lv:
            l.sweep = (lambda ll, o: (lambda v, ff: (lambda j: j + orc.hnet(j - v, ll.geo, hw))(o(v, ff))))(l, l.sweep)
        hist, _ = run_step_hist(mg, u0, f, 5e-5, 60)
        ref = g[f"hjac_hist_{k}"]
        assert len(hist) == len(ref)
        _hist_close(hist, ref, 5, 5e-4)
        for l, o in zip(lv, orig):
            l.sweep = o


def test_hrelax(gold):
    g = gold("mg_test_isopoisson33.npz")
    lvl = orc.Level(32)
    np.testing.assert_allclose(orc.hnet_relax(g["hrelax_u"], g["hrelax_f"], lvl, g["hnet_w"], 1),
                               g["hrelax_out1"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(orc.hnet_relax(g["hrelax_u"], g["hrelax_f"], lvl, g["hnet_w"], 3),
                               g["hrelax_out3"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dt", ["f32", "f64"])
def test_mg_test_synth65(gold, dt):
    g = gold("mg_test_synth65.npz")
    npdt = np.float32 if dt == "f32" else np.float64
    F = g[f"{dt}_F"].astype(npdt)[None, None]
    f = orc.conv3x3(F, orc.fnet_stencil(2 / 64))
    _scale_close(f, g[f"{dt}_fnet_f"], dt, "fnet")
    for L in (6, 3):
        mg = orc.OracleMultigrid(64, "poisson", npdt, levels=L)
        mg.set_boundary(g[f"{dt}_geo"], g[f"{dt}_bc"])
        u0 = np.zeros((1, 1, 65, 65), npdt)
        eps = 1e-9 if dt == "f64" else 5e-6
        hist, u = run_step_hist(mg, u0, f, eps, 40 if L == 6 else 25)
        ref = g[f"{dt}_L{L}_hist"]
        assert abs(len(hist) - len(ref)) <= (0 if dt == "f64" else 1)
        _hist_close(hist, ref, 10, 1e-9 if dt == "f64" else 5e-4, 1e-12 if dt == "f64" else 1e-6)


def test_mm_convergence(gold):
    g = gold("mm_convergence.npz")
    for n in (16, 32, 64):
        for nu in ((1, 1), (0, 1), (1, 0), (2, 1), (1, 2), (2, 2), (0, 2), (2, 0)):
            key = f"n{n}_v{nu[0]}{nu[1]}"
            mg = orc.OracleMultigrid(n, "poisson", np.float32)
            v = g[key + "_init"].reshape(1, 1, n + 1, n + 1)
            f = np.zeros_like(v)
            hist = []
            for _ in range(10):
                v = mg.rec_vcycle(v, f, *nu)
                hist.append(float(mg.residual_norm(v, f)[0]))
            _hist_close(hist, g[key + "_hist"], 6, 2e-3)
        mg = orc.OracleMultigrid(n, "poisson", np.float32, levels=3)
        v = g[f"n{n}_L3_init"].reshape(1, 1, n + 1, n + 1)
        hist = []
        for _ in range(10):
            v = mg.rec_vcycle(v, np.zeros_like(v))
            hist.append(float(mg.residual_norm(v, np.zeros_like(v))[0]))
        _hist_close(hist, g[f"n{n}_L3_hist"], 6, 2e-3)


def test_mm_interface(gold):
    g = gold("mm_interface65.npz")
    rec = gold("recorded_outputs.npz")
    mg = orc.OracleMultigrid(64, "interface", np.float32)
    f = orc.conv3x3(np.ones((1, 1, 65, 65), np.float32), orc.fnet_stencil(2 / 64))
    _scale_close(f, g["f"], "f32", "f")
    v = np.zeros_like(f)
    hist = []
    while (not hist or hist[-1] > 5e-5) and len(hist) < 40:
        v = mg.rec_vcycle(v, f, 1, 1, compat_q2=True)
        hist.append(float(mg.residual_norm(v, f)[0]))
    assert len(hist) == len(g["hist"]) == 14
    _hist_close(hist, g["hist"], 8, 1e-3)
    # the notebook's own stored output (MM_Interface_error.ipynb cell 14)
    _hist_close(hist, rec["mm_interface_res"], 6, 2e-3)


def test_multigrid_py(gold):
    g = gold("multigrid_py_iface65.npz")
    for l in range(6):
        _, pid = orc.interface_mesh((64 >> l) + 1)
        np.testing.assert_array_equal(pid, g[f"pid_level{l}"])
    for tag in ("linear", "learned"):
        mg = orc.OracleMultigrid(64, "interface", np.float32, rtab=g[f"{tag}_rtab"], ptab=g[f"{tag}_ptab"],
                                 w=tuple(float(x) for x in g[f"{tag}_w"]))
        f = g["f"]
        v = np.zeros_like(f)
        hist = [float(mg.residual_norm(v, f)[0])]
        while hist[-1] > 5e-5 and len(hist) < 40:
            v = mg.step(v, f)
            hist.append(float(mg.residual_norm(v, f)[0]))
        assert len(hist) == len(g[f"{tag}_hist"])
        _hist_close(hist, g[f"{tag}_hist"], 8, 1e-3)


@pytest.mark.parametrize("tag", ["f32", "f64"])
@pytest.mark.parametrize("n", [8, 16, 32])
def test_oracle_pbc_jacobi(gold, tag, n):
    """Periodic Jacobi (JacobiBlockPBC, FEANet/jacobi.py:50-97) against the reference's own outputs."""
    g = gold("pbc_jacobi.npz")
    ktab, _ = orc.square_mesh(n + 1)
    u, f = g[f"{tag}_n{n}_u"], g[f"{tag}_n{n}_f"]
    np.testing.assert_array_equal(orc.pbc_pad(u, 1, 2), g[f"{tag}_n{n}_pbc"])
    np.testing.assert_array_equal(orc.pbc_pad(u, 0, 1), g[f"{tag}_n{n}_reset"])
    tol = 1e-5 if tag == "f32" else 1e-13
    u1 = orc.jacobi_sweep_pbc(u, f, ktab)
    np.testing.assert_allclose(u1, g[f"{tag}_n{n}_u1"], rtol=0, atol=tol * max(1, np.abs(u1).max()))
    u3 = orc.jacobi_sweep_pbc(orc.jacobi_sweep_pbc(u1, f, ktab), f, ktab)
    np.testing.assert_allclose(u3, g[f"{tag}_n{n}_u3"], rtol=0, atol=tol * max(1, np.abs(u3).max()))
    # the periodic driver's residual history (FEANet-periodic.ipynb cells 2, 5)
    v = np.zeros_like(u[:1])
    hist = []
    for _ in range(30):
        v = orc.jacobi_sweep_pbc(v, f[:1], ktab)
        r = f[:1] - orc.knet_apply(orc.pbc_pad(v, 1, 2), np.zeros((n + 3, n + 3), np.uint8), ktab)
        hist.append(orc.interior_norm(r).sum())
    np.testing.assert_allclose(hist, g[f"{tag}_n{n}_hist"], rtol=1e-4 if tag == "f32" else 1e-10)
