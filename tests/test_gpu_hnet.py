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


def test_hjac_vcycle_vs_oracle_full_size():
    """The MG-HJac cycle exactly as `bench.py --smoother hjac` times it — 4097^2 fp64, L = 12, the shipped HNet
    weights, the fused schedule (hsweep + restriction, prolongation + hsweep), the fine-level task heights and
    6-step bodies, staged weight loads, the LDS-resident HJac tail — against the oracle's MultiGrid.Step with every
    sweep an HRelax (M-FEANet-mg_test.ipynb:147-155, :27346-27372): three cycles from zero, 1e-10 of max|u| after
    each (~13 s per oracle cycle on the host)."""
    import os
    from feanet_amd.solver import MultigridSolver
    n = 4096
    w = np.load(os.path.join(os.path.dirname(__file__), "..", "multigrid-feanet_amd", "feanet_amd", "weights",
                             "hnet_iso_poisson_33x33.npz"))
    hw = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
    mg = orc.OracleMultigrid(n, "poisson", np.float64)
    for l in mg.levels:
        l.sweep = (lambda ll, o: (lambda v, ff: (lambda j: j + orc.hnet(j - v, ll.geo, hw))(o(v, ff))))(l, l.sweep)
    rng = np.random.default_rng(4097)
    f = rng.standard_normal((1, n + 1, n + 1))
    s = MultigridSolver(n, dtype=torch.float64, smoother="hjac", hnet=hw)
    assert s.L == 12
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(1, 1, n + 1, n + 1))
    s.load()
    v = np.zeros_like(f)
    for k in range(3):
        s.vcycle()
        v = mg.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        err = np.abs(got - v).max() / max(1.0, np.abs(v).max())
        assert err < 1e-10, (k, err)


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,n", [("poisson", 1024), ("poisson", 2048), ("interface", 1024)])
def test_hsweep_vs_oracle_large(T, problem, n):
    """fea_mg_hsweep at the sizes the 4097^2 V-cycle's top levels run (1025^2, 2049^2), whose strip / task geometry
    (rows per task adapted to the level, 17-36 strips) the small cases above do not reach: against the oracle's
    HRelax, one sweep from a random iterate and one from the zero guess.  Two-material maps from the oracle's own
    element/node loop (tests/golden/c3_pattern_maps.npz)."""
    import os
    from feanet_amd import _lib, mesh_setup as ms
    from feanet_amd.solver import _Level
    rng = np.random.default_rng(n + (problem == "interface"))
    H = W = n + 1
    pids = None
    if problem == "interface":
        maps = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pattern_maps.npz"))
        pids = {H: maps[f"pid_{H}"]}
        pid = pids[H]
        assert np.array_equal(pid, ms.interface_pattern_map(H))
    L = _Level(n, n, 1, T, torch.device("cuda"), pid if problem == "interface" else None)
    ktab = ms.stencil_table((1, 20) if problem == "interface" else None)
    omd = ms.omega_over_d(ktab, 2 / 3., npdt(T))
    hw = (0.3 * rng.standard_normal((3, 3, 3))).astype(np.float32)
    geo, _ = orc.square_geometry((H, W), npdt(T))
    lvl = orc.Level(n, problem, npdt(T), pids=pids)
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda().to(T)
    kt, om, hwt = cu(ktab.reshape(-1, 9)), cu(omd), cu(hw.reshape(-1))
    f = rng.standard_normal((1, H, W)).astype(npdt(T))
    L.view(L.f).copy_(torch.from_numpy(f))
    for zero in (False, True):
        u = np.zeros((1, H, W), npdt(T)) if zero else rng.standard_normal((1, H, W)).astype(npdt(T))
        L.view(L.a).copy_(torch.from_numpy(u))
        L.view(L.b).fill_(7.0)
        _lib.call("mg_hsweep", T, None if zero else L.a.data_ptr(), None, L.f.data_ptr(), L.b.data_ptr(),
                  None if L.pid is None else L.pid.data_ptr(), kt.data_ptr(), om.data_ptr(), ktab.shape[0],
                  hwt.data_ptr(), 3, *L.geom(), None)
        out = L.view(L.b).cpu().numpy()
        lvl.bc = u * (1 - geo)
        ref = orc.hnet_relax(u, f, lvl, hw, 1)
        err = np.abs(out[:, 1:-1, 1:-1] - ref[:, 1:-1, 1:-1]).max() / max(1.0, np.abs(ref).max())
        assert err < TOL[T], (zero, err)
        assert (out[:, 0] == 7).all() and (out[:, -1] == 7).all() and (out[:, :, 0] == 7).all()


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,n,B,nl,nu", [("poisson", 32, 2, 3, (1, 1)), ("poisson", 128, 1, 3, (1, 1)),
                                               ("poisson", 256, 1, 2, (2, 1)), ("poisson", 64, 3, 1, (1, 2)),
                                               ("interface", 64, 2, 3, (1, 1)), ("interface", 128, 1, 3, (1, 1)),
                                               ("poisson", 128, 1, 3, (0, 1))])
def test_hjac_tail_bitwise(T, problem, n, B, nl, nu):
    """fea_mg_hjac_tail (the learned-smoother V-cycle's coarse levels in one LDS-resident launch) is bitwise the
    per-level fea_mg_hsweep / fea_mg_residual_restrict / fea_mg_prolong_add sequence it replaces: whole V-cycles
    with and without it, both problems, batches, 1-3 HNet layers, V(1,1), V(2,1), V(1,2), V(0,1)."""
    from feanet_amd.solver import MultigridSolver
    rng = np.random.default_rng(n + B + nl)
    hw = (0.25 * rng.standard_normal((nl, 3, 3))).astype(np.float32)
    f = torch.from_numpy(rng.standard_normal((B, 1, n + 1, n + 1))).to("cuda", T)
    out = []
    for tail in (True, False):
        s = MultigridSolver(n, dtype=T, batch=B, smoother="hjac", hnet=hw, problem=problem, nu1=nu[0], nu2=nu[1],
                            coarse_tail=tail)
        names = [name for name, _ in s._plan("a")[0]]
        assert ("mg_hjac_tail" in names) == tail, names
        if tail:  # the largest level <= 65^2 whose fields fit in LDS: 65^2 in fp32, 33^2 in fp64
            top = 65 if T == torch.float32 else 33
            t = s.hjac_tail_from
            assert s.levels[t].H <= top and (t == 1 or s.levels[t - 1].H > top), (t, s.levels[t].H)
        s.set_rhs(f=f)
        s.load()
        sols = []
        for _ in range(3):
            s.vcycle()
            sols.append(s.solution())
        out.append(sols)
    for k, (a, b) in enumerate(zip(*out)):
        assert torch.equal(a, b), (k, (a - b).abs().max().item())


def _tables(problem, T, rng):
    from feanet_amd import mesh_setup as ms
    ktab = ms.stencil_table((1, 20) if problem == "interface" else None)
    nt = ktab.shape[0]
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda().to(T)
    R = (rng.uniform(0.1, 0.4, (nt, 3, 3))).astype(np.float32)
    P = (rng.uniform(0.1, 0.4, (nt, 3, 3))).astype(np.float32)
    return (cu(ktab.reshape(-1, 9)), cu(ms.omega_over_d(ktab, 2 / 3., npdt(T))), nt, cu(R.reshape(-1, 9)),
            cu(P.reshape(-1, 9)))


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,m,n,B", [("poisson", 8, 8, 1), ("poisson", 64, 64, 2), ("poisson", 300, 130, 1),
                                           ("poisson", 16, 256, 1), ("poisson", 1024, 1024, 1),
                                           ("interface", 32, 32, 3), ("interface", 256, 256, 1)])
@pytest.mark.parametrize("nl", [3, 1])
def test_hsweep_fused_kernels_bitwise(T, problem, m, n, B, nl):
    """fea_mg_hsweep_restrict is bitwise fea_mg_hsweep then fea_mg_residual_restrict (stored iterate), from a
    random iterate, the zero guess and with u_raw; fea_mg_prolong_hsweep is bitwise fea_mg_prolong_add then
    fea_mg_hsweep.  Sizes cover strip and task edges, rows != columns, batches, both problems (per-pattern R/P);
    boundary nodes of every output stay untouched."""
    from feanet_amd import _lib, mesh_setup as ms
    from feanet_amd.solver import _Level
    if problem == "interface" and m != n:
        pytest.skip("two-material problem is square")
    rng = np.random.default_rng(m + 3 * n + B + nl)
    pid = ms.interface_pattern_map(m + 1) if problem == "interface" else None
    pidc = ms.interface_pattern_map(m // 2 + 1) if problem == "interface" else None
    fr = _Level(m, n, B, T, torch.device("cuda"), pid)
    cr = _Level(m // 2, n // 2, B, T, torch.device("cuda"), pidc)
    kt, om, nt, rt, pt = _tables(problem, T, rng)
    hw = torch.from_numpy((0.25 * rng.standard_normal((nl, 3, 3))).astype(np.float32).reshape(-1)).cuda().to(T)
    H, W = m + 1, n + 1
    put = lambda L, buf, x: L.view(L.buf(buf)).copy_(torch.from_numpy(x).to(T))
    get = lambda L, buf: L.view(L.buf(buf)).clone()
    fpid = None if fr.pid is None else fr.pid.data_ptr()
    cpid = None if cr.pid is None else cr.pid.data_ptr()
    put(fr, "f", rng.standard_normal((B, H, W)))
    u = rng.standard_normal((B, H, W))
    put(fr, "a", u)
    put(fr, "zero", rng.standard_normal((B, H, W)))  # used as u_raw below
    hs = (kt.data_ptr(), om.data_ptr(), nt, hw.data_ptr(), nl)
    for variant in ("u", "zero", "raw"):
        uptr = None if variant == "zero" else fr.a.data_ptr()
        raw = fr.buf("zero").data_ptr() if variant == "raw" else None
        # the output buffer's boundary holds the iterate's (Dirichlet) values, as both of the solver's ping-pong
        # buffers do: the separate restriction reads them there (zero guess: a coarse level's zero boundary)
        base = np.zeros((B, H, W)) if variant == "zero" else u
        put(fr, "b", base)
        put(cr, "f", np.full((B, cr.H, cr.W), 5.0))
        _lib.call("mg_hsweep", T, uptr, raw, fr.f.data_ptr(), fr.b.data_ptr(), fpid, *hs, *fr.geom(), None)
        _lib.call("mg_residual_restrict", T, fr.b.data_ptr(), fr.f.data_ptr(), None, cr.f.data_ptr(), fpid,
                  kt.data_ptr(), om.data_ptr(), nt, rt.data_ptr(), nt, 1.25, *fr.geom(), cr.ld, cr.bs, None)
        ref_o, ref_c = get(fr, "b"), get(cr, "f")
        put(fr, "b", base)
        put(cr, "f", np.full((B, cr.H, cr.W), 5.0))
        _lib.call("mg_hsweep_restrict", T, uptr, raw, fr.f.data_ptr(), fr.b.data_ptr(), cr.f.data_ptr(), fpid, *hs,
                  rt.data_ptr(), nt, 1.25, *fr.geom(), cr.ld, cr.bs, None)
        got_o, got_c = get(fr, "b"), get(cr, "f")
        assert torch.equal(got_o, ref_o), (variant, (got_o - ref_o).abs().max().item())
        assert torch.equal(got_c, ref_c), (variant, torch.nonzero(got_c != ref_c)[:5])
        bt = torch.from_numpy(base).to("cuda", T)
        assert torch.equal(got_o[:, 0], bt[:, 0]) and torch.equal(got_o[:, :, -1], bt[:, :, -1])
        assert (got_c[:, 0] == 5).all() and (got_c[:, :, -1] == 5).all()
    # prolongation + correction + sweep
    e = rng.standard_normal((B, cr.H, cr.W))
    e[:, 0] = e[:, -1] = e[:, :, 0] = e[:, :, -1] = 0
    put(cr, "a", e)
    put(fr, "b", np.full((B, H, W), 7.0))
    put(fr, "c", u)  # prolong_add writes the interior: the boundary keeps the iterate's values, as the solver's
    #                  ping-pong buffers both hold the Dirichlet data there
    pp = (pt.data_ptr(), nt, 0.75)
    _lib.call("mg_prolong_add", T, fr.a.data_ptr(), cr.a.data_ptr(), fr.c.data_ptr(), cpid, *pp, *fr.geom(), cr.ld,
              cr.bs, None)
    for raw in (None, fr.buf("zero").data_ptr()):  # the first sweep after a load sees the un-reset guess
        put(fr, "b", np.full((B, H, W), 7.0))
        _lib.call("mg_hsweep", T, fr.c.data_ptr(), raw, fr.f.data_ptr(), fr.b.data_ptr(), fpid, *hs, *fr.geom(), None)
        ref = get(fr, "b")
        put(fr, "b", np.full((B, H, W), 7.0))
        _lib.call("mg_prolong_hsweep", T, fr.a.data_ptr(), raw, cr.a.data_ptr(), fr.f.data_ptr(), fr.b.data_ptr(), fpid,
                  cpid, *hs, *pp, *fr.geom(), cr.ld, cr.bs, None)
        got = get(fr, "b")
        assert torch.equal(got, ref), (raw, (got - ref).abs().max().item())
    assert (got[:, 0] == 7).all() and (got[:, -1] == 7).all()


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,n,B,nu", [("poisson", 128, 2, (1, 1)), ("poisson", 512, 1, (2, 1)),
                                            ("interface", 128, 1, (1, 1)), ("poisson", 64, 1, (0, 2)),
                                            ("poisson", 256, 1, (1, 0))])
def test_hjac_fused_schedule_bitwise(T, problem, n, B, nu):
    """MultigridSolver(smoother="hjac") with the fused level pairs (fuse=True: fea_mg_hsweep_restrict,
    fea_mg_prolong_hsweep) and the coarse tail is bitwise the unfused per-level schedule, first cycle (u_raw from
    a guess with a non-Dirichlet boundary) included."""
    from feanet_amd.solver import MultigridSolver
    rng = np.random.default_rng(n + B)
    hw = (0.25 * rng.standard_normal((3, 3, 3))).astype(np.float32)
    f = torch.from_numpy(rng.standard_normal((B, 1, n + 1, n + 1))).to("cuda", T)
    u0 = torch.from_numpy(rng.standard_normal((B, 1, n + 1, n + 1))).to("cuda", T)
    out = []
    for fused in (True, False):
        s = MultigridSolver(n, dtype=T, batch=B, smoother="hjac", hnet=hw, problem=problem, nu1=nu[0], nu2=nu[1],
                            fuse=fused, coarse_tail=fused)
        kinds = {name for name, _ in s._plan("a")[0]}
        assert ("mg_prolong_hsweep" in kinds) == (fused and nu[1] > 0), kinds
        s.set_rhs(f=f)
        s.load(u0)
        sols = []
        for _ in range(3):
            s.vcycle()
            sols.append(s.solution())
        out.append(sols)
    for k, (a, b) in enumerate(zip(*out)):
        assert torch.equal(a, b), (k, (a - b).abs().max().item())


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,m,n,B,nl,nu", [("poisson", 512, 512, 1, 3, (1, 1)), ("poisson", 1024, 1024, 2, 3, (1, 1)),
                                                 ("poisson", 256, 512, 1, 2, (1, 1)), ("poisson", 512, 512, 1, 1, (2, 1)),
                                                 ("poisson", 512, 512, 2, 3, (1, 2)), ("interface", 512, 512, 1, 3, (1, 1)),
                                                 ("interface", 512, 512, 2, 2, (1, 1))])
@pytest.mark.parametrize("tiles", ["default", "largest", "smallest"])
def test_hjac_hmid_bitwise(T, problem, m, n, B, nl, nu, tiles):
    """fea_mg_hmid_down / fea_mg_hmid_up (two HJac levels per launch, hmid_ops.hip) are bitwise the fused per-level
    kernels they replace (mid=False): whole V-cycles, both problems, batches, 1-3 HNet layers, rows != columns,
    V(2,1) / V(1,2) (only the up / down pairs apply), every tile size the solver may pick."""
    from feanet_amd.solver import MultigridSolver
    rng = np.random.default_rng(m + n + B + nl)
    hw = (0.25 * rng.standard_normal((nl, 3, 3))).astype(np.float32)
    f = torch.from_numpy(rng.standard_normal((B, 1, m + 1, n + 1))).to("cuda", T)
    kw = dict(dtype=T, batch=B, smoother="hjac", hnet=hw, problem=problem, nu1=nu[0], nu2=nu[1],
              rows=None if m == n else m)
    out = []
    for mid in (True, False):
        s = MultigridSolver(n, mid=mid, **kw)
        if tiles != "default":
            s.HMID_MIN_TILES = 1 if tiles == "largest" else 1 << 30
        kinds = [name for name, _ in s._plan("a")[0]]
        assert (kinds.count("mg_hmid_down") > 0) == (mid and nu[0] == 1), kinds
        assert (kinds.count("mg_hmid_up") > 0) == (mid and nu[1] == 1), kinds
        s.set_rhs(f=f)
        s.load()
        sols = []
        for _ in range(3):
            s.vcycle()
            sols.append(s.solution())
        out.append(sols)
    for k, (a, b) in enumerate(zip(*out)):
        assert torch.equal(a, b), (k, (a - b).abs().max().item())


def test_hmid_api_rejects_bad_arguments():
    """fea_mg_hmid_down / _up return FEA_EINVAL (RuntimeError) for even level sizes, a tile whose LDS does not
    fit, missing pattern maps with per-pattern tables, and an output aliasing an input."""
    from feanet_amd import _lib
    from feanet_amd.solver import _Level
    T = torch.float64
    lv = [_Level(256 >> j, 256 >> j, 1, T, torch.device("cuda")) for j in range(3)]
    kt = torch.ones(9, device="cuda", dtype=T)
    om = torch.ones(1, device="cuda", dtype=T)
    hw = torch.zeros(27, device="cuda", dtype=T)
    fs = _lib.PtrArray([l.f.data_ptr() for l in lv])
    us = _lib.PtrArray([lv[0].a.data_ptr(), lv[1].a.data_ptr()])
    ok = (fs, us, None, 1, 257, 257, kt.data_ptr(), om.data_ptr(), 1, hw.data_ptr(), 3, kt.data_ptr(), 1, 1.0)
    assert _lib.hmid_lds_bytes(False, 8, 3, 8, False) > 0 and _lib.hmid_lds_bytes(False, 64, 3, 8, False) == -1
    assert _lib.hmid_lds_bytes(True, 32, 3, 8, False) > 0 and _lib.hmid_lds_bytes(True, 128, 3, 8, False) == -1
    for bad in (dict(H=256), dict(TT=64), dict(ntab=16, nr=16)):
        args = list(ok) + [bad.get("TT", 8), None]
        if "H" in bad:
            args[4] = bad["H"]
        if "ntab" in bad:
            args[8], args[12] = bad["ntab"], bad["nr"]
        with pytest.raises(RuntimeError, match="invalid arguments"):
            _lib.call("mg_hmid_down", T, *args)
    with pytest.raises(RuntimeError, match="invalid arguments"):
        _lib.call("mg_hmid_up", T, _lib.PtrArray([lv[0].f.data_ptr(), lv[1].f.data_ptr()]), us, lv[2].a.data_ptr(),
                  lv[0].a.data_ptr(), None, 1, 257, 257, kt.data_ptr(), om.data_ptr(), 1, hw.data_ptr(), 3,
                  kt.data_ptr(), 1, 1.0, 16, None)


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,m,n,B", [("poisson", 256, 256, 2), ("poisson", 128, 512, 1), ("interface", 256, 256, 1)])
@pytest.mark.parametrize("nl", [0, 1, 2, 3])
def test_hmid_kernels_vs_per_level_calls(T, problem, m, n, B, nl):
    """The C-ABI of the HJac two-level launches against the per-level calls they replace, every HNet depth the ABI
    takes (0-3 layers), per-pattern R/P, rectangles, batches, every tile size that fits: fea_mg_hmid_down is bitwise
    fea_mg_hsweep_restrict(u = NULL) on levels a and a+1 (iterates, both coarse right-hand sides), fea_mg_hmid_up
    bitwise fea_mg_prolong_hsweep on levels a+1 then a; boundary nodes of every output untouched."""
    from feanet_amd import _lib, mesh_setup as ms
    from feanet_amd.solver import _Level
    if problem == "interface" and m != n:
        pytest.skip("two-material problem is square")
    rng = np.random.default_rng(m + n + B + nl)
    dev = torch.device("cuda")
    pids = [ms.interface_pattern_map((m >> j) + 1) if problem == "interface" else None for j in range(3)]
    lv = [_Level(m >> j, n >> j, B, T, dev, pids[j]) for j in range(3)]
    kt, om, nt, rt, pt = _tables(problem, T, rng)
    hw = torch.from_numpy((0.25 * rng.standard_normal((max(nl, 1), 3, 3))).astype(np.float32).reshape(-1)).cuda().to(T)
    put = lambda L, name, x: L.view(L.buf(name)).copy_(torch.from_numpy(x).to(T))
    get = lambda L, name: L.view(L.buf(name)).clone()
    pid = lambda j: None if lv[j].pid is None else lv[j].pid.data_ptr()
    esz = 4 if T == torch.float32 else 8
    hs = (kt.data_ptr(), om.data_ptr(), nt, hw.data_ptr(), nl)
    fa = rng.standard_normal((B, lv[0].H, lv[0].W))
    fa[:, 0] = fa[:, -1] = fa[:, :, 0] = fa[:, :, -1] = 0

    def reset():
        put(lv[0], "f", fa)
        for j in range(3):
            if j:
                put(lv[j], "f", np.full((B, lv[j].H, lv[j].W), 5.0))
            put(lv[j], "a", np.zeros((B, lv[j].H, lv[j].W)))
            put(lv[j], "b", np.full((B, lv[j].H, lv[j].W), 7.0))

    reset()  # per-level reference, down
    for j in range(2):
        _lib.call("mg_hsweep_restrict", T, None, None, lv[j].f.data_ptr(), lv[j].a.data_ptr(), lv[j + 1].f.data_ptr(),
                  pid(j), *hs, rt.data_ptr(), nt, 1.25, *lv[j].geom(), lv[j + 1].ld, lv[j + 1].bs, None)
    ref_down = [get(lv[0], "a"), get(lv[1], "f"), get(lv[1], "a"), get(lv[2], "f")]
    # up from those iterates: e = a random coarse correction with a zero boundary
    e = rng.standard_normal((B, lv[2].H, lv[2].W))
    e[:, 0] = e[:, -1] = e[:, :, 0] = e[:, :, -1] = 0
    put(lv[2], "b", e)
    put(lv[1], "b", np.zeros((B, lv[1].H, lv[1].W)))  # (the solver's coarse buffers hold 0 on the boundary)
    pp = (pt.data_ptr(), nt, 0.75)
    _lib.call("mg_prolong_hsweep", T, lv[1].a.data_ptr(), None, lv[2].b.data_ptr(), lv[1].f.data_ptr(),
              lv[1].b.data_ptr(), pid(1), pid(2), *hs, *pp, *lv[1].geom(), lv[2].ld, lv[2].bs, None)
    put(lv[0], "b", np.full((B, lv[0].H, lv[0].W), 7.0))
    _lib.call("mg_prolong_hsweep", T, lv[0].a.data_ptr(), None, lv[1].b.data_ptr(), lv[0].f.data_ptr(),
              lv[0].b.data_ptr(), pid(0), pid(1), *hs, *pp, *lv[0].geom(), lv[1].ld, lv[1].bs, None)
    ref_up = get(lv[0], "b")
    pids_arr = _lib.PtrArray([pid(j) for j in range(3)]) if nt > 1 else None
    fs = _lib.PtrArray([l.f.data_ptr() for l in lv])
    tds = [t for t in (16, 8, 4, 2) if _lib.hmid_lds_bytes(False, t, nl, esz, nt > 1) > 0]
    tus = [t for t in (64, 32, 16, 8) if _lib.hmid_lds_bytes(True, t, nl, esz, nt > 1) > 0]
    assert tds and tus
    for td in tds:
        reset()
        _lib.call("mg_hmid_down", T, fs, _lib.PtrArray([lv[0].a.data_ptr(), lv[1].a.data_ptr()]), pids_arr, B,
                  lv[0].H, lv[0].W, *hs, rt.data_ptr(), nt, 1.25, td, None)
        got = [get(lv[0], "a"), get(lv[1], "f"), get(lv[1], "a"), get(lv[2], "f")]
        for k, (g_, r_) in enumerate(zip(got, ref_down)):
            assert torch.equal(g_, r_), (td, k, (g_ - r_).abs().max().item())
    put(lv[2], "b", e)
    for tu in tus:
        put(lv[0], "b", np.full((B, lv[0].H, lv[0].W), 7.0))
        _lib.call("mg_hmid_up", T, _lib.PtrArray([lv[0].f.data_ptr(), lv[1].f.data_ptr()]),
                  _lib.PtrArray([lv[0].a.data_ptr(), lv[1].a.data_ptr()]), lv[2].b.data_ptr(), lv[0].b.data_ptr(),
                  pids_arr, B, lv[0].H, lv[0].W, *hs, *pp, tu, None)
        got = get(lv[0], "b")
        assert torch.equal(got, ref_up), (tu, (got - ref_up).abs().max().item())
        assert (got[:, 0] == 7).all() and (got[:, -1] == 7).all() and (got[:, :, 0] == 7).all()


def test_hjac_c3_interface_vs_oracle():
    """The learned smoother on BASELINE C3's two-material problem (SURVEY §8f row 1 on MM_Interface): 2049^2 fp64
    circle inclusion (contrast 20), the learned ratio R / P / w of FEANet/multigrid.py, F = ones, every sweep an
    HRelax with the shipped HNet weights — against the oracle's MultiGrid.Step with HRelax sweeps
    (M-FEANet-mg_test.ipynb:147-155, :27346-27372) on the oracle's own pattern maps (tests/golden/c3_pattern_maps.npz):
    three cycles from zero, 1e-10 of max|u| after each."""
    import os
    from feanet_amd.solver import MultigridSolver
    here = os.path.dirname(__file__)
    n = 2048
    w = np.load(os.path.join(here, "..", "multigrid-feanet_amd", "feanet_amd", "weights", "hnet_iso_poisson_33x33.npz"))
    hw = np.stack([w[f"conv{i}"].reshape(3, 3) for i in range(3)])
    rp = np.load(os.path.join(here, "..", "multigrid-feanet_amd", "feanet_amd", "weights", "multigrid_interface_ratio.npz"))
    s = MultigridSolver(n, problem="interface", dtype=torch.float64, smoother="hjac", hnet=hw, R=rp["R"][0],
                        P=rp["P"][:, 0], w=rp["w"])
    s.set_rhs(F=torch.ones(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64))
    s.load()
    maps = np.load(os.path.join(here, "golden", "c3_pattern_maps.npz"))
    pids = {int(k[4:]): maps[k] for k in maps.files if k.startswith("pid_")}
    mg = orc.OracleMultigrid(n, "interface", np.float64, levels=s.L, pids=pids,
                             rtab=np.broadcast_to(np.asarray(rp["R"][0], np.float32), (16, 3, 3)),
                             ptab=np.asarray(rp["P"][:, 0], np.float32), w=tuple(float(x) for x in rp["w"]))
    for l in mg.levels:
        l.sweep = (lambda ll, o: (lambda v, ff: (lambda j: j + orc.hnet(j - v, ll.geo, hw))(o(v, ff))))(l, l.sweep)
    f = orc.conv3x3(np.ones((1, n + 1, n + 1)), orc.fnet_stencil(2.0 / n))
    v = np.zeros((1, n + 1, n + 1))
    for k in range(3):
        s.vcycle()
        v = mg.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        err = np.abs(got - v).max() / max(1.0, np.abs(v).max())
        assert err < 1e-10, (k, err)
