"""The fused V-cycle schedule (feanet_amd.schedule) is the reference's V-cycle: interpret the
symbolic step list with the CPU oracle's operators and compare with the oracle's own drivers
(MultiGrid.Step / rec_V_cycle / the MM_Interface Q2 variant).  CPU only (host logic)."""
import numpy as np
import pytest

from feanet_amd.schedule import vcycle_schedule
from oracle import feanet_oracle as orc


def interpret(mg, steps, v, f, compat=None):
    """Execute a symbolic schedule with oracle ops. `compat` selects the oracle's transfer flavour."""
    L = mg.L
    lv = mg.levels
    dt = mg.dtype
    B = v.shape[0]
    bufs = [dict() for _ in range(L)]
    bufs[0]["a"] = v
    fs = [None] * L
    fs[0] = f

    def get(l, name):
        if name == "zero":
            return np.zeros((B, lv[l].H, lv[l].W), dt)
        if name == "omdf":  # zero-guess pre-sweep recomputed from f_l
            return lv[l].sweep(np.zeros((B, lv[l].H, lv[l].W), dt), fs[l])
        return bufs[l][name]

    expanded = []
    for st in steps:  # multi-level launches = their per-level steps (feanet_amd.schedule.group_mid)
        if st[0] == "mid_down":
            expanded += [("resid_restrict", l, None, None) for l in range(st[1], st[1] + st[2])]
        elif st[0] == "mid_up":
            a, k, csrc, dst = st[1:5]
            expanded += [("prolong_sweep", l, "omdf", csrc if l == a + k - 1 else "mid", dst if l == a else "mid")
                         for l in range(a + k - 1, a - 1, -1)]
        elif st[0] == "resid_restrict2":  # feanet_amd.schedule.pair_restrictions
            expanded += [("resid_restrict", st[1], None, None), ("resid_restrict", st[1] + 1, None, None)]
        elif st[0] == "prolong_sweep2":  # feanet_amd.schedule.pair_prolongations
            expanded += [("prolong_sweep", st[1] + 1, "omdf", st[2], "mid"), ("prolong_sweep", st[1], "omdf", "mid", st[3])]
        elif st[0] == "coarse_tail_ext":  # feanet_amd.schedule.extend_tail
            expanded += [("resid_restrict", st[1], None, None), ("coarse_tail", st[1] + 1, "ext"),
                         ("prolong_sweep", st[1], "omdf", "ext", st[2])]
        elif st[0] == "hmid_down":  # feanet_amd.schedule.group_hmid
            expanded += [("hsweep_restrict", st[1], None, st[2]), ("hsweep_restrict", st[1] + 1, None, st[3])]
        elif st[0] == "hmid_up":
            a, u0, u1, e, d0 = st[1:6]
            expanded += [("prolong_hsweep", a + 1, u1, e, "mid"), ("prolong_hsweep", a, u0, "mid", d0)]
        else:
            expanded.append(st)
    for st in expanded:
        kind, l = st[0], st[1]
        if kind in ("hsweep", "hsweep_restrict"):  # learned-smoother sweep: the oracle's HRelax with mg.hw
            src = np.zeros((B, lv[l].H, lv[l].W), dt) if st[2] is None else get(l, st[2])
            bufs[l][st[3]] = orc.hnet_relax(src, fs[l], lv[l], mg.hw)
            if kind == "hsweep_restrict":
                fs[l + 1] = orc.restrict(fs[l] - lv[l].K(bufs[l][st[3]]), lv[l].pid, mg.rtab, mg.w[0])
        elif kind == "prolong_hsweep":
            x = get(l, st[2]) + orc.prolong(get(l + 1, st[3]), lv[l + 1].pid, mg.ptab, mg.w[1])
            bufs[l][st[4]] = orc.hnet_relax(x, fs[l], lv[l], mg.hw)
        elif kind == "hjac_tail":
            bufs[l][st[2]] = hjac_tail_oracle(mg, l, fs[l], B)
        elif kind == "sweep":
            src = np.zeros((B, lv[l].H, lv[l].W), dt) if st[2] is None else get(l, st[2])
            bufs[l][st[3]] = lv[l].sweep(src, fs[l])
        elif kind == "resid_restrict":
            if st[2] is None:
                src = lv[l].sweep(np.zeros((B, lv[l].H, lv[l].W), dt), fs[l])
                if st[3] is not None:
                    bufs[l][st[3]] = src
            else:
                src = get(l, st[2])
            r = fs[l] - lv[l].K(src)
            if compat == "mm":
                fs[l + 1] = mg._mm_restrict(r)
            else:
                fs[l + 1] = orc.restrict(r, lv[l].pid, mg.rtab, mg.w[0])
        elif kind == "sweep_restrict":
            out = lv[l].sweep(get(l, st[2]), fs[l])
            bufs[l][st[3]] = out
            r = fs[l] - lv[l].K(out)
            fs[l + 1] = mg._mm_restrict(r) if compat == "mm" else orc.restrict(r, lv[l].pid, mg.rtab, mg.w[0])
        elif kind == "coarse_tail":
            bufs[l][st[2]] = tail_oracle(mg, l, fs[l], compat, B)
        elif kind in ("prolong_sweep", "prolong_add"):
            src = get(l, st[2])
            e = get(l + 1, st[3])
            if compat == "mm":
                corr = orc.bilinear_upsample(e) * lv[l].geo + lv[l].bc
            else:
                corr = orc.prolong(e, lv[l + 1].pid, mg.ptab, mg.w[1])
            x = src + corr
            bufs[l][st[4]] = lv[l].sweep(x, fs[l]) if kind == "prolong_sweep" else x
    return bufs


def tail_oracle(mg, t, f_t, compat, B, nu1=None, nu2=None, q2=None):
    """The coarse_tail kernel's loop (coarse_tail.hip) restated with oracle ops."""
    nu1 = mg.nu[0] if nu1 is None else nu1
    nu2 = mg.nu[1] if nu2 is None else nu2
    q2 = mg.q2 if q2 is None else q2
    lv = mg.levels[t:]
    dt = mg.dtype
    zeros = lambda k: np.zeros((B, lv[k].H, lv[k].W), dt)
    f = [f_t] + [None] * (len(lv) - 1)
    v = [zeros(k) for k in range(len(lv))]
    for k in range(len(lv) - 1):
        if nu1 > 0 and not q2:
            v[k] = lv[k].sweep(zeros(k), f[k])
            for _ in range(nu1 - 1):
                v[k] = lv[k].sweep(v[k], f[k])
        r = f[k] - lv[k].K(v[k])
        f[k + 1] = mg._mm_restrict(r) if compat == "mm" else orc.restrict(r, lv[k].pid, mg.rtab, mg.w[0])
    k = len(lv) - 1
    ncs = nu2 if q2 else nu1 + nu2
    for s in range(ncs):
        v[k] = lv[k].sweep(v[k], f[k])
    for k in range(len(lv) - 2, -1, -1):
        corr = (orc.bilinear_upsample(v[k + 1]) * lv[k].geo if compat == "mm"
                else orc.prolong(v[k + 1], lv[k + 1].pid, mg.ptab, mg.w[1]))
        v[k] = v[k] + corr
        for _ in range(nu2):
            v[k] = lv[k].sweep(v[k], f[k])
    return v[0]


def hjac_tail_oracle(mg, t, f_t, B):
    """The hjac_tail kernel's loop (hjac_tail.hip) restated with oracle ops (HRelax sweeps)."""
    nu1, nu2 = mg.nu
    lv = mg.levels[t:]
    zeros = lambda k: np.zeros((B, lv[k].H, lv[k].W), mg.dtype)
    f = [f_t] + [None] * (len(lv) - 1)
    v = [zeros(k) for k in range(len(lv))]
    for k in range(len(lv) - 1):
        for _ in range(nu1):
            v[k] = orc.hnet_relax(v[k], f[k], lv[k], mg.hw)
        f[k + 1] = orc.restrict(f[k] - lv[k].K(v[k]), lv[k].pid, mg.rtab, mg.w[0])
    k = len(lv) - 1
    for _ in range(nu1 + nu2):
        v[k] = orc.hnet_relax(v[k], f[k], lv[k], mg.hw)
    for k in range(len(lv) - 2, -1, -1):
        v[k] = v[k] + orc.prolong(v[k + 1], lv[k + 1].pid, mg.ptab, mg.w[1])
        for _ in range(nu2):
            v[k] = orc.hnet_relax(v[k], f[k], lv[k], mg.hw)
    return v[0]


@pytest.mark.parametrize("fuse", [False, True])
@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("tail", [None, 1, 2, 4])
def test_hjac_tail_schedule_equals_step(problem, tail, fuse):
    """hjac_schedule (MultiGrid.Step mode='hjac', every relaxation one HRelax) with its coarse levels as one
    "hjac_tail" step (tail_from) is the oracle's Step with every sweep replaced by HRelax."""
    from feanet_amd.schedule import hjac_schedule
    n, L = 32, 5
    rng = np.random.default_rng(13)
    for nu in ((1, 1), (2, 1), (1, 2), (0, 1)):
        mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
        mg.nu, mg.hw = nu, 0.3 * rng.standard_normal((3, 3, 3))
        v = rng.standard_normal((2, n + 1, n + 1))
        f = rng.standard_normal((2, n + 1, n + 1))
        steps, end = hjac_schedule(L, *nu, tail_from=tail, fuse=fuse)
        assert sum(st[0] == "hjac_tail" for st in steps) == (tail is not None)
        kinds = {st[0] for st in steps}
        assert ("hsweep_restrict" in kinds) == (fuse and nu[0] > 0) and ("prolong_hsweep" in kinds) == fuse
        for st in steps:  # a fused prolongation never writes the iterate it reads
            assert st[0] != "prolong_hsweep" or st[2] != st[4]
        out = interpret(mg, steps, v, f)[0][end]
        ref_steps, ref_end = hjac_schedule(L, *nu)
        ref = interpret(mg, ref_steps, v, f)[0][ref_end]
        np.testing.assert_allclose(out, ref, rtol=1e-13, atol=1e-13)
        if nu == (1, 1):  # and the reference's Step with HRelax sweeps
            for lvl in mg.levels:
                lvl.sweep = (lambda ll, o: (lambda x, ff: (lambda j: j + orc.hnet(j - x, ll.geo, mg.hw))(o(x, ff))))(
                    lvl, lvl.sweep)
            np.testing.assert_allclose(out, mg.step(v, f), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("nu", [(1, 1), (2, 1), (1, 2)])
@pytest.mark.parametrize("pairs", [[(1, 8, 32)], [(2, 8, 32)], [(1, 4, 16), (3, 4, 16)]])
def test_hmid_grouping_equals_per_level(problem, nu, pairs):
    """group_hmid (two HJac levels per launch each way, fea_mg_hmid_down / _up) is the fused per-level schedule:
    the down pair only where both levels start from the zero guess (nu1 = 1), the up pair wherever two
    prolongation + sweep steps follow each other (nu2 = 1)."""
    from feanet_amd.schedule import group_hmid, hjac_schedule
    n, L = 64, 6
    rng = np.random.default_rng(17)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    mg.nu, mg.hw = nu, 0.3 * rng.standard_normal((3, 3, 3))
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    ref_steps, end = hjac_schedule(L, *nu, tail_from=5, fuse=True)
    steps = group_hmid(ref_steps, pairs)
    kinds = [st[0] for st in steps]
    assert kinds.count("hmid_down") == (len(pairs) if nu[0] == 1 else 0), steps
    assert kinds.count("hmid_up") == (len(pairs) if nu[1] == 1 else 0), steps
    out = interpret(mg, steps, v, f)[0][end]
    ref = interpret(mg, ref_steps, v, f)[0][end]
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("tail", [None, 1, 2, 4])
def test_tail_schedule_equals_full(problem, tail):
    n = 32
    L = 5
    rng = np.random.default_rng(11)
    for nu, q2 in (((1, 1), False), ((2, 1), False), ((0, 2), False), ((1, 1), True)):
        mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
        mg.nu, mg.q2 = nu, q2
        v = rng.standard_normal((2, n + 1, n + 1))
        f = rng.standard_normal((2, n + 1, n + 1))
        compat = "mm_interface_q2" if q2 else None
        ref_steps, ref_end = vcycle_schedule(L, *nu, compat=compat)
        ref = interpret(mg, ref_steps, v, f)[0][ref_end]
        steps, end = vcycle_schedule(L, *nu, compat=compat, tail_from=tail)
        out = interpret(mg, steps, v, f)[0][end]
        np.testing.assert_allclose(out, ref, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("L", [1, 2, 3, 5])
def test_step_schedule_equals_reference_step(problem, L, fuse):
    n = 32
    rng = np.random.default_rng(L)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    steps, end = vcycle_schedule(L, 1, 1, fuse=fuse)
    out = interpret(mg, steps, v, f)[0][end]
    ref = mg.step(v, f)
    np.testing.assert_allclose(out, ref, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("nu", [(1, 1), (0, 1), (1, 0), (2, 1), (1, 2), (2, 2), (0, 2), (2, 0), (3, 1)])
def test_nu_schedules_equal_rec_vcycle(nu, fuse):
    n = 32
    rng = np.random.default_rng(sum(nu))
    mg = orc.OracleMultigrid(n, "poisson", np.float64)
    v = rng.standard_normal((1, n + 1, n + 1))
    f = rng.standard_normal((1, n + 1, n + 1))
    steps, end = vcycle_schedule(mg.L, *nu, fuse=fuse)
    out = interpret(mg, steps, v, f, compat="mm")[0][end]
    ref = mg.rec_vcycle(v, f, *nu)
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=1e-12)


def test_q2_schedule_equals_mm_interface():
    n = 32
    rng = np.random.default_rng(7)
    mg = orc.OracleMultigrid(n, "interface", np.float64)
    v = rng.standard_normal((1, n + 1, n + 1))
    f = rng.standard_normal((1, n + 1, n + 1))
    steps, end = vcycle_schedule(mg.L, 1, 1, compat="mm_interface_q2")
    out = interpret(mg, steps, v, f, compat="mm")[0][end]
    ref = mg.rec_vcycle(v, f, 1, 1, compat_q2=True)
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=1e-12)


def test_schedule_shape_and_buffers():
    steps, end = vcycle_schedule(12, 1, 1)
    kinds = [s[0] for s in steps]
    # fine sweep fused with its residual-restriction, 10 zero-guess residual-restrictions,
    # 2 coarsest sweeps, 11 fused prolong+sweep
    assert kinds.count("sweep_restrict") == 1 and kinds.count("resid_restrict") == 10
    assert kinds.count("sweep") == 2 and kinds.count("prolong_sweep") == 11 and end == "a"
    # coarse levels keep no iterate between restriction and prolongation (recomputed omd*f)
    assert ("resid_restrict", 1, None, None) in steps
    assert [s[2] for s in steps if s[0] == "prolong_sweep"] == ["omdf"] * 10 + ["b"]
    steps, end = vcycle_schedule(12, 1, 1, recompute=False)
    assert ("resid_restrict", 1, None, "a") in steps and "omdf" not in [s[2] for s in steps]
    steps, end = vcycle_schedule(12, 1, 1, fuse=False)
    kinds = [s[0] for s in steps]
    assert kinds.count("sweep") == 3 and kinds.count("resid_restrict") == 11
    for s in steps:  # no step reads and writes the same buffer
        if s[0] == "sweep":
            assert s[2] != s[3]
        if s[0].startswith("prolong"):
            assert s[2] != s[4]
    # odd number of fine writes alternates the resident buffer
    steps, end = vcycle_schedule(4, 2, 1)
    assert end == "b"


@pytest.mark.parametrize("groups", [[(1, 3)], [(2, 2)], [(1, 2), (3, 2)], [(1, 4)]])
@pytest.mark.parametrize("problem", ["poisson", "interface"])
def test_mid_grouping_equals_per_level(problem, groups):
    """group_mid (multi-level launches) is the per-level schedule: same steps once expanded, same
    V-cycle result with oracle operators, and the grouped steps name the right buffers."""
    from feanet_amd.schedule import group_mid
    n, L = 64, 6
    rng = np.random.default_rng(7)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    mg.nu, mg.q2 = (1, 1), False
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    steps, end = vcycle_schedule(L, 1, 1, tail_from=5)
    pick = lambda levels: [(a, k, 4) for a, k in groups if set(range(a, a + k)) <= set(levels)]
    grouped = group_mid(steps, pick, pick)
    kinds = [s[0] for s in grouped]
    assert kinds.count("mid_down") == len(groups) and kinds.count("mid_up") == len(groups)
    for s in grouped:
        if s[0] == "mid_up":
            a, k, csrc, dst, T = s[1:]
            assert dst == "a" and T == 4 and csrc == ("a" if a + k == 5 else "a")
    ref = interpret(mg, steps, v, f)[0][end]
    out = interpret(mg, grouped, v, f)[0][end]
    np.testing.assert_array_equal(out, ref)
    assert end == "a" or end == "b"
    np.testing.assert_allclose(out, mg.step(v, f), rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("nu", [(1, 1), (2, 1), (1, 2), (0, 2)])
def test_top_zero_schedule_equals_step_from_zero(problem, nu):
    """top_zero (the replicated coarse sub-cycle of the domain-decomposed path): level 0 starts from a zero
    guess; with one pre-sweep its iterate is not kept but recomputed (omd f) by the prolongation, like the
    coarse levels', so the whole sub-cycle can run as multi-level launches — the result is the ordinary
    schedule's from u = 0."""
    n, L = 32, 5
    rng = np.random.default_rng(3)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    mg.nu, mg.q2 = nu, False
    f = rng.standard_normal((2, n + 1, n + 1))
    ref_steps, ref_end = vcycle_schedule(L, *nu)
    ref = interpret(mg, ref_steps, np.zeros_like(f), f)[0][ref_end]
    for tail in (None, 2):
        steps, end = vcycle_schedule(L, *nu, top_zero=True, tail_from=tail)
        if nu == (1, 1):
            assert steps[0] == ("resid_restrict", 0, None, None) and steps[-1][2] == "omdf"
        out = interpret(mg, steps, rng.standard_normal(f.shape), f)[0][end]
        np.testing.assert_allclose(out, ref, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("groups,npairs", [([], 2), ([(3, 2)], 1), ([(1, 2)], 1), ([(2, 3)], 0)])
@pytest.mark.parametrize("problem", ["poisson", "interface"])
def test_level_pairing_equals_per_level(problem, groups, npairs):
    """pair_restrictions / pair_prolongations (fea_mg_zero_restrict2 / fea_mg_prolong2) on the levels the
    multi-level launches leave: the paired schedule is the per-level one (same V-cycle result with oracle
    operators), pairs never overlap a multi-level group, and the intermediate iterate of a paired
    prolongation is never named (it is not stored)."""
    from feanet_amd.schedule import group_mid, pair_prolongations, pair_restrictions
    n, L = 64, 6
    rng = np.random.default_rng(5)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    mg.nu, mg.q2 = (1, 1), False
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    steps, end = vcycle_schedule(L, 1, 1, tail_from=5)
    pick = lambda levels: [(a, k, 4) for a, k in groups if set(range(a, a + k)) <= set(levels)]
    ok = lambda l: l + 2 < L
    paired = pair_prolongations(pair_restrictions(group_mid(steps, pick, pick), ok), ok)
    kinds = [s[0] for s in paired]
    assert kinds.count("resid_restrict2") == kinds.count("prolong_sweep2") == npairs
    for s in paired:
        if s[0] == "prolong_sweep2":
            assert s[2] == "a" and s[3] == "a"
    ref = interpret(mg, steps, v, f)[0][end]
    out = interpret(mg, paired, v, f)[0][end]
    np.testing.assert_array_equal(out, ref)


@pytest.mark.parametrize("finest_first", [True, False])
def test_prolongation_pairing_order(finest_first):
    """A run of three chained recomputed-iterate prolongations (levels 3, 2, 1): finest-first pairs 2-1 and leaves
    level 3 alone (the single-GPU default: the larger iterate stays out of HBM), coarsest-first pairs 3-2 and leaves
    level 1 (the domain decomposition's choice); both are the per-level V-cycle (oracle operators)."""
    from feanet_amd.schedule import OMDF, pair_prolongations
    n, L = 64, 6
    rng = np.random.default_rng(7)
    mg = orc.OracleMultigrid(n, "poisson", np.float64, levels=L)
    mg.nu, mg.q2 = (1, 1), False
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    steps, end = vcycle_schedule(L, 1, 1, tail_from=4)
    ps = [s for s in steps if s[0] == "prolong_sweep" and s[2] == OMDF]
    assert [s[1] for s in ps] == [3, 2, 1]
    paired = pair_prolongations(steps, lambda l: l + 2 < L, finest_first=finest_first)
    pairs = [s[1] for s in paired if s[0] == "prolong_sweep2"]
    singles = [s[1] for s in paired if s[0] == "prolong_sweep" and s[2] == OMDF]
    assert (pairs, singles) == (([1], [3]) if finest_first else ([2], [1]))
    ref = interpret(mg, steps, v, f)[0][end]
    np.testing.assert_array_equal(interpret(mg, paired, v, f)[0][end], ref)


@pytest.mark.parametrize("k", [1, 2, 5, 20, 31, 32, 33, 64, 100, 1000])
def test_vcycle_blocks_cover_k(k):
    """vcycle(k) replays blocks of GRAPH_CYCLES joined cycles plus one block of the rest (pipe_blocks), and
    solve() the binary decomposition (graph_blocks): both cover exactly k cycles with at most G per block."""
    from feanet_amd.solver import MultigridSolver
    G = MultigridSolver.GRAPH_CYCLES
    pb = MultigridSolver.pipe_blocks(k, G)
    assert sum(pb) == k and all(0 < b <= G for b in pb)
    assert sum(b != G for b in pb) <= 1 and (pb[-1] == k % G if k % G else pb[-1] == G)
    gb = MultigridSolver.graph_blocks(k, G)
    assert sum(gb) == k and all(b & (b - 1) == 0 for b in gb)


@pytest.mark.parametrize("problem", ["poisson", "interface"])
@pytest.mark.parametrize("L,tail", [(6, 5), (6, 4), (5, 2), (6, 3)])
def test_extend_tail_equals_per_level(problem, L, tail):
    """extend_tail (fea_mg_coarse_tail_ext: the level right above the coarse tail restricted into it and prolonged
    out of it in the tail's launch) after the level pairing: only a level the pairing left alone is absorbed (an odd
    number of zero-guess restrictions above the tail), and the rewritten schedule is the per-level V-cycle."""
    from feanet_amd.schedule import extend_tail, pair_prolongations, pair_restrictions
    n = 64
    rng = np.random.default_rng(23)
    mg = orc.OracleMultigrid(n, problem, np.float64, levels=L)
    mg.nu, mg.q2 = (1, 1), False
    v = rng.standard_normal((2, n + 1, n + 1))
    f = rng.standard_normal((2, n + 1, n + 1))
    steps, end = vcycle_schedule(L, 1, 1, tail_from=tail)
    ok = lambda l: l + 2 < L
    paired = pair_prolongations(pair_restrictions(steps, ok), ok)
    ext = extend_tail(paired)
    kinds = [s_[0] for s_ in ext]
    assert kinds.count("coarse_tail_ext") == (1 if (tail - 1) % 2 == 1 else 0), ext
    assert kinds.count("coarse_tail") + kinds.count("coarse_tail_ext") == 1
    ref = interpret(mg, steps, v, f)[0][end]
    np.testing.assert_array_equal(interpret(mg, ext, v, f)[0][end], ref)
    assert extend_tail(steps) != steps or tail == 1  # unpaired schedule: the level above the tail is always alone
