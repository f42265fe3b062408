"""BASELINE.json configurations as GPU parity cases: each checked against the oracle or
against the single-GPU path, at the configuration's own size.
  C2  1025^2 Poisson fp64, 6-level V-cycle                      -> oracle, every cycle, 1e-10
  C3  2049^2 two-material, learned R/P ratio (multigrid.py)     -> oracle, three cycles, 1e-10 + convergence
  C4  8193^2 Poisson fp64 over 8 ranks (slabs, 4 x 2 blocks)   -> bitwise the single-GPU V-cycle,
                                                                   which is checked against the oracle
  C5  256 x 1025^2 fp32 batch                                   -> bitwise per-sample independence,
                                                                   oracle fp32 first cycle of 3 samples,
                                                                   their residual norms over 3 cycles
"""
import os

import numpy as np
import pytest
import torch

from oracle import feanet_oracle as orc

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_c2_1025_six_levels_vs_oracle():
    from feanet_amd.solver import MultigridSolver
    n, L = 1024, 6
    rng = np.random.default_rng(2)
    f = rng.standard_normal((1, n + 1, n + 1))
    mg = orc.OracleMultigrid(n, "poisson", np.float64, levels=L)
    s = MultigridSolver(n, levels=L, dtype=torch.float64)
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(1, 1, n + 1, n + 1))
    s.load()
    v = np.zeros_like(f)
    for k in range(3):
        s.vcycle()
        v = mg.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        assert np.abs(got - v).max() / np.abs(v).max() < 1e-10, k
    # Q3: a 6-level cycle whose coarsest grid (33^2) gets 2 sweeps converges slowly but steadily
    r = [float(s.residual_norm()[0])]
    s.vcycle(4)
    r.append(float(s.residual_norm()[0]))
    assert r[1] < r[0]


def test_c3_2049_interface_learned_ratio():
    from feanet_amd.solver import MultigridSolver
    w = np.load(os.path.join(HERE, "..", "multigrid-feanet_amd", "feanet_amd", "weights", "multigrid_interface_ratio.npz"))
    n = 2048
    s = MultigridSolver(n, problem="interface", dtype=torch.float64, R=w["R"][0], P=w["P"][:, 0], w=w["w"])
    F = torch.ones(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64)
    s.set_rhs(F=F)
    s.load()
    r0 = float(s.residual_norm()[0])
    # oracle: same operators; pattern maps computed by the ORACLE's own element/node loop
    # (tests/golden/c3_pattern_maps.npz, made by tests/golden/make_c3_maps.py and re-checked against
    # the loop in the CPU suite, tests/test_setup.py::test_c3_maps_fixture_is_oracle)
    maps = np.load(os.path.join(HERE, "golden", "c3_pattern_maps.npz"))
    pids = {int(k[4:]): maps[k] for k in maps.files if k.startswith("pid_")}
    mg = orc.OracleMultigrid(n, "interface", np.float64, levels=s.L, pids=pids,
                             rtab=np.broadcast_to(np.asarray(w["R"][0], np.float32), (16, 3, 3)),
                             ptab=np.asarray(w["P"][:, 0], np.float32), w=tuple(float(x) for x in w["w"]))
    f = orc.conv3x3(np.ones((1, n + 1, n + 1)), orc.fnet_stencil(2.0 / n))
    v = np.zeros((1, n + 1, n + 1))
    # one plain V-cycle, then two joined ones (fea_mg_cycle_join with the two-material tables)
    for k, cyc in enumerate((1, 2)):
        s.vcycle(cyc)
        for _ in range(cyc):
            v = mg.step(v, f)
        got = s.solution().cpu().numpy()[:, 0]
        assert np.abs(got - v).max() / np.abs(v).max() < 1e-10, k
    res, ref = float(s.residual_norm()[0]), float(mg.residual_norm(v, f)[0])
    assert abs(res - ref) <= 1e-9 * ref, (res, ref)
    # converges, slowly at this size (contrast 20, and the reference's coarsest level is two Jacobi
    # sweeps on 3^2), not strictly monotonically per cycle; over two cycles always
    r = [float(s.residual_norm()[0])]
    for _ in range(13):
        s.vcycle()
        r.append(float(s.residual_norm()[0]))
    assert all(b < a for a, b in zip(r, r[2:])), r
    assert r[-1] / r0 < 0.05, r


@pytest.mark.parametrize("grid", [(8, 1), (4, 2)])
def test_c4_8193_dd_eight_ranks_bitwise(grid):
    """C4: 8193^2 over 8 ranks (row slabs, and the 4 x 2 blocks bench.py runs on 8 GPUs), in-process."""
    from feanet_amd.dd import LocalGroup
    from feanet_amd.solver import MultigridSolver
    n = 8192
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    f = torch.randn(1, 1, n + 1, n + 1, device="cuda", dtype=torch.float64, generator=g)
    s = MultigridSolver(n, dtype=torch.float64)
    s.set_rhs(f=f)
    s.load()
    grp = LocalGroup(n, n, 8, grid=grid)
    grp.set_rhs(f)
    grp.load()
    for k in range(2):
        s.vcycle()
        grp.vcycle()
        assert torch.equal(grp.solution(), s.solution()), k
    torch.testing.assert_close(grp.residual_norm(), s.residual_norm(), rtol=1e-12, atol=0)


def test_c4_8193_single_vs_oracle():
    """C4's grid against the oracle's MultiGrid.Step (M-FEANet-mg_test.ipynb:27346-27372): one V-cycle,
    then two joined ones, 13 levels, 1e-10 of max|u| (~6 s per oracle cycle on the host).  The decomposed
    runs above are bitwise this single-GPU path, so they are pinned to the oracle through it."""
    from feanet_amd.solver import MultigridSolver
    n = 8192
    N = n + 1
    rng = np.random.default_rng(8193)
    f = rng.standard_normal((1, N, N))
    mg_o = orc.OracleMultigrid(n, "poisson", np.float64)
    s = MultigridSolver(n, dtype=torch.float64)
    assert s.L == mg_o.L == 13
    s.set_rhs(f=torch.from_numpy(f).cuda().reshape(1, 1, N, N))
    s.load()
    v = np.zeros_like(f)
    s.vcycle()
    v = mg_o.step(v, f)
    got = s.solution().cpu().numpy()[:, 0]
    assert np.abs(got - v).max() / np.abs(v).max() < 1e-10, "first cycle"
    s.vcycle(2)
    for _ in range(2):
        v = mg_o.step(v, f)
    got = s.solution().cpu().numpy()[:, 0]
    assert np.abs(got - v).max() / np.abs(v).max() < 1e-10, "joined cycles 2-3"
    res, ref = float(s.residual_norm()[0]), float(mg_o.residual_norm(v, f)[0])
    assert abs(res - ref) <= 1e-9 * ref, (res, ref)


def test_c5_batch256_1025_fp32():
    """C5: 256 nodal sources from the six families of the reference's RHS generator
    (Data/RHS/generate_rhs.py:6-56, tools/rhs_families.py), FNet applied on the device."""
    import sys
    sys.path.insert(0, os.path.join(HERE, ".."))
    from tools import rhs_families
    from feanet_amd.solver import MultigridSolver
    n, B = 1024, 256
    F = rhs_families.batch(B, n + 1, torch.float32, "cuda", seed=5)
    s = MultigridSolver(n, dtype=torch.float32, batch=B)
    s.set_rhs(F=F)
    f = s.levels[0].view(s.levels[0].f).unsqueeze(1).clone()
    s.load()
    r0 = s.residual_norm()
    s.vcycle(3)
    ub = s.solution()
    r3 = s.residual_norm()
    assert bool((r3 < 0.1 * r0).all())
    for b in (0, 97, 255):
        s1 = MultigridSolver(n, dtype=torch.float32, batch=1)
        s1.set_rhs(f=f[b:b + 1])
        s1.load()
        s1.vcycle(3)
        assert torch.equal(s1.solution()[0], ub[b]), b
    # the oracle's fp32 MultiGrid.Step on three of the samples, first cycle (as test_gpu_mg's fp32
    # cycles: later fp32 iterates of two implementations drift apart by cond(K) eps32, and with these
    # smooth sources the residual after 3 cycles is already at that rounding floor, so it is not compared);
    # the batch-256 run is bitwise these samples' own runs (above)
    idx = [0, 97, 255]
    s3 = MultigridSolver(n, dtype=torch.float32, batch=3)
    s3.set_rhs(f=f[idx])
    s3.load()
    mg = orc.OracleMultigrid(n, "poisson", np.float32)
    fb = f[idx, 0].cpu().numpy()
    r0 = orc.interior_norm(fb - mg.levels[0].K(np.zeros_like(fb)))
    v = np.zeros_like(fb)
    for k in range(3):
        s3.vcycle()
        v = mg.step(v, fb)
        if k == 0:
            got = s3.solution().cpu().numpy()[:, 0]
            for i in range(3):
                err = np.abs(got[i] - v[i]).max() / np.abs(v[i]).max()
                assert err < 2e-5, (idx[i], err)
        # residual norms of every cycle to 1 % + 1e-3 of the initial residual: with these smooth sources r is a
        # small difference of large K u terms, and two fp32 implementations' iterates differ by cond(K) eps32,
        # so the two residuals differ by ~1e-5 absolute (0.5 % after one cycle, 3 % after three, where r has
        # come down to ~1e-4, measured); a wrong schedule changes the per-cycle contraction (~0.2) far more
        np.testing.assert_allclose(s3.residual_norm().cpu().numpy(), orc.interior_norm(fb - mg.levels[0].K(v)),
                                   rtol=1e-2, atol=1e-3 * float(r0.max()), err_msg=f"cycle {k + 1}")
