"""GPU parity of the multi-level launches (fea_mg_mid_down / fea_mg_mid_up, mid_ops.hip).

They must equal the per-level kernels they replace BITWISE (same per-node expressions, same order):
mid_down against a chain of fea_mg_residual_restrict(u = NULL, v_out = NULL), mid_up against a chain
of fea_mg_prolong_sweep(u = NULL) — on Poisson and two-material grids (distinct per-pattern R/P),
fp32 and fp64, batches 1 and 3, square and rectangular levels, tile sizes that do and do not divide
the interior, k = 1..4 levels per launch.  The solver with and without them is compared bitwise too
(its own V-cycle parity against the oracle is in test_gpu_mg.py)."""
import numpy as np
import pytest
import torch

from test_gpu_mg import Frame, tables

pytestmark = pytest.mark.gpu


def chain(n, m, k, B, T, problem):
    """k+1 framed levels (n x m intervals at the top) with random f / coarse data."""
    lv = []
    for j in range(k + 1):
        lv.append(Frame(n >> j, B, T, problem, m=m >> j))
    return lv


def pid_arr(lv, problem):
    from feanet_amd import _lib
    return _lib.PtrArray([f.pid() for f in lv]) if problem == "interface" else None


CASES = [  # (n, m, k, down tile, up tile); a region row must fit one wave (<= 64 columns)
    (64, 64, 2, 4, 16), (64, 64, 3, 2, 8), (128, 128, 3, 4, 32), (128, 64, 2, 8, 62), (256, 256, 4, 1, 24),
    (256, 128, 3, 5, 7), (512, 512, 3, 4, 32), (32, 32, 1, 3, 5), (1024, 1024, 3, 4, 62),
]


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,learned", [("poisson", False), ("interface", True)])
@pytest.mark.parametrize("n,m,k,tile,tile_up", CASES)
@pytest.mark.parametrize("B", [1, 3])
def test_mid_down_bitwise(T, problem, learned, n, m, k, tile, tile_up, B):
    from feanet_amd import _lib
    if problem == "interface" and n != m:
        pytest.skip("two-material problem is square")
    rng = np.random.default_rng(n + 7 * k + B)
    ktab, omd, R, P, kt, om, rt, pt = tables(problem, T, learned)
    nt = ktab.shape[0]
    w0 = 1.25
    lv = chain(n, m, k, B, T, problem)
    f0 = rng.standard_normal((B, lv[0].H, lv[0].W)).astype(np.float32 if T == torch.float32 else np.float64)
    lv[0].put("f", f0)
    # reference: per-level zero-guess residual + restriction, v not stored
    for j in range(k):
        _lib.call("mg_residual_restrict", T, None, lv[j].L.f.data_ptr(), None, lv[j + 1].L.f.data_ptr(), lv[j].pid(),
                  kt.data_ptr(), om.data_ptr(), nt, rt.data_ptr(), nt, w0, *lv[j].args(), lv[j + 1].L.ld,
                  lv[j + 1].L.bs, None)
    ref = [lv[j].get("f").copy() for j in range(1, k + 1)]
    for j in range(1, k + 1):
        lv[j].put("f", ref[j - 1] * 0 + 5.0)  # sentinel: boundary nodes must stay untouched
    fs = _lib.PtrArray([x.L.f.data_ptr() for x in lv])
    _lib.call("mg_mid_down", T, fs, pid_arr(lv, problem), k, B, lv[0].H, lv[0].W, kt.data_ptr(), om.data_ptr(), nt,
              rt.data_ptr(), nt, w0, tile, tile, None)
    for j in range(1, k + 1):
        out = lv[j].get("f")
        assert np.array_equal(out[:, 1:-1, 1:-1], ref[j - 1][:, 1:-1, 1:-1]), f"f_{j} differs"
        assert (out[:, 0, :] == 5).all() and (out[:, -1, :] == 5).all() and (out[:, :, 0] == 5).all() \
            and (out[:, :, -1] == 5).all(), f"boundary of f_{j} written"


@pytest.mark.parametrize("T", [torch.float32, torch.float64])
@pytest.mark.parametrize("problem,learned", [("poisson", False), ("interface", True)])
@pytest.mark.parametrize("n,m,k,tile_down,tile", CASES)
@pytest.mark.parametrize("B", [1, 3])
def test_mid_up_bitwise(T, problem, learned, n, m, k, tile_down, tile, B):
    from feanet_amd import _lib
    if problem == "interface" and n != m:
        pytest.skip("two-material problem is square")
    rng = np.random.default_rng(3 * n + k + B)
    npdt = np.float32 if T == torch.float32 else np.float64
    ktab, omd, R, P, kt, om, rt, pt = tables(problem, T, learned)
    nt = ktab.shape[0]
    w1 = 0.75
    lv = chain(n, m, k, B, T, problem)
    for j in range(k):
        lv[j].put("f", rng.standard_normal((B, lv[j].H, lv[j].W)).astype(npdt))
    e = rng.standard_normal((B, lv[k].H, lv[k].W)).astype(npdt)
    e[:, 0, :] = e[:, -1, :] = e[:, :, 0] = e[:, :, -1] = 0  # coarse iterates: zero Dirichlet data
    lv[k].put("a", e)
    # reference: per-level prolongation + correction + sweep from the recomputed zero-guess iterate
    for j in range(k - 1, -1, -1):
        lv[j].put("a", np.zeros((B, lv[j].H, lv[j].W), npdt))
        _lib.call("mg_prolong_sweep", T, None, lv[j + 1].L.a.data_ptr(), lv[j].L.f.data_ptr(), lv[j].L.a.data_ptr(),
                  lv[j].pid(), lv[j + 1].pid(), kt.data_ptr(), om.data_ptr(), nt, pt.data_ptr(), nt, w1,
                  *lv[j].args(), lv[j + 1].L.ld, lv[j + 1].L.bs, None)
    ref = lv[0].get("a").copy()
    lv[0].put("b", ref * 0 + 9.0)
    fs = _lib.PtrArray([x.L.f.data_ptr() for x in lv[:k]])
    _lib.call("mg_mid_up", T, fs, lv[k].L.a.data_ptr(), lv[0].L.b.data_ptr(), pid_arr(lv, problem), k, B,
              lv[0].H, lv[0].W, kt.data_ptr(), om.data_ptr(), nt, pt.data_ptr(), nt, w1, tile, tile, None)
    out = lv[0].get("b")
    assert np.array_equal(out[:, 1:-1, 1:-1], ref[:, 1:-1, 1:-1]), \
        f"u_a differs: max {np.abs(out - ref)[:, 1:-1, 1:-1].max():.3e}"
    assert (out[:, 0, :] == 9).all() and (out[:, -1, :] == 9).all() and (out[:, :, 0] == 9).all() \
        and (out[:, :, -1] == 9).all(), "boundary of u_a written"


def test_mid_rejects_oversized_tiles():
    from feanet_amd import _lib
    assert _lib.mid_lds_bytes(False, 4, 64, 64, 8, False) == -1
    assert _lib.mid_lds_bytes(False, 4, 2, 2, 8, False) == -1  # a 77-column region row
    assert _lib.mid_lds_bytes(True, 2, 64, 64, 8, False) == -1
    assert _lib.mid_lds_bytes(True, 2, 32, 32, 8, True) > 0
    lv = chain(256, 256, 2, 1, torch.float64, "poisson")
    ktab, omd, R, P, kt, om, rt, pt = tables("poisson", torch.float64)
    fs = _lib.PtrArray([x.L.f.data_ptr() for x in lv])
    with pytest.raises(RuntimeError, match="invalid arguments"):
        _lib.call("mg_mid_down", torch.float64, fs, None, 2, 1, lv[0].H, lv[0].W, kt.data_ptr(), om.data_ptr(), 1,
                  rt.data_ptr(), 1, 1.0, 200, 200, None)


@pytest.mark.parametrize("problem,n,B,T", [("poisson", 1024, 1, torch.float64), ("poisson", 2048, 1, torch.float64),
                                            ("poisson", 1024, 2, torch.float32), ("interface", 1024, 1, torch.float64)])
def test_solver_mid_bitwise(problem, n, B, T, monkeypatch):
    """MultigridSolver with the multi-level launches == without (bitwise), single and joined cycles.  The default
    grouping threshold (MID_NODES, <= 129^2) forms no group above the 65^2 tail; 300000 (the rounds-2-5 default,
    <= 513^2) makes the solver use them."""
    from feanet_amd.solver import MultigridSolver
    monkeypatch.setattr(MultigridSolver, "MID_NODES", 300000)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    f = torch.randn(B, 1, n + 1, n + 1, device="cuda", dtype=T, generator=g)
    outs = []
    for mid in (True, False):
        s = MultigridSolver(n, problem=problem, dtype=T, batch=B, mid=mid)
        kinds = [c[0] for c in s._plan("a")[0]]
        assert ("mg_mid_down" in kinds) == mid and ("mg_mid_up" in kinds) == mid, kinds
        s.set_rhs(f=f)
        s.load()
        s.vcycle()
        one = s.solution()
        s.vcycle(3)
        outs.append((one, s.solution()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_solver_rect_mid_bitwise():
    from feanet_amd.solver import MultigridSolver
    n, m = 1024, 512
    f = torch.randn(1, 1, m + 1, n + 1, device="cuda", dtype=torch.float64)
    outs = []
    for mid in (True, False):
        s = MultigridSolver(n, rows=m, dtype=torch.float64, mid=mid)
        s.set_rhs(f=f)
        s.load()
        s.vcycle(2)
        outs.append(s.solution())
    assert torch.equal(outs[0], outs[1])
