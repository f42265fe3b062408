"""Symbolic V-cycle schedule (pure host logic, no device code).

One V-cycle of the reference drivers is expressed as a list of fused level steps over named
buffers ("a", "b" ping-pong, "zero" an all-zero field).  The MultigridSolver binds the steps to
C-ABI calls with device pointers; tests interpret the same list with the CPU oracle to show the
fused schedule equals the reference's op sequence.

Steps:
  ("sweep", l, src, dst)               dst = J_l(src, f_l); src None means a zero initial guess
  ("resid_restrict", l, src, vout)     f_{l+1} = w0 R(f_l - K_l src); src None: zero-guess sweep
                                       fused first (v = omd*f_l written to vout, then restricted;
                                       vout None: v is not stored, the level's iterate becomes the
                                       virtual buffer "omdf")
  ("sweep_restrict", l, src, dst)      dst = J_l(src, f_l) and f_{l+1} = w0 R(f_l - K_l dst) in one pass
  ("prolong_sweep", l, src, csrc, dst) dst = J_l(src + w1 P(v_{l+1}[csrc]), f_l); src "omdf": the
                                       zero-guess pre-sweep omd*f_l, recomputed from f_l in the kernel
  ("prolong_add", l, src, csrc, dst)   dst = src + w1 P(v_{l+1}[csrc])
  ("coarse_tail", t, dst)              levels t..L-1 in one launch (coarse_tail.hip): from f_t and a
                                       zero guess, the coarse part of this same schedule; v_t -> dst

Semantics reproduced:
  * nu1 = nu2 = 1: MultiGrid.Step (M-FEANet-mg_test.ipynb:27346-27372) == MultiGrid.iterate
    (FEANet/multigrid.py:159-185): coarse levels start from zero, coarsest gets nu1 + nu2 sweeps.
  * general nu1, nu2: Multigrid.rec_V_cycle (MM_Model_convergence.ipynb:132-148).
  * compat="mm_interface_q2": MM_Interface_error.ipynb:132-150, whose pre-smoothing is applied to
    grids[0] at every depth.
"""


def _other(b):
    return "b" if b == "a" else "a"


OMDF = "omdf"  # virtual buffer: a coarse level's zero-guess pre-sweep omd*f, recomputed where read


def vcycle_schedule(L, nu1=1, nu2=1, compat=None, start="a", tail_from=None, fuse=True, top_zero=False,
                    recompute=True):
    """tail_from = t (1 <= t <= L-1): levels t..L-1 run as one coarse_tail step.
    fuse: the last pre-sweep of a level with a given iterate runs fused with its residual and
    restriction (sweep_restrict).
    top_zero: level 0 starts from a zero guess like the coarse levels (the coarse sub-cycle of a
    domain-decomposed V-cycle, run on the agglomerated level; bitwise the single-grid coarse part).
    recompute: a coarse level (l >= 1) whose only pre-sweep is the zero-guess one keeps no iterate
    between its restriction and its prolongation: the prolongation recomputes omd*f_l (V(nu1=1,
    nu2>=1): 16 B per node less traffic in fp64, bitwise the same)."""
    if tail_from is not None and not (1 <= tail_from <= L - 1):
        raise ValueError("vcycle_schedule: tail_from must be in [1, L-1]")
    if L < 1 or nu1 < 0 or nu2 < 0:
        raise ValueError("vcycle_schedule: need L >= 1, nu1, nu2 >= 0")
    if compat not in (None, "mm_interface_q2"):
        raise ValueError(f"vcycle_schedule: unknown compat mode {compat!r}")
    steps = []
    cur = ["zero"] * L
    cur[0] = "zero" if top_zero else start

    def sweep(l, zero=False):
        dst = "a" if (zero or cur[l] == "zero") else _other(cur[l])
        steps.append(("sweep", l, None if (zero or cur[l] == "zero") else cur[l], dst))
        cur[l] = dst

    if L == 1:
        for _ in range(nu1 + nu2):
            sweep(0)
        return steps, cur[0]
    q2 = compat == "mm_interface_q2"

    def presmooth_restrict(l, nsweeps, from_zero):
        """nsweeps pre-sweeps of level l (the first from zero if from_zero), then residual + restriction."""
        if nsweeps == 0:
            steps.append(("resid_restrict", l, cur[l], None))
            return
        if from_zero and nsweeps == 1:
            if recompute and l >= 1 and nu2 >= 1:
                steps.append(("resid_restrict", l, None, None))
                cur[l] = OMDF
            else:
                steps.append(("resid_restrict", l, None, "a"))
                cur[l] = "a"
            return
        first = True
        for i in range(nsweeps - (1 if fuse else 0)):
            sweep(l, zero=(from_zero and first))
            first = False
        if fuse:
            dst = _other(cur[l]) if cur[l] != "zero" else "a"
            steps.append(("sweep_restrict", l, cur[l], dst))
            cur[l] = dst
        else:
            steps.append(("resid_restrict", l, cur[l], None))

    # ---- down
    if top_zero and nu1 > 0 and not q2:
        presmooth_restrict(0, nu1, True)
    elif top_zero:
        steps.append(("resid_restrict", 0, "zero", None))
    else:
        presmooth_restrict(0, nu1, False)
    if q2:
        for _ in range((L - 1) * nu1):
            sweep(0)
    last_down = L - 1 if tail_from is None else tail_from
    for l in range(1, last_down):
        if q2 or nu1 == 0:
            cur[l] = "zero"
            steps.append(("resid_restrict", l, "zero", None))
        else:
            presmooth_restrict(l, nu1, True)
    if tail_from is not None:
        steps.append(("coarse_tail", tail_from, "a"))
        cur[tail_from] = "a"
        top = tail_from - 1
    else:
        # ---- coarsest
        ncs = nu2 if q2 else nu1 + nu2
        if ncs > 0:
            sweep(L - 1, zero=True)
            for _ in range(ncs - 1):
                sweep(L - 1)
        else:
            cur[L - 1] = "zero"
        top = L - 2
    # ---- up
    for l in range(top, -1, -1):
        dst = "a" if cur[l] in ("zero", OMDF) else _other(cur[l])
        steps.append(("prolong_sweep" if nu2 >= 1 else "prolong_add", l, cur[l], cur[l + 1], dst))
        cur[l] = dst
        for _ in range(max(nu2 - 1, 0)):
            sweep(l)
    return steps, cur[0]


def hjac_schedule(L, nu1=1, nu2=1, start="a"):
    """V-cycle of M-FEANet-mg_test.ipynb MultiGrid.Step with mode='hjac' (:27346-27372 with Relax =
    HJacIterator.HRelax, :147-155): every relaxation is one learned-smoother sweep ("hsweep", l, src,
    dst; src None = zero guess), so nothing is fused with the transfers:
    residual + restriction ("resid_restrict" with the current iterate) and prolongation + correction
    ("prolong_add") run as their own kernels; coarse levels start from zero, the coarsest gets
    nu1 + nu2 sweeps."""
    if L < 1 or nu1 < 0 or nu2 < 0:
        raise ValueError("hjac_schedule: need L >= 1, nu1, nu2 >= 0")
    steps = []
    cur = ["zero"] * L
    cur[0] = start

    def hs(l):
        dst = "a" if cur[l] == "zero" else _other(cur[l])
        steps.append(("hsweep", l, None if cur[l] == "zero" else cur[l], dst))
        cur[l] = dst

    if L == 1:
        for _ in range(nu1 + nu2):
            hs(0)
        return steps, cur[0]
    for _ in range(nu1):
        hs(0)
    for l in range(L - 1):
        steps.append(("resid_restrict", l, cur[l], None))
        if l + 1 < L - 1:
            for _ in range(nu1):
                hs(l + 1)
    for _ in range(nu1 + nu2):
        hs(L - 1)
    for l in range(L - 2, -1, -1):
        dst = "a" if cur[l] == "zero" else _other(cur[l])
        steps.append(("prolong_add", l, cur[l], cur[l + 1], dst))
        cur[l] = dst
        for _ in range(nu2):
            hs(l)
    return steps, cur[0]
