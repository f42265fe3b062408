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
  ("mid_down", a, k, T)                the zero-guess resid_restrict steps of levels a..a+k-1 (vout
                                       None) in one launch (mid_ops.hip, tile T of level a+k)
  ("mid_up", a, k, csrc, dst, T)       the "omdf" prolong_sweep steps of levels a+k-1..a in one
                                       launch: u_a[dst] from u_{a+k}[csrc] (tile T of level a)
                                       (group_mid rewrites a schedule into these)
  ("coarse_tail_ext", l, dst)          the zero-guess restriction of level l, the coarse tail of levels
                                       l+1..L-1 and level l's recomputed-iterate prolongation + sweep in one
                                       launch (fea_mg_coarse_tail_ext; extend_tail rewrites into it)

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
    recompute: a level starting from zero (l >= 1, and level 0 with top_zero) whose only pre-sweep is the
    zero-guess one keeps no iterate between its restriction and its prolongation: the prolongation
    recomputes omd*f_l (V(nu1=1, nu2>=1): 16 B per node less traffic in fp64, bitwise the same; the
    level's two steps can then join the multi-level launches)."""
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
            if recompute and (l >= 1 or top_zero) and nu2 >= 1:
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


def hjac_schedule(L, nu1=1, nu2=1, start="a", tail_from=None, fuse=False):
    """V-cycle of M-FEANet-mg_test.ipynb MultiGrid.Step with mode='hjac' (:27346-27372 with Relax =
    HJacIterator.HRelax, :147-155): every relaxation is one learned-smoother sweep ("hsweep", l, src,
    dst; src None = zero guess), so nothing is fused with the transfers:
    residual + restriction ("resid_restrict" with the current iterate) and prolongation + correction
    ("prolong_add") run as their own kernels; coarse levels start from zero, the coarsest gets
    nu1 + nu2 sweeps.  tail_from = t (1 <= t < L): levels t .. L-1 run as ONE ("hjac_tail", t, dst) step
    (fea_mg_hjac_tail, bitwise the steps it replaces) that reads f_t and writes level t's corrected iterate.
    fuse: a level's last pre-sweep runs with its residual + restriction ("hsweep_restrict", l, src, dst) and its
    prolongation + correction with the first post-sweep ("prolong_hsweep", l, u, e, dst; the corrected iterate
    is never stored) — fea_mg_hsweep_restrict / fea_mg_prolong_hsweep, bitwise the pairs they replace."""
    if L < 1 or nu1 < 0 or nu2 < 0:
        raise ValueError("hjac_schedule: need L >= 1, nu1, nu2 >= 0")
    if tail_from is not None and not 1 <= tail_from < L:
        raise ValueError(f"hjac_schedule: tail_from={tail_from} outside [1, {L - 1}]")
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
    top = L - 1 if tail_from is None else tail_from  # first level not streamed level by level

    def pre_restrict(l):  # nu1 pre-sweeps of level l, then its residual + restriction
        for i in range(nu1):
            if fuse and i == nu1 - 1:
                dst = "a" if cur[l] == "zero" else _other(cur[l])
                steps.append(("hsweep_restrict", l, None if cur[l] == "zero" else cur[l], dst))
                cur[l] = dst
                return
            hs(l)
        steps.append(("resid_restrict", l, cur[l], None))

    for l in range(top):
        pre_restrict(l)
    if tail_from is None:
        for _ in range(nu1 + nu2):
            hs(L - 1)
    else:
        steps.append(("hjac_tail", tail_from, "a"))
        cur[tail_from] = "a"
    for l in range(top - 1, -1, -1):
        dst = "a" if cur[l] == "zero" else _other(cur[l])
        if fuse and nu2 >= 1:
            steps.append(("prolong_hsweep", l, cur[l], cur[l + 1], dst))
            cur[l] = dst
            for _ in range(nu2 - 1):
                hs(l)
            continue
        steps.append(("prolong_add", l, cur[l], cur[l + 1], dst))
        cur[l] = dst
        for _ in range(nu2):
            hs(l)
    return steps, cur[0]


def group_hmid(steps, pairs):
    """Rewrite the fused HJac V(1,1) steps (hjac_schedule(fuse=True)) of two consecutive coarse levels a, a+1 into
    one launch each way, for every (a, T_down, T_up) in `pairs`: the two zero-guess
    ("hsweep_restrict", a, None, da), ("hsweep_restrict", a+1, None, da1) become ("hmid_down", a, da, da1, T_down)
    (fea_mg_hmid_down), and ("prolong_hsweep", a+1, u1, e, d1), ("prolong_hsweep", a, u0, d1, d0) become
    ("hmid_up", a, u0, u1, e, d0, T_up) (fea_mg_hmid_up; level a+1's new iterate is not stored) — bitwise the
    pairs.  Steps that do not have that shape (nu1, nu2 != 1, a stored guess) are left alone."""
    want = {a: (td, tu) for a, td, tu in pairs}
    out = []
    i = 0
    while i < len(steps):
        st = steps[i]
        nx = steps[i + 1] if i + 1 < len(steps) else None
        if (nx is not None and st[0] == "hsweep_restrict" and nx[0] == "hsweep_restrict" and st[1] in want
                and nx[1] == st[1] + 1 and st[2] is None and nx[2] is None):
            out.append(("hmid_down", st[1], st[3], nx[3], want[st[1]][0]))
            i += 2
            continue
        if (nx is not None and st[0] == "prolong_hsweep" and nx[0] == "prolong_hsweep" and nx[1] in want
                and st[1] == nx[1] + 1 and nx[3] == st[4]):
            out.append(("hmid_up", nx[1], nx[2], st[2], st[3], nx[4], want[nx[1]][1]))
            i += 2
            continue
        out.append(st)
        i += 1
    return out


def pair_restrictions(steps, can_pair):
    """Rewrite two consecutive single-level zero-guess restrictions (("resid_restrict", l, None, None), then
    the same at l + 1) into one ("resid_restrict2", l) step — fea_mg_zero_restrict2, bitwise the two —
    where can_pair(l) allows it.  Run after group_mid (the levels it leaves to single-level launches)."""
    out = []
    i = 0
    zr = lambda st: st[0] == "resid_restrict" and st[2] is None and st[3] is None
    while i < len(steps):
        st = steps[i]
        if (zr(st) and i + 1 < len(steps) and zr(steps[i + 1]) and steps[i + 1][1] == st[1] + 1
                and can_pair(st[1])):
            out.append(("resid_restrict2", st[1]))
            i += 2
            continue
        out.append(st)
        i += 1
    return out


def pair_prolongations(steps, can_pair, finest_first=True):
    """Rewrite two consecutive recomputed-iterate prolongations (("prolong_sweep", l+1, OMDF, c, d), then
    ("prolong_sweep", l, OMDF, d, e)) into one ("prolong_sweep2", l, c, e) step — fea_mg_prolong2, bitwise
    the two; the intermediate iterate d of level l+1 is then never stored — where can_pair(l) allows it.
    Within a run of chained prolongations the FINEST levels pair first (the run is paired from its end): the
    iterate a pair keeps out of HBM is the larger one there (C5, 1025^2 x 256: levels 2-1 paired, level 3 alone,
    instead of 3-2 paired and level 1 alone).  finest_first=False pairs from the run's start (the coarsest levels
    first: the domain decomposition keeps that, so the pair right under the agglomeration level reads the coarse
    solution in place, DDSolver._scatter_direct)."""
    ps = lambda st: st[0] == "prolong_sweep" and st[2] == OMDF
    chained = lambda a, b: ps(a) and ps(b) and b[1] == a[1] - 1 and b[3] == a[4]
    out = []
    i = 0
    while i < len(steps):
        if not ps(steps[i]):
            out.append(steps[i])
            i += 1
            continue
        j = i + 1  # the run steps[i:j] of chained prolongations
        while j < len(steps) and chained(steps[j - 1], steps[j]):
            j += 1
        run, paired = steps[i:j], []
        if finest_first:
            k = len(run)
            while k > 0:
                if k >= 2 and can_pair(run[k - 1][1]):
                    paired.append(("prolong_sweep2", run[k - 1][1], run[k - 2][3], run[k - 1][4]))
                    k -= 2
                else:
                    paired.append(run[k - 1])
                    k -= 1
            paired.reverse()
        else:
            k = 0
            while k < len(run):
                if k + 1 < len(run) and can_pair(run[k + 1][1]):
                    paired.append(("prolong_sweep2", run[k + 1][1], run[k][3], run[k + 1][4]))
                    k += 2
                else:
                    paired.append(run[k])
                    k += 1
        out.extend(paired)
        i = j
    return out


def group_mid(steps, pick_down, pick_up):
    """Rewrite runs of consecutive zero-guess restrictions (("resid_restrict", l, None, None), l
    ascending) and of recomputed prolongations (("prolong_sweep", l, OMDF, csrc, dst), l descending)
    into multi-level launches.  pick_down(levels) / pick_up(levels) get the run's levels (ascending)
    and return [(a, k, T), ...]: disjoint groups of consecutive levels (a .. a+k-1, k >= 2) with the
    tile size; levels left out keep their single-level step."""
    out = []
    i = 0
    n = len(steps)
    while i < n:
        st = steps[i]
        if st[0] == "resid_restrict" and st[2] is None and st[3] is None:
            j = i
            while (j + 1 < n and steps[j + 1][0] == "resid_restrict" and steps[j + 1][2] is None
                   and steps[j + 1][3] is None and steps[j + 1][1] == steps[j][1] + 1):
                j += 1
            run = steps[i:j + 1]
            groups = {a: (k, T) for a, k, T in pick_down([s_[1] for s_ in run])}
            m = 0
            while m < len(run):
                l = run[m][1]
                if l in groups:
                    k, T = groups[l]
                    out.append(("mid_down", l, k, T))
                    m += k
                else:
                    out.append(run[m])
                    m += 1
            i = j + 1
            continue
        if st[0] == "prolong_sweep" and st[2] == OMDF:
            j = i
            while (j + 1 < n and steps[j + 1][0] == "prolong_sweep" and steps[j + 1][2] == OMDF
                   and steps[j + 1][1] == steps[j][1] - 1):
                j += 1
            run = steps[i:j + 1]  # levels descending
            by_level = {s_[1]: s_ for s_ in run}
            groups = {a: (k, T) for a, k, T in pick_up(sorted(by_level))}
            m = 0
            while m < len(run):
                l = run[m][1]
                a = next((a_ for a_, (k_, _) in groups.items() if a_ + k_ - 1 == l), None)
                if a is not None:
                    k, T = groups[a]
                    out.append(("mid_up", a, k, by_level[a + k - 1][3], by_level[a][4], T))
                    m += k
                else:
                    out.append(run[m])
                    m += 1
            i = j + 1
            continue
        out.append(st)
        i += 1
    return out


def extend_tail(steps):
    """Rewrite ("resid_restrict", l, None, None), ("coarse_tail", l+1, c), ("prolong_sweep", l, OMDF, c, dst) — the
    level right above the coarse tail going down into it and back up — into ONE ("coarse_tail_ext", l, dst) step
    (fea_mg_coarse_tail_ext, bitwise the three launches).  Run after pair_restrictions / pair_prolongations: only a
    level they left to single-level launches has that shape."""
    out = []
    i = 0
    while i < len(steps):
        st = steps[i]
        if (i + 2 < len(steps) and st[0] == "resid_restrict" and st[2] is None and st[3] is None
                and steps[i + 1][0] == "coarse_tail" and steps[i + 1][1] == st[1] + 1
                and steps[i + 2][0] == "prolong_sweep" and steps[i + 2][1] == st[1] and steps[i + 2][2] == OMDF
                and steps[i + 2][3] == steps[i + 1][2]):
            out.append(("coarse_tail_ext", st[1], steps[i + 2][4]))
            i += 3
            continue
        out.append(st)
        i += 1
    return out
