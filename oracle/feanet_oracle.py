"""CPU oracle for the FEANet geometric-multigrid hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the reference algorithm
(longfish/Multigrid-FEANet, FEANet/{mesh,geo,model,jacobi,multigrid}.py and the
notebook drivers).  It exists to CHECK the HIP product path; it is never the
thing measured (except as the `cpu_baseline` leg of bench.py) and nothing in
`multigrid-feanet_amd/` may import it.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline may use it.

Parity pinning: every function here is checked against golden vectors that
were produced by running the reference itself (tests/golden/make_golden.py,
fixtures under tests/golden/*.npz) in tests/test_oracle_golden.py.

Conventions: fields are [B, 1, N, N] (or [B, N, N]); node (r, c);
boundary = rows/cols 0 and N-1; N = n + 1 nodes per edge.  Arithmetic stays in
the dtype of the inputs (float32 or float64), tables are the reference's
float32 values cast to that dtype.
"""
import numpy as np

# ---------------------------------------------------------------------------
# A1/A2: discretisation setup
# ---------------------------------------------------------------------------
# FEANet/mesh.py:23-26 — quadrant phases [e1, e2, e3, e4] -> pattern id
REF_PATTERNS = {0: (0, 0, 0, 0), 1: (1, 1, 1, 1), 2: (0, 0, 0, 1), 3: (0, 0, 1, 0),
                4: (1, 0, 0, 0), 5: (0, 1, 0, 0), 6: (0, 0, 1, 1), 7: (1, 1, 0, 0),
                8: (0, 1, 1, 0), 9: (1, 0, 0, 1), 10: (0, 1, 0, 1), 11: (1, 0, 1, 0),
                12: (1, 1, 1, 0), 13: (1, 1, 0, 1), 14: (0, 1, 1, 1), 15: (1, 0, 1, 1)}


def element_stiffness():
    """Q1 element stiffness, float32 (FEANet/mesh.py:28-31)."""
    return np.float32(-1.0 / 6.0) * np.array([[-4., 1., 2., 1.],
                                              [1., -4., 1., 2.],
                                              [2., 1., -4., 1.],
                                              [1., 2., 1., -4.]], dtype=np.float32)


def pattern_stencil(a, pattern, Ke=None):
    """3x3 stencil of one node pattern (FEANet/mesh.py:103-117, same float32 op order)."""
    Ke = element_stiffness() if Ke is None else Ke
    a = np.asarray(a, dtype=np.float32)
    p = pattern
    k = np.zeros((3, 3), dtype=np.float32)
    k[0, 0] = a[p[3]] * Ke[1, 3]
    k[0, 1] = a[p[3]] * Ke[1, 2] + a[p[2]] * Ke[0, 3]
    k[0, 2] = a[p[2]] * Ke[0, 2]
    k[1, 0] = a[p[0]] * Ke[2, 3] + a[p[3]] * Ke[1, 0]
    k[1, 1] = a[p[2]] * Ke[0, 0] + a[p[3]] * Ke[1, 1] + a[p[0]] * Ke[2, 2] + a[p[1]] * Ke[3, 3]
    k[1, 2] = a[p[1]] * Ke[3, 2] + a[p[2]] * Ke[0, 1]
    k[2, 0] = a[p[0]] * Ke[2, 0]
    k[2, 1] = a[p[0]] * Ke[2, 1] + a[p[1]] * Ke[3, 0]
    k[2, 2] = a[p[1]] * Ke[3, 1]
    return k


def _hw(N):
    return (N, N) if np.isscalar(N) else tuple(N)


def square_mesh(N):
    """MeshSquare (FEANet/mesh.py:122-189): one pattern (all-background), every node pattern 0.
    N: nodes per edge, or (H, W) for the rectangular extension used by the domain-decomposed path."""
    ktab = pattern_stencil(np.array([1.], np.float32), REF_PATTERNS[0])[None]
    return ktab, np.zeros(_hw(N), np.uint8)


def interface_mesh(N, prop=(1, 20), shape=0, size=2):
    """MeshCenterInterface (FEANet/mesh.py:4-117): element phases from float32 centroids
    (place_circle :62-68 / place_rect :70-76), node pattern from the four surrounding
    elements (identify_patterns :78-93, quadrant tests on centroid vs node), 16 stencils.
    Written as an element loop + node loop (O(N^2)); no vectorised shortcut, so it is an
    independent check on the product's setup code."""
    x = np.linspace(size / 2, -size / 2, N, dtype=np.float32)  # mesh.py:46 (decreasing)
    y = np.linspace(-size / 2, size / 2, N, dtype=np.float32)  # mesh.py:47
    ne = N - 1
    phase = np.zeros((ne, ne), np.int64)
    cx = np.zeros((ne, ne), np.float32)
    cy = np.zeros((ne, ne), np.float32)
    for er in range(ne):
        for ec in range(ne):
            # element nodes (er,ec),(er,ec+1),(er+1,ec+1),(er+1,ec) -> np.mean of float32 points
            px = np.array([x[ec], x[ec + 1], x[ec + 1], x[ec]], np.float32)
            py = np.array([y[er], y[er], y[er + 1], y[er + 1]], np.float32)
            mx, my = np.mean(px), np.mean(py)
            cx[er, ec], cy[er, ec] = mx, my
            if shape == 0:
                if (mx - 0.) ** 2 + (my - 0.) ** 2 < 0.5 ** 2:
                    phase[er, ec] = 1
            else:
                if abs(mx - 0) < 0.5 and abs(my - 0) < 0.5:
                    phase[er, ec] = 1
    lut = {v: k for k, v in REF_PATTERNS.items()}
    pid = np.zeros((N, N), np.uint8)
    for r in range(1, N - 1):          # boundary nodes have < 4 elements -> pattern 0
        for c in range(1, N - 1):
            bits = [0, 0, 0, 0]
            for er, ec in ((r - 1, c - 1), (r - 1, c), (r, c - 1), (r, c)):
                if phase[er, ec] != 1:
                    continue
                ex, ey, px, py = cx[er, ec], cy[er, ec], x[c], y[r]
                if ex < px and ey < py:
                    bits[0] = 1
                if ex > px and ey < py:
                    bits[1] = 1
                if ex > px and ey > py:
                    bits[2] = 1
                if ex < px and ey > py:
                    bits[3] = 1
            pid[r, c] = lut[tuple(bits)]
    a = np.array(prop, np.float32)
    ktab = np.stack([pattern_stencil(a, REF_PATTERNS[k]) for k in range(16)])
    return ktab, pid


def square_geometry(N, dtype=np.float32):
    """Geometry.square_geometry (FEANet/geo.py:13-30): 1 inside, 0 on the boundary; zero bc.
    N: nodes per edge or (H, W)."""
    geo = np.ones(_hw(N), dtype)
    geo[0, :] = geo[-1, :] = geo[:, 0] = geo[:, -1] = 0
    return geo, np.zeros(_hw(N), dtype)


def fnet_stencil(h):
    """FNet mass stencil, float32 (FEANet/model.py:54-56)."""
    return np.array([[h * h / 36., h * h / 9., h * h / 36.],
                     [h * h / 9., 4. * h * h / 9., h * h / 9.],
                     [h * h / 36., h * h / 9., h * h / 36.]], dtype=np.float32)


# ---------------------------------------------------------------------------
# A5-A10: operators
# ---------------------------------------------------------------------------
def _as3(x):
    x = np.asarray(x)
    return x.reshape((-1,) + x.shape[-2:])


def knet_apply(u, pid, ktab):
    """K u (FEANet/model.py:22-30): identity split, per-pattern mask on the INPUT node, then
    per-pattern 3x3 cross-correlation with zero padding:
        y[i] = sum_d W_{p(i+d)}[d] * u[i+d]."""
    shape = np.shape(u)
    u3 = _as3(u)
    dt = u3.dtype
    B, H, W = u3.shape
    tab = np.asarray(ktab, np.float32).astype(dt)
    up = np.zeros((B, H + 2, W + 2), dt)
    up[:, 1:-1, 1:-1] = u3
    pp = np.zeros((H + 2, W + 2), np.int64)
    pp[1:-1, 1:-1] = pid
    y = np.zeros((B, H, W), dt)
    single = tab.shape[0] == 1 or not np.any(pp)
    for dr in range(3):
        for dc in range(3):
            coef = tab[0, dr, dc] if single else tab[pp[dr:dr + H, dc:dc + W], dr, dc]
            y += coef * up[:, dr:dr + H, dc:dc + W]
    return y.reshape(shape)


def split_x(x, pid, nch):
    """KNet.split_x (FEANet/model.py:37-47): x_split[:, p] = mask_p * x  -> [B, C, H, W]."""
    x3 = _as3(x)
    out = np.zeros((x3.shape[0], nch) + x3.shape[1:], x3.dtype)
    for p in range(nch):
        out[:, p] = np.where(pid == p, x3, 0)
    return out


def conv3x3(x, w):
    """Single-channel 3x3 cross-correlation, zero padding 1 (FNet.forward, model.py:60-61; HNet)."""
    N = np.shape(x)[-1]
    return knet_apply(x, np.zeros(np.shape(x)[-2:], np.uint8), np.asarray(w, np.float32)[None])


def omega_over_d(ktab, omega, dtype):
    """omega / d_mat as evaluated in jacobi.py:45 (`self.omega/self.d_mat`): d = centre weight of the
    node's pattern (jacobi.py:31-37); torch evaluates scalar/tensor as reciprocal(d) * omega in dtype."""
    d = np.asarray(ktab, np.float32)[:, 1, 1].astype(dtype)
    return (np.reciprocal(d) * dtype(omega)).astype(dtype)


def jacobi_sweep(u, f, pid, ktab, geo, bc, omega=2. / 3.):
    """JacobiBlock.jacobi_convolution (FEANet/jacobi.py:39-47):
    u0 = u*geo + bc;  r = f - K u0;  u1 = omega/d * r + u0;  return u1*geo + bc."""
    dt = np.asarray(u).dtype.type
    u0 = u * geo + bc
    r = f - knet_apply(u0, pid, ktab)
    omd = omega_over_d(ktab, omega, dt)
    omd = omd[0] if len(omd) == 1 else omd[np.asarray(pid, np.int64)]
    u1 = omd * r + u0
    return u1 * geo + bc


def residual(u, f, pid, ktab):
    return f - knet_apply(u, pid, ktab)


def pbc_pad(u, lo, hi):
    """Circular extension of the periodic part u[..., :-1, :-1] (period n = N-1) by lo rows/columns
    before and hi after: JacobiBlockPBC.pbc_boundary (FEANet/jacobi.py:72-79) is (lo, hi) = (1, 2),
    reset_boundary (:81-84) is (0, 1)."""
    uc = np.asarray(u)[..., :-1, :-1]
    pad = [(0, 0)] * (uc.ndim - 2) + [(lo, hi), (lo, hi)]
    return np.pad(uc, pad, mode="wrap")


def jacobi_sweep_pbc(u, f, ktab, omega=2. / 3.):
    """JacobiBlockPBC.jacobi_convolution (FEANet/jacobi.py:86-97), homogeneous mesh: K applied to the
    (n+3)^2 circular extension with zero padding (KNet.forward, masks padded with 1), cropped to the
    (n+1)^2 nodes; u_new = omega/d * (f - K u_pbc)[1:-1, 1:-1] + reset_boundary(u).  f is (n+3)^2."""
    dt = np.asarray(u).dtype.type
    up = pbc_pad(u, 1, 2)
    r = (np.asarray(f) - knet_apply(up, np.zeros(up.shape[-2:], np.uint8), ktab))[..., 1:-1, 1:-1]
    omd = omega_over_d(ktab, omega, dt)[0]
    return omd * r + pbc_pad(u, 0, 1)


def restrict(r, pid, rtab, w0=1.0):
    """Restriction of an (implicitly split) fine field (FEANet/multigrid.py:50-60, 115-122;
    M-FEANet-mg_test.ipynb:27297-27304): crop [1:-1,1:-1], stride-2 3x3 conv with the FINE node's
    pattern kernel, zero pad, times w0:
        fc[I,J] = w0 * sum_k R_{p(2I-1+ky, 2J-1+kx)}[k] r[2I-1+ky, 2J-1+kx]   (interior I,J)."""
    shape = np.shape(r)
    r3 = _as3(r)
    dt = r3.dtype.type
    B, H, W = r3.shape
    Hc, Wc = (H + 1) // 2, (W + 1) // 2
    tab = np.asarray(rtab, np.float32).astype(dt)
    pid = np.asarray(pid, np.int64)
    acc = np.zeros((B, Hc - 2, Wc - 2), dt)
    for ky in range(3):
        for kx in range(3):
            rs = r3[:, 1 + ky:1 + ky + 2 * (Hc - 2):2, 1 + kx:1 + kx + 2 * (Wc - 2):2]
            ps = pid[1 + ky:1 + ky + 2 * (Hc - 2):2, 1 + kx:1 + kx + 2 * (Wc - 2):2]
            acc += (tab[0, ky, kx] if tab.shape[0] == 1 else tab[ps, ky, kx]) * rs
    out = np.zeros((B, Hc, Wc), dt)
    out[:, 1:-1, 1:-1] = acc
    if w0 != 1.0:
        out = (dt(w0) * out).astype(dt)
    return out.reshape(shape[:-2] + (Hc, Wc))


def prolong(e, pidc, ptab, w1=1.0):
    """Prolongation = stride-2 transposed conv (k=3, pad=1) of the split coarse field with the
    COARSE node's pattern kernel (FEANet/multigrid.py:62-73, 124-130; mg_test :27306-27312):
        ef[y,x] = w1 * sum_{a,b} P_{pc(a,b)}[y-2a+1, x-2b+1] e[a,b]."""
    shape = np.shape(e)
    e3 = _as3(e)
    dt = e3.dtype.type
    B, Hc, Wc = e3.shape
    H, W = 2 * Hc - 1, 2 * Wc - 1
    tab = np.asarray(ptab, np.float32).astype(dt)
    pidc = np.asarray(pidc, np.int64)
    outp = np.zeros((B, H + 2, W + 2), dt)
    for ky in range(3):
        for kx in range(3):
            outp[:, ky:ky + 2 * Hc:2, kx:kx + 2 * Wc:2] += (tab[0, ky, kx] if tab.shape[0] == 1 else
                                                             tab[pidc, ky, kx]) * e3
    out = outp[:, 1:-1, 1:-1]
    if w1 != 1.0:
        out = (dt(w1) * out).astype(dt)
    return np.ascontiguousarray(out).reshape(shape[:-2] + (H, W))


def bilinear_upsample(e):
    """F.interpolate(e, 2m-1, 'bilinear', align_corners=True) (MM_Model_convergence.ipynb:122-130)."""
    shape = np.shape(e)
    e3 = _as3(e)
    dt = e3.dtype.type
    B, m, _ = e3.shape
    M = 2 * m - 1
    h = dt(0.5)
    out = np.zeros((B, M, M), dt)
    out[:, ::2, ::2] = e3
    out[:, ::2, 1::2] = h * e3[:, :, :-1] + h * e3[:, :, 1:]
    rows = h * e3[:, :-1, :] + h * e3[:, 1:, :]
    out[:, 1::2, ::2] = rows
    out[:, 1::2, 1::2] = h * rows[:, :, :-1] + h * rows[:, :, 1:]
    return out.reshape(shape[:-2] + (M, M))


def interior_norm(r):
    """Driver residual norm ||r[..., 1:-1, 1:-1]||_2 per sample (mg_test :27428-27429)."""
    r3 = _as3(r)
    return np.sqrt(np.sum(r3[:, 1:-1, 1:-1].astype(np.float64) ** 2, axis=(1, 2)))


def hnet(x, geo, weights):
    """HNet.forward (M-FEANet-mg_test.ipynb:104-106): three 3x3 convs, each followed by *geo."""
    for w in weights:
        x = conv3x3(x, w) * geo
    return x


# ---------------------------------------------------------------------------
# A11-A14: V-cycles
# ---------------------------------------------------------------------------
class Level:
    """pids: optional {N: pattern map} of the two-material problem computed earlier by interface_mesh (the
    element/node loops are O(N^2) Python: tests/golden/c3_pattern_maps.npz holds their output up to 2049^2)."""

    def __init__(self, n, problem="poisson", dtype=np.float32, prop=(1, 20), shape=0, omega=2. / 3., m=None,
                 pids=None):
        self.n = n
        self.m = n if m is None else m
        self.N = n + 1
        self.H, self.W = self.m + 1, n + 1
        self.dtype = dtype
        if problem == "poisson":
            self.ktab, self.pid = square_mesh((self.H, self.W))
        elif pids is not None and self.N in pids:
            assert self.m == n, "two-material problem: square only"
            a = np.array(prop, np.float32)
            self.ktab = np.stack([pattern_stencil(a, REF_PATTERNS[k]) for k in range(16)])
            self.pid = np.asarray(pids[self.N], np.uint8)
        else:
            assert self.m == n, "two-material problem: square only"
            self.ktab, self.pid = interface_mesh(self.N, prop, shape)
        self.geo, self.bc = square_geometry((self.H, self.W), dtype)
        self.omega = omega

    def sweep(self, v, f):
        return jacobi_sweep(v, f, self.pid, self.ktab, self.geo, self.bc, self.omega)

    def K(self, v):
        return knet_apply(v, self.pid, self.ktab)


class OracleMultigrid:
    """Level hierarchy n, n/2, ..., n/2^(L-1), L = int(log2 n) by default (multigrid.py:87,108-113).

    `step`   — MultiGrid.Step (M-FEANet-mg_test.ipynb:27346-27372) / MultiGrid.iterate
               (FEANet/multigrid.py:159-185): 1 pre-sweep per level (coarse levels from zero),
               coarsest 2 sweeps, prolong+add then 1 post-sweep.  R/P tables and ratios w
               generalise the mg_test P/4 kernels and the learned 16-channel R/P of multigrid.py.
    `rec_vcycle` — Multigrid.rec_V_cycle (MM_Model_convergence.ipynb:132-148): nu1/nu2 sweeps,
               restriction 4*conv(/16), bilinear interpolation + reset; compat_q2 reproduces
               MM_Interface_error.ipynb:141 (pre-smoothing applied to grids[0] at every depth)."""

    def __init__(self, n, problem="poisson", dtype=np.float32, levels=None, rtab=None, ptab=None,
                 w=(1.0, 1.0), prop=(1, 20), shape=0, rows=None, pids=None):
        self.n = n
        m = n if rows is None else rows
        self.L = int(np.log2(min(n, m))) if levels is None else levels
        self.levels = [Level(n >> l, problem, dtype, prop, shape, m=m >> l, pids=pids) for l in range(self.L)]
        lin = np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32)
        nch = len(self.levels[0].ktab)
        self.rtab = (np.broadcast_to(lin / 4, (nch, 3, 3)) if rtab is None else np.asarray(rtab, np.float32))
        self.ptab = (np.broadcast_to(lin / 4, (nch, 3, 3)) if ptab is None else np.asarray(ptab, np.float32))
        self.w = w
        self.dtype = dtype

    def set_boundary(self, geo, bc):
        self.levels[0].geo = np.asarray(geo, self.dtype)
        self.levels[0].bc = np.asarray(bc, self.dtype)

    def step(self, v, f):
        L = self.L
        lv = self.levels
        B = _as3(v).shape[0]
        vs = [None] * L
        fs = [None] * L
        fs[0] = _as3(f).astype(self.dtype)
        vs[0] = lv[0].sweep(_as3(v).astype(self.dtype), fs[0])
        for j in range(L - 1):
            r = fs[j] - lv[j].K(vs[j])
            fs[j + 1] = restrict(r, lv[j].pid, self.rtab, self.w[0])
            z = np.zeros((B, lv[j + 1].H, lv[j + 1].W), self.dtype)
            vs[j + 1] = lv[j + 1].sweep(z, fs[j + 1])
        vs[L - 1] = lv[L - 1].sweep(vs[L - 1], fs[L - 1])
        for j in range(L - 2, -1, -1):
            vs[j] = vs[j] + prolong(vs[j + 1], lv[j + 1].pid, self.ptab, self.w[1])
            vs[j] = lv[j].sweep(vs[j], fs[j])
        return vs[0].reshape(np.shape(v))

    def residual_norm(self, v, f):
        return interior_norm(_as3(f) - self.levels[0].K(_as3(v)))

    def _mm_restrict(self, r):
        k16 = (np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32) / 16.0)[None]
        dt = self.dtype
        return (dt(4) * restrict(r, np.zeros(r.shape[-2:], np.uint8), k16)).astype(dt)

    def rec_vcycle(self, v, f, nu1=1, nu2=1, compat_q2=False):
        lv = self.levels
        L = self.L
        dt = self.dtype
        vs = [None] * L
        fs = [None] * L
        vs[0] = _as3(v).astype(dt)
        fs[0] = _as3(f).astype(dt)
        B = vs[0].shape[0]

        def rec(l):
            if compat_q2:
                for _ in range(nu1):
                    vs[0] = lv[0].sweep(vs[0], fs[0])
            else:
                for _ in range(nu1):
                    vs[l] = lv[l].sweep(vs[l], fs[l])
            if l < L - 1:
                r = fs[l] - lv[l].K(vs[l])
                fs[l + 1] = self._mm_restrict(r)
                vs[l + 1] = np.zeros((B, lv[l + 1].H, lv[l + 1].W), dt)
                rec(l + 1)
                up = bilinear_upsample(vs[l + 1])
                vs[l] = vs[l] + (up * lv[l].geo + lv[l].bc)
                vs[l + 1] = np.zeros_like(vs[l + 1])
            for _ in range(nu2):
                vs[l] = lv[l].sweep(vs[l], fs[l])

        rec(0)
        return vs[0].reshape(np.shape(v))


def hnet_relax(v, f, level, weights, k=1):
    """HJacIterator.HRelax (M-FEANet-mg_test.ipynb:147-155): u <- J(u) + HNet(J(u) - u)."""
    u = v
    for _ in range(k):
        j = level.sweep(u, f)
        u = j + hnet(j - u, level.geo, weights)
    return u
