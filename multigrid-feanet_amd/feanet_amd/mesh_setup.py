"""Setup-time discretisation tables, host side.

Restates the reference's MeshSquare / MeshCenterInterface / FNet / JacobiBlock set-up
(FEANet/mesh.py:4-192, FEANet/model.py:49-58, FEANet/jacobi.py:31-37) in vectorised numpy:
the reference's node-pattern search is O(N^4) (57 s at 257^2, ~64 h at 2049^2); here it is
O(N^2) with identical float32 arithmetic, so BASELINE config 3 (2049^2) sets up in well under
a second.  Outputs are bit-identical to the reference (tests/test_setup.py against the golden
pattern maps and stencils).
"""
import numpy as np

# FEANet/mesh.py:23-26: pattern id -> element phases of quadrants [e1, e2, e3, e4]
PATTERN_BITS = np.array([[0, 0, 0, 0], [1, 1, 1, 1], [0, 0, 0, 1], [0, 0, 1, 0],
                         [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 1], [1, 1, 0, 0],
                         [0, 1, 1, 0], [1, 0, 0, 1], [0, 1, 0, 1], [1, 0, 1, 0],
                         [1, 1, 1, 0], [1, 1, 0, 1], [0, 1, 1, 1], [1, 0, 1, 1]], dtype=np.int64)
# inverse lookup: bits e1 + 2 e2 + 4 e3 + 8 e4 -> pattern id
_BITS_TO_ID = np.zeros(16, np.uint8)
for _pid, _b in enumerate(PATTERN_BITS):
    _BITS_TO_ID[_b[0] + 2 * _b[1] + 4 * _b[2] + 8 * _b[3]] = _pid


def q1_element_stiffness():
    """Q1 Laplace element matrix in float32 (FEANet/mesh.py:28-31)."""
    base = np.array([[-4., 1., 2., 1.], [1., -4., 1., 2.], [2., 1., -4., 1.], [1., 2., 1., -4.]], np.float32)
    return np.float32(-1.0 / 6.0) * base


def node_stencil(coef, bits, Ke):
    """Assemble the 3x3 stencil of a node whose four quadrant elements have phases `bits`,
    summing a_phase * Ke entries in float32 in the reference's order (FEANet/mesh.py:107-116)."""
    a = [np.float32(coef[b]) for b in bits]  # a[q] = coefficient of quadrant element q (e1..e4)
    s = np.zeros((3, 3), np.float32)
    s[0, 0] = a[3] * Ke[1, 3]
    s[0, 1] = a[3] * Ke[1, 2] + a[2] * Ke[0, 3]
    s[0, 2] = a[2] * Ke[0, 2]
    s[1, 0] = a[0] * Ke[2, 3] + a[3] * Ke[1, 0]
    s[1, 1] = a[2] * Ke[0, 0] + a[3] * Ke[1, 1] + a[0] * Ke[2, 2] + a[1] * Ke[3, 3]
    s[1, 2] = a[1] * Ke[3, 2] + a[2] * Ke[0, 1]
    s[2, 0] = a[0] * Ke[2, 0]
    s[2, 1] = a[0] * Ke[2, 1] + a[1] * Ke[3, 0]
    s[2, 2] = a[1] * Ke[3, 1]
    return s


def stencil_table(prop=None):
    """[C, 3, 3] float32 stencils: C = 1 for the homogeneous square (MeshSquare, a = [1]),
    C = 16 for the two-phase mesh (MeshCenterInterface, a = prop)."""
    Ke = q1_element_stiffness()
    if prop is None:
        return node_stencil(np.array([1.], np.float32), PATTERN_BITS[0], Ke)[None]
    coef = np.asarray(prop, np.float32)
    return np.stack([node_stencil(coef, PATTERN_BITS[p], Ke) for p in range(16)])


def element_phase(N, shape=0, size=2.0):
    """Phase (0/1) of each of the (N-1)^2 elements from its float32 centroid
    (place_circle FEANet/mesh.py:62-68 for shape 0, place_rect :70-76 for shape 1)."""
    x = np.linspace(size / 2, -size / 2, N, dtype=np.float32)
    y = np.linspace(-size / 2, size / 2, N, dtype=np.float32)
    four = np.float32(4)
    # np.mean of the 4 float32 element points: ((p0 + p1) + p2) + p3, then / 4 in float32
    cx = (((x[:-1] + x[1:]) + x[1:]) + x[:-1]) / four           # per element column
    cy = (((y[:-1] + y[:-1]) + y[1:]) + y[1:]) / four           # per element row
    CX, CY = np.meshgrid(cx, cy)                                # [row, col]
    if shape == 0:
        inside = (CX - np.float32(0.0)) ** 2 + (CY - np.float32(0.0)) ** 2 < np.float32(0.5) ** 2
    elif shape == 1:
        inside = (np.abs(CX - np.float32(0.0)) < np.float32(0.5)) & (np.abs(CY - np.float32(0.0)) < np.float32(0.5))
    else:
        raise ValueError(f"unknown inclusion shape {shape}")
    return inside.astype(np.int64)


def interface_pattern_map(N, shape=0, size=2.0):
    """uint8 [N, N] pattern id per node (identify_patterns + generate_global_pattern_map,
    FEANet/mesh.py:78-101).  Node (r, c)'s quadrant elements: e1 = (r-1, c), e2 = (r-1, c-1),
    e3 = (r, c-1), e4 = (r, c) (x decreases with c, y increases with r).  Boundary -> 0."""
    ph = element_phase(N, shape, size)
    pid = np.zeros((N, N), np.uint8)
    e1 = ph[:-1, 1:]   # (r-1, c)   for r, c in 1..N-2
    e2 = ph[:-1, :-1]  # (r-1, c-1)
    e3 = ph[1:, :-1]   # (r, c-1)
    e4 = ph[1:, 1:]    # (r, c)
    code = e1 + 2 * e2 + 4 * e3 + 8 * e4
    pid[1:-1, 1:-1] = _BITS_TO_ID[code]
    return pid


def mass_stencil(h):
    """FNet consistent-mass stencil, float32 (FEANet/model.py:54-56)."""
    return np.array([[h * h / 36., h * h / 9., h * h / 36.],
                     [h * h / 9., 4. * h * h / 9., h * h / 9.],
                     [h * h / 36., h * h / 9., h * h / 36.]], dtype=np.float32)


def omega_over_d(ktab, omega, dtype):
    """Per-pattern omega/d with d = centre weight (JacobiBlock.compute_diagonal_matrix,
    FEANet/jacobi.py:31-37), evaluated like the reference's `self.omega/self.d_mat` (:45):
    reciprocal of d in `dtype`, times omega in `dtype`."""
    d = np.asarray(ktab, np.float32)[:, 1, 1].astype(dtype)
    return np.reciprocal(d) * np.asarray(omega, dtype)


def linear_transfer_kernel():
    """[[1,2,1],[2,4,2],[1,2,1]] float32 (M-FEANet-mg_test.ipynb cell 20 before the /4)."""
    return np.array([[1, 2, 1], [2, 4, 2], [1, 2, 1]], np.float32)


def interface_pattern_map_device(N, shape=0, size=2.0, device="cuda", out=None, ld=None):
    """interface_pattern_map computed on the GPU (setup_ops.hip, fea_interface_pattern_map): one
    thread per node, bit-identical to the host restatement / the reference.  Returns a uint8 [N, N]
    tensor, or writes rows of pitch `ld` bytes into the uint8 tensor `out` starting at its first
    element (e.g. a framed level buffer) and returns it."""
    import torch
    from . import _lib
    if out is None:
        out = torch.empty((N, N), dtype=torch.uint8, device=device)
        ld = N
        base = out.data_ptr()
    else:
        base = out.data_ptr() if isinstance(out, torch.Tensor) else int(out)
    st = torch.cuda.current_stream(torch.device(device)).cuda_stream
    rc = _lib.lib().fea_interface_pattern_map(base, int(ld), int(N), int(shape), float(size), st)
    if rc != 0:
        raise RuntimeError(f"feanet_amd: fea_interface_pattern_map failed ({rc})")
    return out


def stencil_mirror_mismatches(ktab, pid):
    """Interior (node, tap) pairs where the stiffness weight of tap t taken from the NEIGHBOUR's pattern (KNet's
    split-then-convolve order, FEANet/model.py:22-30) differs from the mirrored tap 8 - t of the CENTRE's pattern.
    K is a symmetric FE stiffness (K_ij = K_ji), so for the tables of stencil_table() this is 0 bit for bit on any
    pattern map; the framed two-material kernels rely on it (one table row per node).  ktab: [P, 9] or [P, 3, 3];
    pid: [H, W] pattern ids (numpy or torch, any device)."""
    import torch
    p = pid if torch.is_tensor(pid) else torch.from_numpy(np.ascontiguousarray(pid))
    k = torch.as_tensor(np.asarray(ktab, np.float32).reshape(-1, 9) if not torch.is_tensor(ktab) else ktab.reshape(-1, 9),
                        device=p.device)
    p = p.long()
    H, W = p.shape
    if H < 3 or W < 3:
        return 0
    c = p[1:-1, 1:-1]
    bad = 0
    for t in range(9):
        dy, dx = t // 3 - 1, t % 3 - 1
        nb = p[1 + dy:H - 1 + dy, 1 + dx:W - 1 + dx]
        bad += int((k[nb, t] != k[c, 8 - t]).sum().item())
    return bad
