"""Meshes (reference: FEANet/mesh.py:4-192), vectorised.

Same constructor signatures and attributes as the reference (`nnode_edge`, `kernel_dict`,
`global_pattern_center`, `ref_pattern_dict`, `Ke`, `a`, `phase`, `pattern`, `points`, `cells`),
but the node-pattern search is O(N^2) numpy (feanet_amd.mesh_setup) instead of the reference's
O(N^4) loop, and the one-hot `global_pattern_center` maps are built lazily from a uint8
`pattern_id` map (16 int64 N^2 maps are 537 MB at 2049^2).  VTK export (`save_mesh`) needs the
optional `meshio` package and is outside the hot path.
"""
import numpy as np

from feanet_amd import mesh_setup as ms

_REF_PATTERNS = {i: [int(b) for b in ms.PATTERN_BITS[i]] for i in range(16)}


class _LazyPatternMaps(dict):
    """dict pattern id -> int64 one-hot node map [N*N], materialised on first access."""

    def __init__(self, pid, keys):
        super().__init__()
        self._pid = pid
        self._keys = list(keys)

    def _fill(self, k):
        if k in self._keys and not dict.__contains__(self, k):
            dict.__setitem__(self, k, (self._pid.reshape(-1) == k).astype(int))

    def __getitem__(self, k):
        self._fill(k)
        return dict.__getitem__(self, k)

    def __contains__(self, k):
        return k in self._keys

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def keys(self):
        return list(self._keys)

    def items(self):
        return [(k, self[k]) for k in self._keys]

    def values(self):
        return [self[k] for k in self._keys]


def _grid(size, nnode_edge):
    x = np.linspace(size / 2, -size / 2, nnode_edge, dtype=np.float32)
    y = np.linspace(-size / 2, size / 2, nnode_edge, dtype=np.float32)
    mx, my = np.meshgrid(x, y)
    pts = np.stack([mx.ravel(), my.ravel(), np.zeros(mx.size, np.float32)], axis=1)
    nodes = np.arange(nnode_edge * nnode_edge).reshape(nnode_edge, nnode_edge)
    cells = np.stack([nodes[:-1, :-1].ravel(), nodes[:-1, 1:].ravel(), nodes[1:, 1:].ravel(),
                      nodes[1:, :-1].ravel()], axis=1)
    return pts, cells


class _MeshBase:
    def _finish(self, pid, keys):
        self.pattern_id = pid
        self.global_pattern_center = _LazyPatternMaps(pid, keys)

    @property
    def points(self):
        if self._points is None:
            self._points, self._cells = _grid(self.size, self.nnode_edge)
        return self._points

    @property
    def cells(self):
        if self._cells is None:
            self._points, self._cells = _grid(self.size, self.nnode_edge)
        return self._cells

    def save_mesh(self, outfile):
        try:
            import meshio
        except ImportError as e:  # pragma: no cover
            raise RuntimeError("save_mesh needs the optional meshio package (VTK export)") from e
        m = meshio.Mesh(self.points, [("quad", self.cells)])
        m.cell_data["Phase"] = [self.phase]
        m.write(outfile)


class MeshCenterInterface(_MeshBase):
    """Square plate with a central inclusion (circle shape=0 / square shape=1) of coefficient
    prop[1] in a background of prop[0] (FEANet/mesh.py:4-120)."""

    def __init__(self, size=2, prop=(1, 20), nnode_edge=65, shape=0, outfile=None):
        self.size = size
        self.nnode_edge = nnode_edge
        self._points = self._cells = None
        self.a = np.array(prop, dtype=np.float32)
        self.ref_pattern_dict = dict(_REF_PATTERNS)
        self.Ke = ms.q1_element_stiffness()
        self.phase = ms.element_phase(nnode_edge, shape, size).reshape(-1)
        pid = ms.interface_pattern_map(nnode_edge, shape, size)
        self.pattern = ms.PATTERN_BITS[pid.reshape(-1)].copy()
        self.pattern[pid.reshape(-1) == 0] = 0
        tab = ms.stencil_table(prop)
        self.kernel_dict = {k: tab[k] for k in range(16)}
        self._finish(pid, range(16))
        if outfile is not None:
            self.save_mesh(outfile)


class MeshSquare(_MeshBase):
    """Homogeneous square plate, a single stencil (FEANet/mesh.py:122-192)."""

    def __init__(self, size=2, nnode_edge=65, outfile=None):
        self.size = size
        self.nnode_edge = nnode_edge
        self._points = self._cells = None
        self.a = np.array([1.], dtype=np.float32)
        self.ref_pattern_dict = {0: [0, 0, 0, 0]}
        self.Ke = ms.q1_element_stiffness()
        self.phase = np.zeros(((nnode_edge - 1) * (nnode_edge - 1),), dtype=int)
        self.kernel_dict = {0: ms.stencil_table(None)[0]}
        self._finish(np.zeros((nnode_edge, nnode_edge), np.uint8), [0])
        if outfile is not None:
            self.save_mesh(outfile)
