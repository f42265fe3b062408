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

    def save_mesh(self, outfile, point_data=None):
        """VTK export of the quad mesh with its element phases (FEANet/mesh.py:119-120 writes it with
        meshio).  meshio is used when installed; otherwise a legacy binary VTK file (UNSTRUCTURED_GRID,
        VTK_QUAD cells, CELL_DATA "Phase") is written directly.  point_data: optional {name: [N*N]}
        nodal fields (e.g. a solution) — an extension the reference does not have."""
        try:
            import meshio
        except ImportError:
            write_vtk_legacy(outfile, self.points, self.cells, {"Phase": self.phase}, point_data or {})
            return
        m = meshio.Mesh(self.points, [("quad", self.cells)], point_data=point_data or {})
        m.cell_data["Phase"] = [self.phase]
        m.write(outfile)


def write_vtk_legacy(path, points, cells, cell_data, point_data):
    """Legacy binary VTK (big-endian) of a quad mesh: POINTS float32 x 3, CELLS (4 + ids) int32,
    CELL_TYPES 9 (VTK_QUAD), scalar CELL_DATA / POINT_DATA fields (int -> int, float -> double)."""
    pts = np.asarray(points, np.float32).reshape(-1, 3)
    cl = np.asarray(cells, np.int64).reshape(-1, 4)
    nc = cl.shape[0]
    with open(path, "wb") as fh:
        w = fh.write
        w(b"# vtk DataFile Version 3.0\nFEANet mesh (feanet_amd)\nBINARY\nDATASET UNSTRUCTURED_GRID\n")
        w(f"POINTS {pts.shape[0]} float\n".encode())
        w(pts.astype(">f4").tobytes())
        w(f"\nCELLS {nc} {5 * nc}\n".encode())
        conn = np.concatenate([np.full((nc, 1), 4, np.int64), cl], axis=1)
        w(conn.astype(">i4").tobytes())
        w(f"\nCELL_TYPES {nc}\n".encode())
        w(np.full(nc, 9, ">i4").tobytes())
        w(b"\n")

        def fields(kind, n, data):
            if not data:
                return
            w(f"{kind} {n}\n".encode())
            for name, v in data.items():
                v = np.asarray(v).reshape(-1)
                if v.shape[0] != n:
                    raise ValueError(f"write_vtk_legacy: field {name!r} has {v.shape[0]} values, expected {n}")
                if np.issubdtype(v.dtype, np.integer):
                    w(f"SCALARS {name} int 1\nLOOKUP_TABLE default\n".encode())
                    w(v.astype(">i4").tobytes())
                else:
                    w(f"SCALARS {name} double 1\nLOOKUP_TABLE default\n".encode())
                    w(v.astype(">f8").tobytes())
                w(b"\n")

        fields("CELL_DATA", nc, cell_data)
        fields("POINT_DATA", pts.shape[0], point_data)


def read_vtk_legacy(path):
    """Reader for write_vtk_legacy's files (tests): points, cells, cell_data, point_data."""
    raw = open(path, "rb").read()
    pos = 0

    def line():
        nonlocal pos
        e = raw.index(b"\n", pos)
        s_ = raw[pos:e].decode()
        pos = e + 1
        return s_

    def block(n, dt):
        nonlocal pos
        nb = n * np.dtype(dt).itemsize
        a = np.frombuffer(raw[pos:pos + nb], dt).copy()
        pos += nb + 1
        return a

    for _ in range(4):
        line()
    npts = int(line().split()[1])
    pts = block(3 * npts, ">f4").reshape(-1, 3)
    nc = int(line().split()[1])
    conn = block(5 * nc, ">i4").reshape(nc, 5)
    line()
    types = block(nc, ">i4")
    out = {"points": pts, "cells": conn[:, 1:], "types": types, "CELL_DATA": {}, "POINT_DATA": {}}
    sect = None
    while pos < len(raw):
        t = line().split()
        if not t:
            continue
        if t[0] in ("CELL_DATA", "POINT_DATA"):
            sect, n = t[0], int(t[1])
            continue
        name, typ = t[1], t[2]
        line()  # LOOKUP_TABLE
        out[sect][name] = block(n, ">i4" if typ == "int" else ">f8")
    return out


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
