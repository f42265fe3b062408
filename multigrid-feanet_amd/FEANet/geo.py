"""Geometry (reference: FEANet/geo.py:5-48): Dirichlet masks on the default device."""
import torch


class Geometry:
    """`geometry_idx` = 1 at interior nodes, 0 on the boundary; `boundary_value` = Dirichlet data
    (zero by default) — FEANet/geo.py:13-30.  The L-shaped variant of the reference is broken
    (geo.py:41 unpacks a None) and is not provided."""

    def __init__(self, nnode_edge=37, l_shape=False, l_cutout_size=None):
        if l_shape:
            raise NotImplementedError("Geometry(l_shape=True) is broken in the reference (geo.py:41)")
        self.square_geometry(nnode_edge)

    def square_geometry(self, nnode_edge):
        g = torch.ones(1, 1, nnode_edge, nnode_edge)
        g[..., 0, :] = 0
        g[..., -1, :] = 0
        g[..., :, 0] = 0
        g[..., :, -1] = 0
        self.geometry_idx = g
        self.boundary_value = torch.zeros_like(g)

    def set_square_bc(self, bc_values):
        self.boundary_value[:, :, :, :] = bc_values
