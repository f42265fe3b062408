"""JacobiBlock (reference: FEANet/jacobi.py:5-47) with the sweep as one HIP kernel."""
import numpy as np
import torch

from feanet_amd import ops


class JacobiBlock:
    """Weighted Jacobi u <- R(R(u) + omega/d (f - K R(u))), R(u) = u*geometry_idx + boundary_value.

    `d_mat` is computed as the reference does (compute_diagonal_matrix, jacobi.py:31-37); the sweep
    itself runs as fea_jacobi_sweep with omega/d taken per node pattern."""

    def __init__(self, Knet, mesh, omega, geometry_idx, boundary_value):
        self.nnode_edge = geometry_idx.shape[2]
        self.geometry_idx = geometry_idx
        self.boundary_value = boundary_value
        self.omega = omega
        self.mesh = mesh
        self.Knet = Knet
        keys = sorted(mesh.kernel_dict)
        centre = np.array([np.asarray(mesh.kernel_dict[k], np.float32)[1, 1] for k in keys], np.float32)
        dt = geometry_idx.dtype
        self._centre = torch.from_numpy(centre)
        pid = Knet.pattern_id.to(geometry_idx.device).long()
        d = self._centre.to(device=geometry_idx.device, dtype=dt)[pid]
        self.d_mat = d.expand_as(geometry_idx).clone()
        # omega / d per pattern, evaluated as torch does `self.omega / self.d_mat` (reciprocal * omega)
        self._omd = torch.reciprocal(self._centre.to(dt)) * omega

    def reset_boundary(self, u):
        """u * geometry_idx + boundary_value (jacobi.py:27-29)."""
        ops.require_hip(u, "u")
        return u * self.geometry_idx + self.boundary_value

    def jacobi_convolution(self, initial_u, forcing_term):
        """One sweep (jacobi.py:39-47), reset_boundary fused on both sides."""
        ops.require_hip(initial_u, "initial_u")
        # reset_boundary promotes first (float32 coarse buffers meet fp64 masks in the reference)
        dt = torch.promote_types(initial_u.dtype, self.geometry_idx.dtype)
        u = initial_u.to(dt)
        kt = self.Knet._tables(u)
        f = forcing_term.to(dt)
        geo = self.geometry_idx.to(device=u.device, dtype=dt)
        bc = self.boundary_value.to(device=u.device, dtype=dt)
        omd = self._omd.to(device=u.device).to(dt)
        pid = self.Knet._pid(u) if self.Knet.n_channel > 1 else None
        return ops.jacobi_sweep(u, f, kt, omd, pid, geo, bc)
