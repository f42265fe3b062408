"""JacobiBlock / JacobiBlockPBC (reference: FEANet/jacobi.py:5-97) with each sweep as one HIP kernel."""
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


class JacobiBlockPBC:
    """Weighted Jacobi with periodic boundary conditions (FEANet/jacobi.py:50-97; homogeneous meshes).

    Same constructor, attributes (`d_mat` [1,1,N,N] in the default dtype, `omega`, `mesh`, `Knet`) and
    methods as the reference: pbc_boundary(u) -> [.., N+2, N+2] circular extension, reset_boundary(u)
    -> [.., N, N] (last row/column = first), jacobi_convolution(u, forcing_term) with the (N+2)^2
    forcing term of its drivers (f = FNet(pbc_boundary(F))).  Each method is one HIP kernel
    (fea_pbc_pad, fea_jacobi_sweep_pbc); inputs must be GPU tensors."""

    def __init__(self, mesh, Knet=None, omega=2. / 3.):
        self.nnode_edge = mesh.nnode_edge
        self.omega = omega
        self.mesh = mesh
        N = self.nnode_edge
        self.d_mat = torch.zeros((1, 1, N, N))  # compute_diagonal_matrix (:62-70): sum_p mask_p W_p[1,1]
        for pkey in mesh.kernel_dict:
            w = torch.from_numpy(np.asarray(mesh.kernel_dict[pkey], np.float32))
            g = torch.from_numpy(np.asarray(mesh.global_pattern_center[pkey])).reshape(N, N)
            self.d_mat[0, 0] += g * w[1, 1]
        self.Knet = Knet
        if len(mesh.kernel_dict) != 1:
            raise NotImplementedError("JacobiBlockPBC: homogeneous meshes only (as the reference, jacobi.py:51)")
        centre = np.float32(np.asarray(mesh.kernel_dict[sorted(mesh.kernel_dict)[0]], np.float32)[1, 1])
        self._centre = torch.tensor([centre], dtype=torch.float32)

    def pbc_boundary(self, u):
        """[.., n+1, n+1] -> [.., n+3, n+3] circular extension of u[..., :-1, :-1] (jacobi.py:72-79)."""
        ops.require_hip(u, "u")
        return ops.pbc_pad(u, 1, 2)

    def reset_boundary(self, u):
        """[.., n+1, n+1] -> same size, last row/column copied from the first (jacobi.py:81-84)."""
        ops.require_hip(u, "u")
        return ops.pbc_pad(u, 0, 1)

    def jacobi_convolution(self, u, forcing_term):
        """One periodic sweep (jacobi.py:86-97): omega/d (f - K pbc(u))[1:-1, 1:-1] + reset(u)."""
        ops.require_hip(u, "u")
        dt = torch.promote_types(u.dtype, self.d_mat.dtype)
        u = u.to(dt)
        kt = (self.Knet._tables(u) if self.Knet is not None
              else torch.from_numpy(np.asarray(self.mesh.kernel_dict[0], np.float32)).to(u.device, dt))
        # omega/d_mat in d_mat's dtype as torch evaluates it (reciprocal * omega), then promoted
        omd = (torch.reciprocal(self._centre.to(self.d_mat.dtype)) * self.omega).to(dt)
        return ops.jacobi_sweep_pbc(u, forcing_term.to(dt), kt, omd)
