"""The reference's PyTorch-CPU formulation of the V-cycle — CPU BASELINE and TEST INFRASTRUCTURE ONLY.

BASELINE.json's north star times "the reference PyTorch CPU path on the GPU box's own host cores".
The reference itself cannot travel to the GPU box, so this module restates its formulation
operation for operation in PyTorch on the CPU (conv2d / conv_transpose2d / elementwise, the same
ops in the same order as the reference) and bench.py times it as `cpu_baseline` ("kind": "port").
It is never part of the product: nothing in multigrid-feanet_amd/ imports it; only tests/ and
bench.py's cpu_baseline leg do.  Checked against the numpy oracle and the reference-generated
golden fixtures in tests/test_torch_cpu_ref.py.

Restated reference code (file:line):
  KNet.forward            FEANet/model.py:22-30   identity conv (net1), mask by global_pattern, net2
  KNet.split_x            FEANet/model.py:37-47
  JacobiBlock             FEANet/jacobi.py:17-47  d_mat (:31-37), reset_boundary (:27-29),
                                                  jacobi_convolution (:39-47)
  MultiGrid.Restrict      M-FEANet-mg_test.ipynb:27297-27304  conv2d(rF[1:-1,1:-1], P, stride 2), pad 0
  MultiGrid.Interpolate   M-FEANet-mg_test.ipynb:27306-27312  conv_transpose2d(eFC, P, stride 2, pad 1)
  MultiGrid.Step          M-FEANet-mg_test.ipynb:27346-27372  (== FEANet/multigrid.py:159-185 for R = P)
  driver residual norm    M-FEANet-mg_test.ipynb:27428-27429
The only deviation: coarse iterates are created as zeros in the working dtype instead of float32
zeros promoted by reset_boundary (the same values).
"""
import numpy as np
import torch
import torch.nn.functional as F


class TorchLevel:
    """One SingleGrid: KNet (C = #patterns), JacobiBlock with the square geometry (geo.py:13-30)."""

    def __init__(self, ktab, pid, dtype, omega=2.0 / 3.0, geo=None, bc=None):
        ktab = np.asarray(ktab, np.float32)
        C = ktab.shape[0]
        H, W = pid.shape
        self.C = C
        ident = torch.zeros(C, 1, 3, 3)
        ident[:, 0, 1, 1] = 1.0
        # parameters are float32 in the reference; the fp64 runs .double() the modules (MM_poisson.ipynb:117-118)
        self.net1 = ident.to(dtype)
        self.net2 = torch.from_numpy(ktab).reshape(1, C, 3, 3).to(dtype)
        gp = torch.zeros(1, C, H, W)
        pid_t = torch.from_numpy(np.asarray(pid, np.int64))
        for p in range(C):
            gp[0, p] = (pid_t == p).float()
        self.global_pattern = gp  # a plain float32 tensor in the reference (not a buffer)
        if geo is None:
            geo = torch.ones(1, 1, H, W, dtype=dtype)
            geo[..., 0, :] = 0
            geo[..., -1, :] = 0
            geo[..., :, 0] = 0
            geo[..., :, -1] = 0
        self.geo = geo.to(dtype)
        self.bc = torch.zeros(1, 1, H, W, dtype=dtype) if bc is None else bc.to(dtype)
        self.omega = omega
        d = torch.zeros(1, 1, H, W, dtype=dtype)
        for p in range(C):
            d[0, 0] += gp[0, p].to(dtype) * torch.from_numpy(ktab[p])[1, 1]
        self.d_mat = d

    def knet(self, u):
        u_split = F.conv2d(u, self.net1, padding=1) * self.global_pattern
        return F.conv2d(u_split, self.net2, padding=1)

    def split_x(self, x):
        return F.conv2d(x, self.net1, padding=1) * self.global_pattern

    def reset_boundary(self, u):
        return u * self.geo + self.bc

    def jacobi(self, u, f):
        u = self.reset_boundary(u)
        residual = f - self.knet(u)
        u_new = self.omega / self.d_mat * residual + u
        return self.reset_boundary(u_new)


class TorchCPUMultigrid:
    """MultiGrid.Step of M-FEANet-mg_test.ipynb on CPU PyTorch, L = int(log2 n) levels by default,
    R = P = [[1,2,1],[2,4,2],[1,2,1]]/4 (the notebook's `P`)."""

    def __init__(self, n, problem="poisson", dtype=torch.float64, levels=None, tables=None):
        from . import feanet_oracle as orc
        self.n = n
        self.L = int(np.log2(n)) if levels is None else levels
        self.dtype = dtype
        self.levels = []
        for l in range(self.L):
            N = (n >> l) + 1
            if tables is not None:
                ktab, pid = tables(N)
            elif problem == "poisson":
                ktab, pid = orc.square_mesh(N)
            else:
                ktab, pid = orc.interface_mesh(N)
            self.levels.append(TorchLevel(ktab, pid, dtype))
        P = torch.tensor([[1., 2., 1.], [2., 4., 2.], [1., 2., 1.]]) / 4.0
        C = self.levels[0].C
        self.P_conv = P.reshape(1, 1, 3, 3).expand(1, C, 3, 3).contiguous().to(dtype)
        self.P_deconv = P.reshape(1, 1, 3, 3).expand(C, 1, 3, 3).contiguous().to(dtype)

    def set_boundary(self, geo, bc):
        self.levels[0].geo = torch.as_tensor(geo).to(self.dtype).reshape(1, 1, *self.levels[0].geo.shape[-2:])
        self.levels[0].bc = torch.as_tensor(bc).to(self.dtype)
        if self.levels[0].bc.dim() == 2:
            self.levels[0].bc = self.levels[0].bc[None, None]

    def restrict(self, rF):
        rFC = F.conv2d(rF[:, :, 1:-1, 1:-1].clone(), self.P_conv, stride=2)
        return F.pad(rFC, (1, 1, 1, 1), "constant", 0)

    def interpolate(self, eFC):
        return F.conv_transpose2d(eFC.clone(), self.P_deconv, stride=2, padding=1)

    def step(self, v, f):
        lv = self.levels
        L = self.L
        B = v.shape[0]
        vs = [None] * L
        fs = [None] * L
        fs[0] = f
        vs[0] = lv[0].jacobi(v, f)
        for j in range(L - 1):
            rF = fs[j] - lv[j].knet(vs[j])
            rF = lv[j].split_x(rF)
            fs[j + 1] = self.restrict(rF)
            Nn = (self.n >> (j + 1)) + 1
            vs[j + 1] = torch.zeros((B, 1, Nn, Nn), dtype=self.dtype)
            vs[j + 1] = lv[j + 1].jacobi(vs[j + 1], fs[j + 1])
        vs[L - 1] = lv[L - 1].jacobi(vs[L - 1], fs[L - 1])
        for j in range(L - 2, -1, -1):
            eFC = lv[j + 1].split_x(vs[j + 1])
            vs[j] = vs[j] + self.interpolate(eFC)
            vs[j] = lv[j].jacobi(vs[j], fs[j])
        return vs[0]

    def residual_norm(self, v, f):
        r = f - self.levels[0].knet(v)
        return torch.norm(r[:, :, 1:-1, 1:-1], dim=(2, 3)).reshape(-1)
