"""KNet / FNet (reference: FEANet/model.py:8-61) with HIP forward passes.

Parameters keep the reference layout so state_dicts and attribute access carry over:
`net1.weight` [C,1,3,3] (identity split), `net2.weight` [1,C,3,3] (per-pattern stencils),
`net.weight` [1,1,3,3] (FNet mass stencil).  The forward passes call feanet_amd.ops
(fea_knet_apply / fea_split_x); the per-node pattern map is a uint8 buffer instead of the
reference's C dense float masks.
"""
import numpy as np
import torch
import torch.nn as nn

from feanet_amd import ops


def _pattern_id(mesh):
    pid = getattr(mesh, "pattern_id", None)
    if pid is not None:
        return np.asarray(pid, np.uint8)
    n = mesh.nnode_edge
    keys = sorted(mesh.kernel_dict)
    stack = np.stack([np.asarray(mesh.global_pattern_center[k]).reshape(n, n) for k in keys])
    if not (stack.sum(0) == 1).all():
        raise ValueError("KNet: every node must carry exactly one pattern")
    return np.asarray(keys, np.uint8)[np.argmax(stack, axis=0)]


class KNet(nn.Module):
    """Stiffness operator K u as per-node-pattern 3x3 stencils (FEANet/model.py:8-47)."""

    def __init__(self, mesh):
        super().__init__()
        self.nnode_edge = mesh.nnode_edge
        self.kernel_dict = mesh.kernel_dict
        self.n_channel = len(mesh.kernel_dict)
        self.net1 = nn.Conv2d(1, self.n_channel, kernel_size=3, padding=1, bias=False)
        self.net2 = nn.Conv2d(self.n_channel, 1, kernel_size=3, padding=1, bias=False)
        with torch.no_grad():
            ident = torch.zeros(3, 3)
            ident[1, 1] = 1.0
            for pkey in self.kernel_dict:
                self.net1.weight[pkey, 0] = ident
                self.net2.weight[0, pkey] = torch.from_numpy(np.asarray(self.kernel_dict[pkey], np.float32))
        pid = torch.from_numpy(_pattern_id(mesh))
        self.register_buffer("pattern_id", pid.to(self.net2.weight.device), persistent=False)

    @property
    def global_pattern(self):
        """[1, C, N, N] one-hot masks (model.py:32-35), materialised on demand."""
        p = self.pattern_id.long()
        return torch.stack([(p == k).float() for k in range(self.n_channel)])[None]

    def _pid(self, x):
        pid = self.pattern_id
        if pid.device != x.device:
            pid = pid.to(x.device)
            self.pattern_id = pid
        return pid

    def _tables(self, x):
        w = self.net2.weight
        if w.dtype != x.dtype:
            raise RuntimeError(f"KNet: input dtype {x.dtype} != weight dtype {w.dtype} (use .double())")
        return w[0]

    def _check_padded(self, x, what):
        if x.shape[-2] != self.nnode_edge + 2 or x.shape[-1] != self.nnode_edge + 2:
            raise ValueError(f"KNet.{what}: input must be N x N or (N+2) x (N+2) (N = {self.nnode_edge})")

    def _padded_pid(self, x):
        """Pattern map of an (N+2)^2 input: the interior carries the mesh's patterns; on the padding ring
        every mask is 1 (model.py:26-28: F.pad(global_pattern, (1,1,1,1), 'constant', 1))."""
        pp = getattr(self, "_pid_pad", None)
        if pp is None or pp.device != x.device:
            pp = torch.nn.functional.pad(self._pid(x)[None, None].float(), (1, 1, 1, 1))[0, 0].to(torch.uint8)
            self._pid_pad = pp
        return pp

    @staticmethod
    def _ring(x):
        """(interior part, padding-ring part) of a padded field: x = a + b."""
        inner = torch.zeros_like(x)
        inner[..., 1:-1, 1:-1] = x[..., 1:-1, 1:-1]
        return inner, x - inner

    def forward(self, u):
        H = u.shape[-2]
        if H != self.nnode_edge:
            # padded input (JacobiBlockPBC's circular extension, model.py:26-28): on the padding ring every
            # mask is 1, so ring nodes act through the SUM of the pattern stencils; interior nodes through
            # their own pattern's.  K u = K_pid(u inside) + K_sum(u on the ring) — one stencil each.
            self._check_padded(u, "forward")
            tab = self._tables(u)
            if self.n_channel == 1:
                return ops.knet_apply(u, tab, None)
            inner, ring = self._ring(u)
            return (ops.knet_apply(inner, tab, self._padded_pid(u))
                    + ops.knet_apply(ring, tab.sum(0, keepdim=True), None))
        return ops.knet_apply(u, self._tables(u), self._pid(u) if self.n_channel > 1 else None)

    def split_x(self, x):
        """x_split[:, p] = mask_p * x (model.py:37-47); on the ring of a padded (N+2)^2 input every
        channel carries x (masks padded with 1, model.py:42-46)."""
        if x.shape[-2] != self.nnode_edge:
            self._check_padded(x, "split_x")
            if self.n_channel == 1:
                return ops.split_x(x, None, 1)
            inner, ring = self._ring(x)
            return ops.split_x(inner, self._padded_pid(x), self.n_channel) + ring
        return ops.split_x(x, self._pid(x) if self.n_channel > 1 else None, self.n_channel)


class FNet(nn.Module):
    """Consistent-mass right-hand side M f, h^2 [1 4 1; 4 16 4; 1 4 1]/36 (model.py:49-61)."""

    def __init__(self, h):
        super().__init__()
        self.h = h
        self.net = nn.Conv2d(1, 1, kernel_size=3, padding=1, bias=False)
        w = np.array([[h * h / 36., h * h / 9., h * h / 36.],
                      [h * h / 9., 4. * h * h / 9., h * h / 9.],
                      [h * h / 36., h * h / 9., h * h / 36.]], dtype=np.float32).reshape(1, 1, 3, 3)
        self.net.weight = nn.Parameter(torch.from_numpy(w).to(self.net.weight.device))

    def forward(self, x):
        w = self.net.weight
        if w.dtype != x.dtype:
            raise RuntimeError(f"FNet: input dtype {x.dtype} != weight dtype {w.dtype} (use .double())")
        return ops.conv3x3(x, w[0])
