"""HNet — the learned Jacobi correction of M-FEANet-mg_test.ipynb (cell 4, `HNet` :97-106;
used by `HJacIterator.HRelax` :147-155 and trained by `HJacIterator.Train` :161-198) — with every
layer a HIP 3x3 convolution (fea_knet_apply, ntab = 1) and its HIP adjoints (fea_knet_apply_adj,
fea_stencil_weight_grad).  Same constructor, forward signature and state_dict keys
(`convLayers.{i}.weight`, [1, 1, 3, 3]) as the notebook's class, so a notebook can swap it in and
load `Model/learn_iterator/iso_poisson/iso_poisson_33x33.pth` unchanged.

For the V-cycle itself, `MultigridSolver(smoother="hjac", hnet=...)` runs the whole HRelax sweep
as one fused kernel (fea_mg_hsweep); this module is the differentiable, per-layer form.
"""
import torch
import torch.nn as nn

from . import ops


class HNet(nn.Module):
    def __init__(self, nb_layers):
        super().__init__()
        self.convLayers = nn.ModuleList([nn.Conv2d(1, 1, 3, padding=1, bias=False) for _ in range(nb_layers)])

    def forward(self, x, geo_idx):
        """geo_idx: 1 on interior nodes, 0 on the boundary; each layer's output is masked by it."""
        for conv in self.convLayers:
            x = ops.conv3x3(x, conv.weight[0]) * geo_idx
        return x
