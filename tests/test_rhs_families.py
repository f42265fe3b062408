"""tools/rhs_families.py — the C5 benchmark input generator — against the reference's own generator
(tests/golden/rhs_families.npz, made by tests/golden/make_rhs_golden.py from Data/RHS/generate_rhs.py
and gaussian_random_fields.py): each family's formula for the parameters the reference drew."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools import rhs_families as rf  # noqa: E402


def test_families_vs_reference(gold):
    g = gold("rhs_families.npz")
    N = 17
    xx, yy = rf.grid(N)
    for s in range(3):
        c = torch.from_numpy(g[f"trig_coef_{s}"])
        np.testing.assert_allclose(rf.trigonometric(xx, yy, c).numpy(), g[f"trig_{s}"], rtol=1e-12, atol=1e-12)
        c = torch.from_numpy(g[f"poly_coef_{s}"])
        np.testing.assert_allclose(rf.polynomial(xx, yy, c).numpy(), g[f"poly_{s}"], rtol=1e-12, atol=1e-12)
        p = g[f"disc_par_{s}"]
        d = rf.discontinuous(xx, yy, float(p[0]), float(p[1]), torch.from_numpy(p[2:5]), torch.from_numpy(p[5:8]))
        np.testing.assert_allclose(d.numpy(), g[f"disc_{s}"], rtol=1e-12, atol=1e-12)
        noise = torch.complex(torch.from_numpy(g[f"grf_noise_re_{s}"]), torch.from_numpy(g[f"grf_noise_im_{s}"]))
        np.testing.assert_allclose(rf.grf_from_noise(noise, float(g[f"grf_alpha_{s}"])).numpy(), g[f"grf_{s}"],
                                   rtol=1e-10, atol=1e-12)


def test_batch_composition_and_seed():
    assert rf.family_counts(256) == [42, 42, 42, 42, 42, 46]
    a = rf.batch(13, 33, torch.float64, "cpu", seed=3)
    b = rf.batch(13, 33, torch.float64, "cpu", seed=3)
    assert torch.equal(a, b) and a.shape == (13, 1, 33, 33)
    assert not torch.equal(a, rf.batch(13, 33, torch.float64, "cpu", seed=4))
    # random_selected_points: at most N/2 nonzero nodes
    assert int((a[2, 0] != 0).sum()) <= 16
    # Gaussian random field: mean 0, std 1
    assert abs(float(a[4].mean())) < 1e-12 and abs(float(a[4].std(unbiased=False)) - 1) < 1e-12
