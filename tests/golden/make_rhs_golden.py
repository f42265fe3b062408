#!/usr/bin/env python3
"""Golden vectors for tools/rhs_families.py (the benchmark input generator of config C5) from the
reference's own generator, Data/RHS/generate_rhs.py and gaussian_random_fields.py, run in the build
container (numpy/scipy; h5py is only imported by generate_rhs.py and is replaced by an empty module
here, it is used only by its __main__).  The random draws are replayed from the same seeds to record
the parameters each sample used, so the restatement's formulas are checked for given parameters.

Usage:  python tests/golden/make_rhs_golden.py     (writes tests/golden/rhs_families.npz)
"""
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference/Data/RHS"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rhs_families.npz")
sys.modules.setdefault("h5py", types.ModuleType("h5py"))
sys.path.insert(0, REF)
import gaussian_random_fields as gr  # noqa: E402
import generate_rhs as gen  # noqa: E402


def main():
    out = {}
    N = 17
    x = np.linspace(-1, 1, N, dtype=np.float32)
    xx, yy = np.meshgrid(x, x, indexing="xy")
    for s in range(3):
        # trigonometric / polynomial: coefficients 10*rand(k) - 5 from numpy's global generator
        np.random.seed(s)
        out[f"trig_{s}"] = gen.trigonometric_function(xx, yy)
        np.random.seed(s)
        out[f"trig_coef_{s}"] = 10 * np.random.rand(3) - 5
        np.random.seed(s)
        out[f"poly_{s}"] = gen.polynomial_function(xx, yy)
        np.random.seed(s)
        out[f"poly_coef_{s}"] = 10 * np.random.rand(4) - 5
        # discontinuous: a (numpy), b (python random), coef1, coef2 (numpy)
        np.random.seed(s)
        random.seed(s)
        out[f"disc_{s}"] = gen.discontinuous_function(xx, yy)
        np.random.seed(s)
        random.seed(s)
        a = 20 * np.random.random() - 10
        b = 2 * random.random() - 1
        c1 = 10 * np.random.random((3,)) - 5
        c2 = 10 * np.random.random((3,)) - 5
        out[f"disc_par_{s}"] = np.concatenate([[a, b], c1, c2])
        # Gaussian random field for a given alpha: record the complex noise it draws
        alpha = 2.0 + s
        np.random.seed(s)
        out[f"grf_{s}"] = gr.gaussian_random_field(alpha=alpha, size=N)
        np.random.seed(s)
        out[f"grf_noise_re_{s}"] = np.random.normal(size=(N, N))
        out[f"grf_noise_im_{s}"] = np.random.normal(size=(N, N))
        out[f"grf_alpha_{s}"] = np.array(alpha)
    counts = gen.main(N, 12, 6)
    out["main_train_shape"] = np.array(counts["train"].shape)
    np.savez(OUT, **out)
    print("wrote", OUT, len(out), "arrays")


if __name__ == "__main__":
    main()
