"""Benchmark input generator: the six right-hand-side families of the reference's dataset generator
(Data/RHS/generate_rhs.py:6-56, split as in main() :59-109), restated with seeded torch ops on the
device so BASELINE config C5 (256 x 1025^2 fp32) draws its nodal sources the way the reference's
RHS datasets are made.  Not part of the solver: an input generator for bench.py and the C5 test.

  random_data             c0 * U[0,1) + c1                              generate_rhs.py:6-8
  random_selected_points  N/2 random nodes set to U(-5,5) * U[0,1)      :10-17
  Gaussian_random_field   power-law spectrum, alpha ~ U(2,5), std 1     :19-21, gaussian_random_fields.py:47-92
  trigonometric_function  c0 sin(c1 pi x) sin(c2 pi y)                  :23-30
  polynomial_function     c0 x^2 + c1 y^2 + c2 xy + c3                  :32-39
  discontinuous_function  trig above the line a x + b = y, quadratic below  :41-56
Coefficients are U(-5, 5) (10*rand - 5) as in the reference; x, y = float32 linspace(-1, 1, N) on an
'xy' meshgrid.  The reference draws from numpy's global generator (unseeded); here every sample is
drawn from a torch.Generator seeded with (seed, sample index), so batches are reproducible.
"""
import math

import torch

FAMILIES = ("random_data", "random_selected_points", "gaussian_random_field", "trigonometric_function",
            "polynomial_function", "discontinuous_function")


def family_counts(B):
    """Samples per family for a batch of B (generate_rhs.main: B // 6 each, the rest discontinuous)."""
    k = B // 6
    return [k] * 5 + [B - 5 * k]


def grf_from_noise(noise, alpha):
    """gaussian_random_fields.gaussian_random_field(alpha, size=N) for a given complex noise field:
    amplitude |k|^(-alpha/2) on the fftshift-ed integer frequencies (fftind), real part of the inverse
    FFT, normalised to mean 0 and standard deviation 1."""
    N = noise.shape[-1]
    k = torch.arange(N, device=noise.device, dtype=torch.float64) - (N + 1) // 2
    k = torch.fft.fftshift(k)
    kx, ky = k[None, :], k[:, None]
    amp = torch.pow(kx * kx + ky * ky + 1e-10, -alpha / 4.0)
    amp[0, 0] = 0
    f = torch.fft.ifft2(noise * amp).real
    f = f - f.mean()
    return f / f.std(unbiased=False)


def _grf(N, alpha, g, device):
    noise = torch.complex(torch.randn(N, N, generator=g, device=device, dtype=torch.float64),
                          torch.randn(N, N, generator=g, device=device, dtype=torch.float64))
    return grf_from_noise(noise, alpha)


def grid(N, device="cpu"):
    """x, y = float32 linspace(-1, 1, N) on an 'xy' meshgrid (generate_rhs.py:88-90), as float64."""
    x = torch.linspace(-1, 1, N, dtype=torch.float32, device=device).to(torch.float64)
    return x[None, :].expand(N, N), x[:, None].expand(N, N)


def trigonometric(xx, yy, c):
    return c[0] * torch.sin(c[1] * math.pi * xx) * torch.sin(c[2] * math.pi * yy)


def polynomial(xx, yy, c):
    return c[0] * xx ** 2 + c[1] * yy ** 2 + c[2] * xx * yy + c[3]


def discontinuous(xx, yy, a, b, c1, c2):
    """The reference fills a float32 array (np.zeros_like of the float32 grid) node by node, testing
    a x + b > y in float32 arithmetic (Python-float a, b against float32 coordinates)."""
    f32 = torch.float32
    x32, y32 = xx.to(f32), yy.to(f32)
    above = x32 * torch.tensor(a, dtype=f32) + torch.tensor(b, dtype=f32) > y32
    poly = c2[0] * xx ** 2 + c2[1] * yy ** 2 + c2[2] * xx * yy
    return torch.where(above, trigonometric(xx, yy, c1), poly).to(f32).to(xx.dtype)


def sample(family, N, g, device):
    """One N x N nodal source of `family` (float64)."""
    dt = torch.float64
    rand = lambda *s: torch.rand(*s, generator=g, device=device, dtype=dt)  # noqa: E731
    coef = lambda n: 10 * rand(n) - 5  # noqa: E731
    xx, yy = grid(N, device)
    if family == "random_data":
        c = coef(2)
        return c[0] * rand(N, N) + c[1]
    if family == "random_selected_points":
        n = N // 2
        i = torch.randint(N, (n,), generator=g, device=device).tolist()
        j = torch.randint(N, (n,), generator=g, device=device).tolist()
        v = ((10 * rand(n) - 5) * rand(n)).tolist()
        out = torch.zeros(N, N, dtype=dt)
        for a, b, c in zip(i, j, v):  # in order: a repeated node keeps the last value, as the reference's loop
            out[a, b] = c
        return out.to(device)
    if family == "gaussian_random_field":
        alpha = 2.0 + 3.0 * float(rand(1))
        return _grf(N, alpha, g, device)
    if family == "trigonometric_function":
        return trigonometric(xx, yy, coef(3))
    if family == "polynomial_function":
        return polynomial(xx, yy, coef(4))
    if family == "discontinuous_function":
        a = 20 * float(rand(1)) - 10
        b = 2 * float(rand(1)) - 1
        return discontinuous(xx, yy, a, b, coef(3), coef(3))
    raise ValueError(f"unknown RHS family {family!r}")


def batch(B, N, dtype=torch.float32, device="cuda", seed=0):
    """[B, 1, N, N] nodal sources: the six families in the proportions of generate_rhs.main."""
    out = torch.empty(B, 1, N, N, dtype=dtype, device=device)
    i = 0
    for fam, cnt in zip(FAMILIES, family_counts(B)):
        for _ in range(cnt):
            g = torch.Generator(device=device)
            g.manual_seed(seed * 1000003 + i)
            out[i, 0] = sample(fam, N, g, device).to(dtype)
            i += 1
    return out
