"""Accuracy of the fp32 GEMM's libm-free exact-erf GELU (vp_common.h gelu_erfc_fit2) against fp64, emulated
in numpy with one fp32 rounding per device operation (the reciprocal perturbed by up to 1 ulp, as v_rcp_f32),
beside a fp32 GELU built on a correctly rounded erf (what libm's erff approximates).  CPU only.
    python tools/gelu_erfc_accuracy.py
"""
import numpy as np
from scipy.special import erf

F = np.float32
C = [-1.26551223, 1.00002368, 0.37409196, 0.09678418, -0.18628806, 0.27886807, -1.13520398, 1.48851587,
     -0.82215223, 0.17087277]


def fma(a, b, c):
    return (a.astype(np.float64) * b + c).astype(F)


def gelu_fit(x, rng):
    za = (np.abs(x) * F(0.70710678118654752)).astype(F)
    d = fma(F(0.5), za, F(1))
    r = (1.0 / d.astype(np.float64) * (1 + rng.uniform(-1, 1, d.shape) * 2.0 ** -23)).astype(F)
    t = fma(r, fma(-d, r, F(1)), r)
    p = np.full_like(t, F(C[9]))
    for k in range(8, -1, -1):
        p = fma(p, t, F(C[k]))
    y = (fma(-za, za, p) * F(1.4426950408889634)).astype(F)
    hec = ((F(0.5) * t).astype(F) * np.exp2(y.astype(np.float64)).astype(F)).astype(F)
    phi = np.where(x >= 0, (F(1) - hec).astype(F), hec)
    return (x * phi).astype(F)


def gelu_crerf(x):
    z = (x * F(0.70710678118654752)).astype(F)
    e = erf(z.astype(np.float64)).astype(F)
    return (F(0.5) * x * (F(1) + e)).astype(F)


def main():
    rng = np.random.default_rng(0)
    x = np.linspace(-12, 12, 2_000_001).astype(F)
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    for name, v in (("libm-free fit", gelu_fit(x, rng)), ("correctly rounded erf", gelu_crerf(x))):
        d = np.abs(v.astype(np.float64) - ref)
        parts = []
        for lo, hi in ((-12, -4), (-4, -1), (-1, 1), (1, 4), (4, 12)):
            m = (x >= lo) & (x < hi)
            parts.append(f"[{lo},{hi}) max {d[m].max():.2e} mean {d[m].mean():.2e}")
        print(f"{name:22s} " + "  ".join(parts))


if __name__ == "__main__":
    main()
