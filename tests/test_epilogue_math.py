"""The GEMM epilogue's GELU (videoprism-mlx_amd/csrc/gemm_epilogue.h gelu_fast2), restated in
fp32 NumPy with the coefficients parsed from the header, against the exact-erf GELU of the
reference (layers.py:31, jax.nn.gelu(approximate=False)) in fp64.  CPU only: pins the constants
and the error bound the kernel's comment states (relative <= 2.2e-5 where |gelu| > 1e-6, absolute
<= 3.0e-6 on [-30, 30]), far below the bf16 output rounding (2^-9)."""

import os
import re

import numpy as np
from scipy.special import ndtr

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "videoprism-mlx_amd", "csrc",
                   "gemm_epilogue.h")


def _coeffs():
    src = open(HDR).read()
    c = {int(k): float(v.rstrip("f")) for k, v in re.findall(r"#define VP_GELU_P(\d) (\S+)", src)}
    tmax = float(re.search(r"GELU_TMAX = (\S+?)f;", src).group(1))
    return [np.float32(c[i]) for i in range(len(c))], np.float32(tmax)


def gelu_epilogue_f32(x):
    """The kernel's operation sequence in fp32: t = minimum(|x|, TMAX); Horner; exp2; fma (NumPy's
    minimum / maximum propagate NaN like the kernel's v_minimum3_f32 / v_maximum3_f32)."""
    c, tmax = _coeffs()
    x = np.asarray(x, np.float32)
    t = np.minimum(np.abs(x), tmax)
    p = np.full_like(t, c[-1])
    for k in range(len(c) - 2, -1, -1):
        p = (p * t + c[k]).astype(np.float32)
    e = np.exp2(p).astype(np.float32)
    return (np.maximum(x, np.float32(0)) - t * e).astype(np.float32)


def test_gelu_epilogue_error_bound():
    x = np.concatenate([np.linspace(-30, 30, 600001), np.linspace(-6, 6, 400001),
                        np.array([0.0, -0.0, 1e-30, -1e-30, 5.3, -5.3, 5.31, -5.31])]).astype(np.float32)
    g = gelu_epilogue_f32(x).astype(np.float64)
    ref = x.astype(np.float64) * ndtr(x.astype(np.float64))
    err = np.abs(g - ref)
    m = np.abs(ref) > 1e-6
    assert err.max() <= 3.0e-6, err.max()
    assert (err[m] / np.abs(ref[m])).max() <= 2.2e-5, (err[m] / np.abs(ref[m])).max()


def test_gelu_epilogue_limits():
    g = gelu_epilogue_f32(np.array([np.inf, -np.inf, 1e30, -1e30, 40.0, -40.0], np.float32))
    assert g[0] == np.inf and g[2] == np.float32(1e30) and g[4] == np.float32(40.0)
    # -inf: by design the clamp's value gelu(-5.3) (a tiny negative number), not the reference's
    # NaN (-inf * Phi(-inf) = -inf * 0); documented at gelu_fast in gemm_epilogue.h
    assert np.isfinite(g[1]) and -1e-6 < g[1] < 0 and g[1] == gelu_epilogue_f32(np.float32(-5.3))
    assert abs(g[3]) < 1e-6 and abs(g[5]) < 1e-6


def test_gelu_epilogue_nan_propagates():
    """A NaN pre-activation (upstream overflow) must come out NaN, as x * Phi(x) does in the
    reference, not as a small finite value (IEEE minNum / maxNum would absorb it)."""
    with np.errstate(invalid="ignore"):
        g = gelu_epilogue_f32(np.array([np.nan, -np.nan], np.float32))
    assert np.isnan(g).all()
    src = open(HDR).read()
    body = src[src.index("gelu_fast2(f32x2_t x)"):src.index("gelu4(float4 v)")]
    assert "__builtin_fminf" not in body and "__builtin_fmaxf" not in body
    assert body.count("__builtin_elementwise_minimum") == 2 and body.count("__builtin_elementwise_maximum") == 2
