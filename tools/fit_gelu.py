"""Fits the polynomial R(a) of the one-transcendental GELU epilogue:

    Phi(-a) = exp(-a^2 / 2) * R(a),   a = |x| in [0, AMAX]
    gelu(x) = x * Phi(x) = x >= 0 ? x - x*Phi(-a) : x*Phi(-a)

R(a) = erfc(a/sqrt2)/2 * exp(a^2/2) is smooth and positive, so a low-degree polynomial reaches
a relative error far below the bf16 output rounding (2^-9).  Weighted least squares iterated
toward minimax on the relative error; prints the fp32-Horner error per degree and the
coefficients of the chosen degree.   python tools/fit_gelu.py [degree]
"""
import sys

import numpy as np
from scipy.special import erfc

AMAX = 5.5


def fit(deg, a, R):
    V = np.vander(a, deg + 1, increasing=True)
    ww = 1.0 / R
    for _ in range(40):
        c, *_ = np.linalg.lstsq(V * ww[:, None], R * ww, rcond=None)
        err = (V @ c - R) / R
        ww = ww * (1.0 + np.abs(err) / np.abs(err).max()) ** 2
    return c


def horner32(c, a):
    cf = c.astype(np.float32)
    af = a.astype(np.float32)
    p = np.full_like(af, cf[-1])
    for k in range(len(cf) - 2, -1, -1):
        p = p * af + cf[k]
    return p.astype(np.float64)


def main():
    a = np.linspace(0.0, AMAX, 40001)
    R = 0.5 * erfc(a / np.sqrt(2.0)) * np.exp(a * a / 2.0)
    want = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else None
    for deg in range(5, 12):
        c = fit(deg, a, R)
        e32 = np.abs((horner32(c, a) - R) / R).max()
        print(f"degree {deg}: max relative error (fp32 Horner) {e32:.3e}")
        if deg == want:
            print("coefficients (a^0 .. a^n):")
            print(", ".join(f"{float(np.float32(v))!r}f" for v in c))


if __name__ == "__main__":
    main()


def fit_tanh(y0=0.48, deg=3):
    """Capped-softmax numerator exp(cap*tanh(x/cap)) = exp2(log2e * x * T((x/cap)^2)) for
    |x| <= y0*cap, T(v) = tanh(sqrt v)/sqrt v fitted on v in [0, y0^2] (relative error)."""
    v = np.linspace(1e-12, y0 * y0, 20001)
    T = np.tanh(np.sqrt(v)) / np.sqrt(v)
    c = fit(deg, v, T)
    err = np.abs((horner32(c, v) - T) / T).max()
    return c, err


def fit_log2(deg=6, tmax=5.3):
    """Production GELU epilogue (gemm_epilogue.h gelu_fast2, degree 6 on [0, 5.3]; round 2's first
    form was degree 7 on [0, 5.6]): P(t) ~ log2 Phi(-t) on [0, tmax],
    gelu(x) = max(x, 0) - t * exp2(P(t)), t = min(|x|, tmax).  Returns the coefficients and the
    fp32 relative / absolute error of the whole GELU against x*Phi(x) on [-30, 30]."""
    from scipy.special import log_ndtr, ndtr
    t = np.linspace(0.0, tmax, 40001)
    f = log_ndtr(-t) / np.log(2.0)
    V = np.vander(t, deg + 1, increasing=True)
    ww = np.ones_like(t)
    for _ in range(60):
        c, *_ = np.linalg.lstsq(V * ww[:, None], f * ww, rcond=None)
        err = V @ c - f
        ww = ww * (1.0 + np.abs(err) / np.abs(err).max()) ** 2
        ww /= ww.max()
    x = np.concatenate([np.linspace(-30, 30, 600001), np.linspace(-6, 6, 400001)]).astype(np.float32)
    tt = np.minimum(np.abs(x), np.float32(tmax))
    p = horner32(c, tt.astype(np.float64)).astype(np.float32)
    g = (np.maximum(x, np.float32(0)) - tt * np.exp2(p).astype(np.float32)).astype(np.float64)
    gt = x.astype(np.float64) * ndtr(x.astype(np.float64))
    e = np.abs(g - gt)
    m = np.abs(gt) > 1e-6
    return c, float((e[m] / np.abs(gt[m])).max()), float(e.max())


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "log2":
    for deg, tmax in ((6, 5.3), (6, 5.6), (7, 5.6), (8, 5.6)):
        c, rel, ab = fit_log2(deg, tmax)
        print(f"log2 form degree {deg} on [0, {tmax}]: rel {rel:.2e} abs {ab:.2e}:", ", ".join(f"{float(np.float32(v))!r}f" for v in c))


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "tanh":
    for y0 in (0.4, 0.48, 0.6):
        for deg in (2, 3, 4):
            c, err = fit_tanh(y0, deg)
            print(f"tanh y0={y0} deg={deg}: rel err {err:.2e} (x*err*log2e at x=y0*50: {err*y0*50*1.4427:.2e})",
                  ", ".join(f"{float(np.float32(a))!r}" for a in c))
