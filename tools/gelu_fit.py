"""Fit of the rational GELU used by the f16 GEMM epilogues (csrc/gemm_common.h, gelu_rat):
Phi(x) - 1/2 = c P(c^2) / Q(c^2), c = clamp(x, -X, X), deg P = 4, deg Q = 3 (Q(0) = 1).
Linearised least squares (P - f Q = 0, weighted by c) as the start, Levenberg-Marquardt on the
GELU error, coefficients rounded to f32; then the f32 evaluation is checked on [-9, 9].
    python tools/gelu_fit.py [--clamp 5.5]"""
import argparse

import numpy as np
from scipy.optimize import least_squares
from scipy.special import erf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--clamp', type=float, default=5.5)
    a = ap.parse_args()
    X, m, n = a.clamp, 4, 3
    xs = np.linspace(1e-4, X, 20001)
    f = 0.5 * erf(xs / np.sqrt(2)) / xs  # Phi(x) - 1/2 = x f(x^2)
    s = xs * xs

    def rat(c, s):
        return np.polyval(c[:m + 1][::-1], s) / np.polyval(np.r_[1.0, c[m + 1:]][::-1], s)

    A = np.hstack([np.vander(s, m + 1, increasing=True), -f[:, None] * np.vander(s, n + 1, increasing=True)[:, 1:]])
    c0, *_ = np.linalg.lstsq(A * xs[:, None], f * xs, rcond=None)
    c = least_squares(lambda c: (rat(c, s) - f) * xs, c0, xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=20000).x
    c = c.astype(np.float32)
    print('P', [repr(float(v)) for v in c[:m + 1]])
    print('Q', ['1.0'] + [repr(float(v)) for v in c[m + 1:]])
    x = np.linspace(-9, 9, 2000001).astype(np.float32)
    cl = np.clip(x, -X, X).astype(np.float32)
    s32 = (cl * cl).astype(np.float32)
    P = c[m]
    for k in range(m - 1, -1, -1):
        P = (P * s32 + c[k]).astype(np.float32)
    Q = c[m + n]
    for k in range(m + n - 1, m, -1):
        Q = (Q * s32 + c[k]).astype(np.float32)
    Q = (Q * s32 + np.float32(1)).astype(np.float32)
    g = (x * ((cl * P) * (np.float32(1) / Q) + np.float32(0.5))).astype(np.float32)
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    err = np.abs(g - ref)
    print(f'max |err| {err.max():.3g}, max |err| / max(|x|, 1) {(err / np.maximum(np.abs(x), 1)).max():.3g}')


if __name__ == '__main__':
    main()
