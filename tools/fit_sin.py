"""Minimax fit (Lawson's iteratively reweighted least squares, mpmath
reference values) of sin(r) ~ r + r^3 * P(r^2) on [-pi/2, pi/2] in relative
error, for the reduced-by-pi f32 sin/cos of device_ops.h. Prints the f32
coefficients (c1..cK of P). Tool only; run: python tools/fit_sin.py [K]."""
import sys
import numpy as np
import mpmath as mp

mp.mp.dps = 40
K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
half_pi = float(mp.pi / 2)
# sample in s = r^2 on Chebyshev-like nodes, r in (0, pi/2]
m = 4000
t = (1 - np.cos(np.linspace(0, np.pi, m))) / 2
r = np.maximum(t * half_pi, 1e-4)
s = r * r
g = np.array([float((mp.sin(mp.mpf(x)) - mp.mpf(x)) / mp.mpf(x) ** 3) for x in r])
sinr = np.array([float(mp.sin(mp.mpf(x))) for x in r])
A = np.vstack([s ** k for k in range(K)]).T
wrel = r ** 3 / sinr  # error in g scales to relative error of sin by r^3/sin(r)
w = np.ones(m)
for it in range(200):
    W = np.sqrt(w) * wrel
    c, *_ = np.linalg.lstsq(A * W[:, None], g * W, rcond=None)
    e = (A @ c - g) * wrel
    w = w * np.abs(e)
    w /= w.sum()
print("max rel err (double coeffs): %.3e" % np.abs(e).max())
c32 = c.astype(np.float32)
# refit the higher coefficients after rounding the leading ones (greedy)
for k in range(K):
    c32[k] = np.float32(c[k])
    if k + 1 < K:
        rest = g - A[:, : k + 1] @ c32[: k + 1].astype(np.float64)
        B = A[:, k + 1 :]
        cc, *_ = np.linalg.lstsq(B * wrel[:, None], rest * wrel, rcond=None)
        c[k + 1 :] = cc
e32 = (A @ c32.astype(np.float64) - g) * wrel
print("max rel err (f32 coeffs): %.3e" % np.abs(e32).max())
print(", ".join("%.9ef" % v for v in c32))
