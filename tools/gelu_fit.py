"""Fit of the bf16-output GELU's normal tail (csrc/mapa_common.h gelu_bf16out): P(s) ~ log2 Phi(-12 s) on s in
[0, 1] (|x| <= 12), degree 9, Chebyshev least squares reweighted towards minimax; prints the fp32 coefficients (highest
degree first), the fp32-evaluated GELU's errors against the exact-erf GELU (fp64) — every point within 2^-8 relative
or 1e-30 absolute, the max relative error where |GELU| > 1e-30 — and the bf16 rounding-flip rate."""
import numpy as np
from scipy.special import log_ndtr, ndtr

T, DEG = 12.0, 9
t = np.linspace(0, T, 600001)
s = t / T
R = log_ndtr(-t) / np.log(2)
w = np.ones_like(s)
for _ in range(40):
    cheb = np.polynomial.chebyshev.Chebyshev.fit(s, R, DEG, domain=[0, 1], w=w)
    e = np.abs(cheb(s) - R)
    w = w * (1 + e / e.max())
c32 = cheb.convert(kind=np.polynomial.Polynomial).coef[::-1].astype(np.float32)
print("coefficients (highest degree first):", [float(v) for v in c32])


def gelu_fit(x):
    ss = (np.minimum(np.abs(x), np.float32(T)) * np.float32(1 / T)).astype(np.float32)
    p = np.full_like(ss, c32[0])
    for k in c32[1:]:
        p = (p.astype(np.float64) * ss + k).astype(np.float32)  # fma: one rounding
    xq = (x * np.exp2(p.astype(np.float64)).astype(np.float32)).astype(np.float32)
    return np.where(x >= 0, (x - xq).astype(np.float32), xq)


def bf16(a):
    a = np.asarray(a, np.float32).view(np.uint32)
    return ((a + ((a >> 16) & 1) + 0x7FFF) & 0xFFFF0000).view(np.float32)


x = np.linspace(-14, 14, 4000001).astype(np.float32)
g, ex = gelu_fit(x), x.astype(np.float64) * ndtr(x.astype(np.float64))
print("every point within 2^-8 relative or 1e-30 absolute:", bool((np.abs(g - ex) <= np.abs(ex) * 2.0 ** -8 + 1e-30).all()))
m = np.abs(ex) > 1e-30
print("max relative error where |GELU| > 1e-30:", (np.abs(g - ex)[m] / np.abs(ex)[m]).max())
xn = (np.random.default_rng(0).standard_normal(4000000) * 1.5).astype(np.float32)
exn = xn.astype(np.float64) * ndtr(xn.astype(np.float64))
print("bf16 flip rate vs exactly rounded GELU:", (bf16(gelu_fit(xn)) != bf16(exn.astype(np.float32))).mean())
