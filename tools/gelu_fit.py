"""Fit of the bf16-output GELU's normal tail (csrc/mapa_common.h gelu_bf16out): P(t) ~ log2 Phi(-t) on t in [0, 12],
degree DEG (argv[1], default 9), Chebyshev least squares reweighted towards minimax, then rewritten in powers of t
(no 1/12 scaling in the kernel); prints the fp32 coefficients (highest degree first), the fp32-evaluated
GELU = max(x, 0) - |x| exp2(P(min(|x|, 12))) errors against the exact-erf GELU (fp64) — every point within 2^-8 relative
or 1e-30 absolute, the max relative error where |GELU| > 1e-30 — and the bf16 rounding-flip rate."""
import sys

import numpy as np
from scipy.special import log_ndtr, ndtr

T = 12.0
DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 9
t = np.linspace(0, T, 600001)
s = t / T
R = log_ndtr(-t) / np.log(2)
w = np.ones_like(s)
for _ in range(40):
    cheb = np.polynomial.chebyshev.Chebyshev.fit(s, R, DEG, domain=[0, 1], w=w)
    e = np.abs(cheb(s) - R)
    w = w * (1 + e / e.max())
a = cheb.convert(kind=np.polynomial.Polynomial).coef  # powers of s = t / 12, lowest first
c32 = (a / T ** np.arange(DEG + 1))[::-1].astype(np.float32)  # powers of t, highest first
print("coefficients (highest degree first):", [repr(float(v)) for v in c32])


def gelu_fit(x):
    tt = np.minimum(np.abs(x), np.float32(T)).astype(np.float32)
    p = np.full_like(tt, c32[0])
    for k in c32[1:]:
        p = (p.astype(np.float64) * tt + k).astype(np.float32)  # fma: one rounding
    e2 = np.exp2(p.astype(np.float64)).astype(np.float32)
    pos = np.maximum(x, np.float32(0))
    return (pos.astype(np.float64) - np.abs(x).astype(np.float64) * e2).astype(np.float32)  # fma: one rounding


def bf16(v):
    v = np.asarray(v, np.float32).view(np.uint32)
    return ((v + ((v >> 16) & 1) + 0x7FFF) & 0xFFFF0000).view(np.float32)


x = np.linspace(-14, 14, 4000001).astype(np.float32)
g, ex = gelu_fit(x), x.astype(np.float64) * ndtr(x.astype(np.float64))
print("every point within 2^-8 relative or 1e-30 absolute:", bool((np.abs(g - ex) <= np.abs(ex) * 2.0 ** -8 + 1e-30).all()))
m = np.abs(ex) > 1e-30
print("max relative error where |GELU| > 1e-30:", (np.abs(g - ex)[m] / np.abs(ex)[m]).max())
xn = (np.random.default_rng(0).standard_normal(4000000) * 1.5).astype(np.float32)
exn = xn.astype(np.float64) * ndtr(xn.astype(np.float64))
print("bf16 flip rate vs exactly rounded GELU:", (bf16(gelu_fit(xn)) != bf16(exn.astype(np.float32))).mean())
