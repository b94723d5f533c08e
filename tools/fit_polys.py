"""Fit the fixed-coefficient polynomials of the deterministic fp32 math used by
BOTH the C oracle and the HIP kernels (atan2, log2, exp2).  The coefficients are
part of the declared numeric contract (DESIGN.md "Deterministic math"): any
change here must be mirrored in oracle/gsm_oracle_math.h and
gsm-renderer_amd/csrc/gsm_detmath.h.  Run: python tools/fit_polys.py"""
import numpy as np

def cheb_fit(f, a, b, deg, n=4000):
    k = np.arange(n)
    x = np.cos((2 * k + 1) * np.pi / (2 * n))
    s = (a + b) / 2 + (b - a) / 2 * x
    V = np.vander(s, deg + 1, increasing=True)
    w = 1.0 / np.maximum(np.abs(f(s)), 1e-300)
    c, *_ = np.linalg.lstsq(V * w[:, None], f(s) * w, rcond=None)
    return c

def show(name, c):
    c32 = c.astype(np.float32)
    print(name, ", ".join(float(v).hex() for v in c32))
    return c32

# atan(t)/t = P(t^2) on s in [0,1]
ca = show("atan P(s)", cheb_fit(lambda s: np.where(s > 0, np.arctan(np.sqrt(s)) / np.sqrt(np.maximum(s, 1e-300)), 1.0), 0.0, 1.0, 11))
# log2(m) = u * Q(u^2), u=(m-1)/(m+1), m in [sqrt(.5), sqrt(2)] -> u in [-0.1716, 0.1716]
umax = (np.sqrt(2) - 1) / (np.sqrt(2) + 1)
cl = show("log2 Q(u2)", cheb_fit(lambda u2: np.where(u2 > 0, np.log2((1 + np.sqrt(u2)) / (1 - np.sqrt(u2))) / np.sqrt(np.maximum(u2, 1e-300)), 2 / np.log(2)), 0.0, umax ** 2, 5))
# 2^f on f in [-0.5, 0.5]
ce = show("exp2 R(f)", cheb_fit(lambda f: 2.0 ** f, -0.5, 0.5, 7))

def horner(c, x):
    p = np.float32(c[-1])
    for v in c[-2::-1]:
        p = np.float32(p * x + v)
    return p
t = np.linspace(0, 1, 10001, dtype=np.float32)
err = np.max(np.abs(t * horner(ca, t * t) - np.arctan(t.astype(np.float64))))
print("atan max abs err", err)
