"""Fit of the fp64 normal quantile's central polynomial (tmh_math.h ndtri64):
f(w) = erfinv(x) / x with x = 2p - 1, w = -log(1 - x^2) = -log(4 p (1 - p)), as a
polynomial in t = w - W0 over w in [0, WMAX] (p in ~[5e-4, 1 - 5e-4] for WMAX = 6.25:
99.9 % of the per-second draws); the rest take ocml's quantile out of line.
Chebyshev interpolation at 80-digit precision (mpmath), converted to monomials in t,
rounded to fp64; the printed error is that of an fp64 Horner evaluation (fma emulated
in long double) against mpmath's erfinv, relative, over 20,000 points of the interval.
  python3 scripts/fit_ndtri_f64.py [DEGREE]"""
import sys

import mpmath as mp
import numpy as np

mp.mp.dps = 80
W0, WMAX = mp.mpf("3.125"), mp.mpf("6.25")
DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 24


def f(w):
    if w == 0:
        return mp.sqrt(mp.pi) / 2
    x = mp.sqrt(-mp.expm1(-w))
    return mp.erfinv(x) / x


# Chebyshev interpolation on [0, WMAX] in u = (w - W0) / W0 in [-1, 1]
N = DEG + 1
nodes = [mp.cos(mp.pi * (k + mp.mpf(1) / 2) / N) for k in range(N)]
vals = [f(W0 + W0 * u) for u in nodes]
cheb = []
for j in range(N):
    s = mp.fsum(vals[k] * mp.cos(mp.pi * j * (k + mp.mpf(1) / 2) / N) for k in range(N))
    cheb.append(s * (1 if j == 0 else 2) / N)
# Chebyshev -> monomials in u (exact in mp), then in t = W0 u
T = [[mp.mpf(1)], [mp.mpf(0), mp.mpf(1)]]
for j in range(2, N):
    a = [mp.mpf(0)] + [2 * c for c in T[j - 1]]
    b = T[j - 2] + [mp.mpf(0)] * (len(a) - len(T[j - 2]))
    T.append([a[i] - b[i] for i in range(len(a))])
mono = [mp.mpf(0)] * N
for j in range(N):
    for i, c in enumerate(T[j]):
        mono[i] += cheb[j] * c
coef = [float(mono[i] / W0 ** i) for i in range(N)]   # in t
LD = np.longdouble


def horner(t):
    acc = coef[-1]
    for c in coef[-2::-1]:
        acc = float(np.float64(LD(acc) * LD(t) + LD(c)))
    return acc


ws = np.linspace(0.0, float(WMAX), 20000)
err = 0.0
for w in ws:
    ref = f(mp.mpf(w))
    got = horner(float(np.float64(w - float(W0))))
    err = max(err, abs(float((got - ref) / ref)))
print(f"degree {DEG}: max relative error {err:.3e} ({err / 2 ** -53:.2f} ulp)")
print("coefficients in t = w - 3.125, highest degree first:")
for c in coef[::-1]:
    print(f"    {c!r},")
