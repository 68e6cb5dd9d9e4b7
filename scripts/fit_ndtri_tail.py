"""Fit of the fp32 normal quantile's extreme-tail polynomial (tmh_math.h erfinv_tail):
P(s) = ndtri(t) / (sqrt(2) (1 - 2t)) as a polynomial in s - 4.3, s = sqrt(w),
w = -log(4t(1-t)), over w in [15.9, 21.5] (t down to 2^-33, the smallest 32-bit
midpoint uniform), weighted for relative error; prints the fp32 coefficients
(highest degree first) and the max relative error of an fp32 Horner evaluation.
Giles' two polynomials cover w < 16; beyond, his tail polynomial is 4e-4 off."""
import numpy as np
from scipy.special import ndtri

t = np.logspace(np.log10(2.0 ** -33), np.log10(2e-7), 400000)
w = -np.log(4 * t * (1 - t))
m = w >= 15.9
t, w = t[m], w[m]
P = -ndtri(t) / (np.sqrt(2) * (1 - 2 * t))
s = np.sqrt(w)
S0, DEG = 4.3, 5
coef = np.polynomial.polynomial.polyfit(s - S0, P, DEG, w=1 / P).astype(np.float32)
v = (s.astype(np.float32) - np.float32(S0)).astype(np.float32)
acc = np.full_like(v, coef[-1])
for k in range(DEG - 1, -1, -1):
    acc = (acc.astype(np.float64) * v + coef[k]).astype(np.float32)
print("coefficients (highest first):", [repr(float(c)) for c in coef[::-1]])
print("max rel error (fp32 Horner): %.3e over w in [%.2f, %.2f]" % ((np.abs(acc - P) / P).max(), w.min(), w.max()))
