"""CPU emulation of the fp64 PV chain's table functions (tmh_math.h log_tab, exp_tab,
ndtri64): the same operations in numpy (fma emulated in long double, exact for these
products), the table built as tmh_engine_create builds it and the quantile's
coefficients parsed from the header, against numpy / scipy.  The GPU probes
(tmh_probe fn 11-13, tests/test_gpu_parity.py::test_probe_math) check the device code
against the oracle; this pins the algorithm and its accuracy without a GPU."""
import math
import os
import re

import numpy as np
from scipy.special import ndtri

HERE = os.path.dirname(os.path.abspath(__file__))
MATH_H = os.path.join(HERE, "..", "tmhpvsim_amd", "csrc", "tmh_math.h")
LD = np.longdouble
LOG_TAB, EXP_TAB = 128, 64


def fma(a, b, c):
    return float(np.float64(LD(a) * LD(b) + LD(c)))


def coefs():
    """(centers, coefficient rows) of ndtri64's pieces, parsed from the header"""
    src = open(MATH_H).read()
    centers = re.search(r"NDTRI_CENTER\[NDTRI_PIECES\] = \{([^}]*)\};", src).group(1)
    body = re.search(r"NDTRI_COEF\[NDTRI_PIECES\]\[NDTRI_DEG \+ 1\] = \{[^\n]*\n(.*?)\}\};", src, re.S).group(1)
    rows = [[float(x) for x in re.findall(r"[-+]?[0-9][-+0-9.eE]*", r)] for r in body.split("},")]
    return [float(x) for x in centers.split(",")], rows


TAB = [(1.0 / (1.0 + (i + 0.5) / LOG_TAB), math.log(1.0 + (i + 0.5) / LOG_TAB)) for i in range(LOG_TAB)]
EXP = [2.0 ** (i / EXP_TAB) for i in range(EXP_TAB)]


def log_tab(x):
    bits = int(np.float64(x).view(np.uint64))
    hi = bits >> 32
    e = (hi >> 20) - 1023
    i = (hi >> 13) & (LOG_TAB - 1)
    m = float(np.uint64((((hi & 0xFFFFF) | 0x3FF00000) << 32) | (bits & 0xFFFFFFFF)).view(np.float64))
    r, lc = TAB[i]
    u = fma(m, r, -1.0)
    h = fma(u, 1 / 7, -1 / 6)
    for c in (1 / 5, -1 / 4, 1 / 3, -1 / 2):
        h = fma(h, u, c)
    return fma(float(e), 0.693147180559945309417, lc) + fma(u * u, h, u)


def exp_tab(x):
    kf = float(np.rint(x * 92.332482616893656768))
    r = fma(-kf, float.fromhex("0x1.62e42fefa0000p-7"), x)
    r = fma(-kf, 2.572804640231345e-14, r)
    p = fma(r, 1 / 720, 1 / 120)
    for c in (1 / 24, 1 / 6, 0.5, 1.0, 1.0):
        p = fma(p, r, c)
    k = int(kf)
    return math.ldexp(EXP[k & (EXP_TAB - 1)] * p, k >> 6)


def ndtri64(w, c):
    p = (w + 0.5) * 2.0 ** -32
    x = 2.0 * p - 1.0
    ww = -log_tab(4.0 * p * (1.0 - p))
    if not ww < 6.25:
        return None                      # the device takes ocml's quantile here
    centers, rows = c
    q = (1 if ww >= 2.0 else 0) + (1 if ww >= 4.0 else 0)   # the lane's piece
    u = ww - centers[q]
    f = rows[q][-1]
    for k in range(len(rows[q]) - 2, -1, -1):
        f = fma(f, u, rows[q][k])
    return (1.4142135623730950488 * x) * f


def test_log_tab_accuracy():
    xs = np.concatenate([10.0 ** np.random.default_rng(1).uniform(-10, 0.4, 4000), [1.0, 0.5, 2.0, 1 - 2 ** -52]])
    err = max(abs(log_tab(x) - math.log(x)) for x in xs)
    assert err <= 4e-15, err


def test_exp_tab_accuracy():
    xs = np.random.default_rng(2).uniform(-40, 3, 4000)
    err = max(abs(exp_tab(x) - math.exp(x)) / math.exp(x) for x in xs)
    assert err <= 4e-16, err


def test_ndtri64_accuracy_and_coefficients():
    c = coefs()
    centers, rows = c
    assert centers == [1.0, 3.0, 5.125] and [len(r) for r in rows] == [14, 14, 14]
    # degree 0 first: f at each piece's center
    assert abs(rows[1][0] - 1.6235420064648298) < 1e-15 and abs(rows[0][0] - 1.1273743936892275) < 1e-15
    rng = np.random.default_rng(3)
    # uniform words, plus 3,000 in the lower tail (p < 0.031: the pieces from w' = 2 and 4 on)
    ws = np.concatenate([rng.integers(0, 2 ** 32, 6000), 2 ** 32 - 1 - rng.integers(0, 2 ** 27, 1500),
                         rng.integers(0, 2 ** 27, 1500), [2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1]])
    n, worst = 0, 0.0
    for w in ws:
        z = ndtri64(int(w), c)
        if z is None:
            continue
        ref = float(ndtri((int(w) + 0.5) * 2.0 ** -32))
        worst = max(worst, abs(z - ref) / max(abs(ref), 1e-300))
        n += 1
    assert n > 0.95 * len(ws) and worst <= 2e-15, (n, worst)
