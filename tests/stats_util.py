"""Statistics of covered-bit sequences and CSI samples shared by the statistical
equivalence tests (tests/test_stats_cpu.py, tests/test_gpu_stats.py).

The fixture tests/golden/stats_seeded.npz holds the reference's own seeded-mode
runs (tests/golden/make_stats.py): covered bits as run lengths, the CSI of
second 30 of every minute and the hourly cloud-cover draws.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# p-value floor of every two-sample test: the samples are deterministic (keyed
# seeds, a committed fixture), so a pass or a fail is reproducible; 1e-4 keeps a
# true match from failing by chance across the handful of tests.
P_MIN = 1e-4


def load_reference():
    d = np.load(os.path.join(HERE, "golden", "stats_seeded.npz"), allow_pickle=False)
    first, nrun, runs = d["first"], d["nrun"], d["runs"]
    per_chain = np.split(runs, np.cumsum(nrun)[:-1])
    return dict(first=first, runs=per_chain, csi_min=d["csi_min"], cc_hourly=d["cc_hourly"],
                n_steps=int(d["n_steps"]))


def runs_of(cov_chain):
    """(first bit, run lengths) of one chain's covered sequence."""
    c = np.asarray(cov_chain).astype(np.int8)
    change = np.flatnonzero(np.diff(c)) + 1
    starts = np.r_[0, change]
    return int(c[0]), np.diff(np.r_[starts, c.size])


def summarize(firsts, runs_per_chain):
    """Per-chain statistics of the covered sequence, one value per chain-day:
    mean and median length of the interior cloud (covered = 1) and clear (0)
    segments (the two edge runs are censored by the window and dropped), clouds
    per day (0 -> 1 transitions) and the covered fraction.

    Only chain-level values are independent samples: the segments of one chain
    share its daily wind speed and hourly cloud cover (cloud_cover_binary.py:25-40,
    70-74), so a KS test on pooled segments would overstate its confidence."""
    out = {k: [] for k in ("cloud_mean", "cloud_median", "clear_mean", "clear_median", "n_on", "frac")}
    for f, r in zip(firsts, runs_per_chain):
        bits = (np.arange(r.size) + (1 - int(f))) % 2 == 0   # covered value of run i
        inner = np.zeros(r.size, dtype=bool)
        inner[1:-1] = True
        cl, cr = r[inner & bits], r[inner & ~bits]
        out["cloud_mean"].append(cl.mean() if cl.size else np.nan)
        out["cloud_median"].append(np.median(cl) if cl.size else np.nan)
        out["clear_mean"].append(cr.mean() if cr.size else np.nan)
        out["clear_median"].append(np.median(cr) if cr.size else np.nan)
        out["n_on"].append(int(np.sum(bits[1:] & ~bits[:-1])))
        out["frac"].append(r[bits].sum() / r.sum())
    return {k: np.asarray(v, dtype=np.float64) for k, v in out.items()}


def summarize_trace(cov):
    """summarize() of a time-major covered trace [steps, chains] (uint8 0/1)."""
    firsts, runs = [], []
    for c in range(cov.shape[1]):
        f, r = runs_of(cov[:, c])
        firsts.append(f)
        runs.append(r)
    return summarize(firsts, runs)


def ks(a, b):
    from scipy import stats
    a, b = np.asarray(a), np.asarray(b)
    return stats.ks_2samp(a[np.isfinite(a)], b[np.isfinite(b)]).pvalue


SEGMENT_KEYS = ("cloud_mean", "cloud_median", "clear_mean", "clear_median", "n_on", "frac")
