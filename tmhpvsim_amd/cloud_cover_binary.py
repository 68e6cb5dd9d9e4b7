"""Drop-in for tmhpvsim.cloud_cover_binary (reference: tmhpvsim/cloud_cover_binary.py).

Host-side helpers with the reference's names, signatures and random-number
consumption (numpy's global RandomState, as the reference draws), for callers
that use them directly.  They are not on the engine's path: inside the batched
simulator the same process runs per chain on the GPU (tmh_engine.hip
`segments_kernel`, `next_cloud`), keyed by Philox instead of the global stream.
Checked draw for draw against the reference (tests/test_shims_cpu.py,
fixture tests/golden/shims.npz).
"""
from __future__ import annotations

import logging

import numpy as np

logger = logging.getLogger(__name__)

# cloud length law (Wood & Field 2011): P(x) ~ x^-1.66 on [100 m, 1000 km]
# (cloud_cover_binary.py:35-38); the inverse CDF is (alpha + delta u)^(1/(1-beta))
_BETA = 1.66
_XMIN, _XMAX = 0.1e3, 1e6
_ALPHA = _XMAX ** (1 - _BETA)
_DELTA = _XMIN ** (1 - _BETA) - _ALPHA


def random_windspeed(size=None):
    """Wind speed in m/s ~ Gamma(2.69, 2.14) (cloud_cover_binary.py:5-23; Mathiesen et al. 2013)."""
    return np.random.gamma(2.69, 2.14)


def random_cloudlength_in_s(windspeed, shape=(1,)):
    """Duration in s of `shape` clouds passing at `windspeed` m/s (cloud_cover_binary.py:25-40)."""
    return (_ALPHA + _DELTA * np.random.random(shape)) ** (1 / (1 - _BETA)) / windspeed


class CloudCoverBinary:
    """Per-second cloud (1) / clear (0) sequence whose hourly mean follows the
    hourly cloud cover (cloud_cover_binary.py:42-117).

    State: the current cloud and clear lengths, the second counter within them,
    and sigma_cloud / sigma_clear, the cumulated cloud and clear lengths of the
    latest segments (newest first), which next_cloud extends so the clouded
    share of the last ~hour matches the cover.
    """

    def __init__(self, hourly_cloudcover, windspeed=None):
        self.update_parameters(hourly_cloudcover, windspeed)
        self.reset_sigma()
        self.next_cloud()
        # a random position inside the first segment (:68; the lengths are shape-(1,) arrays there)
        self.sec = int(np.ravel((self.cloud_length + self.clear_length) * np.random.random())[0])

    def update_parameters(self, hourly_cloudcover, windspeed=None):
        """Cover capped at 0.95 (:70-74).  The reference's windspeed=None branch calls an
        undefined name; here it draws a wind speed, as that branch intends."""
        self.hourly_cloudcover = min(hourly_cloudcover, 0.95)
        self.windspeed = random_windspeed() if windspeed is None else windspeed

    def reset_sigma(self):
        """int(12 h) segments of 300 s cloud each, clear time in proportion (:76-78)."""
        k = int(self.hourly_cloudcover * 12)
        self.sigma_cloud = 300.0 * np.arange(1, k + 1, dtype=np.float64)
        self.sigma_clear = (1 / self.hourly_cloudcover - 1) * self.sigma_cloud

    def _candidate(self):
        """One try: a new cloud length, the extended cumulated lengths and which
        prefixes are admissible (clear time grows, whole span under 90 min)."""
        cl = random_cloudlength_in_s(self.windspeed)
        cum_cloud = self.sigma_cloud + cl
        cum_clear = cum_cloud * (1 / self.hourly_cloudcover - 1)
        span = cum_cloud + cum_clear
        ok = ((cum_clear - self.sigma_clear) > 0) & (span < 5400)
        return cl, cum_cloud, cum_clear, span, ok

    def next_cloud(self, recurse=False):
        """Draw the next cloud + clear segment (:80-107): up to 20 cloud lengths until
        one admits a prefix; the prefix whose span is nearest one hour wins (the
        first on ties).  20 failures reset sigma and retry once, then assert."""
        for _ in range(20):
            cl, cum_cloud, cum_clear, span, ok = self._candidate()
            if ok.any():
                break
        else:
            assert not recurse
            logger.error("20 random cloud lengths rejected at windspeed %s and cloud cover %s; "
                         "resetting sigma_cloud, sigma_clear", self.windspeed, self.hourly_cloudcover)
            self.reset_sigma()
            return self.next_cloud(recurse=True)
        idx = np.flatnonzero(ok)
        last = idx[np.argmin(np.abs(span[idx] - 3600))]
        self.cloud_length = cl
        self.clear_length = cum_clear[last] - self.sigma_clear[last]
        self.sigma_cloud = np.concatenate([cl, cum_cloud[:last + 1]])
        self.sigma_clear = np.concatenate([np.atleast_1d(self.clear_length), cum_clear[:last + 1]])
        self.sec = 0
        return self.cloud_length, self.clear_length

    def __iter__(self):
        return self

    def __next__(self):
        """1 while inside the cloud, 0 in the clear part, then the next segment (:109-117)."""
        while True:
            self.sec += 1
            if self.sec < self.cloud_length:
                return 1
            if self.sec < self.cloud_length + self.clear_length:
                return 0
            self.next_cloud()
