"""Drop-in for tmhpvsim.clearskyindexmodel (reference: tmhpvsim/clearskyindexmodel.py).

`ClearskyindexModel(time).next(time) -> float` keeps the reference's
per-second, stateful calling convention (clearskyindexmodel.py:57,128): it must
be called for consecutive seconds starting at the constructor time (the
reference advances its samplers on wall-clock field changes, :113-126; the
engine runs the same schedule on the GPU).  Values are produced in look-ahead
blocks by the HIP engine (tmhpvsim_amd.engine.BatchedSim, one chain), fp64.

Randomness: the reference draws from numpy's global RandomState; here each
model is one keyed-Philox chain whose seed is taken from that same global
state when not given, so `np.random.seed(s)` still makes runs reproducible.

Faults keep the reference's exception types: a constructor whose initial cloud
cover falls in [0.75, 0.875) raises NameError (:72-80); a CloudCoverBinary
that cannot place a cloud raises AssertionError (cloud_cover_binary.py:90-98)
from the next() call of that second.
"""
from __future__ import annotations

import datetime as _dt
from collections import namedtuple

import numpy as np

from .params import ModelParams

Time = namedtuple("Time", ["time", "day_fraction", "hour_fraction", "min_fraction"])


class InterpolatedSampler:
    """Interpolation between two successive samples (clearskyindexmodel.py:12-40).

    Host-side helper with the reference's exact semantics; the batched engine
    keeps the six samplers of every chain as SoA (before, after) pairs on the GPU.
    """

    def __init__(self, next_sample_func):
        self.next_sample_func = next_sample_func
        self.before = next_sample_func()
        self.after = next_sample_func()

    def __next__(self):
        self.before = self.after
        self.after = self.next_sample_func()
        return self.before

    def interpolate(self, fraction):
        return fraction * self.after + (1 - fraction) * self.before


def _utc_seconds(t):
    if t.tzinfo is None:
        return (t - _dt.datetime(1970, 1, 1)).total_seconds()
    return t.timestamp()


def _draw_seed():
    return int(np.random.randint(0, 2 ** 31 - 1)) << 20 | int(np.random.randint(0, 2 ** 20))


class _StreamedChain:
    """One chain on the GPU, consumed second by second from look-ahead blocks.

    The engine's clock rolls forward with the blocks (BatchedSim installs a new
    DST table when a block runs past the current one), so a stream has no end.
    The current and the previous block stay readable, like the tail of the
    reference's cache that populate_cache keeps (pvmodel.py:39-43)."""

    def __init__(self, time, params, tz, block, precision, device, fields):
        from .engine import BatchedSim
        self._t0 = time
        self._u0 = _utc_seconds(time)
        self._block = int(block)
        self._fields = fields
        self.sim = BatchedSim(1, time, tz=tz, params=params, precision=precision, device=device,
                              horizon=max(self._block, 400 * 86400))
        st = int(self.sim.status()[0])
        if st == 1:
            raise NameError("name 'x' is not defined")        # clearskyindexmodel.py:80
        if st == 2:
            raise AssertionError()                            # cloud_cover_binary.py:91
        self._bufs = []       # [(first step, {field: np.ndarray})], at most two blocks
        self._hi = 0          # one past the last step computed

    def _fill(self, upto):
        while self._hi <= upto:
            out = self.sim.run(self._block, trace=self._fields)
            self._bufs = self._bufs[-1:] + [(self._hi, {k: v[:, 0].cpu().numpy() for k, v in out.items()})]
            self._hi += self._block

    def value(self, step, field):
        self._fill(step)
        for lo, buf in self._bufs:
            if lo <= step < lo + self._block:
                i = step - lo
                cov = buf.get("covered")
                if cov is not None and cov[i] == 255:
                    raise AssertionError()                     # CloudCoverBinary could not place a cloud
                return float(buf[field][i])
        raise KeyError(f"second {step} is before the look-ahead window (only forward access is supported)")


class ClearskyindexModel:
    """Clear-sky-index model (Bright et al. 2015, streaming), one chain on the GPU.

    Parameters beyond the reference signature are keyword-only:
    seed (default: drawn from numpy's global RandomState), params
    (tmhpvsim_amd.params.ModelParams), block (look-ahead seconds per GPU
    launch), device, precision ("fp64" default).
    """

    time = None

    def __init__(self, time, *, seed=None, params: ModelParams | None = None, block=3600, device=None,
                 precision="fp64"):
        p = params or ModelParams()
        p = ModelParams(**{**p.__dict__, "with_pv": False, "seed": _draw_seed() if seed is None else int(seed)})
        self._set_time(time)
        tz = time.tzinfo
        self._chain = _StreamedChain(time, p, tz, block, precision, device, ("csi", "covered"))
        self._k = 0

    def _set_time(self, time):
        min_fraction = time.second / 60
        hour_fraction = (time.minute + min_fraction) / 60
        day_fraction = (time.hour + hour_fraction) / 24
        self.time = Time(time, day_fraction, hour_fraction, min_fraction)

    def next(self, time):
        """Clear-sky index for `time` (the next consecutive second)."""
        k = int(round(_utc_seconds(time) - self._chain._u0))
        if k != self._k:
            raise ValueError(f"ClearskyindexModel.next must be called for consecutive seconds: expected "
                             f"{self._k} s after the constructor time, got {k} s")
        self._set_time(time)
        v = self._chain.value(k, "csi")
        self._k += 1
        return v
