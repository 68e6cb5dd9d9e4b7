"""Wall clock of a batched run -> tmh_clock (include/tmhpvsim.h).

The reference advances its samplers on changes of the LOCAL wall-clock fields
of consecutive times (clearskyindexmodel.py:113-126): naive datetimes in the
reference's own test (tests/test_clearskyindexmodel.py:8), Europe/Berlin-aware
ones inside PVModel (pvmodel.py:45-48).  A run starts at the constructor time
(step 0) and step s is s seconds later in UTC; local time is
local0 + s + (sum of the DST shifts that happened by step s).
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass

EPOCH = _dt.datetime(1970, 1, 1)


def _tz(tz):
    if tz is None or isinstance(tz, _dt.tzinfo):
        return tz
    from zoneinfo import ZoneInfo
    return ZoneInfo(tz)


@dataclass
class RunClock:
    utc0: int
    local0: int
    shifts: list          # [(step, delta_seconds)]
    tz: object = None

    def as_struct(self):
        from ._lib import Clock
        ck = Clock()
        ck.utc0, ck.local0, ck.n_shifts = self.utc0, self.local0, len(self.shifts)
        for i, (s, d) in enumerate(self.shifts):
            ck.shift_step[i], ck.shift_delta[i] = s, d
        return ck

    def local_at(self, step):
        return self.local0 + step + sum(d for s, d in self.shifts if step >= s)

    def time_at(self, step):
        """Datetime of `step` as the reference's caller would pass it."""
        if self.tz is None:
            return EPOCH + _dt.timedelta(seconds=self.local0 + step)
        return (_dt.datetime.fromtimestamp(self.utc0 + step, tz=_dt.timezone.utc)).astimezone(self.tz)


def make_clock(start, n_steps, tz=None) -> RunClock:
    """Clock for `n_steps` consecutive seconds from `start`.

    start: naive or aware datetime (or anything pandas.Timestamp accepts).
    tz: None -> naive wall clock (no DST; UTC used for solar geometry);
        name/tzinfo -> a naive start is localised there (like pd.Timestamp(t, tz=...)).
    """
    if not isinstance(start, _dt.datetime):
        import pandas as pd
        start = pd.Timestamp(start).to_pydatetime()
    tzi = _tz(tz) if tz is not None else start.tzinfo
    if tzi is None:
        t0 = int((start.replace(tzinfo=None) - EPOCH).total_seconds())
        return RunClock(utc0=t0, local0=t0, shifts=[], tz=None)
    if start.tzinfo is None:
        import pandas as pd
        start = pd.Timestamp(start).tz_localize(tzi).to_pydatetime()   # pvmodel.py:39,83 semantics
    utc0 = int(start.timestamp())

    def offset(u):
        return int(_dt.datetime.fromtimestamp(u, tz=tzi).utcoffset().total_seconds())

    off0 = offset(utc0)
    local0 = utc0 + off0
    shifts = []
    prev, s = off0, 0
    step_h = 3600
    while s < n_steps:                       # scan hourly, bisect each change to the second
        nxt = min(s + step_h, n_steps - 1) if s < n_steps - 1 else n_steps
        if nxt >= n_steps:
            break
        o = offset(utc0 + nxt)
        if o != prev:
            lo, hi = s, nxt
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if offset(utc0 + mid) == prev:
                    lo = mid
                else:
                    hi = mid
            shifts.append((hi, o - prev))
            prev = o
        s = nxt
    if len(shifts) > 8:
        raise ValueError("more than 8 DST changes in one run: split the run")
    return RunClock(utc0=utc0, local0=local0, shifts=shifts, tz=tzi)
