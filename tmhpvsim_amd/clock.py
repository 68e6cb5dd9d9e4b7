"""Wall clock of a batched run -> tmh_clock (include/tmhpvsim.h).

The reference advances its samplers on changes of the LOCAL wall-clock fields
of consecutive times (clearskyindexmodel.py:113-126): naive datetimes in the
reference's own test (tests/test_clearskyindexmodel.py:8), Europe/Berlin-aware
ones inside PVModel (pvmodel.py:45-48).  A run starts at the constructor time
(step 0) and step s is s seconds later in UTC; local time is
local0 + s + (sum of the DST shifts that happened by step s).

The engine's clock holds at most 8 DST shifts (4 years of Europe/Berlin), so a
long or open-ended run (a streamed PVModel, a multi-year sweep) uses a rolling
clock: make_clock(..., step0=s) describes steps s-1 .. s + n_steps - 1 only, with
the shifts before s folded into local0, and BatchedSim installs a new one
(tmh_set_clock) whenever a run goes past the current one.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass

EPOCH = _dt.datetime(1970, 1, 1)
MAX_SHIFTS = 8


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
    step0: int = 0        # first step this clock describes (steps step0 - 1 .. end)
    end: int = 0          # one past the last step it describes

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


def _start(start, tz):
    if not isinstance(start, _dt.datetime):
        import pandas as pd
        start = pd.Timestamp(start).to_pydatetime()
    tzi = _tz(tz) if tz is not None else start.tzinfo
    if tzi is not None and start.tzinfo is None:
        import pandas as pd
        start = pd.Timestamp(start).tz_localize(tzi).to_pydatetime()   # pvmodel.py:39,83 semantics
    return start, tzi


def make_clock(start, n_steps, tz=None, step0=0) -> RunClock:
    """Clock for the consecutive seconds step0 .. step0 + n_steps - 1 of a run from `start`.

    start: naive or aware datetime (or anything pandas.Timestamp accepts).
    tz: None -> naive wall clock (no DST; UTC used for solar geometry);
        name/tzinfo -> a naive start is localised there (like pd.Timestamp(t, tz=...)).
    step0: first step described (a rolling clock); the offset in force at step
        step0 - 1 is folded into local0, so boundary detection at step0 (which
        compares with step0 - 1) stays exact.
    """
    start, tzi = _start(start, tz)
    step0, n_steps = int(step0), int(n_steps)
    end = step0 + n_steps
    if tzi is None:
        t0 = int((start.replace(tzinfo=None) - EPOCH).total_seconds())
        return RunClock(utc0=t0, local0=t0, shifts=[], tz=None, step0=step0, end=end)
    utc0 = int(start.timestamp())

    def offset(s):   # UTC offset in force at step s
        return int(_dt.datetime.fromtimestamp(utc0 + s, tz=tzi).utcoffset().total_seconds())

    base = step0 - 1 if step0 > 0 else 0
    prev = offset(base)
    local0 = utc0 + prev
    shifts = []
    s = base
    while s < end - 1:               # scan hourly, bisect each change to the second
        nxt = min(s + 3600, end - 1)
        o = offset(nxt)
        if o != prev:
            lo, hi = s, nxt
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if offset(mid) == prev:
                    lo = mid
                else:
                    hi = mid
            shifts.append((hi, o - prev))
            prev = o
        s = nxt
    if len(shifts) > MAX_SHIFTS:
        raise ValueError(f"more than {MAX_SHIFTS} DST changes in {n_steps} steps: use a shorter rolling horizon")
    return RunClock(utc0=utc0, local0=local0, shifts=shifts, tz=tzi, step0=step0, end=end)
