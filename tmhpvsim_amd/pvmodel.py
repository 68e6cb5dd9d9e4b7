"""Drop-in for tmhpvsim.pvmodel.PVModel (reference: tmhpvsim/pvmodel.py:11-87).

Same construction (`PVModel(time=None)`: the Munich system of pvmodel.py:19-30,
time defaults to now() truncated to seconds, :32-33) and the same lookup
`next(time) -> float` (AC power in W, clipped >= 0 with NaN -> 0, :80-87).
The reference fills a 5,000-second pandas cache with a Python loop over
ClearskyindexModel.next plus pvlib; here the same look-ahead block is one GPU
launch of the fused chain kernel (CSI x clear-sky PV chain).  Naive times are
read as Europe/Berlin wall clock exactly like pd.Timestamp(time, tz=...) (:83).
"""
from __future__ import annotations

import datetime

from .clearskyindexmodel import _StreamedChain, _draw_seed
from .params import ModelParams


class PVModel:
    def __init__(self, time=None, *, seed=None, params: ModelParams | None = None, block=5000, device=None,
                 precision="fp64"):
        import pandas as pd
        p = params or ModelParams()
        p = ModelParams(**{**p.__dict__, "with_pv": True, "seed": _draw_seed() if seed is None else int(seed)})
        self.tz = p.site.tz
        if time is None:
            time = datetime.datetime(*datetime.datetime.now().timetuple()[:6])
        t0 = pd.Timestamp(time, tz=self.tz) if getattr(time, "tzinfo", None) is None else pd.Timestamp(time)
        self._t0 = t0
        self._chain = _StreamedChain(t0.to_pydatetime(), p, self.tz, block, precision, device,
                                     ("pv", "covered"))

    def next(self, time):
        import pandas as pd
        t = pd.Timestamp(time, tz=self.tz) if getattr(time, "tzinfo", None) is None else pd.Timestamp(time)
        k = int((t - self._t0).total_seconds())
        if k < 0:
            raise KeyError(t)
        return self._chain.value(k, "pv")
