"""Diagnostic: the stats expansion with and without the residual histogram (C3 shape,
262,144 chains x one day): what the per-workgroup LDS-histogram flush costs."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmhpvsim_amd import _lib  # noqa: E402
from tmhpvsim_amd.engine import BatchedSim  # noqa: E402

n, steps = 262144, 86400
for hist in (True, False, True, False):
    sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", device="cuda:0", horizon=steps)
    sim.enable_stats(histogram=hist)
    L = _lib.load()
    _lib.check(L.tmh_profile_enable(sim._eng, 1))
    sim.run(steps, trace=())
    torch.cuda.synchronize()
    ms, cnt = _lib.profile_read(sim._eng, _lib.K_EXPAND)
    print(f"histogram={hist}: expand {ms / max(cnt, 1):.2f} ms per launch ({cnt} launches)", flush=True)
