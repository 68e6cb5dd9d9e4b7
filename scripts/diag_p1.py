"""Diagnostic (never the product): cycles per section of the P1 segment walk from a
-DTMH_DIAG_P1 build (scripts/diag_variants.sh builds libtmh_p1diag.so)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TMHPVSIM_LIB"] = os.path.join(ROOT, "tmhpvsim_amd", "libtmh_p1diag.so")
from tmhpvsim_amd import _lib  # noqa: E402
from tmhpvsim_amd.engine import BatchedSim  # noqa: E402

n = 4096
sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", device="cuda:0", horizon=86400)
L = _lib.load()
for rep in range(2):
    sim2 = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", device="cuda:0", horizon=86400)
    sim2.run(86400, trace=("pv",))
    torch.cuda.synchronize()
nw = (n + 3) // 4
out = np.zeros(nw * 8, dtype=np.uint64)
L.tmh_diag_p1(out.ctypes.data_as(C.c_void_p), C.c_uint32(nw * 8))
d = out.reshape(nw, 8).astype(np.float64)
names = ["events+fractions", "h/ws/f/cand", "tries(scan+min)", "fault checks", "last+shift", "state+record",
         "loop top", "iterations"]
it = d[:, 7]
print("waves", nw, "iterations mean %.0f max %.0f" % (it.mean(), it.max()))
tot = d[:, :7].sum(1)
print("cycles/wave mean %.3g max %.3g" % (tot.mean(), tot.max()))
for i in range(7):
    print(f"{names[i]:18s} cycles/iter mean {np.mean(d[:, i] / np.maximum(it, 1)):8.1f}")
