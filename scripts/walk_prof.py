"""Diagnostic: where the segment walk's time goes, per loop section (s_memtime stamps).

Needs the diagnostic build: scripts/build_variant.sh is not used; build with
  hipcc ... -DTMH_WALK_PROF -o tmhpvsim_amd/libtmh_wprof.so tmhpvsim_amd/csrc/tmh_engine.hip
and run with TMHPVSIM_LIB=tmhpvsim_amd/libtmh_wprof.so python scripts/walk_prof.py [--chains N ...].
Prints, per configuration: the walk's time (HIP events), iterations of the slowest wave and the
mean, and cycles per iteration of each section (the busiest lane of each wave, which takes part in
every iteration), for the slowest wave and weighted over all waves."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tmhpvsim_amd import _lib  # noqa: E402
from tmhpvsim_amd.engine import BatchedSim  # noqa: E402
from tmhpvsim_amd.params import ModelParams  # noqa: E402

SECTIONS = ["top (ballot, Lmax)", "events+fractions+h/ws/f+cand", "tries (scan+argmin)", "faults+nclr+shift",
            "state+record", "-"]
ap = argparse.ArgumentParser()
ap.add_argument("--chains", type=int, nargs="+", default=[4096, 2048])
ap.add_argument("--lanes", type=int, nargs="+", default=[16])
ap.add_argument("--order", type=int, nargs="+", default=[1, 0])
ap.add_argument("--days", type=int, default=1)
args = ap.parse_args()
L = _lib.load()
assert hasattr(L, "tmh_debug_walk_prof"), "needs the -DTMH_WALK_PROF build (TMHPVSIM_LIB)"
L.tmh_debug_walk_prof.argtypes = [C.c_void_p, C.c_uint32]
dev = "cuda:0"
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
for n in args.chains:
    secs = 86400 * args.days
    sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", params=ModelParams(), precision="fp32", device=dev,
                     horizon=secs, kernel_path="time_parallel")
    state = torch.zeros(L.tmh_state_bytes(n), dtype=torch.uint8, device=dev)
    plan = torch.empty(L.tmh_plan_bytes(secs), dtype=torch.uint8, device=dev)
    scratch = torch.empty(L.tmh_scratch_bytes(n, secs), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    sp = C.c_void_p(s.cuda_stream)
    for lanes in args.lanes:
        for order in args.order:
            _lib.check(L.tmh_set_walk_lanes(sim._eng, lanes))
            _lib.check(L.tmh_set_walk_order(sim._eng, order))
            ms = []
            for r in range(3):
                _lib.check(L.tmh_init(sim._eng, P(state), r * n, n, None, sp))
                _lib.check(L.tmh_plan(sim._eng, 0, secs, P(plan), sp))
                _lib.check(L.tmh_walk_part(sim._eng, P(state), r * n, n, 0, secs, P(plan), P(scratch),
                                           scratch.numel(), None, 0, _lib.WALK_DRAWS, sp))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                _lib.check(L.tmh_walk_part(sim._eng, P(state), r * n, n, 0, secs, P(plan), P(scratch),
                                           scratch.numel(), None, 0, _lib.WALK_SEGMENTS, sp))
                e1.record(s)
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            threads = ((n + 15) // 16) * 16 * lanes
            buf = np.zeros((threads, 8), dtype=np.uint64)
            _lib.check(L.tmh_debug_walk_prof(buf.ctypes.data_as(C.c_void_p), threads))
            w = buf.reshape(-1, 64, 8)
            best = np.argmax(w[:, :, 6], axis=1)                 # the busiest lane of each wave
            rows = w[np.arange(w.shape[0]), best].astype(np.float64)
            it = rows[:, 6]
            slow = int(np.argmax(rows[:, 7]))
            print(f"chains {n} lanes {lanes} order {order} days {args.days}: walk {' '.join('%.3f' % m for m in ms)} ms; "
                  f"waves {w.shape[0]}, iterations mean {it.mean():.0f} max {it.max():.0f}; slowest wave "
                  f"{rows[slow, 7]:.3g} cycles, {rows[slow, 7] / max(1, rows[slow, 6]):.0f} per iteration")
            for i, name in enumerate(SECTIONS[:5]):
                print(f"   {name:32s} slowest {rows[slow, i] / max(1, rows[slow, 6]):8.1f}   all "
                      f"{rows[:, i].sum() / max(1, it.sum()):8.1f} cycles/iter")
