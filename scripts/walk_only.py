"""Diagnostic: the C2 segment walk alone (construction + draws outside it), REPS times, for
PMC passes on segments_kernel.  Usage: python scripts/walk_only.py [--walk-lanes G] [--reps R]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tmhpvsim_amd import _lib  # noqa: E402
from tmhpvsim_amd.engine import BatchedSim  # noqa: E402
from tmhpvsim_amd.params import ModelParams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--walk-lanes", type=int, default=0)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--chains", type=int, default=4096)
args = ap.parse_args()
L = _lib.load()
dev = "cuda:0"
n, secs = args.chains, 86400
sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", params=ModelParams(), precision="fp32", device=dev,
                 horizon=secs, kernel_path="time_parallel")
if args.walk_lanes:
    _lib.check(L.tmh_set_walk_lanes(sim._eng, args.walk_lanes))
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
state = torch.zeros(L.tmh_state_bytes(n), dtype=torch.uint8, device=dev)
plan = torch.empty(L.tmh_plan_bytes(secs), dtype=torch.uint8, device=dev)
scratch = torch.empty(L.tmh_scratch_bytes(n, secs), dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)
sp = C.c_void_p(s.cuda_stream)
ms = []
for r in range(args.reps):
    _lib.check(L.tmh_init(sim._eng, P(state), r * n, n, None, sp))
    _lib.check(L.tmh_plan(sim._eng, 0, secs, P(plan), sp))
    _lib.check(L.tmh_walk_part(sim._eng, P(state), r * n, n, 0, secs, P(plan), P(scratch), scratch.numel(), None, 0,
                               _lib.WALK_DRAWS, sp))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    _lib.check(L.tmh_walk_part(sim._eng, P(state), r * n, n, 0, secs, P(plan), P(scratch), scratch.numel(), None, 0,
                               _lib.WALK_SEGMENTS, sp))
    e1.record(s)
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
print(f"walk lanes {args.walk_lanes or 'default'}: {' '.join('%.3f' % m for m in ms)} ms")
