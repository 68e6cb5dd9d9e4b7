"""Diagnostic: what slows the C2 expansion down in the pipeline?  Times one batch's
expansion kernel (EXPAND_KERNEL, HIP events on its stream) alone and beside each of
the other pipelined pieces launched on a second stream just before it: the next
batch's segment walk, its construction (tmh_init), its plan (tmh_plan: geom_kernel
and the event tables), its draws.  Usage: python scripts/contend.py [--walk-lanes G]"""
import argparse
import ctypes as C
import json
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
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--occupy", action="store_true", help="also beside scripts/micro/libocc*.so (resident dummy waves)")
args = ap.parse_args()
L = _lib.load()
dev = "cuda:0"
n, secs = 4096, 86400
sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", params=ModelParams(), precision="fp32", device=dev,
                 horizon=secs, kernel_path="time_parallel")
if args.walk_lanes:
    _lib.check(L.tmh_set_walk_lanes(sim._eng, args.walk_lanes))
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731


class Ctx:
    def __init__(self, k):
        self.chain0 = k * n
        self.state = torch.zeros(L.tmh_state_bytes(n), dtype=torch.uint8, device=dev)
        self.plan = torch.empty(L.tmh_plan_bytes(secs), dtype=torch.uint8, device=dev)
        self.scratch = torch.empty(L.tmh_scratch_bytes(n, secs), dtype=torch.uint8, device=dev)
        self.trace = {f: torch.empty(secs, n, dtype=torch.float32, device=dev) for f in ("pv", "meter", "residual")}
        self.tr = _lib.Trace(None, None, *(self.trace[f].data_ptr() for f in ("pv", "meter", "residual")), n)


def init(cx, sp):
    _lib.check(L.tmh_init(sim._eng, P(cx.state), cx.chain0, n, None, sp))


def plan(cx, sp):
    _lib.check(L.tmh_plan(sim._eng, 0, secs, P(cx.plan), sp))


def draws(cx, sp):
    _lib.check(L.tmh_walk_part(sim._eng, P(cx.state), cx.chain0, n, 0, secs, P(cx.plan), P(cx.scratch),
                               cx.scratch.numel(), None, 0, _lib.WALK_DRAWS, sp))


def walk(cx, sp):
    _lib.check(L.tmh_walk_part(sim._eng, P(cx.state), cx.chain0, n, 0, secs, P(cx.plan), P(cx.scratch),
                               cx.scratch.numel(), None, 0, _lib.WALK_SEGMENTS, sp))


def expand(cx, sp):
    _lib.check(L.tmh_expand_part(sim._eng, P(cx.state), cx.chain0, n, 0, secs, None, C.byref(cx.tr), None,
                                 P(cx.plan), P(cx.scratch), cx.scratch.numel(), _lib.EXPAND_KERNEL, sp))


def build(cx, sp):
    init(cx, sp)
    plan(cx, sp)
    draws(cx, sp)


a, b = Ctx(0), Ctx(1)
s1, s2, s3 = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
p1, p2, p3 = C.c_void_p(s1.cuda_stream), C.c_void_p(s2.cuda_stream), C.c_void_p(s3.cuda_stream)
build(a, p1)
walk(a, p1)
for _ in range(5):   # warm-up (clocks, code objects): the first variant is not the slow one
    expand(a, p1)
torch.cuda.synchronize()

variants = {
    "alone": None,
    "walk": lambda sp: walk(b, sp),
    "build": lambda sp: build(b, sp),
    "init": lambda sp: init(b, sp),
    "plan": lambda sp: plan(b, sp),
    "draws": lambda sp: draws(b, sp),
    "walk+build": lambda sp: (walk(b, sp), build(Ctx.spare, p3)),
}
Ctx.spare = Ctx(2)
if args.occupy:   # dummy waves, one per SIMD, ~1.5 ms: sleeping with 138 / 70 VGPRs, or fp64 FMA chains
    occ_out = torch.zeros(256, dtype=torch.float64, device=dev)
    for tag, so in (("138", "libocc.so"), ("70", "libocc72.so")):
        lib = C.CDLL(os.path.join(ROOT, "scripts", "micro", so))
        lib.launch_occupy.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        variants[f"sleep{tag}"] = (lambda l: lambda sp: l.launch_occupy(0, 250, 256, sp, P(occ_out)))(lib)
        variants[f"fma{tag}"] = (lambda l: lambda sp: l.launch_occupy(1, 20000, 256, sp, P(occ_out)))(lib)
res = {}
for name, other in variants.items():
    ts, to = [], []
    for r in range(args.reps + 1):
        build(b, p2)          # fresh chains for the walk (outside the timed region)
        torch.cuda.synchronize()
        e0, e1, o0, o1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        if other is not None:
            o0.record(s2)
            other(p2)
            o1.record(s2)
        e0.record(s1)
        expand(a, p1)
        e1.record(s1)
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
            to.append(o0.elapsed_time(o1) if other is not None else 0.0)
    res[name] = (sorted(ts)[len(ts) // 2], sorted(to)[len(to) // 2])
    print(f"{name:11s} expansion {res[name][0]:.3f} ms   other {res[name][1]:.3f} ms", flush=True)
print(json.dumps({k: v[0] for k, v in res.items()}))
