"""Diagnostic: the fixup kernel's load per workgroup (records, flagged seconds, 64-lane passes)
on one C2 batch.  Needs a diagnostic library: the counters are a patch kept out of the product
source (whose text the PMC records' build stamp hashes):
  d=$(mktemp -d); cp -r include tmhpvsim_amd/csrc "$d"; (cd "$d" && patch -p2 < .../scripts/diag/fix_prof.patch)
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DTMH_FIX_PROF -I "$d/include" \
      -o tmhpvsim_amd/libtmh_fprof.so "$d/csrc/tmh_engine.hip"
then TMHPVSIM_LIB=tmhpvsim_amd/libtmh_fprof.so python scripts/diag/fix_prof.py.  Round 5 (build
b13604d6): 276 workgroups, ~5,500 records of ~1 flagged second each, 67 workgroups with two
record groups in a row (the grid-stride), i.e. the kernel two redo latencies long."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from tmhpvsim_amd import _lib
from tmhpvsim_amd.engine import BatchedSim
from tmhpvsim_amd.params import ModelParams

L = _lib.load()
L.tmh_debug_fix_prof.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
n, secs = 4096, 86400
for chain0 in (1_000_000, 2_000_000):
    sim = BatchedSim(n, "2019-09-05 00:00:00", tz="Europe/Berlin", params=ModelParams(), precision="fp32",
                     chain0=chain0, device="cuda:0", horizon=secs)
    _lib.check(L.tmh_debug_fix_prof(None, 0, 1))
    sim.run(secs, trace=("pv", "meter", "residual"))
    torch.cuda.synchronize()
    buf = np.zeros((65536, 3), dtype=np.uint32)
    _lib.check(L.tmh_debug_fix_prof(buf.ctypes.data_as(C.c_void_p), 65536, 0))
    used = buf[buf[:, 0] > 0]
    rec, fl, ps = used[:, 0], used[:, 1], used[:, 2]
    print(f"chain0 {chain0}: workgroups {len(used)}, records {rec.sum()}, flagged seconds {fl.sum()} "
          f"({fl.sum() / max(1, rec.sum()):.1f} per record); passes per workgroup: "
          + ", ".join(f"{k}: {int((ps == k).sum())}" for k in range(0, int(ps.max()) + 1) if (ps == k).sum())
          + f"; max flagged per workgroup {fl.max()}")
