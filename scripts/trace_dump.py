"""Diagnostic: fp32 C2-style traces of 128 chains x 4 h (keyed, time-parallel) saved to
gpurun_out/trace_<tag>.npz, for bit-for-bit comparisons between library builds
(TMHPVSIM_LIB).  Usage: python scripts/trace_dump.py TAG [--compare OTHER_TAG]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

tag = sys.argv[1]
out = os.path.join(ROOT, "gpurun_out", f"trace_{tag}.npz")
if "--compare" in sys.argv:
    other = np.load(os.path.join(ROOT, "gpurun_out", f"trace_{sys.argv[sys.argv.index('--compare') + 1]}.npz"))
    mine = np.load(out)
    for k in mine.files:
        same = np.array_equal(mine[k], other[k], equal_nan=True)
        print(k, "bit-identical" if same else f"DIFFERS at {int((mine[k] != other[k]).sum())} points")
    sys.exit(0)
import torch  # noqa: E402

from tmhpvsim_amd.engine import BatchedSim  # noqa: E402
from tmhpvsim_amd.params import ModelParams  # noqa: E402

sim = BatchedSim(128, "2019-09-05 08:00:00", tz="Europe/Berlin", params=ModelParams(), precision="fp32",
                 device="cuda:0", horizon=14400, kernel_path="time_parallel")
res = sim.run(14400, trace=("csi", "pv", "meter", "residual"))
torch.cuda.synchronize()
np.savez(out, **{k: v.cpu().numpy() for k, v in res.items()})
print("saved", out)
