"""Diagnostic (GPU): where the fp32 kernel's PV / residual differ from the fp64 oracle.
Prints per case the max errors; dumps every point with a PV error > 1e-6 (relative,
1 W floor) to gpurun_out/diag_fp32.npz."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from tmhpvsim_amd.engine import BatchedSim  # noqa: E402
from tmhpvsim_amd.params import ModelParams, site_grid  # noqa: E402

out = {}
cases = [("sep", "2019-09-05 00:00:00", 86400, 512, None, 0x5EED),
         ("jun", "2019-06-21 00:00:00", 86400, 512, None, 0x5EEE),
         ("dec", "2019-12-21 00:00:00", 86400, 512, None, 0x5EEF),
         ("mar", "2019-03-31 00:00:00", 86400, 256, None, 0x5EF0),
         ("grid", "2019-06-21 02:30:00", 14400, 128, site_grid(16, 8), 0x51E),
         ("grid2", "2019-10-10 05:00:00", 43200, 256, site_grid(16, 16), 0x51F)]
for name, start, steps, n, sites, seed in cases:
    mp = ModelParams(seed=seed)
    ref = O.run(mp, 0, n, steps, start, tz="Europe/Berlin", n_threads=16, sites=sites)
    sim = BatchedSim(n, start, tz="Europe/Berlin", params=mp, precision="fp32", device="cuda:0", horizon=steps,
                     sites=sites)
    r = sim.run(steps)
    g = {k: v.double().cpu().numpy() for k, v in r.items()}
    ok = ref["status"] == 0
    e_pv = np.abs(g["pv"] - ref["pv"]) / np.maximum(np.abs(ref["pv"]), 1.0)
    e_res = np.abs(g["residual"] - ref["residual"]) / np.maximum(np.abs(ref["meter"]) + np.abs(ref["pv"]), 1.0)
    e_csi = np.abs(g["csi"] - ref["csi"]) / np.abs(ref["csi"])
    for e in (e_pv, e_res, e_csi):
        e[:, ~ok] = 0
    idx = np.nonzero(e_pv > 1e-6)
    print(name, "pv max %.3e" % e_pv.max(), "n>1e-5", int((e_pv > 1e-5).sum()), "n>1e-6", len(idx[0]),
          "res max %.3e" % e_res.max(), "csi max %.3e" % np.nanmax(e_csi), flush=True)
    out[name + "_step"], out[name + "_chain"] = idx[0], idx[1]
    for k in ("csi", "pv"):
        out[name + "_g" + k] = g[k][idx]
        out[name + "_r" + k] = ref[k][idx]
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/diag_fp32.npz", **out)
