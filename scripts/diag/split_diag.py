"""Diagnostic: where the gated schedule's split first batch differs from one tmh_run,
and whether BatchedSim.run over two half-day windows (engine.run_windows) equals one window."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from tmhpvsim_amd.engine import BatchedSim
from tmhpvsim_amd.params import ModelParams
from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults

START, TZ, n, secs = "2019-09-05 00:00:00", "Europe/Berlin", 4096, 86400
F = ("pv", "meter", "residual")


def sim(chain0):
    return BatchedSim(n, START, tz=TZ, params=ModelParams(), precision="fp32", chain0=chain0, device="cuda:0",
                      horizon=secs)


def diff(a, b, tag):
    for f in F:
        x, y = torch.nan_to_num(a[f], nan=-12345.0), torch.nan_to_num(b[f], nan=-12345.0)
        d = (x != y)
        if bool(d.any()):
            idx = d.nonzero()
            rows = idx[:, 0]
            print(tag, f, "differs at", int(d.sum()), "points; rows", int(rows.min()), "-", int(rows.max()),
                  "chains", int(idx[:, 1].unique().numel()), "first", idx[0].tolist(),
                  float(x[tuple(idx[0].tolist())]), float(y[tuple(idx[0].tolist())]))
        else:
            print(tag, f, "equal")


a, b = sim(7000), sim(7000)
ra = a.run(secs, trace=F, window=secs)
rb = b.run(secs, trace=F, window=43200)
torch.cuda.synchronize()
diff(ra, rb, "engine windows 43200 vs 86400:")

s = sim(0)
pipe = BatchPipeline(s, n, secs, pipeline_defaults("c2", "fp32"), lambda k: 3_000_000 + k * n, torch.device("cuda:0"))
pipe.run(0, 1)
pipe.sync()
ref = sim(3_000_000)
rr = ref.run(secs, trace=F)
torch.cuda.synchronize()
diff(pipe.ctxs[0].trace, rr, "split batch vs tmh_run:")
s.state = pipe.ctxs[0].state
print("status equal", bool(np.array_equal(s.status(), ref.status())))
