"""Debug: DPP probes + first divergence between time-parallel and sequential paths."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tmhpvsim_amd.engine import BatchedSim, probe
from tmhpvsim_amd.params import ModelParams

rng = np.random.default_rng(1)
x = rng.random(128)
x[[5, 40]] = 0.01; x[77] = 0.005; x[100] = 0.005
km = probe(5, 0.0, x)
print("argmin wave0 got", km[0], "want", np.argmin(x[:64]), "| wave1 got", km[64], "want", 64 + np.argmin(x[64:]) - 64)
sh = probe(6, -7.0, x)
print("wave_shr lane0", sh[0], "lanes1..3", sh[1:4], "want", x[0:3], "| lane64", sh[64])
rl = probe(7, 0.0, x)
print("readlane63", rl[0], x[63], rl[64], x[127])

start, n, steps = "2019-06-21 03:00:00", 64, 7200
a = BatchedSim(n, start, precision="fp64", horizon=steps, kernel_path="time_parallel")
b = BatchedSim(n, start, precision="fp64", horizon=steps, kernel_path="sequential")
ra, rb = a.run(steps, trace=("covered", "csi")), b.run(steps, trace=("covered", "csi"))
ca, cb = ra["covered"].cpu().numpy(), rb["covered"].cpu().numpy()
bad = np.nonzero((ca != cb).any(0))[0]
print("chains differing:", len(bad), bad[:10])
for c in bad[:4]:
    j = np.nonzero(ca[:, c] != cb[:, c])[0][0]
    print(f" chain {c}: first diff step {j}; tp {ca[max(0,j-3):j+3, c]} seq {cb[max(0,j-3):j+3, c]}")
print("L tp", a.state_field("sigma_len").cpu().numpy()[:8], "seq", b.state_field("sigma_len").cpu().numpy()[:8])
print("cl tp", a.state_field("cloud_length").cpu().numpy()[:4], "seq", b.state_field("cloud_length").cpu().numpy()[:4])
