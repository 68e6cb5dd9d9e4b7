"""The BASELINE.json configurations on the GPU at (or near) their full size, against
the C oracle:

  * C2 with injected uniforms: 4,096 chains x 86,400 s, fp32 and fp64, the covered
    bit and the stream position bit-exact on every chain (the sequential path,
    which consumes the reference's draw order), CSI / PV / meter / residual of
    every chain and second within the north-star tolerance;
  * stats mode (C3's outputs) on 512 chains x one day: per-chain energies and peak
    residual, and the residual histogram, against the oracle's statistics;
  * a C4 slice: 256 chains x the whole year 2019 in day windows, statistics only,
    no capacity fault, 16 of the chains against the oracle's year.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tmhpvsim_amd.params import RNG_INJECTED, ModelParams

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HIST = dict(n_bins=4096, lo=-300.0, hi=9000.0)


def _sim(n, start, **kw):
    from tmhpvsim_amd.engine import BatchedSim
    return BatchedSim(n, start, tz="Europe/Berlin", device="cuda:0", **kw)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c2_injected_full_size(prec):
    """per-chain injected streams of 92,160 uniforms (Philox key (0x5EED, chain)),
    4,096 chains x 86,400 s from 2019-09-05 00:00 Europe/Berlin, with PV.  Every chain, every
    second: covered bit and stream position bit-exact; CSI, PV, meter and residual within the
    north-star tolerance (fp64 1e-12, fp32 1e-5).  PV is relative to max(|pv|, 1 W) (dawn
    watts); the residual meter - pv to |meter| + |pv| (the fp32 difference of two ~kW
    values cannot hold 1e-5 of |residual| where they cancel)."""
    n, steps, start = 4096, 86400, "2019-09-05 00:00:00"
    inj = O.injected_streams(0x5EED, 0, n, 92160)
    mp = ModelParams(rng_mode=RNG_INJECTED)
    ref = O.run(mp, 0, n, steps, start, tz="Europe/Berlin", inj=inj, n_threads=16,
                outputs=("covered", "pos", "csi", "pv", "meter", "residual"))
    sim = _sim(n, start, params=mp, precision=prec, injected=inj, horizon=steps)
    assert sim.path == "sequential"
    out = sim.run(steps, trace=("covered", "csi", "pv", "meter", "residual"))
    torch.cuda.synchronize()
    st = sim.status()
    np.testing.assert_array_equal(st, ref["status"])
    cov = out["covered"].cpu().numpy()
    np.testing.assert_array_equal(cov, ref["covered"])                     # every chain, every second
    pos = sim.state_field("pos").cpu().numpy().astype(np.int64)
    np.testing.assert_array_equal(pos[st == 0], ref["pos"][-1, st == 0])    # uniforms consumed
    tol = 1e-12 if prec == "fp64" else 1e-5
    worst = dict(csi=0.0, pv=0.0, meter=0.0, residual=0.0)
    for c0 in range(0, n, 512):   # all chains, streamed in blocks of 512 (354 MB per fp64 field)
        cols = np.arange(c0, c0 + 512)
        good = st[cols] == 0
        g = {k: out[k][:, c0:c0 + 512].double().cpu().numpy()[:, good] for k in worst}
        r = {k: ref[k][:, cols[good]] for k in worst}
        assert np.isnan(out["csi"][:, c0:c0 + 512].double().cpu().numpy()[:, ~good]).all()   # faulted chains: NaN
        worst["csi"] = max(worst["csi"], float((np.abs(g["csi"] - r["csi"]) / np.abs(r["csi"])).max(initial=0)))
        worst["pv"] = max(worst["pv"], float((np.abs(g["pv"] - r["pv"]) / np.maximum(np.abs(r["pv"]), 1.0)).max(initial=0)))
        worst["meter"] = max(worst["meter"], float((np.abs(g["meter"] - r["meter"]) / np.abs(r["meter"])).max(initial=0)))
        scale = np.abs(r["meter"]) + np.abs(r["pv"])
        worst["residual"] = max(worst["residual"], float((np.abs(g["residual"] - r["residual"]) / scale).max(initial=0)))
    assert all(v <= tol for v in worst.values()), worst


def _check_stats(sim, ref, prec):
    st = sim.status()
    np.testing.assert_array_equal(st, ref["status"])
    ok = st == 0
    acc = sim.chain_acc.cpu().numpy().T                  # [n, 4]
    tol = 1e-12 if prec == "fp64" else 1e-5
    for k in range(3):                                   # energies: sum pv, sum meter, sum residual
        scale = np.abs(ref["acc"][ok, 1]) + np.abs(ref["acc"][ok, 0])
        assert (np.abs(acc[ok, k] - ref["acc"][ok, k]) / scale).max() <= tol, k
    assert (np.abs(acc[ok, 3] - ref["acc"][ok, 3]) / 9000.0).max() <= tol    # peak residual
    h, rh = sim.hist.cpu().numpy().astype(np.int64), ref["hist"].sum(0).astype(np.int64)
    assert h.sum() == rh.sum()
    # a bin may differ only by seconds whose residual lies within the tolerance of a bin edge
    assert np.abs(h - rh).sum() <= 2 * int(ref["amb"].sum()), (np.abs(h - rh).sum(), int(ref["amb"].sum()))


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_stats_mode_vs_oracle(prec):
    """Stats mode (no trace: the OUT_STATS expansion) on 512 chains x the C2 day."""
    n, steps, start = 512, 86400, "2019-09-05 00:00:00"
    mp = ModelParams(seed=0x5EED + 3)
    sim = _sim(n, start, params=mp, precision=prec, chain0=4096, horizon=steps)
    sim.enable_stats(**HIST)
    sim.run(steps, trace=())
    amb = 1e-6 if prec == "fp64" else 2e-3      # bins: 1e-12 / 1e-5 of ~9,000 W over 2.27 W bins, with margin
    ref = O.run(mp, 4096, n, steps, start, tz="Europe/Berlin", n_threads=16, outputs=(), stats=dict(HIST, amb_eps=amb))
    _check_stats(sim, ref, prec)


def test_c4_year_slice():
    """SURVEY §8d C4 in small: 256 chains x 31,536,000 s (2019, both DST changes, 365 day
    windows pipelined), stats only; no SIGMA / SEGMENT / GUARD overflow anywhere; chains
    0-15 against the oracle's year (fp32 kernel, 1e-5)."""
    n, steps, start = 256, 365 * 86400, "2019-01-01 00:00:00"
    mp = ModelParams()
    sim = _sim(n, start, params=mp, precision="fp32", horizon=steps)
    sim.enable_stats(**HIST)
    sim.run(steps, trace=(), window=86400)
    st = sim.status()
    assert set(np.unique(st)) <= {0, 1}, np.unique(st)    # only the reference's NameError
    ref = O.run(mp, 0, 16, steps, start, tz="Europe/Berlin", n_threads=16, outputs=(), stats=dict(HIST, amb_eps=2e-3))
    np.testing.assert_array_equal(st[:16], ref["status"])
    ok = ref["status"] == 0
    acc = sim.chain_acc[:, :16].cpu().numpy().T
    scale = np.abs(ref["acc"][ok, 1]) + np.abs(ref["acc"][ok, 0])
    for k in range(3):
        assert (np.abs(acc[ok, k] - ref["acc"][ok, k]) / scale).max() <= 1e-5, k
    assert (np.abs(acc[ok, 3] - ref["acc"][ok, 3]) / 9000.0).max() <= 1e-5
    assert int(sim.hist.sum()) == int((st == 0).sum()) * steps   # NameError chains fault at construction
