"""Statistical equivalence of the keyed (Philox) mode with the reference's own
seeded mode, on the CPU: the C oracle (the same keyed contract the HIP kernels
follow bit for bit, tests/test_gpu_parity.py) against the reference's seeded runs
in tests/golden/stats_seeded.npz (tests/golden/make_stats.py).

North star: "in independent-seed mode, statistical equivalence is shown by
transition-count and KS tests".  Tested quantities (Munich, 2019-09-05, one day
at 1 s, different random streams on each side):
  * per chain-day: mean and median cloud and clear segment lengths
    (cloud_cover_binary.py:80-117) - KS;
  * clouds per chain-day, i.e. 0 -> 1 transitions of the covered bit - KS;
  * covered fraction per chain-day - KS;
  * the clear-sky index at second 30 of every minute (clearskyindexmodel.py:128-160) - KS;
  * the hourly cloud-cover draw (cloud_cover_hourly.py:309-316, the faithful
    fresh-generator quirk) against the oracle's AL quantile - KS, and its atom at 1.0.
"""
import numpy as np
import pytest

from stats_util import P_MIN, SEGMENT_KEYS, ks, load_reference, summarize, summarize_trace

N_CHAINS = 512


@pytest.fixture(scope="module")
def ref():
    r = load_reference()
    r["summary"] = summarize(r["first"], r["runs"])
    return r


@pytest.fixture(scope="module")
def oracle_run():
    from oracle import oracle as O
    from tmhpvsim_amd.params import ModelParams
    return O.run(ModelParams(with_pv=False), 10_000, N_CHAINS, 86400, "2019-09-05 00:00:00", tz="Europe/Berlin",
                 n_threads=8, outputs=("csi", "covered"))


def test_segment_and_transition_statistics(ref, oracle_run):
    assert (oracle_run["status"] == 0).all()
    got = summarize_trace(oracle_run["covered"])
    exp = ref["summary"]
    for key in SEGMENT_KEYS:
        p = ks(got[key], exp[key])
        assert p > P_MIN, f"{key}: KS p = {p:.2e} (keyed {np.mean(got[key]):.4g} vs reference {np.mean(exp[key]):.4g})"


def csi_chain_stats(csi_min):
    """Per-chain statistics of the minute-sampled CSI [chains, 1440]: the samples of
    one chain share its daily / hourly draws and the cloudy-hour value frozen at
    construction (clearskyindexmodel.py:105-107), so only chain-level values are
    independent samples."""
    return dict(mean=csi_min.mean(1), std=csi_min.std(1), noon=csi_min[:, 720], q10=np.quantile(csi_min, 0.1, 1))


def test_clear_sky_index_distribution(ref, oracle_run):
    got_min = oracle_run["csi"][30::60].T
    assert (oracle_run["csi"] > 0).all() and (oracle_run["csi"] < 2).all()   # tests/test_clearskyindexmodel.py:13
    got, exp = csi_chain_stats(got_min), csi_chain_stats(ref["csi_min"])
    for key in got:
        p = ks(got[key], exp[key])
        assert p > P_MIN, f"csi {key}: KS p = {p:.2e} ({np.mean(got[key]):.4g} vs {np.mean(exp[key]):.4g})"


def test_the_tests_reject_a_different_model(ref):
    """Negative control: the same statistics separate the reference from the
    persistent hourly Markov chain (get_cloud_cover as a chain, markov mode)."""
    from oracle import oracle as O
    from tmhpvsim_amd.params import CC_MARKOV, ModelParams
    r = O.run(ModelParams(with_pv=False, cc_mode=CC_MARKOV), 20_000, 256, 86400, "2019-09-05 00:00:00",
              tz="Europe/Berlin", n_threads=8, outputs=("covered",))
    ok = r["status"] == 0
    got = summarize_trace(r["covered"][:, ok])
    assert min(ks(got[k], ref["summary"][k]) for k in SEGMENT_KEYS) < 1e-6


def test_hourly_cloud_cover_draw(ref):
    """The reference's hourly draws vs the restated mapping clip(1 + AL(u) scale + loc)."""
    from oracle import oracle as O
    from tmhpvsim_amd.params import SHAPES
    loc, scale, kappa, _ = SHAPES[5]
    u = (np.arange(200_000) + 0.5) / 200_000
    mine = np.clip(1.0 + (O.al_ppf(u, kappa) * scale + loc), 0.0, 1.0)
    exp = ref["cc_hourly"]
    at_one = np.mean(exp == 1.0)
    assert abs(at_one - 1 / (1 + kappa ** 2)) < 4 * np.sqrt(at_one * (1 - at_one) / exp.size)
    p = ks(mine, exp)
    assert p > P_MIN, f"hourly cc KS p = {p:.2e}"
