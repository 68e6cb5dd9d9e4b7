"""The driver's secondary configurations as the bench runs them, against the C oracle.

bench.py's C4 and C5 lines run BatchPipeline with pipeline_defaults("c4") /
pipeline_defaults("c5"): C4 in 30-day windows (a window's segment capacity, overflow
pool, fixed-point unit and plan all follow its length), C5 with markov cloud cover,
per-site tables, per-site PV geometry and windows compacted to the live chains.
These tests run exactly those schedules and compare their per-chain statistics and
histograms with the oracle's (tmh_oracle.c), not with another GPU run:

  * C4: the year 2019 through the pipeline at 256 chains (day and 30-day windows), at
    the N = 8 shard (2,048 chains, 16 walk lanes) and at the N = 1 batch (16,384
    chains, 8 walk lanes, bench.py's choice above 8,192): chains spread over each
    batch (first, middle and last walk rows / workgroups) against the oracle's year,
    fp32 within 1e-5; and 64 chains x 60 days in 30-day windows (across the spring DST
    change) with every chain and the whole histogram against the oracle;
  * C5: 512 sites x 3 days (markov, per-site tables and sites, compacted windows, the
    group schedule, eight contexts at this batch size), fp32 (1e-5) and fp64 (1e-12): every chain's
    energies and peak -- the faulted chains' seconds before their fault included --,
    status, and the histogram, whose count equals the oracle's chain-seconds, so
    energies and histogram cover the same chain-seconds (dist.chain_totals).

Reference: /root/reference/tmhpvsim/pvsim.py:80-83 (the residual the statistics
reduce), cloud_cover_hourly.py:290-316 (markov), cloud_cover_binary.py:90-98 (the
AssertionError that ends markov chains).
"""
import functools

import numpy as np
import pytest

from oracle import oracle as O
from tmhpvsim_amd.params import CC_MARKOV, ModelParams, site_grid, site_shape_tables

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TZ = "Europe/Berlin"
HIST = dict(n_bins=4096, lo=-300.0, hi=9000.0)
YEAR, Y0 = 365 * 86400, "2019-01-01 00:00:00"
AMB = {"fp32": 2e-3, "fp64": 1e-6}     # bin-edge tolerance (1e-5 / 1e-12 of ~9 kW over 2.27 W bins, with margin)
TOL = {"fp32": 1e-5, "fp64": 1e-12}


def _pipeline(workload, n, secs, start, prec="fp32", chain0=0, lanes=0, mp=None, window=None, batches=None, **kw):
    """BatchPipeline with bench.py's schedule for `workload` (pipeline_defaults, the batch
    size of one GPU) and bench.py's walk-lane choice; every context runs one batch (batch k
    = chains chain0 + k n ...): returns the pipeline after sync."""
    from tmhpvsim_amd import _lib
    from tmhpvsim_amd.engine import BatchedSim
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    cfg = pipeline_defaults(workload, prec, chains=n, seconds=secs, window=window)
    sim = BatchedSim(n, start, tz=TZ, params=mp or ModelParams(), precision=prec, chain0=chain0, device="cuda:0",
                     horizon=secs, **kw)
    if lanes:
        _lib.check(sim.L.tmh_set_walk_lanes(sim._eng, lanes))
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: chain0 + k * n, torch.device("cuda:0"))
    pipe.run(0, batches or len(pipe.ctxs))
    pipe.sync()
    return pipe


def _check_chains(acc, st, ref, prec, label):
    """per-chain energies (relative to |sum meter| + |sum pv|) and peak residual (relative
    to 9 kW) of every chain, a faulted chain's seconds before its fault included"""
    np.testing.assert_array_equal(st, ref["status"], err_msg=label)
    tol = TOL[prec]
    racc = ref["acc"]
    scale = np.maximum(np.abs(racc[:, 1]) + np.abs(racc[:, 0]), 1.0)
    for k in range(3):
        err = np.abs(acc[:, k] - racc[:, k]) / scale
        assert err.max() <= tol, (label, k, float(err.max()))
    has = np.isfinite(racc[:, 3])
    np.testing.assert_array_equal(np.isfinite(acc[:, 3]), has, err_msg=label)
    assert (np.abs(acc[has, 3] - racc[has, 3]) / 9000.0).max(initial=0.0) <= tol, label


def _check_hist(hist, ref, prec, label):
    h, rh = hist.cpu().numpy().astype(np.int64), ref["hist"].sum(0).astype(np.int64)
    assert h.sum() == rh.sum(), (label, int(h.sum()), int(rh.sum()))        # the same chain-seconds
    # a bin may differ only by seconds whose residual lies within the tolerance of a bin edge
    assert np.abs(h - rh).sum() <= 2 * int(ref["amb"].sum()), (label, int(np.abs(h - rh).sum()), int(ref["amb"].sum()))


# ------------------------------------------------------------------ C4
# chains compared per configuration: (batch size, walk lanes) -> local chain indices
C4_CONFIGS = {(256, 0): np.arange(16), (2048, 16): np.r_[0:4, 1020:1024, 2044:2048],
              (16384, 8): np.r_[0:4, 8190:8194, 16380:16384]}


@functools.lru_cache(maxsize=1)
def _c4_oracle_year():
    """one oracle year over the union of the compared global chains (chain0 = 0 batches)"""
    ids = np.unique(np.concatenate(list(C4_CONFIGS.values()))).astype(np.uint64)
    ref = O.run(ModelParams(), 0, len(ids), YEAR, Y0, tz=TZ, n_threads=16, outputs=(),
                stats=dict(HIST, amb_eps=AMB["fp32"]), chain_ids=ids)
    return ids, ref


def _c4_ref(local):
    ids, ref = _c4_oracle_year()
    pos = np.searchsorted(ids, local.astype(np.uint64))
    return {"status": ref["status"][pos], "acc": ref["acc"][pos]}


@pytest.mark.parametrize("window", [86400, 30 * 86400])
def test_c4_year_pipeline_256_vs_oracle(window):
    """256 chains x the year 2019 through BatchPipeline with pipeline_defaults("c4") at
    day and at 30-day windows (bench.py's C4 default): no capacity fault anywhere, and
    chains 0-15 against the oracle's year, fp32 within 1e-5."""
    n = 256
    pipe = _pipeline("c4", n, YEAR, Y0, window=window, batches=2)
    assert pipe.cfg.window == window and pipe.cfg.mode == "stats" and pipe.nwin == -(-YEAR // window)
    cx = pipe.ctxs[0]
    pipe.sim.state = cx.state
    st = pipe.sim.status()
    assert set(np.unique(st)) <= {0, 1}, np.unique(st)     # only the reference's NameError at construction
    loc = C4_CONFIGS[(256, 0)]
    _check_chains(cx.acc[:, loc].cpu().numpy().T, st[loc], _c4_ref(loc), "fp32", f"c4 256 w={window}")
    assert int(cx.hist.sum()) == int((st == 0).sum()) * YEAR


@pytest.mark.parametrize("n,lanes", [(2048, 16), (16384, 8)])
def test_c4_year_pipeline_shard_vs_oracle(n, lanes):
    """bench.py's C4 batches as the driver runs them: the N = 8 shard (2,048 chains, 16
    walk lanes) and the N = 1 batch (16,384 chains, 8 walk lanes), 30-day windows,
    every context in flight (pipeline_defaults("c4", chains=n)); chains at the start,
    middle and end of context 0's batch against the oracle's year."""
    pipe = _pipeline("c4", n, YEAR, Y0, lanes=lanes)
    assert pipe.cfg.window == 30 * 86400 and pipe.nwin == 13
    cx = pipe.ctxs[0]
    pipe.sim.state = cx.state
    st = pipe.sim.status()
    loc = C4_CONFIGS[(n, lanes)]
    acc = cx.acc.cpu().numpy().T
    _check_chains(acc[loc], st[loc], _c4_ref(loc), "fp32", f"c4 {n}/{lanes}")
    # a chain-year in faithful mode can end in the reference's AssertionError (20 + 20 rejected
    # cloud lengths, cloud_cover_binary.py:90-98: 0.02 % of the N = 1 batch's chain-years);
    # every chain faulting during the year is checked against the oracle too
    odd = np.flatnonzero(~np.isin(st, (0, 1)))
    assert set(np.unique(st[odd])) <= {2} and len(odd) <= n // 1000, (len(odd), np.unique(st))
    if len(odd):
        ref = O.run(ModelParams(), 0, len(odd), YEAR, Y0, tz=TZ, n_threads=16, outputs=(),
                    stats=dict(HIST, amb_eps=AMB["fp32"]), chain_ids=odd.astype(np.uint64))
        _check_chains(acc[odd], st[odd], ref, "fp32", f"c4 {n}/{lanes} faulted")
    # the histogram counts every chain's seconds before its fault: the oracle's count for the
    # faulted ones, a full year for the rest
    want = int((st == 0).sum()) * YEAR + (int(ref["hist"].sum()) if len(odd) else 0)
    assert int(cx.hist.sum()) == want


def test_c4_thirty_day_windows_every_chain_vs_oracle():
    """64 chains x 60 days from 2019-03-10 in two 30-day windows (the spring-forward DST
    change inside the first), pipeline_defaults("c4"): every chain's energies, peak and
    status and the whole residual histogram against the oracle."""
    n, secs, start = 64, 60 * 86400, "2019-03-10 00:00:00"
    pipe = _pipeline("c4", n, secs, start, chain0=3_000_000)
    assert pipe.cfg.window == 30 * 86400 and pipe.nwin == 2
    ref = O.run(ModelParams(), 3_000_000, n, secs, start, tz=TZ, n_threads=16, outputs=(),
                stats=dict(HIST, amb_eps=AMB["fp32"]))
    cx = pipe.ctxs[0]
    pipe.sim.state = cx.state
    _check_chains(cx.acc.cpu().numpy().T, pipe.sim.status(), ref, "fp32", "c4 60 d")
    _check_hist(cx.hist, ref, "fp32", "c4 60 d")


# ------------------------------------------------------------------ C5
C5_N, C5_SECS, C5_START, C5_CHAIN0 = 512, 3 * 86400, "2019-09-05 00:00:00", 7_000_000


def _c5_inputs():
    return site_shape_tables(C5_N), site_grid(32, 16)


@functools.lru_cache(maxsize=4)
def _c5_oracle(chain0, prec):
    tables, sites = _c5_inputs()
    return O.run(ModelParams(cc_mode=CC_MARKOV), chain0, C5_N, C5_SECS, C5_START, tz=TZ, n_threads=16, outputs=(),
                 tables=tables, sites=sites, stats=dict(HIST, amb_eps=AMB[prec]))


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_c5_pipeline_vs_oracle(prec):
    """bench.py's C5 schedule (pipeline_defaults("c5"): markov cc, per-site tables and
    sites, day windows compacted to the live chains, the batches of every context advanced
    window by window together): the first and the last context against the oracle -- every chain's energies and
    peak (faulted chains' seconds before the fault included), status (a quarter or more
    of the chains fault: the reference's AssertionError), and the histogram, whose count
    equals the oracle's count of those chain-seconds."""
    from tmhpvsim_amd.dist import chain_totals
    tables, sites = _c5_inputs()
    pipe = _pipeline("c5", C5_N, C5_SECS, C5_START, prec=prec, chain0=C5_CHAIN0, lanes=16,
                     mp=ModelParams(cc_mode=CC_MARKOV), shape_tables=tables, sites=sites)
    # a 512-site batch is below the one-GPU C5 batch: pipeline_defaults keeps more contexts in flight
    assert pipe.cfg.compact and pipe.cfg.window == 86400 and len(pipe.ctxs) == pipe.cfg.pipeline >= 5
    for ci in (0, len(pipe.ctxs) - 1):
        cx = pipe.ctxs[ci]
        ref = _c5_oracle(C5_CHAIN0 + ci * C5_N, prec)
        pipe.sim.state = cx.state
        st = pipe.sim.status()
        assert (st != 0).sum() >= C5_N // 4
        _check_chains(cx.acc.cpu().numpy().T, st, ref, prec, f"c5 {prec} ctx{ci}")
        _check_hist(cx.hist, ref, prec, f"c5 {prec} ctx{ci}")
        # energies and histogram over the same chain-seconds: the node totals' count is the
        # oracle's number of accumulated seconds, and their meter energy its sum over them
        tot = chain_totals(cx.acc, cx.hist)
        assert int(tot["hist"].sum()) == int(ref["hist"].sum())
        assert abs(float(tot["energy_meter"]) - float(ref["acc"][:, 1].sum())) <= TOL[prec] * float(ref["acc"][:, 1].sum())
