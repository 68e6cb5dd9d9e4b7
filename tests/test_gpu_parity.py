"""GPU parity: the HIP kernels (through the C-ABI) against the C oracle and the
reference's golden fixtures.

Bars (DESIGN.md "Parity"):
  * discrete Markov state (covered bit, uniforms consumed, fault status): bit-exact;
  * fp64 kernel: every continuous output within 1e-12 relative (PV / residual
    relative to max(|ref|, 1 W));
  * fp32 kernel: within 1e-5 relative (same floor), pointwise, no outlier allowance
    (the seconds in a guard band of the PV chain's discontinuities are recomputed
    in fp64 by fixup_kernel);
  * reference fixtures (injected uniforms): CSI within 1e-12 relative.
"""
import os

import numpy as np
import pytest

from golden_util import CHAIN_CASES, load, streams
from oracle import oracle as O
from tmhpvsim_amd.params import CC_MARKOV, RNG_INJECTED, SHAPES, ModelParams

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _sim(n, start, tz=None, mp=None, prec="fp64", chain0=0, inj=None, horizon=None, kernel_path="auto", tables=None,
         sites=None):
    from tmhpvsim_amd.engine import BatchedSim
    return BatchedSim(n, start, tz=tz, params=mp or ModelParams(), precision=prec, chain0=chain0,
                      device="cuda:0", injected=inj, horizon=horizon or 400 * 86400, kernel_path=kernel_path,
                      shape_tables=tables, sites=sites)


def _np(t):
    return t.double().cpu().numpy() if t.dtype != torch.uint8 else t.cpu().numpy()


def _rel(got, ref, floor=1.0):
    return np.abs(got - ref) / np.maximum(np.abs(ref), floor)


def _err(field, got, ref):
    """Relative error with the scale each output is conditioned on:
    residual = meter - pv cancels, so it is measured against |meter| + |pv|."""
    if field == "residual":
        return np.abs(got["residual"] - ref["residual"]) / np.maximum(np.abs(ref["meter"]) + np.abs(ref["pv"]), 1.0)
    return _rel(got[field], ref[field])


def _where(err, tol):
    i = np.unravel_index(np.argmax(err), err.shape)
    return f"max {err.max():.3e} at step {i[0]} chain {i[1]}; {(err > tol).sum()} points > {tol}"


# ------------------------------------------------------------------ device math
def test_probe_math():
    from tmhpvsim_amd.engine import probe
    F = load("functions")
    u = F["u"][(F["u"] >= 2.0 ** -53)]
    np.testing.assert_allclose(probe(0, 0, u), O.ndtri(u), rtol=1e-14)
    np.testing.assert_allclose(probe(1, 2.69, u), O.gammaincinv(2.69, u), rtol=1e-13)
    np.testing.assert_allclose(probe(1, 3.5624, u), O.gammaincinv(3.5624, u), rtol=1e-13)
    m = np.abs(u - 0.5) > 1e-9
    np.testing.assert_allclose(probe(2, SHAPES[2][3], u[m]), O.stdtrit(SHAPES[2][3], u[m]), rtol=1e-12)
    for b in (0, 1, 3, 4, 5):
        np.testing.assert_allclose(probe(3, SHAPES[b][2], u), O.al_ppf(u, SHAPES[b][2]), rtol=1e-14)
    z32 = probe(4, 0, u)
    np.testing.assert_allclose(z32, O.ndtri(u), rtol=2e-6, atol=1e-6)
    w = np.random.default_rng(1).integers(0, 2 ** 32, 20000, dtype=np.uint64)
    u32 = (w.astype(np.float64) + 0.5) * 2.0 ** -32            # the fp64 per-second noise's uniforms
    np.testing.assert_allclose(probe(8, 0, u32), O.ndtri(u32), rtol=2e-15)
    # the fp64 PV chain's table functions (round 4): the noise quantile of the 32-bit word
    # itself (refitted erfinv polynomial, ocml's beyond p ~ 5e-4), the word range's extremes
    # included; log and exp over the ranges the PV chain feeds them (Ee, DISC's c am)
    wx = np.concatenate([w, [0, 1, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 2, 2 ** 32 - 1]]).astype(np.float64)
    ux = (wx + 0.5) * 2.0 ** -32
    np.testing.assert_allclose(probe(11, 0, wx), O.ndtri(ux), rtol=2e-15)
    xl = np.concatenate([10.0 ** np.random.default_rng(2).uniform(-12, 0.5, 20000), [1.0, 0.5, 2.0, 1 - 2 ** -52]])
    np.testing.assert_allclose(probe(12, 0, xl), np.log(xl), rtol=0, atol=4e-15)
    edge = probe(12, 0, np.array([0.0, -1.0, np.nan, np.inf, 5e-324]))
    np.testing.assert_array_equal(edge[:4], [-np.inf, np.nan, np.nan, np.inf])
    np.testing.assert_allclose(edge[4], np.log(5e-324), rtol=1e-15)
    xe = np.concatenate([np.random.default_rng(3).uniform(-45, 5, 20000), [0.0, -700.5, 710.0]])
    with np.errstate(over="ignore"):   # exp(710) = inf on both sides
        np.testing.assert_allclose(probe(13, 0, xe), np.exp(xe), rtol=5e-16, atol=0)
    # pv_power_f's final clamp relies on v_med3_f32(NaN, 0, Paco) = 0 (min3 on a NaN operand)
    x = np.array([np.nan, -5.0, 0.5, 3000.0, 1e9])
    np.testing.assert_array_equal(probe(9, 2500.0, x), [0.0, 0.0, 0.5, 2500.0, 2500.0])
    # and its min(csi, csimax) = v_med3_f32(csi, -inf, csimax): csimax on a NaN csi (measured on
    # MI355X, round 4), as fminf(NaN, csimax) gave
    np.testing.assert_array_equal(probe(10, 1.25, x), [1.25, -5.0, 0.5, 1.25, 1.25])
    # round 6: the fp32 kernels' min(csi, csimax) as a plain v_min_f32 with the bound in an SGPR
    # (pv_power_f<true>): the same results, csimax on a NaN csi
    np.testing.assert_array_equal(probe(16, 1.25, x), [1.25, -5.0, 0.5, 1.25, 1.25])


def test_probe_noise_table_quantile():
    """Round 6: the fp32 kernels' per-second noise quantile from the segment table
    (ndtri_t: a cubic per 1/32 octave of min(u, 1 - u), the log form below 2^-15) against
    the fp64 quantile of the same 32-bit words: <= 6e-7 absolute on the table's range over
    random words, every segment's ends, both halves and the word range's extremes; below
    2^-15 it is round 5's log form (ndtri_w, probe 15) bit for bit, <= 1.5e-6 there.  Reference: the per-second noise
    draw, /root/reference/tmhpvsim/clearskyindexmodel.py:146-147."""
    from tmhpvsim_amd.engine import probe
    rng = np.random.default_rng(11)
    w = rng.integers(0, 2 ** 32, 200000, dtype=np.uint64)
    # every segment's first and last words (both halves) and the log form's range (u < 2^-15)
    e = np.arange(112, 126)
    top = np.arange(32)
    lo = (2.0 ** (e[:, None] - 127) * (1 + top[None, :] / 32.0)).ravel()
    hi = (2.0 ** (e[:, None] - 127) * (1 + (top[None, :] + 1) / 32.0)).ravel()
    words = np.concatenate([lo * 2.0 ** 32, hi * 2.0 ** 32 - 1]).astype(np.int64).clip(0, 2 ** 31 - 1)
    words = np.concatenate([words, rng.integers(0, 2 ** 17, 5000), [0, 1, 2, 2 ** 31 - 2, 2 ** 31 - 1]])
    words = np.concatenate([words, 2 ** 32 - 1 - words, w.astype(np.int64)]).astype(np.float64)
    u = (words + 0.5) * 2.0 ** -32
    ref = O.ndtri(u)
    z = probe(14, 0, words)
    err = np.abs(z - ref)
    tab = np.minimum(u, 1 - u) >= 2.0 ** -15     # the table's range; below it the log form
    assert err[tab].max() <= 6e-7, (err[tab].max(), words[tab][err[tab].argmax()])
    zw = probe(15, 0, words)                     # round 5's form on the same words
    np.testing.assert_array_equal(z[~tab], zw[~tab])
    # the log form's own accuracy in the far tails (|z| > 4.1): <= 1.5e-6 absolute (3e-7 relative)
    assert np.abs(zw - ref).max() <= 1.5e-6 and err.max() <= 1.5e-6, (np.abs(zw - ref).max(), err.max())
    assert (np.sign(z[np.abs(ref) > 1e-6]) == np.sign(ref[np.abs(ref) > 1e-6])).all()


# ------------------------------------------------------------------ reference fixtures
@pytest.mark.parametrize("case", CHAIN_CASES)
def test_injected_vs_reference_fixture(case):
    d = load(case)
    n = int(d["n_steps"])
    chains = d["chains"]
    mp = ModelParams(rng_mode=RNG_INJECTED, cc_mode=CC_MARKOV if bool(d["markov"]) else 0, with_pv=False)
    sim = _sim(len(chains), str(d["start"]), tz=str(d["tz"]) or None, mp=mp, inj=streams(d), horizon=n)
    out = sim.run(n, trace=("csi", "covered"))
    csi, cov = _np(out["csi"]).T, _np(out["covered"]).T
    ok = np.isfinite(d["csi"])
    np.testing.assert_array_equal(np.isnan(csi), ~ok)
    np.testing.assert_array_equal(cov[ok], d["covered"][ok])
    assert (_rel(csi[ok], d["csi"][ok], 0) <= 1e-12).all()
    codes = {"": 0, "NameError": 1, "AssertionError": 2}
    assert list(sim.status()) == [codes[str(e)] for e in d["error"]]
    pos = sim.state_field("pos").cpu().numpy().astype(np.int64)
    good = sim.status() == 0
    np.testing.assert_array_equal(pos[good], d["pos"][good, -1])


# ------------------------------------------------------------------ keyed mode vs oracle
CASES_KEYED = [
    ("2019-09-05 00:00:00", "Europe/Berlin", 86400, 0),      # C2 day (scaled chains)
    ("2019-10-27 00:00:00", "Europe/Berlin", 14400, 1),      # DST fall-back night
    ("2019-06-21 03:00:00", None, 7200, 0),                  # naive clock, sunrise
]


@pytest.mark.parametrize("start,tz,steps,variant", CASES_KEYED)
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_keyed_vs_oracle(start, tz, steps, variant, prec):
    n = 256 if steps <= 14400 else 128
    mp = ModelParams(seed=0x5EED + variant)
    ref = O.run(mp, 1000, n, steps, start, tz=tz, n_threads=8)
    sim = _sim(n, start, tz=tz, mp=mp, prec=prec, chain0=1000, horizon=steps)
    out = sim.run(steps)
    np.testing.assert_array_equal(sim.status(), ref["status"])   # NameError chains (~1e-4) included
    ok = ref["status"] == 0
    np.testing.assert_array_equal(_np(out["covered"]), ref["covered"])
    tol = 1e-12 if prec == "fp64" else 1e-5
    got = {f: _np(out[f])[:, ok] for f in ("csi", "pv", "meter", "residual")}
    rf = {f: ref[f][:, ok] for f in ("csi", "pv", "meter", "residual")}
    for f in ("csi", "pv", "meter", "residual"):
        assert np.array_equal(np.isnan(_np(out[f])), np.isnan(ref[f])), f
        err = _err(f, got, rf)
        assert err.max() <= tol, (f, _where(err, tol), got["pv"][np.unravel_index(np.argmax(err), err.shape)])


@pytest.mark.parametrize("path", ["sequential", "time_parallel"])
def test_markov_keyed_vs_oracle(path):
    mp = ModelParams(cc_mode=CC_MARKOV, seed=77)
    n, steps, start = 128, 43200, "2019-09-05 06:00:00"
    ref = O.run(mp, 0, n, steps, start, tz="Europe/Berlin", n_threads=8)
    sim = _sim(n, start, tz="Europe/Berlin", mp=mp, horizon=steps, kernel_path=path)
    assert sim.path == path
    out = sim.run(steps)
    np.testing.assert_array_equal(sim.status(), ref["status"])
    ok = ref["status"] == 0
    np.testing.assert_array_equal(_np(out["covered"])[:, ok], ref["covered"][:, ok])
    got = {f: _np(out[f])[:, ok] for f in ("csi", "pv", "meter", "residual")}
    rf = {f: ref[f][:, ok] for f in ("csi", "pv", "meter", "residual")}
    for f in ("csi", "pv", "residual"):
        err = _err(f, got, rf)
        assert err.max() <= 1e-12, (f, _where(err, 1e-12), got["pv"][np.unravel_index(np.argmax(err), err.shape)])


@pytest.mark.parametrize("path", ["sequential", "time_parallel"])
@pytest.mark.parametrize("markov", [True, False])
def test_site_tables_vs_oracle(markov, path):
    """Per-chain shape tables (C5's lat/lon sweep: one mc_dist_shapes table x U(0.9, 1.1) per
    site) through tmh_set_shape_tables, both cc modes and both kernel paths, against the oracle
    with the same tables; chains > n_tab are refused."""
    from tmhpvsim_amd.params import site_shape_tables
    mp = ModelParams(cc_mode=CC_MARKOV if markov else 0, seed=0x7AB1E + 1)
    n, steps, start = 128, 30000, "2019-09-05 04:00:00"
    tab = site_shape_tables(n, site0=3000)
    ref = O.run(mp, 3000, n, steps, start, tz="Europe/Berlin", n_threads=8, tables=tab)
    sim = _sim(n, start, tz="Europe/Berlin", mp=mp, chain0=3000, horizon=steps, kernel_path=path, tables=tab)
    out = sim.run(steps, window=10000)
    np.testing.assert_array_equal(sim.status(), ref["status"])
    ok = ref["status"] == 0
    np.testing.assert_array_equal(_np(out["covered"])[:, ok], ref["covered"][:, ok])
    got = {f: _np(out[f])[:, ok] for f in ("csi", "pv", "meter", "residual")}
    rf = {f: ref[f][:, ok] for f in ("csi", "pv", "meter", "residual")}
    for f in ("csi", "pv", "residual"):
        err = _err(f, got, rf)
        assert err.max() <= 1e-12, (f, _where(err, 1e-12))
    plain = O.run(mp, 3000, n, steps, start, tz="Europe/Berlin", n_threads=8, outputs=("covered",))
    assert (plain["covered"][:, ok] != ref["covered"][:, ok]).any()    # the tables are in effect
    rc = sim.L.tmh_init(sim._eng, _ptr_of(sim.state), 0, n + 1, None, sim._stream())   # batch > tables
    assert rc != 0 and b"shape tables" in sim.L.tmh_last_error()


def _ptr_of(t):
    import ctypes as C
    return C.c_void_p(t.data_ptr())


def _check_vs_oracle(out, ref, prec):
    np.testing.assert_array_equal(_np(out["covered"]), ref["covered"])
    ok = ref["status"] == 0
    tol = 1e-12 if prec == "fp64" else 1e-5
    got = {f: _np(out[f])[:, ok] for f in ("csi", "pv", "meter", "residual")}
    rf = {f: ref[f][:, ok] for f in ("csi", "pv", "meter", "residual")}
    for f in ("csi", "pv", "meter", "residual"):
        assert np.array_equal(np.isnan(_np(out[f])), np.isnan(ref[f])), f
        err = _err(f, got, rf)
        assert err.max() <= tol, (f, _where(err, tol))


@pytest.mark.parametrize("path,prec,linke", [("time_parallel", "fp64", False), ("time_parallel", "fp32", True),
                                             ("sequential", "fp64", True), ("sequential", "fp32", False)])
def test_site_grid_vs_oracle(path, prec, linke):
    """Per-chain PV sites (tmh_set_sites; C5's lat/lon grid, 35-60 N x 10 W-30 E): geometry per
    chain-second in the kernels vs the oracle's per-chain geometry, across sunrise at every longitude."""
    from tmhpvsim_amd.params import site_grid
    n, steps, start = 128, 14400, "2019-06-21 02:30:00"
    sites = site_grid(16, 8)
    lk = None
    if linke:   # per-site monthly Linke turbidity (pvlib's lookup table is per lat/lon)
        lk = np.asarray(ModelParams().linke)[None, :] * (0.8 + 0.4 * np.random.default_rng(3).random((n, 1)))
    mp = ModelParams(seed=0x51E)
    ref = O.run(mp, 0, n, steps, start, tz="Europe/Berlin", n_threads=8, sites=(sites, lk))
    sim = _sim(n, start, tz="Europe/Berlin", mp=mp, prec=prec, horizon=steps, kernel_path=path, sites=(sites, lk))
    out = sim.run(steps, window=5000)
    np.testing.assert_array_equal(sim.status(), ref["status"])
    _check_vs_oracle(out, ref, prec)
    pv = ref["pv"][:, ref["status"] == 0]
    first = np.argmax(pv > 0, axis=0)
    assert first.max() - first.min() > 60 * 60      # sunrise spreads over the grid's longitudes / latitudes


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_sites_all_default_equal_single_site(prec):
    """Every chain given the engine's own site: the per-chain-second geometry reproduces the
    plan's per-site geometry (same functions), so the traces agree to rounding."""
    n, steps, start = 64, 6000, "2019-09-05 10:00:00"
    sites = np.broadcast_to(ModelParams().site.as_array(), (n, 8)).copy()
    a = _sim(n, start, tz="Europe/Berlin", prec=prec, horizon=steps).run(steps)
    b = _sim(n, start, tz="Europe/Berlin", prec=prec, horizon=steps, sites=sites).run(steps)
    assert _same(a["covered"], b["covered"]) and _same(a["csi"], b["csi"]) and _same(a["meter"], b["meter"])
    tol = 1e-13 if prec == "fp64" else 1e-6
    d = (a["pv"].double() - b["pv"].double()).abs().max().item()
    assert d <= tol * 250.0, d


def test_c5_slice_time_parallel_equals_sequential_and_oracle():
    """C5 in small: markov cc with per-site tables and per-site PV geometry on a lat/lon grid;
    the time-parallel path == the sequential kernel bit for bit (fp32), and both == the oracle."""
    from tmhpvsim_amd.params import site_grid, site_shape_tables
    n, start, windows = 192, "2019-03-30 20:00:00", [9000, 21000, 6000]     # across the DST spring-forward
    steps = sum(windows)
    mp = ModelParams(cc_mode=CC_MARKOV, seed=0xC5)
    sites, tab = site_grid(16, 12), site_shape_tables(n)
    kw = dict(tz="Europe/Berlin", mp=mp, horizon=steps, tables=tab, sites=sites)
    a = _sim(n, start, prec="fp32", kernel_path="time_parallel", **kw)
    b = _sim(n, start, prec="fp32", kernel_path="sequential", **kw)
    ra = [a.run(w, window=w) for w in windows]
    rb = [b.run(w, window=w) for w in windows]
    for f in ("csi", "covered", "pv", "meter", "residual"):
        assert _same(torch.cat([r[f] for r in ra]), torch.cat([r[f] for r in rb])), f
    c = _sim(n, start, prec="fp64", **kw)
    ref = O.run(mp, 0, n, steps, start, tz="Europe/Berlin", n_threads=8, tables=tab, sites=sites)
    out = c.run(steps, window=12000)
    np.testing.assert_array_equal(c.status(), ref["status"])
    _check_vs_oracle(out, ref, "fp64")


def test_geometry_table_vs_oracle():
    from tmhpvsim_amd.params import ModelParams
    mp = ModelParams()
    steps, start, tz = 86400, "2019-09-05 00:00:00", "Europe/Berlin"
    sim = _sim(1, start, tz=tz, mp=mp, horizon=steps)
    tab = sim.geometry(0, steps).cpu().numpy()
    cal, utc = O.calendar(start, steps, tz)
    P = O.make_params(mp)
    import ctypes as C
    idx = np.arange(0, steps, 97)
    for s in idx:
        g = np.zeros(16)
        O.lib().orc_geometry(C.byref(P), int(utc[s]), int(cal[s, 4]), int(cal[s, 5]), g.ctypes.data_as(C.c_void_p))
        # oracle geom_t order: cosz csi_max ghi_cs i0h i0 knc am disc_ok cos_zen rb dni_extra term2 gfac cos_aoi f1 f2
        mine = tab[s, [4, 5, 6, 7, 8, 9, 10, 18, 4, 12, 13, 14, 15, 16, 17, 11]]   # G_DISCOK 18, G_F2 11
        m = np.isfinite(g)
        np.testing.assert_allclose(mine[m], g[m], rtol=1e-11, atol=1e-13)
    np.testing.assert_array_equal(tab[:, 0], cal[:, 3] / 60.0)


# ------------------------------------------------------------------ invariances
def _same(a, b):
    """bitwise equality with NaN == NaN (faulted chains emit NaN)"""
    if a.dtype == torch.uint8:
        return torch.equal(a, b)
    return torch.equal(torch.nan_to_num(a, nan=-12345.0), torch.nan_to_num(b, nan=-12345.0))


def test_window_and_partition_invariance():
    start, steps = "2019-09-05 10:00:00", 5000
    a = _sim(128, start, tz="Europe/Berlin", prec="fp32", horizon=steps)
    ra = a.run(steps, window=steps)
    b = _sim(128, start, tz="Europe/Berlin", prec="fp32", horizon=steps)
    parts = [b.run(k, window=333) for k in (1, 999, 4000)]
    for f in ("csi", "pv", "covered", "residual"):
        joined = torch.cat([p[f] for p in parts])
        assert _same(ra[f], joined), f
    c0 = _sim(64, start, tz="Europe/Berlin", prec="fp32", horizon=steps)
    c1 = _sim(64, start, tz="Europe/Berlin", prec="fp32", chain0=64, horizon=steps)
    r0, r1 = c0.run(steps), c1.run(steps)
    for f in ("csi", "pv", "covered", "residual"):
        assert _same(ra[f], torch.cat([r0[f], r1[f]], dim=1)), f


@pytest.mark.parametrize("prec,markov", [("fp32", False), ("fp64", False), ("fp32", True)])
def test_time_parallel_equals_sequential(prec, markov):
    """P1 segments + P2 (chain x 128 s) expansion == one-lane-per-chain sequential kernel, bit for bit,
    over uneven windows crossing midnight and the DST fall-back (state carried between windows);
    markov: the hourly Markov cc (markov_cc_kernel) with per-site tables."""
    from tmhpvsim_amd.params import site_shape_tables
    start, n = "2019-10-26 21:00:00", 192
    windows = [7001, 30000, 1, 20000]
    steps = sum(windows)
    mp = ModelParams(cc_mode=CC_MARKOV) if markov else None
    tab = site_shape_tables(n) if markov else None
    a = _sim(n, start, tz="Europe/Berlin", mp=mp, prec=prec, horizon=steps, kernel_path="time_parallel", tables=tab)
    b = _sim(n, start, tz="Europe/Berlin", mp=mp, prec=prec, horizon=steps, kernel_path="sequential", tables=tab)
    assert a.path == "time_parallel" and b.path == "sequential"
    for w in windows:
        ra, rb = a.run(w, window=w), b.run(w, window=w)
        for f in ("csi", "covered", "pv", "meter", "residual"):
            assert _same(ra[f], rb[f]), (w, f)
    np.testing.assert_array_equal(a.status(), b.status())
    ok = torch.as_tensor(a.status() == 0, device="cuda:0")   # a faulted chain's state is frozen, not defined
    for f in ("sb_cc", "sa_cc", "sb_clear_day", "sa_clear_day", "sb_cloudy_noise", "sa_clear_noise", "sa_ws",
              "cloud_length", "clear_length", "sec", "sigma_len", "markov_state"):
        assert _same(a.state_field(f)[ok], b.state_field(f)[ok]), f
    L = a.state_field("sigma_len").long()
    live = torch.arange(a.state_field("sigma_cloud").shape[1], device="cuda:0")[None, :] < L[:, None]
    live &= ok[:, None]
    for f in ("sigma_cloud", "sigma_clear"):   # entries past len(sigma) are dead storage
        assert torch.equal(a.state_field(f)[live], b.state_field(f)[live]), f


@pytest.mark.parametrize("path", ["time_parallel", "sequential"])
def test_walk_then_expand_equals_step(path):
    """tmh_walk + tmh_expand (the split bench.py pipelines) == tmh_run, bit for bit."""
    import ctypes as C
    from tmhpvsim_amd import _lib
    start, steps, n = "2019-09-05 05:00:00", 7000, 96
    a = _sim(n, start, tz="Europe/Berlin", prec="fp32", horizon=steps, kernel_path=path)
    b = _sim(n, start, tz="Europe/Berlin", prec="fp32", horizon=steps, kernel_path=path)
    ra = a.run(steps, window=steps)
    L = b.L
    out = {f: torch.empty(steps, n, dtype=torch.float32, device="cuda:0") for f in ("csi", "pv", "meter", "residual")}
    cov = torch.empty(steps, n, dtype=torch.uint8, device="cuda:0")
    tr = _lib.Trace(out["csi"].data_ptr(), cov.data_ptr(), out["pv"].data_ptr(), out["meter"].data_ptr(),
                    out["residual"].data_ptr(), n)
    plan = torch.empty(L.tmh_plan_bytes(steps), dtype=torch.uint8, device="cuda:0")
    scr = torch.empty(max(1, L.tmh_scratch_bytes(n, steps)), dtype=torch.uint8, device="cuda:0")
    p = lambda t: C.c_void_p(t.data_ptr())
    s = b._stream()
    _lib.check(L.tmh_plan(b._eng, 0, steps, p(plan), s))
    _lib.check(L.tmh_walk(b._eng, p(b.state), 0, n, 0, steps, p(plan), p(scr), scr.numel(), s))
    _lib.check(L.tmh_expand(b._eng, p(b.state), 0, n, 0, steps, None, C.byref(tr), None, p(plan), p(scr),
                            scr.numel(), s))
    torch.cuda.synchronize()
    for f in ("csi", "pv", "meter", "residual"):
        assert _same(ra[f], out[f]), f
    assert _same(ra["covered"], cov)
    np.testing.assert_array_equal(a.status(), b.status())
    assert _same(a.state_field("sa_cc"), b.state_field("sa_cc"))


@pytest.mark.parametrize("markov", [False, True])
def test_pipelined_windows_equal_one_window(markov):
    """BatchedSim.run over several windows (walk of window w+1 via tmh_walk_next beside the
    expansion of window w) == one window: traces bit for bit, state, per-chain statistics."""
    from tmhpvsim_amd.params import site_shape_tables
    start, steps, n = "2019-03-30 22:00:00", 3 * 7001, 160
    mp = ModelParams(cc_mode=CC_MARKOV) if markov else None
    tab = site_shape_tables(n) if markov else None
    a = _sim(n, start, tz="Europe/Berlin", mp=mp, prec="fp32", horizon=steps, tables=tab)
    b = _sim(n, start, tz="Europe/Berlin", mp=mp, prec="fp32", horizon=steps, tables=tab)
    a.enable_stats()
    b.enable_stats()
    ra = a.run(steps, window=steps)
    rb = b.run(steps, window=3000)            # 8 windows, the last one short
    for f in ("csi", "covered", "pv", "meter", "residual"):
        assert _same(ra[f], rb[f]), f
    np.testing.assert_array_equal(a.status(), b.status())
    ok = torch.as_tensor(a.status() == 0, device="cuda:0")
    for f in ("sa_cc", "sb_ws", "sa_clear_noise", "cloud_length", "sec", "sigma_len", "markov_state"):
        assert _same(a.state_field(f)[ok], b.state_field(f)[ok]), f
    assert torch.equal(a.hist, b.hist)
    np.testing.assert_allclose(a.chain_acc[:, ok].cpu().numpy(), b.chain_acc[:, ok].cpu().numpy(), rtol=1e-12)


def test_stats_match_trace():
    start, steps, n = "2019-09-05 00:00:00", 20000, 512
    s = _sim(n, start, tz="Europe/Berlin", prec="fp32", horizon=steps)
    s.enable_stats(4096, -300.0, 9000.0)
    out = s.run(steps, trace=("pv", "meter", "residual"))
    ok = torch.as_tensor(s.status() == 0, device="cuda:0")
    for k in out:
        out[k] = out[k][:, ok]
    s.chain_acc = s.chain_acc[:, ok]
    res = out["residual"].double()
    np.testing.assert_allclose(s.chain_acc[0].cpu().numpy(), out["pv"].double().sum(0).cpu().numpy(), rtol=1e-9)
    np.testing.assert_allclose(s.chain_acc[2].cpu().numpy(), res.sum(0).cpu().numpy(), rtol=1e-9)
    np.testing.assert_array_equal(s.chain_acc[3].cpu().numpy(), res.max(0).values.cpu().numpy())
    # the fp32 kernels' bin position: one fp32 FMA of res with the fp32-rounded scale and
    # offset (hist_bin; exact in fp64 here, 48 + 24 bits, then rounded once like the FMA)
    scale = 4096 / 9300.0
    x = (res.cpu().numpy() * np.float64(np.float32(scale)) + np.float64(np.float32(300.0 * scale))).astype(np.float32)
    bins = np.clip(np.floor(x), 0, 4095).astype(np.int64)
    np.testing.assert_array_equal(s.hist.cpu().numpy(), np.bincount(bins.ravel(), minlength=4096))


# ------------------------------------------------------------------ full size (C2) properties
def test_c2_full_size_properties():
    """4,096 chains x 86,400 s, fp32: reference invariants + oracle spot checks."""
    n, steps, start, tz = 4096, 86400, "2019-09-05 00:00:00", "Europe/Berlin"
    sim = _sim(n, start, tz=tz, prec="fp32", horizon=steps)
    out = sim.run(steps)
    torch.cuda.synchronize()
    st = sim.status()
    assert set(np.unique(st)) <= {0, 1} and (st == 1).mean() < 2e-3   # only the reference's NameError
    ok = torch.as_tensor(st == 0, device="cuda:0")
    out = {k: v[:, ok] for k, v in out.items()}
    csi = out["csi"]
    assert bool(((csi > 0) & (csi < 2)).all())                       # tests/test_clearskyindexmodel.py:13
    assert bool((out["pv"] >= 0).all())                              # tests/test_pvmodel.py:10
    assert bool(((out["meter"] >= 0) & (out["meter"] < 9000)).all())  # metersim.py:51
    assert torch.equal(out["residual"], out["meter"] - out["pv"])    # pvsim.py:83
    assert bool(out["covered"].le(1).all())
    peak = out["pv"].max().item()
    assert 0 < peak <= 250.0                                          # Paco of the micro-inverter
    pick = [c for c in (0, 1, 777, 2048, 4095) if st[c] == 0]
    cols = {c: int(np.nonzero(st == 0)[0].tolist().index(c)) for c in pick}
    for c in pick:
        ref = O.run(ModelParams(), c, 1, steps, start, tz=tz)
        np.testing.assert_array_equal(_np(out["covered"][:, cols[c]]), ref["covered"][:, 0])
        assert _rel(_np(out["csi"][:, cols[c]]), ref["csi"][:, 0]).max() <= 1e-5


@pytest.mark.parametrize("lanes", [16, 4])
def test_segment_overflow_pool(lanes):
    """Segment records past a chain's row go to the shared overflow pool (the windy
    tail of cloud_cover_binary.py:80-107's call count).  With the row cut to 16
    records every chain spills ~24 chunks' worth and the outputs stay bit-identical.
    With the row cut to 400 records (only the windier chains spill) and a pool of
    2 chunks, the fault is deterministic: exactly the chains with more than 400
    records end with TMH_CHAIN_SEGMENT_OVERFLOW (5), at their first record past the
    row (their outputs equal the unconstrained run's before that step and are NaN
    from it), and every other chain is unchanged -- whichever claims of the
    atomic pool counter the waves won.  Both walk widths (16 and 4 lanes per chain)."""
    from tmhpvsim_amd import _lib
    L = _lib.load()
    n, steps, start = 256, 86400, "2019-09-05 00:00:00"

    def run():
        s = _sim(n, start, tz="Europe/Berlin", prec="fp32", kernel_path="time_parallel", horizon=steps)
        _lib.check(L.tmh_set_walk_lanes(s._eng, lanes))
        calls0 = s.state_field("ncalls").cpu().numpy().astype(np.int64)
        out = s.run(steps, trace=("covered", "pv"))
        torch.cuda.synchronize()
        calls = s.state_field("ncalls").cpu().numpy().astype(np.int64) - calls0
        return s.status(), _np(out["covered"]), _np(out["pv"]), calls

    st0, cov0, pv0, calls = run()
    try:
        _lib.check(L.tmh_test_set_segment_capacity(16, 4 * n))
        st1, cov1, pv1, _ = run()
        _lib.check(L.tmh_test_set_segment_capacity(400, 2))
        st2, cov2, pv2, _ = run()
    finally:
        L.tmh_test_set_segment_capacity(0, 0)
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(cov1, cov0)
    np.testing.assert_array_equal(pv1, pv0)
    records = calls + 1                       # the window-start segment + one record per next_cloud call
    ok0 = st0 == 0
    want = ok0 & (records > 400)
    assert 2 < want.sum() < ok0.sum()         # a pool of 2 chunks is short for them
    hit = st2 == 5
    np.testing.assert_array_equal(hit, want)  # exactly the chains that reached the pool
    keep = ~hit
    np.testing.assert_array_equal(st2[keep], st0[keep])
    np.testing.assert_array_equal(cov2[:, keep], cov0[:, keep])
    np.testing.assert_array_equal(pv2[:, keep], pv0[:, keep])
    for c in np.nonzero(hit)[0]:               # equal up to the fault, NaN (covered 255) from it on
        f = int(np.argmax(cov2[:, c] == 255))
        assert 0 < f and (cov2[f:, c] == 255).all() and np.isnan(pv2[f:, c]).all()
        np.testing.assert_array_equal(cov2[:f, c], cov0[:f, c])
        np.testing.assert_array_equal(pv2[:f, c], pv0[:f, c])


@pytest.mark.parametrize("window", [86400, 7200])
def test_walk_chains_per_row_invariance(window):
    """tmh_set_walk_chains_per_row: rows that take the next chain from the window's
    queue when theirs is done give bit-identical segment walks (covered bit, PV,
    status, state) for 1, 3 and 64 chains per row, one window or 12 chained windows."""
    from tmhpvsim_amd import _lib
    L = _lib.load()
    n, steps, start = 700, 86400, "2019-09-05 00:00:00"
    outs = []
    for cpr in (1, 3, 64):
        s = _sim(n, start, tz="Europe/Berlin", prec="fp32", kernel_path="time_parallel", horizon=steps)
        _lib.check(L.tmh_set_walk_chains_per_row(s._eng, cpr))
        out = s.run(steps, trace=("covered", "pv"), window=window)
        torch.cuda.synchronize()
        outs.append((s.status(), _np(out["covered"]), _np(out["pv"]), s.state_field("ncalls").cpu().numpy()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("window,markov,start", [(86400, False, "2019-09-05 00:00:00"),
                                                 (7200, False, "2019-09-05 00:00:00"),
                                                 (7200, False, "2019-10-26 12:00:00"),   # DST fall-back
                                                 (86400, True, "2019-09-05 00:00:00")])
def test_walk_lanes_invariance(window, markov, start):
    """tmh_set_walk_lanes: the segment walk with 4, 8 or 16 lanes per chain (sigma
    entries spread over fewer lanes, more register chunks per lane; entries past
    the registers in the chain's global row) gives bit-identical results -- covered
    bit, PV, status, call counts and the window-end sigma arrays -- alone and with
    groups that take queued chains, with the rows in wind order (tmh_set_walk_order) or
    in chain order, in one window or in chained windows.  2,000
    chain-days reach sigma lengths past 64 (~0.5 % of the calls) on every path.  Markov
    cloud cover with per-site tables (C5's walk inputs) too, and chained windows across the
    DST fall-back (the walk's clock shift)."""
    from tmhpvsim_amd import _lib
    from tmhpvsim_amd.params import site_shape_tables
    L = _lib.load()
    n, steps = 2000, 86400
    mp = ModelParams(cc_mode=CC_MARKOV, seed=0x7AB1E) if markov else None
    tab = site_shape_tables(n) if markov else None
    outs = []
    # tp: the 8-lane walk's throughput variant (32 register entries, 4 waves per SIMD: C3's
    # batches), forced on this small batch through the engine's row threshold; mk: markov mode's
    # hour quantiles precomputed by event_draws_kernel (the default at this size) or drawn in
    # markov_cc_kernel's walk (0: a full C5 batch's path)
    for lanes, cpr, order, tp, mk in ((16, 1, 1, 0, 1), (16, 1, 0, 0, 1), (8, 1, 1, 0, 1), (4, 1, 1, 0, 1),
                                      (4, 3, 1, 0, 1), (4, 3, 0, 0, 1), (8, 2, 1, 0, 1), (8, 1, 1, 1, 1),
                                      (8, 1, 0, 1, 1), (16, 1, 1, 0, 0)):
        env = {"TMH_WALK_TP_ROWS": "1" if tp else "4294967295", "TMH_MK_PRE_MAX": "4294967295" if mk else "0"}
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            s = _sim(n, start, tz="Europe/Berlin", mp=mp, prec="fp32", kernel_path="time_parallel", horizon=steps,
                     tables=tab)
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        _lib.check(L.tmh_set_walk_lanes(s._eng, lanes))
        _lib.check(L.tmh_set_walk_chains_per_row(s._eng, cpr))
        _lib.check(L.tmh_set_walk_order(s._eng, order))   # rows windiest chain first, or in chain order
        out = s.run(steps, trace=("covered", "pv"), window=window)
        torch.cuda.synchronize()
        outs.append((s.status(), _np(out["covered"]), _np(out["pv"]), s.state_field("ncalls").cpu().numpy(),
                     s.state_field("sigma_len").cpu().numpy(), s.state_field("sigma_cloud").cpu().numpy(),
                     s.state_field("sigma_clear").cpu().numpy()))
    Lend = outs[0][4]
    assert Lend.max() > 40 or markov   # markov: most chains end in the low-cover AssertionError
    for o in outs[1:]:
        for i, (a, b) in enumerate(zip(outs[0], o)):
            if i >= 5:   # sigma rows: entries < L only
                m = np.arange(a.shape[1])[None, :] < Lend[:, None]
                a, b = np.where(m, a, 0), np.where(m, b, 0)
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("markov", [False, True])
def test_parts_minutes_ahead_equal_step(markov):
    """bench.py's gated order through the C-ABI -- draws, the minute table ahead
    (TMH_EXPAND_MINUTES), the segment walk with queued rows, the expansion without
    its minute table (KERNEL | NO_MINUTES), the commit on another stream -- equals
    tmh_run bit for bit (traces, statistics, state)."""
    import ctypes as C
    from tmhpvsim_amd import _lib
    start, steps, n = "2019-09-05 04:00:00", 9000, 300
    mp = ModelParams(cc_mode=CC_MARKOV) if markov else ModelParams()
    a = _sim(n, start, tz="Europe/Berlin", mp=mp, prec="fp32", horizon=steps, kernel_path="time_parallel")
    b = _sim(n, start, tz="Europe/Berlin", mp=mp, prec="fp32", horizon=steps, kernel_path="time_parallel")
    a.enable_stats()
    b.enable_stats()
    ra = a.run(steps, window=steps)
    L = b.L
    out = {f: torch.empty(steps, n, dtype=torch.float32, device="cuda:0") for f in ("csi", "pv", "meter", "residual")}
    cov = torch.empty(steps, n, dtype=torch.uint8, device="cuda:0")
    tr = _lib.Trace(out["csi"].data_ptr(), cov.data_ptr(), out["pv"].data_ptr(), out["meter"].data_ptr(),
                    out["residual"].data_ptr(), n)
    st = b._stats_struct()
    plan = torch.empty(L.tmh_plan_bytes(steps), dtype=torch.uint8, device="cuda:0")
    scr = torch.empty(L.tmh_scratch_bytes(n, steps), dtype=torch.uint8, device="cuda:0")
    p = lambda t: C.c_void_p(t.data_ptr())
    s = b._stream()
    s2 = torch.cuda.Stream()
    _lib.check(L.tmh_set_walk_chains_per_row(b._eng, 5))
    args = (b._eng, p(b.state), 0, n, 0, steps, None, C.byref(tr), C.byref(st), p(plan), p(scr), scr.numel())
    _lib.check(L.tmh_plan(b._eng, 0, steps, p(plan), s))
    _lib.check(L.tmh_walk_part(b._eng, p(b.state), 0, n, 0, steps, p(plan), p(scr), scr.numel(), None, 0,
                               _lib.WALK_DRAWS, s))
    _lib.check(L.tmh_expand_part(*args, _lib.EXPAND_MINUTES, s))
    _lib.check(L.tmh_walk_part(b._eng, p(b.state), 0, n, 0, steps, p(plan), p(scr), scr.numel(), None, 0,
                               _lib.WALK_SEGMENTS, s))
    _lib.check(L.tmh_expand_part(*args, _lib.EXPAND_KERNEL | _lib.EXPAND_NO_MINUTES, s))
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())      # b._stream() is torch's current stream
    s2.wait_event(ev)
    _lib.check(L.tmh_expand_part(*args, _lib.EXPAND_COMMIT, C.c_void_p(s2.cuda_stream)))
    torch.cuda.synchronize()
    for f in ("csi", "pv", "meter", "residual"):
        assert _same(ra[f], out[f]), f
    assert _same(ra["covered"], cov)
    np.testing.assert_array_equal(a.status(), b.status())
    assert torch.equal(a.hist, b.hist)
    assert torch.equal(a.chain_acc, b.chain_acc)
    for fld in ("sa_cc", "sigma_len", "ncalls", "sec"):
        assert _same(a.state_field(fld), b.state_field(fld)), fld


@pytest.mark.parametrize("path", ["time_parallel", "sequential"])
def test_compacted_windows_equal_full_batch(path):
    """BatchedSim.run(compact=True): windows after the first run on the chains still
    live (markov cc with per-site tables and sites, where the reference's
    AssertionError ends many chains); per-chain statistics, histogram, status and
    state are bit-identical to the uncompacted run."""
    from tmhpvsim_amd.params import site_grid, site_shape_tables
    n, steps, start = 512, 3 * 86400, "2019-09-05 00:00:00"
    mp = ModelParams(cc_mode=CC_MARKOV, seed=0xC5)
    kw = dict(tz="Europe/Berlin", mp=mp, horizon=steps, tables=site_shape_tables(n), sites=site_grid(32, 16),
              prec="fp32", kernel_path=path)
    a = _sim(n, start, **kw)
    b = _sim(n, start, **kw)
    a.enable_stats()
    b.enable_stats()
    a.run(steps, trace=(), window=86400)
    b.run(steps, trace=(), window=86400, compact=True)
    torch.cuda.synchronize()
    sa, sb = a.status(), b.status()
    assert (sa != 0).sum() > n // 8, "the test needs faulting chains"
    np.testing.assert_array_equal(sa, sb)
    assert torch.equal(a.hist, b.hist)
    assert _same(a.chain_acc, b.chain_acc)
    for fld in ("sa_cc", "sb_ws", "cloud_length", "sigma_len", "ncalls", "sec", "pos"):
        assert _same(a.state_field(fld), b.state_field(fld)), fld
    Ls = a.state_field("sigma_len").long()
    used = torch.arange(a.state_field("sigma_cloud").shape[1], device="cuda:0")[None, :] < Ls[:, None]
    for fld in ("sigma_cloud", "sigma_clear"):   # entries past a chain's length are not state
        assert _same(torch.where(used, a.state_field(fld), 0.0), torch.where(used, b.state_field(fld), 0.0)), fld
