"""The kernel and the schedule the headline bench line times, against the oracle.

bench.py's C2 line traces exactly pv, meter and residual with no statistics, which
selects the OUT_TRACE3 instantiation of the expansion (expand_kernel<float, 1,
false>; <double, 1, false> for the fp64 line): its own launch bounds, buffer-
resource stores with lanes past the last chain parked out of range, and the fp32
guard-band fixup writing through those trace pointers.  These tests run exactly
that instantiation (tmh_engine_last_expand says so) and the bench's gated
schedule (tmhpvsim_amd.pipeline.BatchPipeline with bench.py's C2 defaults):

  * every chain and second of the C2 batch (4,096 keyed chains x 86,400 s) against
    the C oracle: fp32 <= 1e-5, fp64 <= 1e-12 (PV relative to max(|pv|, 1 W),
    residual to |meter| + |pv|, DESIGN.md "Parity"), NaN pattern and status equal;
  * n = 4,000 (not a multiple of 64 or 256: a partial last wavefront whose lanes
    past the last chain are parked at voff = 2^31 and must never record a
    guard-band second), fp32 and fp64, against the oracle;
  * statistics with n = 1,000 (the same partial wavefront in the OUT_STATS kernel);
  * the gated schedule (five contexts, two walks in flight, construction four
    batches ahead, the first walk in chain order, the rest in wind order, contexts
    reused) == one tmh_run (OUT_ANY) per batch, bit for bit.

Reference: /root/reference/tmhpvsim/pvmodel.py:62-80 (PV), metersim.py:49-51
(meter), pvsim.py:83 (residual).
"""
import numpy as np
import pytest

from oracle import oracle as O
from tmhpvsim_amd.params import ModelParams

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

START, TZ = "2019-09-05 00:00:00", "Europe/Berlin"
FIELDS = ("pv", "meter", "residual")


def _sim(n, prec, chain0=0, steps=86400, mp=None):
    from tmhpvsim_amd.engine import BatchedSim
    return BatchedSim(n, START, tz=TZ, params=mp or ModelParams(), precision=prec, chain0=chain0, device="cuda:0",
                      horizon=steps)


def _compare(out, ref, status, tol, block=1024):
    """every chain and second on the GPU: err of each field (DESIGN.md scales) <= tol,
    NaN exactly where the oracle has NaN (faulted chains)"""
    worst = dict.fromkeys(FIELDS, 0.0)
    n = status.shape[0]
    for c0 in range(0, n, block):
        c1 = min(n, c0 + block)
        r = {f: torch.from_numpy(np.ascontiguousarray(ref[f][:, c0:c1])).to("cuda:0") for f in FIELDS}
        g = {f: out[f][:, c0:c1].double() for f in FIELDS}
        for f in FIELDS:
            assert torch.equal(torch.isnan(g[f]), torch.isnan(r[f])), (f, c0)
        ok = torch.from_numpy(status[c0:c1] == 0).to("cuda:0")
        if not bool(ok.any()):
            continue
        g = {f: g[f][:, ok] for f in FIELDS}
        r = {f: r[f][:, ok] for f in FIELDS}
        errs = {
            "pv": (g["pv"] - r["pv"]).abs() / r["pv"].abs().clamp_min(1.0),
            "meter": (g["meter"] - r["meter"]).abs() / r["meter"].abs().clamp_min(1.0),
            "residual": (g["residual"] - r["residual"]).abs() / (r["meter"].abs() + r["pv"].abs()).clamp_min(1.0),
        }
        for f, e in errs.items():
            worst[f] = max(worst[f], float(e.max()))
    assert all(v <= tol for v in worst.values()), worst
    return worst


def _run_trace3(sim, steps=86400):
    from tmhpvsim_amd import _lib
    out = sim.run(steps, trace=FIELDS)
    torch.cuda.synchronize()
    want = _lib.OUT_TRACE3 | (_lib.OUT_FP64 if sim.real == torch.float64 else 0)
    assert sim.L.tmh_engine_last_expand(sim._eng) == want    # the bench's instantiation ran
    return out


@pytest.mark.parametrize("n,prec", [(4096, "fp32"), (4096, "fp64"), (4000, "fp32"), (4000, "fp64")])
def test_trace3_c2_day_vs_oracle(n, prec):
    """OUT_TRACE3 on the C2 day, every chain and second vs the oracle (keyed mode)."""
    mp = ModelParams()
    chain0 = 40960 + n                        # fresh global ids, as the bench's batches
    sim = _sim(n, prec, chain0=chain0)
    assert sim.path == "time_parallel"
    out = _run_trace3(sim)
    ref = O.run(mp, chain0, n, 86400, START, tz=TZ, n_threads=16, outputs=FIELDS)
    st = sim.status()
    np.testing.assert_array_equal(st, ref["status"])
    assert (st == 0).mean() > 0.99
    _compare(out, ref, st, 1e-12 if prec == "fp64" else 1e-5)


def test_trace3_equals_any_odd_count():
    """The OUT_TRACE3 and OUT_ANY instantiations of the fp32 expansion give the same
    pv / meter / residual bits, with 1,000 chains (a partial last wavefront)."""
    n = 1000
    a = _sim(n, "fp32", chain0=777)
    b = _sim(n, "fp32", chain0=777)
    ra = _run_trace3(a)
    rb = b.run(86400, trace=("csi",) + FIELDS)
    torch.cuda.synchronize()
    assert b.L.tmh_engine_last_expand(b._eng) == 0
    for f in FIELDS:
        assert torch.equal(torch.nan_to_num(ra[f], nan=-1.0), torch.nan_to_num(rb[f], nan=-1.0)), f
    np.testing.assert_array_equal(a.status(), b.status())


# histogram specs: the default; 21 kW in 2,048 bins (wider than [-300, 9000), still binned
# in fp32: the fp32 bin position's error bound 3.6e-4 bins); a 100 W range far from 0
# and a 500 kW range in 16,384 bins, both beyond the 1e-3-bin bound, so the fp32 kernel
# bins them in fp64 (StatsView::bin64, hist_bin)
HISTS = {"default": dict(n_bins=4096, lo=-300.0, hi=9000.0), "wide": dict(n_bins=2048, lo=-1000.0, hi=20000.0),
         "offset": dict(n_bins=1024, lo=4000.0, hi=4100.0), "huge": dict(n_bins=16384, lo=-2e5, hi=3e5)}


@pytest.mark.parametrize("spec", list(HISTS))
@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_stats_odd_count_vs_oracle(prec, spec):
    """OUT_STATS with 1,000 chains (a partial last wavefront: lanes past the last chain
    must not record guard-band seconds or touch another chain's corrections): per-chain
    energies, peak residual and the histogram against the oracle's statistics, for
    histogram ranges that bin in fp32 and ranges that fall back to fp64 binning.  The
    bin-edge tolerance is a residual tolerance in W (fp32 4.5e-3 W, fp64 2.3e-6 W) times
    the spec's bins per W."""
    from tmhpvsim_amd import _lib
    n = 1000
    hist = HISTS[spec]
    mp = ModelParams(seed=0x0DD)
    sim = _sim(n, prec, chain0=123, mp=mp)
    sim.enable_stats(**hist)
    sim.run(86400, trace=())
    torch.cuda.synchronize()
    assert sim.L.tmh_engine_last_expand(sim._eng) == _lib.OUT_STATS | (_lib.OUT_FP64 if prec == "fp64" else 0)
    amb = (2.3e-6 if prec == "fp64" else 4.5e-3) * hist["n_bins"] / (hist["hi"] - hist["lo"])
    ref = O.run(mp, 123, n, 86400, START, tz=TZ, n_threads=16, outputs=(), stats=dict(hist, amb_eps=amb))
    st = sim.status()
    np.testing.assert_array_equal(st, ref["status"])
    ok = st == 0
    acc = sim.chain_acc.cpu().numpy().T
    tol = 1e-12 if prec == "fp64" else 1e-5
    scale = np.abs(ref["acc"][ok, 1]) + np.abs(ref["acc"][ok, 0])
    for k in range(3):
        assert (np.abs(acc[ok, k] - ref["acc"][ok, k]) / scale).max() <= tol, k
    assert (np.abs(acc[ok, 3] - ref["acc"][ok, 3]) / 9000.0).max() <= tol
    assert np.isnan(acc[~ok, 0]).all() or (acc[~ok, :3] == 0).all()
    h, rh = sim.hist.cpu().numpy().astype(np.int64), ref["hist"].sum(0).astype(np.int64)
    assert h.sum() == rh.sum() == int(ok.sum()) * 86400
    assert np.abs(h - rh).sum() <= 2 * int(ref["amb"].sum())


def _same(a, b):
    return torch.equal(torch.nan_to_num(a, nan=-12345.0), torch.nan_to_num(b, nan=-12345.0))


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_bench_gated_schedule_equals_tmh_run(prec):
    """bench.py's C2 schedule as timed (BatchPipeline with pipeline_defaults("c2")):
    4,096 chains x 86,400 s per batch, eight batches through five contexts (batches 5-7
    reuse contexts 0-2 after their commit), two walks in flight, construction four
    batches ahead, the first walk in chain order and the rest in wind order, minute
    table and commit on the expansion stream.  Each context's last batch equals a
    separate tmh_run of the same chains (OUT_ANY: csi traced too) bit for bit."""
    from tmhpvsim_amd import _lib
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    n, secs = 4096, 86400
    cfg = pipeline_defaults("c2", prec)
    sim = _sim(n, prec)
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 1_000_000 + k * n, torch.device("cuda:0"))
    assert pipe.gated() and len(pipe.ctxs) == 5 and pipe.W == 2 and pipe.A == 4
    nb = 8
    pipe.run(0, nb)
    pipe.sync()
    assert sim.L.tmh_engine_last_expand(sim._eng) == _lib.OUT_TRACE3 | (_lib.OUT_FP64 if prec == "fp64" else 0)
    last = {k % len(pipe.ctxs): k for k in range(nb)}     # context -> the batch it holds
    for ci, k in sorted(last.items()):
        cx = pipe.ctxs[ci]
        assert cx.chain0 == 1_000_000 + k * n
        ref = _sim(n, prec, chain0=cx.chain0)
        r = ref.run(secs, trace=("csi",) + FIELDS)
        torch.cuda.synchronize()
        for f in FIELDS:
            assert _same(cx.trace[f], r[f]), (k, f)
        sim.state = cx.state
        np.testing.assert_array_equal(sim.status(), ref.status())
        del ref, r


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_gated_first_batch_split_equals_tmh_run(prec):
    """The gated schedule's first batch of each run as two half-day windows
    (`first_split=2`, a bench.py A/B option: the windows' walks chained through the
    previous window's scratch, their expansions in order, the second window's trace rows
    from row 43,200): two runs (batches 0-1, then 2-4), so batches 0 and 2 are split and
    batch 1 is not; each equals a separate tmh_run of the same chains bit for bit."""
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    n, secs = 4096, 86400
    cfg = pipeline_defaults("c2", prec, first_split=2)
    sim = _sim(n, prec)
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 3_000_000 + k * n, torch.device("cuda:0"))
    assert pipe.gated() and pipe.split == [(0, 43200), (43200, 43200)]
    pipe.run(0, 2)
    pipe.run(2, 3)
    pipe.sync()
    for k in (0, 1, 2):
        cx = pipe.ctxs[k]
        assert cx.chain0 == 3_000_000 + k * n
        ref = _sim(n, prec, chain0=cx.chain0)
        r = ref.run(secs, trace=("csi",) + FIELDS)
        torch.cuda.synchronize()
        for f in FIELDS:
            assert _same(cx.trace[f], r[f]), (k, f)
        sim.state = cx.state
        np.testing.assert_array_equal(sim.status(), ref.status())
        del ref, r


def test_stats_pipeline_c3_shape_equals_batches():
    """The stats schedule bench.py's C3 line runs (pipeline_defaults("c3"): two contexts,
    one walk in flight, so the staggered schedule: construction ahead on the expansion
    stream, the walk on the context's high-priority stream, the commit beside the next
    expansion) on 8,192 chains x one day, four batches: each context's accumulated
    per-chain statistics and histogram equal the sum of separate runs of its batches."""
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    n, secs = 8192, 86400
    cfg = pipeline_defaults("c3")
    assert cfg.mode == "stats" and cfg.pipeline == 2
    sim = _sim(n, "fp32")
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 5_000_000 + k * n, torch.device("cuda:0"))
    assert not pipe.gated()
    pipe.run(0, 4)
    pipe.sync()
    for ci, cx in enumerate(pipe.ctxs):
        acc = torch.zeros(4, n, dtype=torch.float64, device="cuda:0")
        acc[3].fill_(-float("inf"))
        hist = torch.zeros(4096, dtype=torch.int64, device="cuda:0")
        for k in (ci, ci + 2):
            s = _sim(n, "fp32", chain0=5_000_000 + k * n)
            s.enable_stats()
            s.run(secs, trace=())
            torch.cuda.synchronize()
            acc[:3] += s.chain_acc[:3]
            acc[3] = torch.maximum(acc[3], s.chain_acc[3])
            hist += s.hist
        assert torch.equal(cx.hist, hist), ci
        assert _same(cx.acc, acc), ci


def test_c4_shape_pipeline_equals_batches():
    """The multi-window schedule of bench.py's C4 line (pipeline_defaults("c4"): 30-day
    windows, each window's walk beside the previous window's expansion, batches on
    their contexts' streams) on 2,048 chains x 34 days from 2019-03-10 (a 30-day window
    across the DST spring-forward, then 4 days): per-chain statistics equal
    BatchedSim.run of the same chains."""
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    from tmhpvsim_amd.engine import BatchedSim
    n, secs, start = 2048, 34 * 86400, "2019-03-10 00:00:00"
    cfg = pipeline_defaults("c4", seconds=secs)
    assert cfg.window == 30 * 86400 and cfg.mode == "stats"
    sim = BatchedSim(n, start, tz=TZ, device="cuda:0", horizon=secs)
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 9_000_000 + k * n, torch.device("cuda:0"))
    pipe.run(0, len(pipe.ctxs))
    pipe.sync()
    for ci, cx in enumerate(pipe.ctxs):
        s = BatchedSim(n, start, tz=TZ, device="cuda:0", horizon=secs, chain0=9_000_000 + ci * n)
        s.enable_stats()
        s.run(secs, trace=(), window=cfg.window)   # the same windows (the fixed-point unit follows the window length)
        torch.cuda.synchronize()
        assert torch.equal(cx.hist, s.hist), ci
        assert _same(cx.acc, s.chain_acc), ci


def test_c5_shape_compacted_group_equals_batches():
    """bench.py's C5 schedule (pipeline_defaults("c5"): markov cc with per-site tables and
    sites, day windows compacted to the live chains) with three batches advanced window by
    window together (BatchPipeline.compact_batches: one host read of the live counts per
    window for the group, per-context chain ids set around each context's launches) ==
    BatchedSim.run(compact=True) of each batch alone: statistics and histogram bit for bit."""
    from tmhpvsim_amd.engine import BatchedSim
    from tmhpvsim_amd.params import CC_MARKOV, site_grid, site_shape_tables
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    n, secs, start = 512, 3 * 86400, "2019-09-05 00:00:00"
    mp = ModelParams(cc_mode=CC_MARKOV)
    kw = dict(shape_tables=site_shape_tables(n), sites=site_grid(32, 16))
    cfg = pipeline_defaults("c5", seconds=secs)
    assert cfg.compact and cfg.window == 86400
    sim = BatchedSim(n, start, tz=TZ, params=mp, device="cuda:0", horizon=secs, **kw)
    pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 7_000_000 + k * n, torch.device("cuda:0"))
    pipe.run(0, len(pipe.ctxs))
    pipe.sync()
    faulted = 0
    for ci, cx in enumerate(pipe.ctxs):
        s = BatchedSim(n, start, tz=TZ, params=mp, device="cuda:0", horizon=secs, chain0=7_000_000 + ci * n, **kw)
        s.enable_stats()
        s.run(secs, trace=(), window=86400, compact=True)
        torch.cuda.synchronize()
        faulted += int((s.status() != 0).sum())
        assert torch.equal(cx.hist, s.hist), ci
        assert _same(cx.acc, s.chain_acc), ci
    assert faulted > n // 4, "the test needs chains that fault (markov AssertionError)"


def test_pipelines_closed_in_turn_release_their_streams():
    """Lifecycle (round 6): a long-lived process builds pipelines in turn (the GPU test
    session, a pvsim service).  Each BatchPipeline owns dedicated CU-masked streams (a
    hardware queue each); `close()` / the context manager drains and releases them, so
    twelve pipelines built and closed one after another never hold more streams than
    one pipeline does, and the last pipeline's batches still equal tmh_run bit for bit.
    Reference: /root/reference/tmhpvsim/pvsim.py:86-101 (the long-lived process that owns
    the model)."""
    from tmhpvsim_amd import _lib
    from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults
    n, secs = 512, 3600
    cfg = pipeline_defaults("c2", "fp32", seconds=secs)
    sim = _sim(n, "fp32", steps=secs)
    base = _lib.live_streams()
    peak = per = 0
    for i in range(12):
        with BatchPipeline(sim, n, secs, cfg, lambda k, i=i: 20_000_000 + (i * 8 + k) * n, torch.device("cuda:0")) as pipe:
            assert pipe.gated()
            pipe.run(0, 6)
            pipe.sync()
            now = _lib.live_streams() - base
            per = per or now
            peak = max(peak, now)
            assert now > 0, "the dedicated queues are CU-masked streams"
            if i == 11:   # the last pipeline's batches against separate runs
                last = {k % len(pipe.ctxs): k for k in range(6)}
                for ci, k in sorted(last.items()):
                    cx = pipe.ctxs[ci]
                    ref = _sim(n, "fp32", chain0=cx.chain0, steps=secs)
                    r = ref.run(secs, trace=("csi",) + FIELDS)
                    torch.cuda.synchronize()
                    for f in FIELDS:
                        assert _same(cx.trace[f], r[f]), (k, f)
        assert _lib.live_streams() == base, "close() released every stream the pipeline created"
        with pytest.raises(RuntimeError, match="closed"):
            pipe.run(0, 1)
    assert peak == per, (peak, per)


def test_compacted_pipeline_closed_exits_cleanly(tmp_path):
    """Lifecycle: a compacted (C5-shape) pipeline copies each window's live count to pinned
    host memory on its context's stream; PyTorch's host allocator records an event on that
    stream when the buffer is freed.  close() frees those buffers before it releases the
    streams, so a process that closes its pipeline and exits ends with status 0 (round 6:
    bench.py --workload c5 printed its line, then aborted at exit with 'invalid resource
    handle').  Run in a child process: the failure is an abort at interpreter exit."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "c5_close.py"
    script.write_text(
        "import sys, torch\n"
        f"sys.path.insert(0, {root!r})\n"
        "from tmhpvsim_amd.engine import BatchedSim\n"
        "from tmhpvsim_amd.params import CC_MARKOV, ModelParams, site_grid, site_shape_tables\n"
        "from tmhpvsim_amd.pipeline import BatchPipeline, pipeline_defaults\n"
        "n, secs = 256, 2 * 86400\n"
        "kw = dict(shape_tables=site_shape_tables(n), sites=site_grid(16, 16))\n"
        "sim = BatchedSim(n, '2019-09-05 00:00:00', tz='Europe/Berlin', params=ModelParams(cc_mode=CC_MARKOV),\n"
        "                 device='cuda:0', horizon=secs, **kw)\n"
        "cfg = pipeline_defaults('c5', seconds=secs)\n"
        "pipe = BatchPipeline(sim, n, secs, cfg, lambda k: 9_000_000 + k * n, torch.device('cuda:0'))\n"
        "pipe.run(0, len(pipe.ctxs))\n"
        "pipe.sync()\n"
        "pipe.close()\n"
        "print('closed', flush=True)\n")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "closed" in r.stdout, (r.returncode, r.stderr[-2000:])
