#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the IMPORTED reference.

Build-container only (needs /root/reference); the fixtures are committed and
the reference never travels.  Run:  python tests/golden/make_golden.py

Every chain case drives the reference's own ClearskyindexModel
(tmhpvsim/clearskyindexmodel.py:57-160) through oracle/ref_harness.py with an
injected uniform stream (oracle/philox.py `injected_stream`, key = (seed, chain)),
so each fixture pins: per-second CSI, covered bit, stream position, every
next_cloud call (cloud_cover_binary.py:80-107) and every sampler push.

Function-level fixtures pin the variate mappings (scipy ndtri / gammaincinv /
stdtrit), the asymmetric-Laplace ppf (cloud_cover_hourly.py:100-104), cloud
lengths (cloud_cover_binary.py:25-40) and the loaded shape table bits
(cloud_cover_hourly.py:278-288).
"""
from __future__ import annotations

import json
import os
import platform
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.philox import injected_stream  # noqa: E402
from oracle.ref_harness import Harness, SAMPLERS  # noqa: E402

SEED = 0x5EED


def pack_chains(logs, n_steps):
    """Stack per-chain logs into fixed arrays + flattened event tables."""
    n = len(logs)
    csi = np.full((n, n_steps), np.nan)
    covered = np.full((n, n_steps), 255, dtype=np.uint8)
    sec = np.full((n, n_steps), -1, dtype=np.int32)
    pos = np.full((n, n_steps), -1, dtype=np.int64)
    calls, pushes, err, err_step = [], [], [], []
    init_samplers = np.full((n, 6, 2), np.nan)
    init_bin = np.full((n, 4), np.nan)     # sec, cloud_length, clear_length, pos
    sig_c = np.full((n, 64), np.nan)
    sig_l = np.full((n, 64), np.nan)
    for c, lg in enumerate(logs):
        k = len(lg.csi)
        csi[c, :k] = lg.csi
        covered[c, :k] = lg.covered
        sec[c, :k] = lg.sec
        pos[c, :k] = lg.pos[:k]
        for row in lg.calls:
            calls.append((c,) + tuple(row))
        for row in lg.pushes:
            pushes.append((c,) + tuple(row))
        err.append(lg.error)
        err_step.append(lg.error_step)
        if lg.init:
            init_samplers[c] = lg.init["samplers"]
            init_bin[c] = (lg.init["sec"], lg.init["cloud_length"], lg.init["clear_length"], lg.init["pos"])
            L = len(lg.init["sigma_cloud"])
            sig_c[c, :L] = lg.init["sigma_cloud"]
            sig_l[c, :L] = lg.init["sigma_clear"]
        elif lg.pos:
            init_bin[c, 3] = lg.pos[-1]
    return dict(
        csi=csi, covered=covered, sec=sec, pos=pos,
        # next_cloud calls: chain, step, pos_before, pos_after, h, ws, L_before, cl, clr, L_after
        calls=np.array(calls, dtype=np.float64).reshape(-1, 10),
        # sampler pushes: chain, step, sampler id (SAMPLERS order), new `after`
        pushes=np.array(pushes, dtype=np.float64).reshape(-1, 4),
        error=np.array(err), error_step=np.array(err_step, dtype=np.int64),
        init_samplers=init_samplers, init_bin=init_bin,
        init_sigma_cloud=sig_c, init_sigma_clear=sig_l,
    )


def times_for(start, n, tz=None):
    import pandas as pd
    return pd.date_range(start, periods=n, freq="s", tz=tz).to_pydatetime()


def chain_case(h, name, start, n_steps, chains, tz=None, markov=False, streams=None):
    times = times_for(start, n_steps, tz)
    logs = []
    for i, c in enumerate(chains):
        u = streams[i] if streams is not None else injected_stream(SEED, c, int(n_steps * 1.1) + 400)
        logs.append(h.run_chain(times, u, markov=markov))
    d = pack_chains(logs, n_steps)
    d["chains"] = np.array(chains, dtype=np.int64)
    d["n_steps"] = np.int64(n_steps)
    d["seed"] = np.int64(SEED)
    d["start"] = np.array(start)
    d["tz"] = np.array(tz or "")
    d["markov"] = np.bool_(markov)
    if streams is not None:
        d["streams"] = np.array(streams, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **d)
    bad = [e for e in d["error"] if e]
    print(f"{name}: chains={len(chains)} steps={n_steps} calls={len(d['calls'])} "
          f"pushes={len(d['pushes'])} errors={bad}")


def functions_case(h):
    from scipy import special
    u = injected_stream(SEED, 999, 4000)
    tails = np.array([2.0 ** -53, 1e-300, 1e-100, 1e-30, 1e-16, 1e-10, 1e-5, 1e-3, 0.02425,
                      0.1, 0.3, 0.5, 0.5 + 2 ** -40, 0.7, 0.97575, 0.999, 1 - 1e-10, 1 - 2.0 ** -53])
    u = np.concatenate([tails, u])
    dists, edges = h.distributions()
    df = dists[2, 3]
    out = dict(
        u=u,
        ndtri=special.ndtri(u),
        gammaincinv_269=special.gammaincinv(2.69, u),
        gammaincinv_35624=special.gammaincinv(3.5624, u),
        stdtrit_bin2=special.stdtrit(df, u),
        shapes=dists, edges=edges,
        al_ppf=np.stack([h.al_ppf(u, dists[b, 2]) if b != 2 else np.full_like(u, np.nan)
                         for b in range(6)]),
    )
    ws = np.abs(injected_stream(SEED, 998, 512)) * 15 + 0.05
    uc = injected_stream(SEED, 997, 512)
    out["cl_ws"], out["cl_u"] = ws, uc
    out["cloudlength"] = h.cloudlength(ws, uc)
    # standalone hourly Markov chain get_cloud_cover (markov-mode transition reference)
    chains_u = [injected_stream(SEED, 900 + k, 2048) for k in range(16)]
    states, used = [], []
    for uu in chains_u:
        s, p = h.cloud_cover_chain(uu, 2000)
        states.append(s)
        used.append(p)
    out["mc_states"] = np.array(states)
    out["mc_used"] = np.array(used)
    out["mc_chain_ids"] = np.arange(900, 916)
    np.savez_compressed(os.path.join(HERE, "functions.npz"), **out)
    print("functions: ok", out["mc_states"].shape)


def crafted_streams():
    """Streams that drive the reference into its two fault branches."""
    base = injected_stream(SEED, 77, 1200)
    # NameError (clearskyindexmodel.py:72-80): both cc init draws with
    # AL(u) * scale5 + loc5 in [-0.25, -0.125)  ->  u ~ 1e-5 (bin 5, kappa 2.2375)
    name_err = base.copy()
    name_err[0] = name_err[1] = 1e-5
    # AssertionError (cloud_cover_binary.py:90-98): cc < 1/12 -> int(12 h) == 0
    # -> empty sigma -> 20 + 20 rejected tries.  u = 1e-30 gives cc ~ 0.027.
    assert_err = base.copy()
    assert_err[0] = assert_err[1] = 1e-30
    # low-cover N(0.6784, 0.2046) branch (c < 0.75), no fault: u ~ 1e-12
    low = base.copy()
    low[0] = low[1] = 1e-12
    return [name_err, assert_err, low]


def main():
    h = Harness()
    meta = dict(
        generator="tests/golden/make_golden.py", reference="/root/reference (coroa/tmhpvsim)",
        cpu=platform.processor() or platform.machine(), python=platform.python_version(),
        numpy=np.__version__, seed=SEED, samplers=SAMPLERS,
    )
    import scipy
    import pandas
    meta["scipy"], meta["pandas"] = scipy.__version__, pandas.__version__
    try:
        with open("/proc/cpuinfo") as f:
            meta["cpu"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    functions_case(h)
    chain_case(h, "faithful_2h", "2019-09-05 00:00:00", 7200, list(range(8)))
    chain_case(h, "faithful_midnight", "2019-09-05 23:00:00", 7200, [8, 9, 10, 11])
    chain_case(h, "faithful_25h", "2019-09-05 12:00:00", 90001, [12, 13])
    chain_case(h, "dst_fall", "2019-10-27 01:30:00", 9000, [14, 15], tz="Europe/Berlin")
    chain_case(h, "dst_spring", "2019-03-31 01:30:00", 3600, [16, 17], tz="Europe/Berlin")
    chain_case(h, "faults", "2019-09-05 10:00:00", 600, [77, 78, 79], streams=crafted_streams())
    chain_case(h, "markov_6h", "2019-09-05 06:00:00", 21600, [20, 21, 22, 23], markov=True)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
