#!/usr/bin/env python3
"""Generate tests/golden/stats_seeded.npz: statistics of the IMPORTED reference
running in its own seeded mode (numpy's global legacy RandomState, np.random.seed),
the fixture that pins the keyed (Philox) mode statistically.

Build-container only (needs /root/reference; the reference never travels).
Run:  python tests/golden/make_stats.py   (about 2 minutes on 8 cores)

Each chain c is one reference ClearskyindexModel (tmhpvsim/clearskyindexmodel.py:57)
driven with .next(t) (:128) for one day at 1 s from 2019-09-05 00:00 (local wall
clock, as tests/test_clearskyindexmodel.py:8 builds its times), after
np.random.seed(BASE + c).  Only the reference's own code and RNG run here; the
offline-fitting modules are stubbed as in oracle/ref_harness.py.

Stored per chain: the covered bit as run lengths, the CSI of second 30 of every
minute, the hourly cloud cover draws (cloudcover_hour.after after each hour change).
"""
from __future__ import annotations

import datetime as dt
import json
import multiprocessing as mp
import os
import platform
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

N_CHAINS = 256
BASE = 20190905
START = dt.datetime(2019, 9, 5, 0, 0, 0)
N_STEPS = 86400


def one_chain(c):
    from oracle.ref_harness import import_reference
    csm, _, _ = import_reference()
    np.random.seed(BASE + c)
    try:
        model = csm.ClearskyindexModel(START)
    except NameError:   # the construction quirk at clearskyindexmodel.py:72-80 (p ~ 2.6e-5)
        return None
    cov = np.empty(N_STEPS, dtype=np.uint8)
    csi_min = np.empty(N_STEPS // 60)
    cc = []
    last_hour = START.hour
    for s in range(N_STEPS):
        t = START + dt.timedelta(seconds=s)
        v = model.next(t)
        # covered: CloudCoverBinary.__next__ returned 1 (clearskyindexmodel.py:137)
        b = model.cloudcover_binary
        cov[s] = 1 if b.sec < b.cloud_length else 0
        if s % 60 == 30:
            csi_min[s // 60] = v
        if t.hour != last_hour:
            cc.append(model.cloudcover_hour.after)
            last_hour = t.hour
    # run-length encode the covered bits
    change = np.flatnonzero(np.diff(cov.astype(np.int8))) + 1
    starts = np.r_[0, change]
    lens = np.diff(np.r_[starts, N_STEPS])
    return cov[0], lens.astype(np.int32), csi_min, np.asarray(cc)


def main():
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        res = [r for r in pool.map(one_chain, range(N_CHAINS)) if r is not None]
    first = np.array([r[0] for r in res], dtype=np.uint8)
    nrun = np.array([len(r[1]) for r in res], dtype=np.int32)
    runs = np.concatenate([r[1] for r in res])
    csi = np.stack([r[2] for r in res])
    cc = np.concatenate([r[3] for r in res])
    out = os.path.join(HERE, "stats_seeded.npz")
    np.savez_compressed(out, first=first, nrun=nrun, runs=runs, csi_min=csi, cc_hourly=cc,
                        n_steps=N_STEPS, start=str(START))
    meta = {"generator": "tests/golden/make_stats.py", "reference": "/root/reference (coroa/tmhpvsim)",
            "rng": "numpy legacy RandomState, np.random.seed(%d + chain)" % BASE, "chains": N_CHAINS,
            "cpu": platform.processor() or platform.machine(), "python": platform.python_version(),
            "numpy": np.__version__}
    json.dump(meta, open(os.path.join(HERE, "stats_seeded.json"), "w"), indent=1)
    print(out, runs.size, "runs", cc.size, "hourly cc")


if __name__ == "__main__":
    main()
