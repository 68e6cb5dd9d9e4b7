"""TEST INFRASTRUCTURE ONLY — ctypes wrapper around oracle/liboracle.so.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, only
as the checker.  The calendar (local wall-clock fields per step) is built here
with pandas, exactly like the reference's callers build their times
(tests/test_clearskyindexmodel.py:8, pvmodel.py:45), independently of the
product's own clock arithmetic.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OrcParams(C.Structure):
    _fields_ = [
        ("cc_mode", C.c_int32), ("rng_mode", C.c_int32), ("seed", C.c_uint64),
        ("with_pv", C.c_int32), ("n_threads", C.c_int32),
        ("shapes", (C.c_double * 4) * 6), ("shape_is_t", C.c_int32 * 6), ("edges", C.c_double * 6),
        ("site", C.c_double * 8), ("linke", C.c_double * 12), ("module", C.c_double * 26),
        ("inverter", C.c_double * 9),
    ]


def build(force=False):
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "tmh_oracle.c")):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        d, p = C.c_double, C.c_void_p
        for name, args in [("orc_ndtri", [d]), ("orc_gammaincinv", [d, d]), ("orc_stdtrit", [d, d]),
                           ("orc_al_ppf", [d, d])]:
            getattr(L, name).restype = d
            getattr(L, name).argtypes = args
        L.orc_pv.restype = d
        L.orc_pv.argtypes = [p, C.c_int64, C.c_int, C.c_int, d]
        L.orc_geometry.argtypes = [p, C.c_int64, C.c_int, C.c_int, p]
        L.orc_solpos.argtypes = [C.c_int64, d, d, d, d, p, p, p]
        L.orc_constants.argtypes = [p]
        L.orc_philox.argtypes = [p, p, p]
        L.orc_run.restype = C.c_int
        L.orc_run.argtypes = [p, C.c_uint64, C.c_uint32, C.c_uint32, p, p, p, C.c_uint64,
                              p, p, p, p, p, p, p, p]
        L.orc_set_tables.argtypes = [p, p, C.c_uint32]
        L.orc_set_sites.argtypes = [p, p, C.c_uint32]
        L.orc_set_chain_ids.argtypes = [p, C.c_uint32]
        L.orc_injected_streams.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, p, C.c_int]
        L.orc_set_stats.argtypes = [p, p, p, C.c_uint32, C.c_double, C.c_double, C.c_double]
        _lib = L
    return _lib


def make_params(mp, n_threads=1):
    """tmhpvsim_amd.params.ModelParams-like object -> OrcParams."""
    P = OrcParams()
    P.cc_mode, P.rng_mode, P.seed = int(mp.cc_mode), int(mp.rng_mode), int(mp.seed)
    P.with_pv, P.n_threads = int(bool(mp.with_pv)), int(n_threads)
    sh = np.asarray(mp.shapes, dtype=np.float64)
    for i in range(6):
        for j in range(4):
            P.shapes[i][j] = sh[i, j]
        P.shape_is_t[i] = int(mp.shape_is_t[i])
        P.edges[i] = float(mp.edges[i])
    for i, v in enumerate(mp.site.as_array()):
        P.site[i] = v
    for i, v in enumerate(mp.linke):
        P.linke[i] = v
    for i, v in enumerate(mp.module_array()):
        P.module[i] = v
    for i, v in enumerate(mp.inverter_array()):
        P.inverter[i] = v
    return P


def calendar(start, n_steps, tz=None):
    """Local wall-clock fields for consecutive seconds, as the reference sees them.

    Returns cal int32 [n, 6] = (day, hour, minute, second, dayofyear, is_leap)
    and utc int64 [n] (unix seconds; naive times are taken as `tz` local or UTC).
    """
    import pandas as pd
    idx = pd.date_range(start, periods=n_steps, freq="s", tz=tz)
    cal = np.stack([idx.day, idx.hour, idx.minute, idx.second, idx.dayofyear,
                    idx.is_leap_year.astype(np.int32)], axis=1).astype(np.int32)
    if idx.tz is None:
        utc = (idx.asi8 // 10**9).astype(np.int64)
    else:
        utc = (idx.tz_convert("UTC").tz_localize(None).asi8 // 10**9).astype(np.int64)
    return np.ascontiguousarray(cal), np.ascontiguousarray(utc)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def run(mp, chain0, n_chains, n_steps, start, tz=None, inj=None, n_threads=1,
        outputs=("csi", "covered", "pv", "meter", "residual", "pos"), tables=None, sites=None, stats=None,
        chain_ids=None):
    """Run the oracle; returns dict of time-major [n_steps, n_chains] arrays + status/init.

    tables: optional per-chain shape tables (shapes [n_chains, 6, 4] float64,
    is_t [n_chains, 6] int32); chain c draws its hourly cloud cover from row c.
    sites: optional per-chain PV sites [n_chains, 8] (or (sites, linke [n_chains, 12])).
    stats: optional dict(n_bins, lo, hi, amb_eps): per-chain statistics of the good
    seconds as the GPU's stats mode keeps them -> res["acc"] [n, 4] (sum pv, sum
    meter, sum residual, max residual), res["hist"] [n, n_bins], res["amb"] [n].
    chain_ids: optional global ids [n_chains] (chain c is chain_ids[c], not chain0 + c)."""
    P = make_params(mp, n_threads)
    cal, utc = calendar(start, n_steps, tz)
    out = {}
    shapes = {"csi": np.float64, "covered": np.uint8, "pv": np.float64, "meter": np.float64,
              "residual": np.float64, "pos": np.uint32}
    for k, dt in shapes.items():
        out[k] = np.empty((n_steps, n_chains), dtype=dt) if k in outputs else None
    status = np.empty(n_chains, dtype=np.uint8)
    init = np.empty((n_chains, 16), dtype=np.float64)
    stride = 0
    if inj is not None:
        inj = np.ascontiguousarray(inj, dtype=np.float64)
        assert inj.shape[0] == n_chains
        stride = inj.shape[1]
    if tables is not None:
        tsh = np.ascontiguousarray(tables[0], dtype=np.float64)
        tit = np.ascontiguousarray(tables[1], dtype=np.int32)
        assert tsh.shape == (n_chains, 6, 4) and tit.shape == (n_chains, 6)
        lib().orc_set_tables(_ptr(tsh), _ptr(tit), n_chains)
    if sites is not None:
        ssi, sli = sites if isinstance(sites, tuple) else (sites, None)
        ssi = np.ascontiguousarray(ssi, dtype=np.float64)
        assert ssi.shape == (n_chains, 8)
        if sli is not None:
            sli = np.ascontiguousarray(sli, dtype=np.float64)
            assert sli.shape == (n_chains, 12)
        lib().orc_set_sites(_ptr(ssi), _ptr(sli), n_chains)
    ids = None
    if chain_ids is not None:
        ids = np.ascontiguousarray(chain_ids, dtype=np.uint64)
        assert ids.shape == (n_chains,)
        lib().orc_set_chain_ids(_ptr(ids), n_chains)
    if stats is not None:
        acc = np.zeros((n_chains, 4))
        hist = np.zeros((n_chains, int(stats["n_bins"])), dtype=np.uint64)
        amb = np.zeros(n_chains, dtype=np.uint64)
        lib().orc_set_stats(_ptr(acc), _ptr(hist), _ptr(amb), int(stats["n_bins"]), float(stats["lo"]),
                            float(stats["hi"]), float(stats.get("amb_eps", 0.0)))
    try:
        rc = lib().orc_run(C.byref(P), chain0, n_chains, n_steps, _ptr(cal), _ptr(utc), _ptr(inj), stride,
                           _ptr(out["csi"]), _ptr(out["covered"]), _ptr(out["pv"]), _ptr(out["meter"]),
                           _ptr(out["residual"]), _ptr(out["pos"]), _ptr(status), _ptr(init))
    finally:
        if tables is not None:
            lib().orc_set_tables(None, None, 0)
        if sites is not None:
            lib().orc_set_sites(None, None, 0)
        if stats is not None:
            lib().orc_set_stats(None, None, None, 0, 0.0, 1.0, 0.0)
        if ids is not None:
            lib().orc_set_chain_ids(None, 0)
    if rc != 0:
        raise RuntimeError(f"orc_run failed: {rc}")
    res = {k: v for k, v in out.items() if v is not None}
    res["status"], res["init"] = status, init
    if stats is not None:
        res["acc"], res["hist"], res["amb"] = acc, hist, amb
    return res


def injected_streams(seed, chain0, n_chains, length, n_threads=16):
    """[n_chains, length] injected uniforms (philox.injected_stream of chains chain0..), in C."""
    out = np.empty((n_chains, length), dtype=np.float64)
    lib().orc_injected_streams(int(seed), int(chain0), int(n_chains), int(length), _ptr(out), int(n_threads))
    return out


def ndtri(u):
    f = lib().orc_ndtri
    return np.array([f(float(x)) for x in np.ravel(u)]).reshape(np.shape(u))


def gammaincinv(a, u):
    f = lib().orc_gammaincinv
    return np.array([f(float(a), float(x)) for x in np.ravel(u)]).reshape(np.shape(u))


def stdtrit(df, u):
    f = lib().orc_stdtrit
    return np.array([f(float(df), float(x)) for x in np.ravel(u)]).reshape(np.shape(u))


def al_ppf(u, kappa):
    f = lib().orc_al_ppf
    return np.array([f(float(x), float(kappa)) for x in np.ravel(u)]).reshape(np.shape(u))


def constants():
    o = np.zeros(4)
    lib().orc_constants(_ptr(o))
    return o


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().orc_philox(_ptr(c), _ptr(k), _ptr(o))
    return o


def solpos(utc, lat, lon, pressure=100920.0, temp=12.0):
    z, az_, a = C.c_double(), C.c_double(), C.c_double()
    lib().orc_solpos(int(utc), lat, lon, pressure, temp, C.byref(z), C.byref(az_), C.byref(a))
    return z.value, az_.value, a.value
