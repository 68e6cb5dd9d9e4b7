"""The C-ABI library without a GPU: it loads, exports every entry point that
include/tmhpvsim.h declares, and its host-side logic (layout, validation)
behaves.  No compute calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from tmhpvsim_amd import _lib
from tmhpvsim_amd.params import ModelParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "tmhpvsim.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(tmh_\w+)\s*\(", src, re.M)))


def test_exports_every_declared_symbol():
    L = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 15, syms
    for s in syms:
        assert hasattr(L, s), f"{s} declared in include/tmhpvsim.h but not exported"
    assert set(syms) == set(_lib.EXPORTS)


def test_abi_version_and_layout():
    L = _lib.load()
    assert L.tmh_abi_version() == 1
    for n in (1, 63, 64, 4096, 1 << 20):
        off = _lib.state_offsets(n)
        total = L.tmh_state_bytes(n)
        assert (np.diff(off.astype(np.int64)) >= 0).all()
        assert all(int(o) % 256 == 0 for o in off)
        # sigma arrays hold CAP doubles per chain
        assert int(off[21]) - int(off[20]) >= 8 * n * _lib.TMH_SIGMA_CAP
        assert total >= int(off[21]) + 8 * n * _lib.TMH_SIGMA_CAP
    assert L.tmh_plan_bytes(86400) >= 86400 * 20 * 12
    assert L.tmh_workspace_bytes(4096, 86400) == L.tmh_plan_bytes(86400) + L.tmh_scratch_bytes(4096, 86400)
    # no engine: the bound that fits any engine (an fp32 engine's minute table is half of it)
    assert L.tmh_engine_scratch_bytes(None, 4096, 86400) == L.tmh_scratch_bytes(4096, 86400)
    # a day window's scratch per chain (DESIGN.md "Data layout"): under 70 KB at the fp64 bound
    assert L.tmh_scratch_bytes(1 << 20, 86400) < 70_000 * (1 << 20)


def test_engine_create_validates_before_touching_device():
    L = _lib.load()
    ck = _lib.Clock()
    eng = C.c_void_p()
    for field, bad in (("cc_mode", 7), ("rng_mode", 9), ("precision", 3), ("kernel_path", 5)):
        P = _lib.make_params(ModelParams(), 0)
        setattr(P, field, bad)
        rc = L.tmh_engine_create(C.byref(P), C.byref(ck), 0, C.byref(eng))
        assert rc == -1
        assert field in L.tmh_last_error().decode()
    ck.n_shifts = 99
    P = _lib.make_params(ModelParams(), 0)
    assert L.tmh_engine_create(C.byref(P), C.byref(ck), 0, C.byref(eng)) == -1
    assert L.tmh_engine_create(None, C.byref(ck), 0, C.byref(eng)) == -1


def test_null_arguments_rejected():
    L = _lib.load()
    assert L.tmh_init(None, None, 0, 1, None, None) == -1
    assert L.tmh_run(None, None, 0, 1, 0, 1, None, None, None, None, 0, None) == -1
    assert L.tmh_step(None, None, 0, 1, 0, 1, None, None, None, None, None, 0, None) == -1
    assert L.tmh_plan(None, 0, 1, None, None) == -1
    assert L.tmh_engine_path(None) == -1
    assert L.tmh_probe(0, 0.0, None, None, 1, None) == -1
    assert L.tmh_state_offsets(4, None) == -1
    assert L.tmh_set_shape_tables(None, None, None, 0) == -1
    assert L.tmh_set_sites(None, None, None, 0) == -1
    assert L.tmh_walk(None, None, 0, 1, 0, 1, None, None, 0, None) == -1
    assert L.tmh_expand(None, None, 0, 1, 0, 1, None, None, None, None, None, 0, None) == -1
    assert L.tmh_walk_part(None, None, 0, 1, 0, 1, None, None, 0, None, 0, 3, None) == -1
    assert L.tmh_walk_part(None, None, 0, 1, 0, 1, None, None, 0, None, 0, 8, None) == -1
    assert b"parts" in L.tmh_last_error()
    assert L.tmh_set_walk_lanes(None, 4) == -1
    assert L.tmh_set_walk_chains_per_row(None, 2) == -1


def test_params_struct_matches_header():
    # tmh_params: 6 int32 + u64 + 24 + 6 int32 + 6 + 8 + 12 + 26 + 9 doubles
    assert C.sizeof(_lib.Params) == 24 + 8 + 24 * 8 + 6 * 4 + 6 * 8 + 8 * 8 + 12 * 8 + 26 * 8 + 9 * 8
    assert C.sizeof(_lib.Clock) == 8 + 8 + 4 + 4 + 64 + 32


def test_no_cpu_fallback():
    from tmhpvsim_amd.engine import BatchedSim
    with pytest.raises(Exception):
        BatchedSim(4, "2019-09-05 00:00:00", device="cpu")


def test_loaded_library_carries_the_sources_stamp():
    """Provenance (round 6): the library exports the build stamp it was compiled with
    (tmh_build_stamp), build.lib_stamp reads it from the file, and it equals the stamp of
    the sources in the tree -- the loader refuses an in-tree library built from other
    sources, so a stale pushed binary can neither be tested nor benchmarked."""
    from tmhpvsim_amd import build
    _lib.load()
    assert _lib.loaded_stamp() == build.build_stamp() == build.lib_stamp()


def test_loader_refuses_a_stale_library(monkeypatch):
    from tmhpvsim_amd import build
    L = _lib.load()
    monkeypatch.delenv("TMHPVSIM_LIB", raising=False)
    monkeypatch.delenv("TMHPVSIM_ALLOW_STALE", raising=False)
    monkeypatch.setattr(build, "build_stamp", lambda: "0123456789abcdef")
    with pytest.raises(_lib.StaleLibraryError, match="other sources"):
        _lib._check_stamp(L)
    monkeypatch.setenv("TMHPVSIM_ALLOW_STALE", "1")
    _lib._check_stamp(L)   # diagnostics override
