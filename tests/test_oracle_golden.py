"""The C oracle against the reference's own outputs (golden fixtures).

Pins oracle/tmh_oracle.c to the imported reference (tests/golden/make_golden.py):
discrete state (covered bit, stream position = uniforms consumed, fault
status) bit-exact; continuous CSI <= 1e-12 relative (observed ~1e-15: the
reference's numpy SIMD log/pow differ from glibc by an ulp).
"""
import numpy as np
import pytest

from golden_util import CHAIN_CASES, load, streams
from oracle import oracle as O
from tmhpvsim_amd.params import CC_MARKOV, RNG_INJECTED, SHAPES, ModelParams

FAULT_CODE = {"": 0, "NameError": 1, "AssertionError": 2}


@pytest.mark.parametrize("case", CHAIN_CASES)
def test_chain_fixture(case):
    d = load(case)
    n, chains = int(d["n_steps"]), d["chains"]
    mp = ModelParams(rng_mode=RNG_INJECTED, cc_mode=CC_MARKOV if bool(d["markov"]) else 0,
                     with_pv=False)
    r = O.run(mp, 0, len(chains), n, str(d["start"]), tz=str(d["tz"]) or None, inj=streams(d))
    ok = np.isfinite(d["csi"])
    csi, cov, pos = r["csi"].T, r["covered"].T, r["pos"].T.astype(np.int64)
    np.testing.assert_array_equal(np.isnan(csi), ~ok)
    np.testing.assert_array_equal(cov[ok], d["covered"][ok])
    np.testing.assert_array_equal(pos[ok], d["pos"][ok])
    rel = np.abs(csi[ok] - d["csi"][ok]) / np.abs(d["csi"][ok])
    assert rel.max(initial=0) <= 1e-12
    assert [FAULT_CODE[str(e)] for e in d["error"]] == list(r["status"])
    # constructor state: samplers + binary (sec exact, lengths 1e-12)
    good = r["status"] == 0
    np.testing.assert_allclose(r["init"][good, :12], d["init_samplers"].reshape(-1, 12)[good], rtol=1e-12)
    np.testing.assert_array_equal(r["init"][good, 12], d["init_bin"][good, 0])
    np.testing.assert_allclose(r["init"][good, 13:15], d["init_bin"][good, 1:3], rtol=1e-12)


def test_reference_invariant_range():
    """tests/test_clearskyindexmodel.py:13 — 0 < csi < 2 over 25 h (keyed mode, 64 chains)."""
    r = O.run(ModelParams(with_pv=False), 0, 64, 90001, "2019-09-05 12:00:00", n_threads=4,
              outputs=("csi",))
    assert (r["status"] == 0).all()
    assert (r["csi"] > 0).all() and (r["csi"] < 2).all()


def test_functions_fixture():
    F = load("functions")
    u = F["u"]
    np.testing.assert_array_equal(np.nan_to_num(F["shapes"][:, :4]), np.nan_to_num(np.array(SHAPES)))
    np.testing.assert_array_equal(F["edges"], [0.1, 0.3, 0.7, 0.9, 0.99, 1.0])
    np.testing.assert_allclose(O.ndtri(u), F["ndtri"], rtol=1e-14, atol=0)
    np.testing.assert_allclose(O.gammaincinv(2.69, u), F["gammaincinv_269"], rtol=1e-13)
    np.testing.assert_allclose(O.gammaincinv(3.5624, u), F["gammaincinv_35624"], rtol=1e-13)
    # scipy's stdtrit itself is only ~1e-11 accurate (CDF residual 1.6e-12); the
    # oracle's is ~1e-16 — compare at 1e-9 inside the range our uniforms reach.
    m = (u >= 2.0 ** -53) & (np.abs(u - 0.5) > 1e-6)
    np.testing.assert_allclose(O.stdtrit(SHAPES[2][3], u[m]), F["stdtrit_bin2"][m], rtol=1e-9)
    for b in (0, 1, 3, 4, 5):
        np.testing.assert_allclose(O.al_ppf(u, SHAPES[b][2]), F["al_ppf"][b], rtol=1e-14)
    alpha, delta, expo, s6 = O.constants()
    assert alpha == float.fromhex("0x1.cbe5732814218p-14")
    assert delta == float.fromhex("0x1.87320eb153222p-5")
    assert expo == -1.5151515151515154 and s6 == 2.449489742783178
    cl = (alpha + delta * F["cl_u"]) ** expo / F["cl_ws"]
    np.testing.assert_allclose(cl, F["cloudlength"], rtol=1e-14)


def test_standalone_markov_chain():
    """get_cloud_cover (cloud_cover_hourly.py:290-316) as a 6-bin chain: oracle draw_cc
    restated in numpy on the same streams reproduces the reference's hourly states."""
    from oracle.philox import injected_stream
    F = load("functions")
    edges = np.array([0.1, 0.3, 0.7, 0.9, 0.99, 1.0])
    for k, cid in enumerate(F["mc_chain_ids"]):
        u = injected_stream(0x5EED, int(cid), 2048)
        ref = F["mc_states"][k]
        state, out = 1.0, []
        for i in range(len(ref)):
            b = int(np.searchsorted(edges, state))
            loc, scale, kap, df = SHAPES[b]
            v = O.stdtrit(df, u[i]) if b == 2 else O.al_ppf(u[i], kap)
            state = min(max(state + (float(v) * scale + loc), 0.0), 1.0)
            out.append(state)
        # scipy stdtrit's ~1e-11 error is carried along the chain: absolute gate,
        # plus the discrete bin sequence exactly.
        np.testing.assert_allclose(out, ref, rtol=0, atol=5e-11)
        np.testing.assert_array_equal(np.searchsorted(edges, out), np.searchsorted(edges, ref))


def test_fast_clock_fractions_are_exact():
    """The device's division-free wall-clock fractions equal the reference's
    IEEE divisions (clearskyindexmodel.py:114-116) for all 86,400 seconds."""
    import ctypes as C
    from oracle import oracle as O
    f = O.lib().orc_check_fractions
    f.restype = C.c_int
    assert f() == 0
