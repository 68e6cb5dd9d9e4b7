"""Philox4x32-10 known-answer tests (Random123 KATs) for both
the numpy restatement and the C oracle, plus the uniform-conversion contract."""
import numpy as np

from oracle import oracle as O
from oracle.philox import injected_stream, keyed_uniform, philox4x32_10, u52

KATS = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def test_kats_numpy_and_c():
    for ctr, key, exp in KATS:
        assert list(philox4x32_10(ctr, key)) == exp
        assert list(O.philox(ctr, key)) == exp


def test_u52_range_and_exactness():
    assert u52(0, 0) == 2.0 ** -53
    assert u52(0xFFFFFFFF, 0xFFFFFFFF) == 1.0 - 2.0 ** -53
    u = injected_stream(0x5EED, 0, 10000)
    assert (u > 0).all() and (u < 1).all()
    k = u * 2.0 ** 53
    assert np.array_equal(k, np.round(k)) and (k % 2 == 1).all()


def test_keyed_distinct_families():
    a = keyed_uniform(1, 5, 10, 1, 0, 0)
    b = keyed_uniform(1, 5, 10, 2, 0, 0)
    c = keyed_uniform(1, 6, 10, 1, 0, 0)
    assert len({float(a), float(b), float(c)}) == 3
