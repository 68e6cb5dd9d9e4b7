"""TEST INFRASTRUCTURE ONLY — numpy restatement of Philox4x32-10 (Random123).

Pinned by the Random123 known-answer vectors listed in SURVEY.md App. B
(checked in tests/test_oracle_philox.py).

Uniform conversion (shared contract with the HIP kernels and the C oracle,
see DESIGN.md "Random numbers"): a 64-bit value v = (hi << 32) | lo maps to

    u = (2 * (v >> 12) + 1) * 2**-53        in (0, 1), exact in fp64,

i.e. the midpoint of one of 2**52 equal cells; never 0, never 1.

Streams
-------
* injected stream (config C2): uniform k of chain c is half (k & 1) of
  philox(ctr=(k >> 1 lo32, k >> 1 hi32, 0, 0), key=(seed, c)).
* keyed mode: philox(ctr=(step, tag << 28 | sub, chain lo32, chain hi32),
  key=(seed lo32, seed hi32)); each block gives two uniforms (halves).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# keyed-mode draw families (ctr1 = tag << 28 | sub)
TAG_STEP = 1        # injected-mode bookkeeping only (per-second draws are TAG_METER4 / TAG_NOISE4)
TAG_BOUNDARY = 2    # sub 0 day (clear_day, ws), 1 hour (cc, clear_day), 2 minute (cloudy, clear noise)
TAG_CLOUD = 3       # ctr0 = next_cloud call number (0 = ctor), sub = try >> 1, half = try & 1
TAG_INIT = 4        # step 0, sub = draw >> 1, half = draw & 1 (14 ctor draws)
TAG_INIT_CLOUD = 5  # ctor next_cloud (call 0): ctr0 = 0, sub = try >> 1, half = try & 1
TAG_INIT_SEC = 6    # ctor start offset draw: sub 0, half 0
TAG_METER4 = 8      # per-second meter draws: ctr0 = step >> 2, word step & 3; u = (w + 1/2) 2^-32
TAG_NOISE4 = 9      # per-second noise draws: the same layout (a night second draws no noise word)


def philox4x32_10(ctr, key):
    """Vectorised Philox4x32-10.  ctr: (..., 4) uint32, key: (..., 2) uint32."""
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    x0 = ctr[..., 0].astype(np.uint64)
    x1 = ctr[..., 1].astype(np.uint64)
    x2 = ctr[..., 2].astype(np.uint64)
    x3 = ctr[..., 3].astype(np.uint64)
    k0 = key[..., 0].astype(np.uint64)
    k1 = key[..., 1].astype(np.uint64)
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(W0)) & MASK32
            k1 = (k1 + np.uint64(W1)) & MASK32
        p0 = M0 * x0
        p1 = M1 * x2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        x0 = hi1 ^ x1 ^ k0
        x1 = lo1
        x2 = hi0 ^ x3 ^ k1
        x3 = lo0
    return np.stack([x0, x1, x2, x3], axis=-1).astype(np.uint32)


def u52(lo, hi):
    """(lo, hi) uint32 pair -> fp64 uniform (2*(v>>12)+1) * 2**-53."""
    v = (np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)
    k = (v >> np.uint64(11)) | np.uint64(1)
    return k.astype(np.float64) * 2.0 ** -53


def block_uniforms(blocks):
    """(..., 4) uint32 philox output -> (..., 2) fp64 uniforms (two halves)."""
    b = np.asarray(blocks, dtype=np.uint32)
    return np.stack([u52(b[..., 0], b[..., 1]), u52(b[..., 2], b[..., 3])], axis=-1)


def injected_stream(seed: int, chain: int, n: int) -> np.ndarray:
    """First n uniforms of the injected stream of `chain` (key = (seed, chain))."""
    nb = (n + 1) // 2
    blk = np.arange(nb, dtype=np.uint64)
    ctr = np.zeros((nb, 4), dtype=np.uint32)
    ctr[:, 0] = (blk & MASK32).astype(np.uint32)
    ctr[:, 1] = (blk >> np.uint64(32)).astype(np.uint32)
    key = np.array([seed & 0xFFFFFFFF, chain & 0xFFFFFFFF], dtype=np.uint32)
    out = block_uniforms(philox4x32_10(ctr, np.broadcast_to(key, (nb, 2))))
    return out.reshape(-1)[:n].copy()


def keyed_uniform(seed: int, chain, step, tag: int, sub, half):
    """Keyed-mode uniform(s); chain/step/sub/half broadcast."""
    chain = np.asarray(chain, dtype=np.uint64)
    step = np.asarray(step, dtype=np.uint64)
    sub = np.asarray(sub, dtype=np.uint64)
    half = np.asarray(half)
    chain, step, sub, half = np.broadcast_arrays(chain, step, sub, half)
    ctr = np.zeros(chain.shape + (4,), dtype=np.uint32)
    ctr[..., 0] = (step & MASK32).astype(np.uint32)
    ctr[..., 1] = ((np.uint64(tag) << np.uint64(28)) | (sub & np.uint64(0x0FFFFFFF))).astype(np.uint32)
    ctr[..., 2] = (chain & MASK32).astype(np.uint32)
    ctr[..., 3] = (chain >> np.uint64(32)).astype(np.uint32)
    key = np.empty(chain.shape + (2,), dtype=np.uint32)
    key[..., 0] = seed & 0xFFFFFFFF
    key[..., 1] = (seed >> 32) & 0xFFFFFFFF
    u = block_uniforms(philox4x32_10(ctr, key))
    return np.where(half == 0, u[..., 0], u[..., 1])
