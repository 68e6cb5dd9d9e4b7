"""Shared loaders for the golden fixtures (tests/golden/*.npz)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CHAIN_CASES = ["faithful_2h", "faithful_midnight", "faithful_25h", "dst_fall", "dst_spring",
               "faults", "markov_6h"]


def load(case):
    return dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))


def streams(d):
    """Injected uniform streams [chains, n] for a chain fixture."""
    from oracle.philox import injected_stream
    if "streams" in d:
        return np.asarray(d["streams"], dtype=np.float64)
    n = int(d["n_steps"])
    return np.stack([injected_stream(int(d["seed"]), int(c), int(n * 1.1) + 400) for c in d["chains"]])
