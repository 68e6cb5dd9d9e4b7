#!/usr/bin/env python3
"""Generate tests/golden/shims.npz from the IMPORTED reference (build container only).

Pins the host-side helper shims (tmhpvsim_amd.cloud_cover_binary /
cloud_cover_hourly) against the reference's own functions run in their own
seeded mode (numpy's legacy global RandomState): random_windspeed,
random_cloudlength_in_s (cloud_cover_binary.py:5-40), CloudCoverBinary driven
second by second with hourly parameter updates (:42-117), the loaded shape
table's distributions and get_cloud_cover's chain (cloud_cover_hourly.py:93-106,
269-316).  Run:  python tests/golden/make_shims.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.ref_harness import import_reference  # noqa: E402

# hourly (cover, wind speed) schedule of the CloudCoverBinary case
SCHEDULE = [(0.9, 3.1), (0.55, 6.0), (0.95, 1.2), (0.3, 9.5), (1.0, 2.4), (0.7, 4.4)]
STEPS_PER_HOUR = 3600


def main():
    _, ccb, cch = import_reference()
    out = {}
    np.random.seed(11)
    out["windspeed"] = np.array([ccb.random_windspeed() for _ in range(500)])
    np.random.seed(12)
    out["cloudlength_1"] = np.array([ccb.random_cloudlength_in_s(3.0)[0] for _ in range(500)])
    out["cloudlength_5"] = ccb.random_cloudlength_in_s(2.5, shape=(5,))
    np.random.seed(13)
    b = ccb.CloudCoverBinary(*SCHEDULE[0])
    out["ccb_init"] = np.array([b.sec, float(np.ravel(b.cloud_length)[0]), float(b.clear_length)])
    bits, lengths = [], []
    for h, (cc, ws) in enumerate(SCHEDULE):
        b.update_parameters(cc, ws)
        for _ in range(STEPS_PER_HOUR):
            bits.append(next(b))
        lengths.append((float(np.ravel(b.cloud_length)[0]), float(b.clear_length), b.sec, len(b.sigma_cloud)))
    out["ccb_bits"] = np.array(bits, dtype=np.uint8)
    out["ccb_lengths"] = np.array(lengths)
    out["ccb_sigma_cloud"] = np.asarray(b.sigma_cloud, dtype=np.float64)
    out["ccb_sigma_clear"] = np.asarray(b.sigma_clear, dtype=np.float64)
    d = cch.get_distributions_from_shapes_file()
    out["edges"] = np.array([iv.right for iv in d.index])
    x = np.linspace(-0.3, 0.3, 61)
    out["al_pdf"] = cch.asymmetric_laplace.pdf(x, 1.3)
    out["al_ppf"] = cch.asymmetric_laplace.ppf(np.linspace(0.01, 0.99, 99), 1.3)
    np.random.seed(14)
    g = cch.get_cloud_cover(d)
    out["cc_chain"] = np.array([next(g) for _ in range(3000)])
    np.random.seed(15)
    g = cch.get_cloud_cover(d, initial_state=0.45)
    out["cc_chain_045"] = np.array([next(g) for _ in range(500)])
    np.savez(os.path.join(HERE, "shims.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
