"""Meter side (reference: tmhpvsim/metersim.py:49-51).

`get_meter_value()` keeps the reference's scalar API (9000 W x U[0, 1) from
numpy's global RandomState).  In batched runs the same draw is fused into the
chain kernel: meter = 9000 * U with U from the chain's keyed Philox stream
(its own stream, as metersim is its own process), residual = meter - pv
(pvsim.py:83) computed in the same kernel.
"""
import numpy as np


def get_meter_value():
    """Sample a single meter value from a uniform random distribution [0, 9000]"""
    return 9000 * np.random.random()
