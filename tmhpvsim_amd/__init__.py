"""tmhpvsim_amd — MI355X-native batched simulator of tmhpvsim's clear-sky-index
chain and PV model.

    from tmhpvsim_amd import BatchedSim, ClearskyindexModel, PVModel

The compute path is libtmhpvsim.so (HIP, gfx950) behind include/tmhpvsim.h.
"""
from .params import ModelParams, Site  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    if name == "BatchedSim":
        from .engine import BatchedSim
        return BatchedSim
    if name == "ClearskyindexModel":
        from .clearskyindexmodel import ClearskyindexModel
        return ClearskyindexModel
    if name == "PVModel":
        from .pvmodel import PVModel
        return PVModel
    raise AttributeError(name)
