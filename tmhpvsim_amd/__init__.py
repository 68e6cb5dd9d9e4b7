"""tmhpvsim_amd — MI355X-native batched simulator of tmhpvsim's clear-sky-index
chain and PV model.

    from tmhpvsim_amd import BatchedSim, ClearskyindexModel, PVModel, get_meter_value

The compute path is libtmhpvsim.so (HIP, gfx950) behind include/tmhpvsim.h.
The drop-in names resolve lazily, so importing the package
loads neither torch nor the library.
"""
import importlib

from .params import ModelParams, Site  # noqa: F401

__version__ = "0.1.0"

# name -> submodule that defines it (the reference's module in brackets)
_EXPORTS = {
    "BatchedSim": "engine",
    "ClearskyindexModel": "clearskyindexmodel",   # tmhpvsim.clearskyindexmodel
    "InterpolatedSampler": "clearskyindexmodel",
    "Time": "clearskyindexmodel",
    "PVModel": "pvmodel",                         # tmhpvsim.pvmodel
    "get_meter_value": "metersim",                # tmhpvsim.metersim
    "random_windspeed": "cloud_cover_binary",     # tmhpvsim.cloud_cover_binary
    "random_cloudlength_in_s": "cloud_cover_binary",
    "CloudCoverBinary": "cloud_cover_binary",
    "get_cloud_cover": "cloud_cover_hourly",      # tmhpvsim.cloud_cover_hourly
    "get_distributions_from_shapes": "cloud_cover_hourly",
    "get_distributions_from_shapes_file": "cloud_cover_hourly",
    "asymmetric_laplace": "cloud_cover_hourly",
}

__all__ = ["ModelParams", "Site"] + sorted(_EXPORTS)


def __getattr__(name):
    mod = _EXPORTS.get(name)
    if mod is None:
        raise AttributeError(f"module 'tmhpvsim_amd' has no attribute {name!r}")
    return getattr(importlib.import_module(f".{mod}", __name__), name)


def __dir__():
    return sorted(set(globals()) | set(_EXPORTS))
