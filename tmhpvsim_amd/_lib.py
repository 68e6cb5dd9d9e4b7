"""ctypes binding of libtmhpvsim.so (include/tmhpvsim.h).

The shared library is built in-tree (tmhpvsim_amd/build.py, driven by
__graft_entry__.build()).  There is no CPU fallback: if the library is
missing or fails to load, every compute entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMHPVSIM_LIB") or os.path.join(HERE, "libtmhpvsim.so")

TMH_ABI_VERSION = 1
TMH_SIGMA_CAP = 512
TMH_GEOM_FIELDS = 22
TMH_STATE_NFIELDS = 24
TMH_FP32, TMH_FP64 = 0, 1
PATH_AUTO, PATH_SEQUENTIAL, PATH_TIME_PARALLEL = 0, 1, 2
CHAIN_STATUS = {0: "ok", 1: "NameError (init)", 2: "AssertionError (CloudCoverBinary)",
                3: "sigma capacity exceeded", 4: "injected stream exhausted",
                5: "segment capacity exceeded", 6: "fp32 guard-band records exceeded"}
STATE_FIELDS = ["sb_cc", "sb_clear_day", "sb_cloudy_hour", "sb_cloudy_noise", "sb_clear_noise", "sb_ws",
                "sa_cc", "sa_clear_day", "sa_cloudy_hour", "sa_cloudy_noise", "sa_clear_noise", "sa_ws",
                "cloud_length", "clear_length", "markov_state", "sec", "sigma_len", "pos", "status",
                "ncalls", "sigma_cloud", "sigma_clear", "fn_cloudy", "fn_clear"]
STATE_DTYPES = {**{f: np.float64 for f in STATE_FIELDS[:15]}, "sec": np.int32, "sigma_len": np.int32,
                "pos": np.uint32, "status": np.uint32, "ncalls": np.uint32, "sigma_cloud": np.float64,
                "sigma_clear": np.float64, "fn_cloudy": np.float32, "fn_clear": np.float32}


class Params(C.Structure):
    _fields_ = [
        ("cc_mode", C.c_int32), ("rng_mode", C.c_int32), ("precision", C.c_int32), ("with_pv", C.c_int32),
        ("kernel_path", C.c_int32), ("reserved", C.c_int32), ("seed", C.c_uint64), ("shapes", (C.c_double * 4) * 6), ("shape_is_t", C.c_int32 * 6),
        ("edges", C.c_double * 6), ("site", C.c_double * 8), ("linke", C.c_double * 12),
        ("module", C.c_double * 26), ("inverter", C.c_double * 9),
    ]


class Clock(C.Structure):
    _fields_ = [("utc0", C.c_int64), ("local0", C.c_int64), ("n_shifts", C.c_int32), ("reserved", C.c_int32),
                ("shift_step", C.c_int64 * 8), ("shift_delta", C.c_int32 * 8)]


class UStream(C.Structure):
    _fields_ = [("u", C.c_void_p), ("stride", C.c_uint64), ("len", C.c_uint64)]


class Trace(C.Structure):
    _fields_ = [("csi", C.c_void_p), ("covered", C.c_void_p), ("pv", C.c_void_p), ("meter", C.c_void_p),
                ("residual", C.c_void_p), ("ld", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("hist", C.c_void_p), ("n_bins", C.c_uint32), ("reserved", C.c_uint32), ("lo", C.c_double),
                ("hi", C.c_double), ("chain_acc", C.c_void_p)]


EXPORTS = ["tmh_abi_version", "tmh_last_error", "tmh_build_stamp", "tmh_state_bytes", "tmh_state_offsets", "tmh_plan_bytes",
           "tmh_scratch_bytes", "tmh_engine_scratch_bytes", "tmh_workspace_bytes", "tmh_engine_create", "tmh_engine_destroy", "tmh_engine_path",
           "tmh_init", "tmh_run", "tmh_plan", "tmh_step", "tmh_probe", "tmh_profile_enable", "tmh_profile_read",
           "tmh_set_shape_tables", "tmh_set_sites", "tmh_walk", "tmh_expand",
           "tmh_walk_part", "tmh_expand_part", "tmh_set_clock", "tmh_test_set_segment_capacity",
           "tmh_set_walk_chains_per_row", "tmh_set_walk_lanes", "tmh_set_chain_ids", "tmh_live_chains", "tmh_state_move",
           "tmh_stream_create_cus", "tmh_stream_destroy", "tmh_set_walk_order", "tmh_engine_last_expand"]
K_EXPAND, K_SEGMENTS, K_CANDIDATES, K_STEP = 0, 1, 2, 3
WALK_DRAWS, WALK_SEGMENTS = 1, 2
EXPAND_KERNEL, EXPAND_COMMIT, EXPAND_MINUTES, EXPAND_NO_MINUTES = 1, 2, 4, 8
OUT_ANY, OUT_TRACE3, OUT_STATS, OUT_SITES, OUT_FP64 = 0, 1, 2, 16, 32   # tmh_engine_last_expand

_lib = None


class TmhError(RuntimeError):
    pass


class StaleLibraryError(ImportError):
    pass


def loaded_stamp():
    """The build stamp compiled into the loaded library ("unstamped" without one)."""
    L = load()
    if not hasattr(L, "tmh_build_stamp"):
        return "unstamped"
    raw = L.tmh_build_stamp().decode()
    return raw.split(":", 1)[1] if raw.startswith("TMHSTAMP:") else raw


def _check_stamp(L):
    """The in-tree library must carry the stamp of the sources beside it (build.build_stamp):
    a stale pushed binary is refused instead of being tested or benchmarked silently.
    A library named by TMHPVSIM_LIB (same-box A/B builds of other sources) is not checked;
    TMHPVSIM_ALLOW_STALE=1 skips the check (diagnostics only)."""
    if os.environ.get("TMHPVSIM_LIB") or os.environ.get("TMHPVSIM_ALLOW_STALE") == "1":
        return
    from .build import build_stamp
    want = build_stamp()
    have = None
    if hasattr(L, "tmh_build_stamp"):
        L.tmh_build_stamp.restype = C.c_char_p
        raw = L.tmh_build_stamp().decode()
        have = raw.split(":", 1)[1] if raw.startswith("TMHSTAMP:") else raw
    if have != want:
        raise StaleLibraryError(f"{LIB_PATH} was built from other sources (stamp {have}, sources {want}): "
                                "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")


def load():
    """Load libtmhpvsim.so (raises if it is missing or stale: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch first: the library must bind to the HIP runtime torch already uses
    # (one libamdhip64 per process), never load a second one ahead of it.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    _check_stamp(L)
    if hasattr(L, "tmh_build_stamp"):
        L.tmh_build_stamp.restype = C.c_char_p
    p, u32, u64, i64, sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int64, C.c_size_t
    L.tmh_abi_version.restype = C.c_int
    L.tmh_last_error.restype = C.c_char_p
    L.tmh_state_bytes.restype = sz
    L.tmh_state_bytes.argtypes = [u32]
    L.tmh_state_offsets.argtypes = [u32, p]
    L.tmh_plan_bytes.restype = sz
    L.tmh_plan_bytes.argtypes = [u32]
    L.tmh_scratch_bytes.restype = sz
    L.tmh_scratch_bytes.argtypes = [u32, u32]
    L.tmh_engine_scratch_bytes.restype = sz
    L.tmh_engine_scratch_bytes.argtypes = [p, u32, u32]
    L.tmh_workspace_bytes.restype = sz
    L.tmh_test_set_segment_capacity.argtypes = [u32, u32]
    if hasattr(L, "tmh_set_walk_chains_per_row"):
        L.tmh_set_walk_chains_per_row.argtypes = [p, u32]
    if hasattr(L, "tmh_set_walk_lanes"):
        L.tmh_set_walk_lanes.argtypes = [p, u32]
    if hasattr(L, "tmh_set_walk_order"):
        L.tmh_set_walk_order.argtypes = [p, C.c_int]
    if hasattr(L, "tmh_stream_create_cus"):
        L.tmh_stream_create_cus.argtypes = [u32, u32, C.POINTER(p)]
        L.tmh_stream_destroy.argtypes = [p]
    if hasattr(L, "tmh_set_chain_ids"):
        L.tmh_set_chain_ids.argtypes = [p, p, u32]
        L.tmh_live_chains.argtypes = [p, p, u32, p, p, p, p]
        L.tmh_state_move.argtypes = [p, p, u32, p, u32, p, p, u32, C.c_int, p]
    L.tmh_workspace_bytes.argtypes = [u32, u32]
    L.tmh_engine_path.argtypes = [p]
    if hasattr(L, "tmh_engine_last_expand"):
        L.tmh_engine_last_expand.argtypes = [p]
        L.tmh_engine_last_expand.restype = C.c_int
    L.tmh_engine_create.argtypes = [C.POINTER(Params), C.POINTER(Clock), C.c_int, C.POINTER(p)]
    L.tmh_engine_destroy.argtypes = [p]
    if hasattr(L, "tmh_set_clock"):
        L.tmh_set_clock.argtypes = [p, C.POINTER(Clock)]
    L.tmh_init.argtypes = [p, p, u64, u32, C.POINTER(UStream), p]
    L.tmh_run.argtypes = [p, p, u64, u32, i64, u32, C.POINTER(UStream), C.POINTER(Trace), C.POINTER(Stats), p, sz, p]
    L.tmh_step.argtypes = [p, p, u64, u32, i64, u32, C.POINTER(UStream), C.POINTER(Trace), C.POINTER(Stats), p, p,
                           sz, p]
    L.tmh_plan.argtypes = [p, i64, u32, p, p]
    L.tmh_walk.argtypes = [p, p, u64, u32, i64, u32, p, p, sz, p]
    L.tmh_walk_part.argtypes = [p, p, u64, u32, i64, u32, p, p, sz, p, u32, C.c_int, p]
    L.tmh_expand.argtypes = [p, p, u64, u32, i64, u32, C.POINTER(UStream), C.POINTER(Trace), C.POINTER(Stats), p, p,
                             sz, p]
    if hasattr(L, "tmh_expand_part"):   # (absent from round-1 builds, which same-box A/B runs still load)
        L.tmh_expand_part.argtypes = [p, p, u64, u32, i64, u32, C.POINTER(UStream), C.POINTER(Trace),
                                      C.POINTER(Stats), p, p, sz, C.c_int, p]
    L.tmh_probe.argtypes = [C.c_int, C.c_double, p, p, u32, p]
    L.tmh_profile_enable.argtypes = [p, C.c_int]
    L.tmh_set_shape_tables.argtypes = [p, p, p, u32]
    L.tmh_set_sites.argtypes = [p, p, p, u32]
    L.tmh_profile_read.argtypes = [p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    for name in ("tmh_state_offsets", "tmh_engine_create", "tmh_engine_destroy", "tmh_engine_path", "tmh_init",
                 "tmh_run", "tmh_step", "tmh_plan", "tmh_probe", "tmh_profile_enable", "tmh_profile_read",
                 "tmh_set_shape_tables", "tmh_set_sites", "tmh_walk", "tmh_expand", "tmh_walk_part",
                 "tmh_expand_part", "tmh_set_clock"):
        if hasattr(L, name):
            getattr(L, name).restype = C.c_int
    if L.tmh_abi_version() != TMH_ABI_VERSION:
        raise ImportError(f"libtmhpvsim ABI {L.tmh_abi_version()} != {TMH_ABI_VERSION}")
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise TmhError(f"libtmhpvsim error {rc}: {load().tmh_last_error().decode()}")
    return rc


_streams = []   # (device, handle) of the live streams cu_stream created (process-wide)


def _destroy_streams():
    """At interpreter exit: drain and destroy the streams cu_stream created that nobody
    released (release_stream), before the HIP runtime's own teardown (a CU-masked stream
    still alive when the runtime is finalised crashed the process's exit under
    rocprofv3's kernel trace)."""
    import torch
    while _streams:
        dev, h = _streams.pop()
        try:
            torch.cuda.synchronize(dev)
            load().tmh_stream_destroy(h)
        except Exception:   # exit path: nothing to report to
            pass


def live_streams():
    """How many streams cu_stream created are alive (not yet released)."""
    return len(_streams)


def cu_stream(cu_first, cu_count, device):
    """A torch stream over a HIP stream restricted to CU-mask bits cu_first ..
    cu_first + cu_count - 1 of `device` (tmh_stream_create_cus; cu_count 0 = all CUs).
    Created with `device` current (the HIP call builds the mask and the stream on the
    current device).  Release it with release_stream (BatchPipeline.close does); what is
    still alive at interpreter exit is destroyed then (_destroy_streams).  A CU-masked HIP
    stream is blocking (it synchronises with the legacy null stream); the pipelines issue
    nothing on the null stream."""
    import atexit
    import torch
    dev = torch.device(device)
    h = C.c_void_p()
    with torch.cuda.device(dev):
        check(load().tmh_stream_create_cus(cu_first, cu_count, C.byref(h)))
    if not _streams and not getattr(cu_stream, "_atexit", False):
        atexit.register(_destroy_streams)   # registered after torch's handlers, so it runs before them (LIFO)
        cu_stream._atexit = True
    _streams.append((dev, h.value))
    return torch.cuda.ExternalStream(h.value, device=dev)


def release_stream(stream):
    """Drain and destroy a stream cu_stream / dedicated_stream created (no-op for others)."""
    for i, (dev, h) in enumerate(_streams):
        if h == stream.cuda_stream:
            stream.synchronize()
            _streams.pop(i)
            check(load().tmh_stream_destroy(h))
            return True
    return False


def dedicated_stream(device):
    """A torch stream on a hardware queue of its own: a CU-masked HIP stream whose mask
    holds every CU (tmh_stream_create_cus(0, all)).  HIP maps plain streams onto a pool
    of GPU_MAX_HW_QUEUES hardware queues (4 by default) shared round-robin by every
    stream of the process -- torch's stream pool included -- and a queue runs its
    packets in order across the streams sharing it; a CU-masked stream always gets a
    queue of its own, so the pipeline's streams never wait behind each other's kernels
    whatever GPU_MAX_HW_QUEUES is.  Released by release_stream (cu_stream)."""
    import torch
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    return cu_stream(0, ncu, device)


def profile_read(eng, kernel):
    """(total ms, launches) of one kernel since the last read (tmh_profile_read)."""
    ms, n = C.c_double(), C.c_int()
    check(load().tmh_profile_read(eng, int(kernel), C.byref(ms), C.byref(n)))
    return ms.value, n.value


def state_offsets(n):
    off = np.zeros(TMH_STATE_NFIELDS, dtype=np.uint64)
    check(load().tmh_state_offsets(n, off.ctypes.data_as(C.c_void_p)))
    return off


def make_params(mp, precision, kernel_path=PATH_AUTO):
    """tmhpvsim_amd.params.ModelParams -> Params."""
    P = Params()
    P.kernel_path = int(kernel_path)
    P.cc_mode, P.rng_mode, P.precision = int(mp.cc_mode), int(mp.rng_mode), int(precision)
    P.with_pv, P.seed = int(bool(mp.with_pv)), int(mp.seed) & (2 ** 64 - 1)
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
