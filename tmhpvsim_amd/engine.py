"""Batched simulator: N chains (site x scenario) advanced on one MI355X.

PyTorch-ROCm is used only for device memory and the stream; all compute runs
in libtmhpvsim.so (HIP, gfx950) through the C-ABI of include/tmhpvsim.h.
Chain state is a structure-of-arrays buffer owned by this object; traces are
time-major [step, chain] tensors; statistics are accumulated on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .clock import make_clock
from .params import ModelParams, RNG_INJECTED

TRACE_FIELDS = ("csi", "covered", "pv", "meter", "residual")
ROLL_MAX = 731 * 86400   # steps per rolling clock (<= 6 DST changes in two years)
DEFAULT_HIST = dict(n_bins=4096, lo=-300.0, hi=9000.0)


def _torch():
    import torch
    return torch


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class BatchedSim:
    """Advance chains [chain0, chain0 + n_chains) second by second.

    Parameters
    ----------
    n_chains : chains on this device (each is one ClearskyindexModel + PVModel
        + meter, tmhpvsim/clearskyindexmodel.py:44, pvmodel.py:11, metersim.py:49)
    start : constructor time of every chain (datetime / str); step 0 = next(start)
    tz : None (naive wall clock) or a zone name ("Europe/Berlin", as pvmodel.py:19)
    params : tmhpvsim_amd.params.ModelParams (modes, seed, shape table, site, PV system)
    precision : "fp32" (per-second CSI/PV math in fp32; Markov state fp64) or "fp64"
    chain0 : global id of the first chain (keyed RNG -> partition-independent results)
    injected : optional device tensor [n_chains, L] of uniforms (RNG_INJECTED mode)
    horizon : steps covered by one wall clock (its DST table holds 8 changes); a run
        past it installs the next rolling clock (tmh_set_clock), so runs are unbounded
    shape_tables : optional per-chain hourly cloud-cover tables (shapes [n, 6, 4],
        is_t [n, 6]; e.g. params.site_shape_tables) in place of params.shapes —
        one table per site of a lat/lon sweep (tmh_set_shape_tables)
    sites : optional per-chain PV sites [n, 8] in Site.as_array() order (e.g.
        params.site_grid), or (sites, linke [n, 12]); columns 0-5 vary per chain,
        temp_air and wind stay params.site's (tmh_set_sites)
    """

    def __init__(self, n_chains, start, tz=None, params: ModelParams | None = None, precision="fp32",
                 chain0=0, device=None, injected=None, horizon=400 * 86400, kernel_path="auto",
                 shape_tables=None, sites=None):
        torch = _torch()
        L = _lib.load()
        self.L = L
        self.params = params or ModelParams()
        self.n = int(n_chains)
        self.chain0 = int(chain0)
        self.precision = _lib.TMH_FP64 if precision in ("fp64", "f64", 64) else _lib.TMH_FP32
        self.real = torch.float64 if self.precision == _lib.TMH_FP64 else torch.float32
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("BatchedSim runs on a GPU device (there is no CPU path)")
        self.horizon = int(horizon)
        self._start, self._tz = start, tz
        self.clock = make_clock(start, self.horizon, tz)
        kp = {"auto": _lib.PATH_AUTO, "sequential": _lib.PATH_SEQUENTIAL,
              "time_parallel": _lib.PATH_TIME_PARALLEL}[kernel_path]
        P = _lib.make_params(self.params, self.precision, kp)
        ck = self.clock.as_struct()
        eng = C.c_void_p()
        _lib.check(L.tmh_engine_create(C.byref(P), C.byref(ck), self.device.index or 0, C.byref(eng)))
        self._eng = eng
        self.path = {1: "sequential", 2: "time_parallel"}[L.tmh_engine_path(eng)]
        self.state = torch.zeros(L.tmh_state_bytes(self.n), dtype=torch.uint8, device=self.device)
        self._offsets = _lib.state_offsets(self.n)
        self.injected = None
        self._us = None
        if self.params.rng_mode == RNG_INJECTED:
            if injected is None:
                raise ValueError("RNG_INJECTED mode needs `injected` uniforms [n_chains, L]")
            inj = torch.as_tensor(injected, dtype=torch.float64, device=self.device).contiguous()
            if inj.shape[0] != self.n:
                raise ValueError("injected must have one row per chain")
            self.injected = inj
            self._us = _lib.UStream(inj.data_ptr(), inj.shape[1], inj.shape[1])
        self.tables = None
        if shape_tables is not None:
            sh, it = shape_tables if isinstance(shape_tables, tuple) else (shape_tables, None)
            sh = torch.as_tensor(np.asarray(sh, dtype=np.float64) if not torch.is_tensor(sh) else sh,
                                 dtype=torch.float64, device=self.device).contiguous()
            if tuple(sh.shape) != (self.n, 6, 4):
                raise ValueError(f"shape_tables must be [n_chains, 6, 4], got {tuple(sh.shape)}")
            if it is not None:
                it = torch.as_tensor(np.asarray(it) if not torch.is_tensor(it) else it,
                                     dtype=torch.int32, device=self.device).contiguous()
                if tuple(it.shape) != (self.n, 6):
                    raise ValueError(f"shape_tables is_t must be [n_chains, 6], got {tuple(it.shape)}")
            self.tables = (sh, it)   # the engine reads them on every launch: keep them alive
            _lib.check(L.tmh_set_shape_tables(self._eng, _ptr(sh), _ptr(it) if it is not None else None, self.n))
        self.sites = None
        if sites is not None:
            si, li = sites if isinstance(sites, tuple) else (sites, None)
            si = torch.as_tensor(np.asarray(si, dtype=np.float64) if not torch.is_tensor(si) else si,
                                 dtype=torch.float64, device=self.device).contiguous()
            if tuple(si.shape) != (self.n, 8):
                raise ValueError(f"sites must be [n_chains, 8], got {tuple(si.shape)}")
            if li is not None:
                li = torch.as_tensor(np.asarray(li, dtype=np.float64) if not torch.is_tensor(li) else li,
                                     dtype=torch.float64, device=self.device).contiguous()
                if tuple(li.shape) != (self.n, 12):
                    raise ValueError(f"sites linke must be [n_chains, 12], got {tuple(li.shape)}")
            self.sites = (si, li)
            _lib.check(L.tmh_set_sites(self._eng, _ptr(si), _ptr(li) if li is not None else None, self.n))
        self.step = 0
        self.hist = None
        self.chain_acc = None
        self._hist_spec = None
        with torch.cuda.device(self.device):
            _lib.check(L.tmh_init(self._eng, _ptr(self.state), self.chain0, self.n,
                                  C.byref(self._us) if self._us is not None else None, self._stream()))

    def _stream(self):
        return C.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def __del__(self):
        try:
            if getattr(self, "_eng", None):
                self.L.tmh_engine_destroy(self._eng)
                self._eng = None
        except Exception:
            pass

    # ------------------------------------------------------------------ state
    def state_field(self, name):
        """Device view of one SoA state field ([n], or [n, TMH_SIGMA_CAP] for the sigma arrays)."""
        torch = _torch()
        i = _lib.STATE_FIELDS.index(name)
        dt = {np.float64: torch.float64, np.int32: torch.int32, np.uint32: torch.int32,
              np.float32: torch.float32}[_lib.STATE_DTYPES[name]]
        esz = 8 if dt == torch.float64 else 4
        rows = _lib.TMH_SIGMA_CAP if name.startswith("sigma_c") else (2 if name.startswith("fn_") else 1)
        o = int(self._offsets[i])
        v = self.state[o:o + esz * self.n * rows].view(dt)
        return v.view(self.n, rows) if rows > 1 else v

    def status(self):
        return self.state_field("status").cpu().numpy().astype(np.uint32)

    # ------------------------------------------------------------------ stats
    def enable_stats(self, n_bins=4096, lo=-300.0, hi=9000.0, histogram=True):
        torch = _torch()
        self._hist_spec = (int(n_bins), float(lo), float(hi), bool(histogram))
        self.hist = torch.zeros(int(n_bins), dtype=torch.int64, device=self.device) if histogram else None
        self.chain_acc = torch.zeros(4, self.n, dtype=torch.float64, device=self.device)
        self.chain_acc[3].fill_(-float("inf"))

    def _stats_struct(self):
        if self.chain_acc is None:
            return None
        n_bins, lo, hi, _ = self._hist_spec
        return _lib.Stats(self.hist.data_ptr() if self.hist is not None else None, n_bins, 0, lo, hi,
                          self.chain_acc.data_ptr())

    # ------------------------------------------------------------------ run
    def workspace(self, n_steps):
        """plan + scratch of one window (tmh_engine_scratch_bytes: this engine's precision)"""
        nb = self.L.tmh_plan_bytes(n_steps) + self.L.tmh_engine_scratch_bytes(self._eng, self.n, n_steps)
        return _torch().empty(nb, dtype=torch_uint8(), device=self.device)

    def run(self, n_steps, trace=TRACE_FIELDS, window=86400, out=None, compact=False):
        """Advance n_steps seconds.  Returns {field: tensor[n_steps, n_chains]} for `trace`.

        compact=True (statistics runs, trace=()): each window after the first runs
        on the chains still live at its start only (tmh_live_chains, tmh_state_move,
        tmh_set_chain_ids), so chains the reference's AssertionError ended
        (cloud_cover_binary.py:91; most C5 chains within the week) cost nothing
        more.  Every chain's state and statistics come out as without compaction."""
        torch = _torch()
        n_steps = int(n_steps)
        trace = tuple(trace or ())
        if compact and (trace or self._us is not None):
            raise ValueError("compact=True needs a keyed statistics run (trace=(), no injected uniforms)")
        if n_steps > ROLL_MAX:   # one rolling clock covers at most ROLL_MAX steps: run in pieces (same bits)
            res = out if out is not None else self._alloc(n_steps, trace)
            done = 0
            while done < n_steps:
                k = min(ROLL_MAX, n_steps - done)
                self.run(k, trace, window, {f: res[f][done:done + k] for f in trace}, compact=compact)
                done += k
            return res
        if self.step + n_steps > self.clock.end:
            self._roll(n_steps)
        for f in trace:
            if f not in TRACE_FIELDS:
                raise ValueError(f"unknown trace field {f!r}")
        res = out if out is not None else self._alloc(n_steps, trace)
        st = self._stats_struct()
        win = max(1, min(int(window), n_steps))
        if compact and n_steps > win:
            with torch.cuda.device(self.device):
                self._run_compacted(n_steps, win, st)
            self.step += n_steps
            return res
        if self.path == "time_parallel" and n_steps > win:
            with torch.cuda.device(self.device):
                self._run_pipelined(n_steps, win, trace, res, st)
            self.step += n_steps
            return res
        ws = self.workspace(win)
        with torch.cuda.device(self.device):
            done = 0
            while done < n_steps:
                k = min(win, n_steps - done)
                tr = _lib.Trace(*(res[f][done:done + k].data_ptr() if f in trace else None
                                  for f in ("csi", "covered", "pv", "meter", "residual")), self.n)
                _lib.check(self.L.tmh_run(self._eng, _ptr(self.state), self.chain0, self.n, self.step + done, k,
                                          C.byref(self._us) if self._us is not None else None,
                                          C.byref(tr), C.byref(st) if st is not None else None,
                                          _ptr(ws), ws.numel(), self._stream()))
                done += k
        self.step += n_steps
        return res

    def _run_compacted(self, n_steps, win, st):
        """Windows in order; from the second on, only the chains live at the window
        start run, gathered into a dense working state and scattered back after it."""
        torch = _torch()
        L, s = self.L, self._stream()
        ws = self.workspace(win)
        work = torch.empty_like(self.state)
        ids = torch.empty(self.n, dtype=torch.int32, device=self.device)
        nlive = torch.zeros(1, dtype=torch.int32, device=self.device)
        tr = _lib.Trace(None, None, None, None, None, self.n)
        done = 0
        while done < n_steps:
            k = min(win, n_steps - done)
            nl, cur = self.n, self.state
            if done > 0:
                _lib.check(L.tmh_live_chains(self._eng, _ptr(self.state), self.n, None, _ptr(ids), _ptr(nlive), s))
                nl = int(nlive.item())
                if nl < self.n:
                    cur = work
                    if nl:
                        _lib.check(L.tmh_state_move(self._eng, _ptr(self.state), self.n, _ptr(work), nl, _ptr(ids),
                                                    _ptr(nlive), nl, 0, s))
                        _lib.check(L.tmh_set_chain_ids(self._eng, _ptr(ids), self.n))
            try:
                if nl:
                    _lib.check(L.tmh_run(self._eng, _ptr(cur), self.chain0, nl, self.step + done, k, None, C.byref(tr),
                                         C.byref(st) if st is not None else None, _ptr(ws), ws.numel(), s))
                if nl and cur is work:
                    _lib.check(L.tmh_state_move(self._eng, _ptr(work), nl, _ptr(self.state), self.n, _ptr(ids),
                                                _ptr(nlive), nl, 1, s))
            finally:
                _lib.check(L.tmh_set_chain_ids(self._eng, None, 0))
            done += k

    def _alloc(self, n_steps, trace):
        torch = _torch()
        return {f: torch.empty(n_steps, self.n, dtype=torch.uint8 if f == "covered" else self.real, device=self.device)
                for f in trace}

    def _roll(self, n_steps):
        """The next rolling wall clock, from the current step (tmh_set_clock)."""
        self.clock = make_clock(self._start, max(int(n_steps), min(self.horizon, ROLL_MAX)), self._tz, step0=self.step)
        _lib.check(self.L.tmh_set_clock(self._eng, C.byref(self.clock.as_struct())))

    def _run_pipelined(self, n_steps, win, trace, res, st):
        """Windows of the time-parallel path, pipelined (run_windows): each window's plan,
        draws and segment walk on a walk stream that runs up to two windows ahead of the
        expansions on the current stream.  Same bits as one tmh_run per window
        (tests/test_gpu_parity.py)."""
        torch = _torch()
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_wstream", None) is None:
            self._wstream = torch.cuda.Stream(self.device, priority=torch.cuda.Stream.priority_range()[1])
            self._pstream = torch.cuda.Stream(self.device)
        wins = []
        done = 0
        while done < n_steps:
            k = min(win, n_steps - done)
            wins.append((self.step + done, k, done))
            done += k
        bufs = [self.workspace(win) for _ in range(min(WINDOW_BUFFERS, len(wins)))]

        def trace_of(w):
            off, k = wins[w][2], wins[w][1]
            return _lib.Trace(*(res[f][off:off + k].data_ptr() if f in trace else None
                                for f in ("csi", "covered", "pv", "meter", "residual")), self.n)

        run_windows(self.L, self._eng, self.state, self.chain0, self.n, [(a, k) for a, k, _ in wins], bufs, main,
                    self._wstream, trace_of, st, plan_stream=self._pstream)
        self._keep = bufs   # allocated on the main stream, whose last work is the last expansion

    def plan(self, step0, n_steps):
        """Build the chain-independent plan of a window (tmh_plan); returns the uint8 buffer."""
        torch = _torch()
        plan = torch.empty(self.L.tmh_plan_bytes(int(n_steps)), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(self.L.tmh_plan(self._eng, int(step0), int(n_steps), _ptr(plan), self._stream()))
        return plan

    def geometry(self, step0, n_steps):
        """The clock/geometry table rows [n_steps, TMH_GEOM_FIELDS] (fp64) of a window."""
        torch = _torch()
        plan = self.plan(step0, n_steps)
        return plan[: n_steps * _lib.TMH_GEOM_FIELDS * 8].view(torch.float64).view(n_steps, _lib.TMH_GEOM_FIELDS)

    def stats_totals(self):
        """Node-local totals: histogram, energy sums (W*s, exact fixed-point limbs and the
        fp64 values of them) and peak residual (W) over every chain's accumulated
        seconds -- a faulted chain's seconds before its fault included, in energies
        and histogram alike (dist.chain_totals)."""
        from .dist import chain_totals
        return chain_totals(self.chain_acc, self.hist.clone() if self.hist is not None else None)


WINDOW_BUFFERS = 3   # plan + scratch sets of the multi-window pipeline (run_windows)


def run_windows(L, eng, state, chain0, n, wins, bufs, main, walk, trace_of, st, plan_stream=None):
    """Consecutive windows [(step0, n_steps)] of the same chains, software-pipelined over
    len(bufs) workspace buffers (plan + scratch each, window w in buffer w % K):

      plan stream: plan(w) (chain-independent: clock and geometry rows) as soon as buffer
                   w % K is free;
      walk stream: draws(w) chained to window w-1's walk (tmh_walk_part with
                   prev_scratch), segment walk(w) -- up to K-1 windows ahead;
      main stream: expansion + commit of window w once its walk is done.

    The walk of a window needs only the previous window's walk (its end status,
    cloud-cover and wind pairs, call counts, sigma arrays), never its expansion, so the
    walks run back to back while the expansions follow; buffer w % K is reused once the
    expansion of window w - K is done.  With small batches (the walk latency-bound) the
    per-window tail (fixup, commit, plan, draws) is off the walk's path.  trace_of(w):
    the window's tmh_trace; st: tmh_stats or None.  Same bits as one tmh_run per window."""
    import ctypes as C
    torch = _torch()
    K = len(bufs)
    pst = plan_stream or walk
    mptr, wptr, pptr = C.c_void_p(main.cuda_stream), C.c_void_p(walk.cuda_stream), C.c_void_p(pst.cuda_stream)
    nb = bufs[0].numel()
    pbytes = [L.tmh_plan_bytes(int(max(k for _, k in wins)))] * K
    walked = [torch.cuda.Event() for _ in range(K)]
    expanded = [torch.cuda.Event() for _ in range(K)]
    planned = [torch.cuda.Event() for _ in range(K)]

    def views(w):
        b = bufs[w % K]
        return C.c_void_p(b.data_ptr()), C.c_void_p(b.data_ptr() + pbytes[w % K]), nb - pbytes[w % K]

    def prev_of(w):
        return (views(w - 1)[1], wins[w - 1][1]) if w > 0 else (None, 0)

    def issue_walk(w):   # plan, draws and segment walk of window w, on the walk stream
        s0, k = wins[w]
        plan, scr, sb = views(w)
        if w >= K:
            pst.wait_event(expanded[w % K])    # the expansion of window w - K has read this buffer
            if pst is not walk:
                walk.wait_event(expanded[w % K])
        _lib.check(L.tmh_plan(eng, s0, k, plan, pptr))
        if pst is not walk:
            planned[w % K].record(pst)
            walk.wait_event(planned[w % K])
        ps, pk = prev_of(w)
        _lib.check(L.tmh_walk_part(eng, _ptr(state), chain0, n, s0, k, plan, scr, sb, ps, pk,
                                   _lib.WALK_DRAWS | _lib.WALK_SEGMENTS, wptr))
        walked[w % K].record(walk)

    # everything already issued on the main stream (the chains' construction, a previous
    # run's last commit) precedes this run's plans, draws and walks
    begun = torch.cuda.Event()
    begun.record(main)
    walk.wait_event(begun)
    if pst is not walk:
        pst.wait_event(begun)
    for w in range(min(K - 1, len(wins))):
        issue_walk(w)
    for w in range(len(wins)):
        if w + K - 1 < len(wins):
            issue_walk(w + K - 1)
        s0, k = wins[w]
        plan, scr, sb = views(w)
        main.wait_event(walked[w % K])
        tr = trace_of(w)
        _lib.check(L.tmh_expand(eng, _ptr(state), chain0, n, s0, k, None, C.byref(tr) if tr is not None else None,
                                C.byref(st) if st is not None else None, plan, scr, sb, mptr))
        expanded[w % K].record(main)


def torch_uint8():
    return _torch().uint8


def probe(fn, a, x, device="cuda"):
    """Device math probe (parity tests): fn 0 ndtri, 1 gammaincinv, 2 stdtrit, 3 al_ppf, 4 ndtri fp32."""
    torch = _torch()
    L = _lib.load()
    xt = torch.as_tensor(np.asarray(x, dtype=np.float64), device=device)
    out = torch.empty_like(xt)
    _lib.check(L.tmh_probe(int(fn), float(a), _ptr(xt), _ptr(out), xt.numel(),
                           C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    return out.cpu().numpy()
