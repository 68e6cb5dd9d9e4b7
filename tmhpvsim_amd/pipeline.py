"""Batches of chains in flight on one GPU: the schedules bench.py times.

A batch = one BatchedSim engine's n chains constructed fresh (tmh_init, new global
ids every batch) and advanced over `secs` seconds (tmh_plan + tmh_walk_part +
tmh_expand_part, or tmh_step per window).  Several batches are in flight at once,
each in its own context (state, plan, scratch, outputs), so the latency-bound
segment walks of the next batches run beside this batch's expansion
(DESIGN.md "The C2 pipeline").  bench.py times `BatchPipeline.run`; the GPU tests
(tests/test_gpu_trace3.py) run the same object and compare every batch's trace
with a separate tmh_run of the same chains, so the timed schedule is the tested
one.

Reference: the batch replaces n chains of `pvsim`'s per-second loop
(/root/reference/tmhpvsim/pvsim.py:72-84: PVModel.next, get_meter_value,
meter - pv), one ClearskyindexModel per chain (clearskyindexmodel.py:57-160).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib
from .engine import WINDOW_BUFFERS, run_windows


@dataclass
class PipelineConfig:
    """How batches overlap (bench.py's flags; `pipeline_defaults` gives each workload's)."""
    mode: str = "trace"          # "trace": pv, meter, residual traces; "stats": on-GPU statistics
    window: int = 86400          # steps per tmh_step window (a batch of secs > window runs windows in order)
    pipeline: int = 5            # contexts (batches in flight)
    walks: int = 2               # gated schedule: segment walks in flight
    build_ahead: int = 4         # gated: construction of batch k + A released when walk k ends
    plan_stream: bool = False    # gated: each construction's plan on a stream of its own, beside its
                                 # chains' init (the draws wait for both)
    build_streams: int = 1       # gated: constructions on this many streams in turn (2: consecutive
                                 # batches' constructions may overlap; their kernels are latency-bound)
    stagger: bool = True         # one-window batches software-pipelined (else one tmh_step each, in turn)
    schedule: str = "gated"      # "gated" or round 1's "stagger"
    build_on: str = "walk"       # stagger schedule: construction on the walk or the expansion stream
    walk_priority: str = "normal"
    expand_priority: str = "normal"
    build_priority: str = "normal"
    commit_stream: bool = False  # gated: fixup + commit on a stream of their own
    walk_order: bool = True      # walk rows windiest chain first (the run's first walk in chain order)
    drain_order: int = 1         # gated: the run's last walks in chain order too (they drain the pipeline)
    walk_cus: int = 0            # gated: segment walks on CU-mask bits 0 .. K-1 (0 = all CUs)
    other_cus: str = "all"       # with walk_cus: the other streams on all CUs or the rest
    compact: bool = False        # multi-window stats batches: later windows on the live chains only
    timeline: bool = False       # gated: HIP events around every build, walk and expansion
    first_split: int = 1         # gated: the run's first batch in this many consecutive windows (its walk
                                 # is the pipeline's fill; the windows' walks run ahead of their expansions)
    queues: str = "dedicated"    # "dedicated": normal-priority streams on hardware queues of their own
                                 # (_lib.dedicated_stream); "shared": plain streams (GPU_MAX_HW_QUEUES pool)
    hist_bins: int = 4096
    hist_lo: float = -300.0
    hist_hi: float = 9000.0


def pipeline_defaults(workload, precision="fp32", seconds=None, window=None, walks=None, build_ahead=None,
                      pipeline=None, compact=None, mode=None, chains=None, **overrides):
    """The measured-best schedule of each BASELINE.json workload (DESIGN.md "The C2
    pipeline", "C3, C4, C5"): bench.py's defaults, shared with the tests that check
    the timed schedule.  chains: the chains of one batch on this GPU (a rank's shard of
    a strong-scaled workload); C4 / C5 shards smaller than the one-GPU batch keep more
    batches in flight (their windows' walks are latency-bound at small batches, so the
    GPU has room for several: as many contexts as keep ~3 one-GPU batches' chains in
    flight, at most 8)."""
    c5, c4 = workload == "c5", workload == "c4"
    secs = seconds or {"c2": 86400, "c3": 86400, "c4": 365 * 86400, "c5": 604800}[workload]
    mode = mode or ("trace" if workload == "c2" else "stats")
    # C2: two walks in flight (r02, same-box A/B: 1.71-1.72 ms per batch against 1.81 with one)
    walks = walks if walks is not None else (2 if workload == "c2" else 1)
    # construction released walks + 2 batches ahead (round 3, 16 queues, same box, 3 reps:
    # 1.41-1.44 ms per C2 batch at 4, 5 or 6 ahead against 1.48-1.55 at 3, 1.86-1.90 at 2)
    build_ahead = build_ahead or max(1, walks) + (2 if walks > 1 else 1)
    # c3: two 1 M-chain batches in flight (2 x ~27 GB of state + scratch): +3 % over one (r02)
    if not pipeline:
        # c5: five compacted batches in flight (round 4, same box: 3.40 / 3.46 / 3.51 / 3.51e10
        # live chain-s/s with 3 / 4 / 5 / 6; the compacted windows shrink as chains fault)
        pipeline = 2 if workload == "c3" else (5 if c5 else build_ahead + 1)
        if (c4 or c5) and chains:
            full = 16384 if c4 else 65536
            pipeline = max(pipeline, min(8, -(-3 * full // int(chains))))
    # C4: 30-day windows (round 4, same box: 2.41e11 chain-s/s with day windows, 2.73e11 with
    # 7-day, 2.78e11 with 30-day; the N = 8 shard alone 1.24e11 / 2.36e11 / 2.47e11 -- the
    # per-window plan, draws and walk latency no longer dominate a small shard's day)
    cfg = PipelineConfig(
        mode=mode,
        window=min(window or (30 * 86400 if c4 else 86400 if c5 else secs), secs),
        pipeline=pipeline, walks=walks, build_ahead=build_ahead,
        # C2 (same-box A/B, r01): construction on the walk stream at normal priority
        # 1.94e11 chain-s/s vs 1.82e11 on the expansion stream with high-priority walks
        build_on="walk" if workload == "c2" else "expand",
        walk_priority="normal" if workload == "c2" else "high",
        # (first_split 2 for C2 -- the run's first batch as two half-day windows -- starts the
        # first expansion after half a day's walk, but the second half's draws and walk then
        # run beside that expansion, the next batch's walk and three constructions: the first
        # batch ends 0.6 ms later, 2.39-2.44 against 2.46-2.47e11, round 5, same box)
        compact=bool(c5 if compact is None else compact),
    )
    for k, v in overrides.items():
        if v is not None:
            setattr(cfg, k, v)
    return cfg


class BatchPipeline:
    """`cfg.pipeline` contexts of `n` chains each over `secs` seconds on `sim`'s engine.
    chain0_of(k): global id of the first chain of batch k (fresh chains every batch)."""

    def __init__(self, sim, n, secs, cfg: PipelineConfig, chain0_of, device):
        import torch
        self.torch = torch
        self.L = L = _lib.load()
        self.sim, self.n, self.secs, self.cfg, self.chain0_of, self.dev = sim, n, secs, cfg, chain0_of, device
        self.win = win = min(cfg.window, secs)
        self.nwin = nwin = (secs + win - 1) // win
        prio_lo, prio_hi = torch.cuda.Stream.priority_range()
        self._prio = lambda s: prio_hi if s == "high" else prio_lo
        pipe = self
        # every stream this pipeline creates: close() drains them and releases the CU-masked
        # ones (a long-lived process that builds pipelines in turn -- the GPU test session, a
        # pvsim service -- would otherwise accumulate hardware queues until exit)
        self._owned, self._closed = [], False

        def own(st):
            pipe._owned.append(st)
            return st

        def mk(prio="normal"):
            # HIP maps plain streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by
            # default) and a queue runs its packets in order across the streams sharing it:
            # with 4, the C2 expansion stream shared a queue with another pipeline stream and
            # waited for its kernels (1.74-1.76 ms per batch against 1.47-1.51 with 16 queues,
            # round 3).  A dedicated stream (CU-masked over every CU) has a queue of its own
            # at any GPU_MAX_HW_QUEUES.  (High-priority streams keep HIP's priority pool: the
            # CU-masked constructor takes no priority.)
            if cfg.queues == "dedicated" and prio != "high":
                return own(_lib.dedicated_stream(device))
            return own(torch.cuda.Stream(device, priority=pipe._prio(prio)))
        self._mk = mk

        class Ctx:   # one batch in flight: its own state, plan, scratch, outputs and HIP streams
            # The context's own streams are created on first use: the gated schedule runs on
            # shared streams, and every extra stream shares one of HIP's few hardware queues
            # with a busy one (a queue runs its packets in order, across streams).
            @property
            def stream(self):
                if self._stream is None:
                    self._stream = mk()
                return self._stream

            @property
            def sptr(self):
                return C.c_void_p(self.stream.cuda_stream)

            @property
            def wstream(self):   # the walk runs on a stream of its own
                if self._wstream is None:
                    self._wstream = mk(cfg.walk_priority)
                return self._wstream

            @property
            def wptr(self):
                return C.c_void_p(self.wstream.cuda_stream)

            def __init__(self):
                self._stream = self._wstream = None
                self.chain0 = None
                self.walked = torch.cuda.Event()
                self.done = torch.cuda.Event()
                self.kernel_done = torch.cuda.Event()
                self.expanded = None   # recorded after this context's last expansion
                self.state = torch.zeros(L.tmh_state_bytes(n), dtype=torch.uint8, device=device)
                compacted = cfg.compact and cfg.mode == "stats" and nwin > 1
                # multi-window batches of the time-parallel path run on the window buffers
                # (engine.run_windows) only: no plan + scratch set of their own (a 30-day window
                # of 16,384 chains is ~10 GB of scratch)
                windowed = nwin > 1 and not compacted and sim.path == "time_parallel"
                self.plan = self.scratch = None
                if not windowed:
                    self.plan = torch.empty(L.tmh_plan_bytes(win), dtype=torch.uint8, device=device)
                    self.scratch = torch.empty(L.tmh_engine_scratch_bytes(sim._eng, n, win), dtype=torch.uint8,
                                               device=device)
                if compacted:   # compacted windows: a working state
                    self.work = torch.empty_like(self.state)
                    self.ids = torch.empty(n, dtype=torch.int32, device=device)
                    self.nlive = torch.zeros(1, dtype=torch.int32, device=device)
                if windowed:
                    # plan + scratch sets of the multi-window pipeline (engine.run_windows): the
                    # walks of the next windows run ahead of this window's expansion
                    wb = L.tmh_plan_bytes(win) + L.tmh_engine_scratch_bytes(sim._eng, n, win)
                    self.wbufs = [torch.empty(wb, dtype=torch.uint8, device=device)
                                  for _ in range(min(WINDOW_BUFFERS, nwin))]
                self.trace = {f: torch.empty(win, n, dtype=sim.real, device=device) for f in ("pv", "meter", "residual")} \
                    if cfg.mode == "trace" else {}
                self.tr = _lib.Trace(None, None, *(self.trace[f].data_ptr() if f in self.trace else None
                                                   for f in ("pv", "meter", "residual")), n)
                self.st = None
                if cfg.mode == "stats":
                    self.hist = torch.zeros(cfg.hist_bins, dtype=torch.int64, device=device)
                    self.acc = torch.zeros(4, n, dtype=torch.float64, device=device)
                    self.acc[3].fill_(-float("inf"))
                    self.st = _lib.Stats(self.hist.data_ptr(), cfg.hist_bins, 0, cfg.hist_lo, cfg.hist_hi,
                                         self.acc.data_ptr())

        self.ctxs = [Ctx() for _ in range(max(1, cfg.pipeline))]
        # One-window batches (C2, C3): one stream for every batch's expansion (expansions run
        # back to back, in order: they fill the chip on their own) and, on the gated schedule,
        # walk / construction / commit streams shared by the batches.  Multi-window batches
        # (C4, C5) run on their contexts' own streams (main, walk, plan): HIP maps streams
        # round-robin onto GPU_MAX_HW_QUEUES hardware queues and a queue runs its packets in
        # order across the streams sharing it, so streams nobody uses are not created (bench.py
        # raises the queues to 32 for these workloads' 3 streams per context).
        W = self.W = max(1, cfg.walks)
        self.estream = self.bst = self._cst = self.psts = None
        self.wsts = []
        if nwin == 1:
            self.estream = mk(cfg.expand_priority)
            self.wsts = [mk(cfg.walk_priority) for _ in range(W)]
            self.bst = mk(cfg.build_priority)
            self.bsts = [self.bst] + [mk(cfg.build_priority) for _ in range(max(1, cfg.build_streams) - 1)]
            self.psts = mk(cfg.build_priority) if cfg.plan_stream else None
            if cfg.walk_cus:   # the walks on a share of every XCD's CUs (CU-masked streams)
                ncu = torch.cuda.get_device_properties(device).multi_processor_count
                self.wsts = [own(_lib.cu_stream(0, cfg.walk_cus, device)) for _ in range(W)]
                if cfg.other_cus == "rest":
                    self.bst, self._cst = (own(_lib.cu_stream(cfg.walk_cus, ncu - cfg.walk_cus, device))
                                           for _ in range(2))
                    self.bsts = [self.bst] + [own(_lib.cu_stream(cfg.walk_cus, ncu - cfg.walk_cus, device))
                                              for _ in range(max(1, cfg.build_streams) - 1)]
                    self.estream = own(_lib.cu_stream(cfg.walk_cus, ncu - cfg.walk_cus, device))
            self.eptr = C.c_void_p(self.estream.cuda_stream)
            self.bst_p = C.c_void_p(self.bst.cuda_stream)
        self.A = cfg.build_ahead
        self.tl = {}   # timeline: per-batch HIP timing events (build done, walk start / end, expansion start / end)
        # gated schedule, the run's first batch in consecutive windows of whole hours (first_split):
        # their plans + scratch, and the events chaining each window's walk to the previous one's
        self.split = []
        if nwin == 1 and cfg.first_split > 1 and sim.path == "time_parallel":
            h = secs // cfg.first_split // 3600 * 3600
            if h > 0:
                bounds = [i * h for i in range(cfg.first_split)] + [secs]
                self.split = [(a, b - a) for a, b in zip(bounds[:-1], bounds[1:])]
                self.sbufs = [(torch.empty(L.tmh_plan_bytes(k), dtype=torch.uint8, device=device),
                               torch.empty(L.tmh_engine_scratch_bytes(sim._eng, n, k), dtype=torch.uint8, device=device))
                              for _, k in self.split]
                self.swalked = [torch.cuda.Event() for _ in self.split]
                self.splanned = [torch.cuda.Event() for _ in self.split]
                self.sdone = None   # the last split batch's expansions are done (its buffers are free)

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        """Drain every stream of the pipeline and release the CU-masked ones
        (_lib.release_stream); the pipeline is unusable afterwards.  Idempotent."""
        if self._closed:
            return
        self.torch.cuda.synchronize(self.dev)
        # a pinned host tensor copied to on a stream (the compacted windows' live counts) records
        # an event on that stream when it is freed: free them while the streams exist (freed after
        # release_stream, the event record fails and aborts the process, e.g. at interpreter exit)
        for cx in self.ctxs:
            if getattr(cx, "nlive_host", None) is not None:
                cx.nlive_host = None
        for st in self._owned:
            st.synchronize()
            _lib.release_stream(st)
        self._owned.clear()
        self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    # ------------------------------------------------------------------ helpers
    @property
    def cst(self):   # the commit stream (gated schedule with commit_stream only): created on first use
        if self._cst is None:
            self._cst = self._mk()
        return self._cst

    def ctx_of(self, k):
        return self.ctxs[k % len(self.ctxs)]

    def _p(self, t):
        return C.c_void_p(t.data_ptr())

    def tl_mark(self, key, j, stream):
        if self.cfg.timeline:
            e = self.torch.cuda.Event(enable_timing=True)
            e.record(stream)
            self.tl.setdefault(key, {})[j] = e

    def expand_args(self, cx):
        return (self.sim._eng, self._p(cx.state), cx.chain0, self.n, 0, self.secs, None, C.byref(cx.tr),
                C.byref(cx.st) if cx.st is not None else None, self._p(cx.plan), self._p(cx.scratch),
                cx.scratch.numel())

    # ------------------------------------------------------------------ one batch at a time
    def one_step(self, k):
        """A whole batch on its context's streams (multi-window batches, or no overlap)."""
        L, sim, n, secs, win, cfg = self.L, self.sim, self.n, self.secs, self.win, self.cfg
        cx = self.ctx_of(k)
        chain0 = cx.chain0 = self.chain0_of(k)                 # fresh global chains every batch
        _lib.check(L.tmh_init(sim._eng, self._p(cx.state), chain0, n, None, cx.sptr))
        if self.nwin == 1 or sim.path != "time_parallel":
            for s0 in range(0, secs, win):   # windows: a trace window is overwritten by the next
                w = min(win, secs - s0)
                _lib.check(L.tmh_plan(sim._eng, s0, w, self._p(cx.plan), cx.sptr))
                _lib.check(L.tmh_step(sim._eng, self._p(cx.state), chain0, n, s0, w, None,
                                      C.byref(cx.tr), C.byref(cx.st) if cx.st is not None else None,
                                      self._p(cx.plan), self._p(cx.scratch), cx.scratch.numel(), cx.sptr))
            return
        if cfg.compact and cfg.mode == "stats":   # windows in order, the live chains of each only
            self.compact_batches([k], init=False)
            return
        # multi-window: each window's plan, draws and walk on the context's walk stream,
        # up to two windows ahead of the expansions on its stream (engine.run_windows)
        wins = [(s0, min(win, secs - s0)) for s0 in range(0, secs, win)]
        if getattr(cx, "pstream", None) is None:   # the context's plan stream (plans are per batch)
            cx.pstream = self._mk()
        run_windows(L, sim._eng, cx.state, chain0, n, wins, cx.wbufs, cx.stream, cx.wstream, lambda w: cx.tr, cx.st,
                    plan_stream=cx.pstream)

    def compact_batches(self, ks, init=True):
        """Compacted multi-window statistics batches (C5), one per context, advanced window
        by window together: every window after the first runs on the chains still live
        (tmh_live_chains -> tmh_state_move gather, tmh_set_chain_ids, tmh_step, scatter).
        The chain ids are engine state read at each launch, so the contexts' launches are
        issued one context at a time while their streams run concurrently.

        Round 6: no host drain per window.  Each context's live count goes to pinned host
        memory behind an event on its own stream, and the host waits for that context's
        count only, just before issuing its next window -- the other contexts' windows keep
        the GPU busy meanwhile (round 5 synchronised every context's stream at every window,
        so all of them drained before any next window was issued).  The window's plan
        (chain-independent: the same clock / geometry table for every batch of the group)
        is built once per window on a plan stream, into one of three rotating buffers,
        instead of once per context."""
        L, sim, n, secs, win = self.L, self.sim, self.n, self.secs, self.win
        torch = self.torch
        cxs = [self.ctx_of(k) for k in ks]
        assert len({id(c) for c in cxs}) == len(cxs), "one batch per context"
        if init:
            for k, cx in zip(ks, cxs):
                cx.chain0 = self.chain0_of(k)
                _lib.check(L.tmh_init(sim._eng, self._p(cx.state), cx.chain0, n, None, cx.sptr))
        wins = [(s0, min(win, secs - s0)) for s0 in range(0, secs, win)]
        NP = 3
        if getattr(self, "_cplans", None) is None:   # the group's plan buffers and stream
            self._cplans = [torch.empty(L.tmh_plan_bytes(win), dtype=torch.uint8, device=self.dev) for _ in range(NP)]
            self._cplan_ev = [torch.cuda.Event() for _ in range(NP)]
            self._cpst = self._mk()
        for cx in cxs:
            if getattr(cx, "nlive_host", None) is None:
                cx.nlive_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                cx.counted = torch.cuda.Event()
                cx.wdone = [torch.cuda.Event() for _ in range(NP)]
                cx.wdone_used = [False] * NP
        pst = self._cpst
        for wi, (s0, w) in enumerate(wins):
            b = wi % NP
            plan = self._cplans[b]
            for cx in cxs:   # the buffer's previous window is done on every context
                if cx.wdone_used[b]:
                    pst.wait_event(cx.wdone[b])
            _lib.check(L.tmh_plan(sim._eng, s0, w, self._p(plan), C.c_void_p(pst.cuda_stream)))
            self._cplan_ev[b].record(pst)
            for cx in cxs:
                nl = n
                if wi > 0:
                    cx.counted.synchronize()           # this context's count only
                    nl = int(cx.nlive_host[0])
                cx.stream.wait_event(self._cplan_ev[b])
                sp, cur = self._p(cx.state), cx.state
                try:
                    if nl < n:
                        cur = cx.work
                        if nl:
                            _lib.check(L.tmh_state_move(sim._eng, sp, n, self._p(cx.work), nl, self._p(cx.ids),
                                                        self._p(cx.nlive), nl, 0, cx.sptr))
                            _lib.check(L.tmh_set_chain_ids(sim._eng, self._p(cx.ids), n))
                    if nl:
                        _lib.check(L.tmh_step(sim._eng, self._p(cur), cx.chain0, nl, s0, w, None, C.byref(cx.tr),
                                              C.byref(cx.st), self._p(plan), self._p(cx.scratch),
                                              cx.scratch.numel(), cx.sptr))
                    if nl and cur is cx.work:
                        _lib.check(L.tmh_state_move(sim._eng, self._p(cx.work), nl, sp, n, self._p(cx.ids),
                                                    self._p(cx.nlive), nl, 1, cx.sptr))
                finally:
                    _lib.check(L.tmh_set_chain_ids(sim._eng, None, 0))
                cx.wdone[b].record(cx.stream)
                cx.wdone_used[b] = True
                if wi + 1 < len(wins):   # the next window's live chains, counted behind this window
                    _lib.check(L.tmh_live_chains(sim._eng, sp, n, None, self._p(cx.ids), self._p(cx.nlive), cx.sptr))
                    with torch.cuda.stream(cx.stream):
                        cx.nlive_host.copy_(cx.nlive, non_blocking=True)
                    cx.counted.record(cx.stream)

    # ------------------------------------------------------------------ round 1's staggered schedule
    def _build(self, k):      # construction of batch k's chains, its plan and draws
        L, sim, cx = self.L, self.sim, self.ctx_of(k)
        cx.chain0 = self.chain0_of(k)
        if self.cfg.build_on == "walk":   # on the batch's walk stream, beside the running expansion
            bs, bp = cx.wstream, cx.wptr
        else:                          # in order on the expansion stream
            bs, bp = self.estream, self.eptr
        if cx.expanded is not None:   # after the commit of the context's previous batch (it reads
            bs.wait_event(cx.expanded)   # and writes the state and scratch this construction resets)
        _lib.check(L.tmh_init(sim._eng, self._p(cx.state), cx.chain0, self.n, None, bp))
        _lib.check(L.tmh_plan(sim._eng, 0, self.secs, self._p(cx.plan), bp))
        _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, 0, self.secs, self._p(cx.plan),
                                   self._p(cx.scratch), cx.scratch.numel(), None, 0, _lib.WALK_DRAWS, bp))
        cx.done.record(bs)

    def _start(self, k):      # the segment walk of batch k, on its context's walk stream
        L, sim, cx = self.L, self.sim, self.ctx_of(k)
        cx.wstream.wait_event(cx.done)
        _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, 0, self.secs, self._p(cx.plan),
                                   self._p(cx.scratch), cx.scratch.numel(), None, 0, _lib.WALK_SEGMENTS, cx.wptr))
        cx.walked.record(cx.wstream)

    def _finish(self, k):     # the expansion on the expansion stream, then its commit on the
        L, cx = self.L, self.ctx_of(k)   # batch's walk stream, beside the next batch's expansion
        self.estream.wait_event(cx.walked)
        args_ = self.expand_args(cx)
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL, self.eptr))
        cx.kernel_done.record(self.estream)
        cx.wstream.wait_event(cx.kernel_done)
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, cx.wptr))
        if cx.expanded is None:
            cx.expanded = self.torch.cuda.Event()
        cx.expanded.record(cx.wstream)

    # ------------------------------------------------------------------ the gated schedule (C2)
    # One walk stream per walk in flight and one construction stream for all batches.
    # When the walk of batch k ends, three streams are released together: the
    # expansion of k, the walk of k + W and the construction of k + A.  Their
    # workgroups are then dispatched interleaved, so the walk (one long-lived wave
    # per SIMD) and the construction kernels are resident beside the expansion
    # instead of queueing behind its 10,800 workgroups (a kernel launched while an
    # expansion fills the CUs waits for its tail: the walks then ran three at a time,
    # between expansions, rocprofv3 kernel trace r02).
    def g_build(self, j, gate):
        L, sim, cfg = self.L, self.sim, self.cfg
        cx = self.ctx_of(j)
        cx.chain0 = self.chain0_of(j)
        bst = self.bsts[j % len(self.bsts)]
        bp = C.c_void_p(bst.cuda_stream)
        if gate is not None:
            bst.wait_event(gate)
        if cx.expanded is not None:                        # the context's previous batch is committed
            bst.wait_event(cx.expanded)
        if self.psts is not None:   # the plan beside the chains' init, on its own stream
            pst = self.psts
            if gate is not None:
                pst.wait_event(gate)
            if cx.expanded is not None:   # the previous batch of this context read the plan
                pst.wait_event(cx.expanded)
            _lib.check(L.tmh_plan(sim._eng, 0, self.secs, self._p(cx.plan), C.c_void_p(pst.cuda_stream)))
            if getattr(cx, "planned", None) is None:
                cx.planned = self.torch.cuda.Event()
            cx.planned.record(pst)
            _lib.check(L.tmh_init(sim._eng, self._p(cx.state), cx.chain0, self.n, None, bp))
            bst.wait_event(cx.planned)
        else:
            _lib.check(L.tmh_init(sim._eng, self._p(cx.state), cx.chain0, self.n, None, bp))
            _lib.check(L.tmh_plan(sim._eng, 0, self.secs, self._p(cx.plan), bp))
        _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, 0, self.secs, self._p(cx.plan),
                                   self._p(cx.scratch), cx.scratch.numel(), None, 0, _lib.WALK_DRAWS, bp))
        cx.done.record(bst)
        self.tl_mark("built", j, bst)

    def g_walk(self, j):
        L, sim = self.L, self.sim
        cx = self.ctx_of(j)
        wst = self.wsts[j % self.W]
        wst.wait_event(cx.done)
        self.tl_mark("walk0", j, wst)
        _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, 0, self.secs, self._p(cx.plan),
                                   self._p(cx.scratch), cx.scratch.numel(), None, 0, _lib.WALK_SEGMENTS,
                                   C.c_void_p(wst.cuda_stream)))
        cx.walked.record(wst)
        self.tl_mark("walk1", j, wst)

    def g_expand(self, j):
        L, cfg = self.L, self.cfg
        cx = self.ctx_of(j)
        es, ep = self.estream, self.eptr
        es.wait_event(cx.walked)
        args_ = self.expand_args(cx)
        self.tl_mark("exp0", j, es)
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL, ep))
        self.tl_mark("exp1", j, es)
        if cx.expanded is None:
            cx.expanded = self.torch.cuda.Event()
        if cfg.commit_stream:   # fixup + commit beside the next expansion
            cx.kernel_done.record(es)
            self.cst.wait_event(cx.kernel_done)
            _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, C.c_void_p(self.cst.cuda_stream)))
            cx.expanded.record(self.cst)
        else:
            _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, ep))
            cx.expanded.record(es)

    # the run's first batch in consecutive windows (first_split): as engine.run_windows, each
    # window's draws + walk chained to the previous window's walk (tmh_walk_part with its
    # scratch as prev), the expansions in order behind them on the expansion stream
    def s_build(self, j):
        L, sim = self.L, self.sim
        cx = self.ctx_of(j)
        cx.chain0 = self.chain0_of(j)
        bst, bp = self.bst, self.bst_p
        if cx.expanded is not None:
            bst.wait_event(cx.expanded)
        if self.sdone is not None:   # a previous run's split batch still reading the window buffers
            bst.wait_event(self.sdone)
        _lib.check(L.tmh_init(sim._eng, self._p(cx.state), cx.chain0, self.n, None, bp))
        (s0, k), (plan, scr) = self.split[0], self.sbufs[0]
        _lib.check(L.tmh_plan(sim._eng, s0, k, self._p(plan), bp))
        _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, s0, k, self._p(plan),
                                   self._p(scr), scr.numel(), None, 0, _lib.WALK_DRAWS, bp))
        cx.done.record(bst)
        self.tl_mark("built", j, bst)
        for w in range(1, len(self.split)):   # the later windows' plans, after the first window's draws
            (s0, k), (plan, _) = self.split[w], self.sbufs[w]
            _lib.check(L.tmh_plan(sim._eng, s0, k, self._p(plan), bp))
            self.splanned[w].record(bst)

    def s_walk(self, j):
        L, sim = self.L, self.sim
        cx = self.ctx_of(j)
        wst = self.wsts[j % self.W]
        wp = C.c_void_p(wst.cuda_stream)
        wst.wait_event(cx.done)
        self.tl_mark("walk0", j, wst)
        for w, ((s0, k), (plan, scr)) in enumerate(zip(self.split, self.sbufs)):
            parts, ps, pk = _lib.WALK_SEGMENTS, None, 0
            if w > 0:
                wst.wait_event(self.splanned[w])
                parts = _lib.WALK_DRAWS | _lib.WALK_SEGMENTS
                ps, pk = self._p(self.sbufs[w - 1][1]), self.split[w - 1][1]
            _lib.check(L.tmh_walk_part(sim._eng, self._p(cx.state), cx.chain0, self.n, s0, k, self._p(plan),
                                       self._p(scr), scr.numel(), ps, pk, parts, wp))
            self.swalked[w].record(wst)
        cx.walked.record(wst)
        self.tl_mark("walk1", j, wst)

    def s_expand(self, j):
        L = self.L
        cx = self.ctx_of(j)
        es, ep = self.estream, self.eptr
        esz = self.torch.finfo(self.sim.real).bits // 8   # the trace rows of window w start at row s0
        last = len(self.split) - 1
        for w, ((s0, k), (plan, scr)) in enumerate(zip(self.split, self.sbufs)):
            es.wait_event(self.swalked[w])
            if w == 0:
                self.tl_mark("exp0", j, es)
            tr = _lib.Trace(None, None, *((cx.trace[f].data_ptr() + s0 * self.n * esz) if f in cx.trace else None
                                          for f in ("pv", "meter", "residual")), self.n)
            args_ = (self.sim._eng, self._p(cx.state), cx.chain0, self.n, s0, k, None, C.byref(tr),
                     C.byref(cx.st) if cx.st is not None else None, self._p(plan), self._p(scr), scr.numel())
            if w < last:
                _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL | _lib.EXPAND_COMMIT, ep))
            else:
                _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL, ep))
                self.tl_mark("exp1", j, es)
                _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, ep))
        if cx.expanded is None:
            cx.expanded = self.torch.cuda.Event()
        cx.expanded.record(es)
        if self.sdone is None:
            self.sdone = self.torch.cuda.Event()
        self.sdone.record(es)

    def run_gated(self, k0, cnt):
        """W walks in flight: when the walk of batch k ends, the expansion of k, the walk
        of k + W (on k's walk stream) and the construction of k + A are released together."""
        L, sim, cfg, W, A = self.L, self.sim, self.cfg, self.W, self.A
        end = k0 + cnt
        for j in range(k0, min(k0 + A, end)):
            # the run's first walk is the pipeline's fill latency (its expansion waits for it with
            # nothing else to do): chain order, whose windiest wavefront is shorter than the wind
            # order's (four windy chains); the wind order for the rest, which run beside expansions
            if cfg.walk_order:
                _lib.check(L.tmh_set_walk_order(sim._eng, 0 if (j == k0 and W > 1) or self._drains(j, end) else 1))
            if j == k0 and self.split:
                self.s_build(j)
            else:
                self.g_build(j, None)
        for j in range(k0, min(k0 + W, end)):
            if j == k0 and self.split:
                self.s_walk(j)
            else:
                self.g_walk(j)
        for k in range(k0, end):
            gate = self.ctx_of(k).walked
            if k + A < end:
                if cfg.walk_order:   # the order is read by the construction's draws
                    _lib.check(L.tmh_set_walk_order(sim._eng, 0 if self._drains(k + A, end) else 1))
                self.g_build(k + A, gate)
            if k + W < end:
                self.g_walk(k + W)
            if k == k0 and self.split:
                self.s_expand(k)
            else:
                self.g_expand(k)

    def _drains(self, j, end):
        """Batch j is among the run's last drain_order: little is left to overlap its walk, so it
        walks in chain order, whose windiest wavefront is shorter than the wind order's."""
        return self.W > 1 and j >= end - int(self.cfg.drain_order)

    def gated(self):
        """Whether `run` takes the gated schedule (one-window, staggered batches)."""
        cfg = self.cfg
        return (self.nwin == 1 and cfg.stagger and cfg.schedule == "gated"
                and len(self.ctxs) >= max(self.A + 1, self.W + 2))

    def run(self, k0, cnt):
        """Batches k0 .. k0 + cnt - 1.  One-window batches are software-pipelined:
        construction + plan and the expansions run in order, the segment walks of the
        next batches on their own streams beside them, so the one-wave-per-SIMD walks
        overlap the expansion instead of running in lockstep with it.  The caller
        synchronises (the outputs of batch k sit in context k % pipeline)."""
        if self._closed:
            raise RuntimeError("BatchPipeline is closed")
        cfg = self.cfg
        if self.nwin > 1 and cfg.compact and cfg.mode == "stats" and self.sim.path == "time_parallel":
            P = len(self.ctxs)   # compacted windows: one group of batches (one per context) at a time
            for g in range(k0, k0 + cnt, P):
                self.compact_batches(list(range(g, min(g + P, k0 + cnt))))
            return
        if self.nwin > 1 or not cfg.stagger:
            for k in range(k0, k0 + cnt):
                self.one_step(k)
            return
        if self.gated():
            self.run_gated(k0, cnt)
            return
        D = len(self.ctxs)
        ahead = D - 1
        for k in range(k0, min(k0 + D, k0 + cnt)):
            self._build(k)
        for k in range(k0, min(k0 + ahead, k0 + cnt)):
            self._start(k)
        for k in range(k0, k0 + cnt):
            if k + ahead < k0 + cnt:
                self._start(k + ahead)
            self._finish(k)
            if k + D < k0 + cnt:
                self._build(k + D)

    # ------------------------------------------------------------------ statistics
    def sync(self):
        torch = self.torch
        torch.cuda.synchronize()
        for cx in self.ctxs:   # (streams a schedule never created have nothing to wait for)
            for st_ in (cx._stream, cx._wstream):
                if st_ is not None:
                    st_.synchronize()

    def totals(self):
        """stats mode: the node-local totals over every context (histogram, energies, peak;
        dist.chain_totals: every chain's accumulated seconds, exact integer energy sums).
        A context's per-chain accumulators keep adding over every batch run on it until
        reset_stats(); the fixed-point grid holds |energy| < 2^42 W s per chain slot (~15
        chain-years at 9 kW): past it chain_totals raises OverflowError, so reset between
        runs longer than that."""
        from .dist import chain_totals
        hist = sum(cx.hist for cx in self.ctxs)
        return chain_totals(self.torch.cat([cx.acc for cx in self.ctxs], dim=1), hist)

    def reset_stats(self):
        for cx in self.ctxs:
            cx.hist.zero_()
            cx.acc[:3].zero_()
            cx.acc[3].fill_(-float("inf"))

    def faulted(self):
        """chains with a nonzero status over the contexts' last batches"""
        bad = 0
        for cx in self.ctxs:
            self.sim.state = cx.state
            bad += int((self.sim.status() != 0).sum())
        return bad
