#!/usr/bin/env python3
"""Benchmark: simulated chain-seconds/sec (BASELINE.json metric) on the C2 workload.

Workload (BASELINE.json configs[1]): 4,096 independent chains
(Munich site, Europe/Berlin clock) x one day (86,400 s) at 1 s, fp32 per-second
arithmetic (fp64 Markov state), keyed Philox uniforms, trace mode: every
chain-second's meter, pv and residual streamed to HBM (12 B / chain-second).
One bench "step" = one batch: build the day's clock/geometry table, construct
4,096 fresh chains (new global chain ids every step) and advance them 86,400 s.

Multi-GPU, one rank per GPU: `--gpus N` run directly (no WORLD_SIZE in the
environment) starts N child ranks itself (`launch_ranks`, before this process
touches torch or the GPU); under torchrun WORLD_SIZE must equal N.  C2 scales
weakly: every rank runs its own 4,096 chains with distinct global ids, no
data-path collective (chains are independent).  C3 / C4 / C5
scale strongly: the node total (1,048,576 chains / 16,384 / 65,536 sites,
BASELINE.json configs[2..4]) is split into contiguous global-id shards
(`dist.shard`), and the RCCL all-reduce of the statistics is in the timed
region.  value = chain-seconds of all ranks / max rank time.

Roofline: the dominant kernel (expand_kernel, P2 of the time-parallel path) is
timed with HIP events the library records on the stream it runs on
(tmh_profile_enable / tmh_profile_read).  Trace mode is HBM-bound: achieved =
12 B x chains x seconds per launch / mean launch time, against 8 TB/s.  Stats
mode writes no trace and is VALU-bound: achieved = the launch's
VALU lane-ops (rocprofv3 SQ_INSTS_VALU x 64, profiles/pmc_kernels.json, measured
on the same workload) / mean launch time, against 256 CU x 4 SIMD x 32 lanes x
2.4 GHz.  `traffic` = HBM bytes per launch from the same PMC record (FETCH_SIZE x
2 + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), null when no record
matches.  cpu_baseline: the C oracle (oracle/tmh_oracle.c, "port") on a bounded
sample of the same workload on this host, rank 0, N = 1: all threads of the
box's share (<= 16) and one thread.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
TRACE_BYTES = 12               # meter + pv + residual, fp32 (24 in fp64)
# VALU issue peak: 256 CUs x 4 SIMD-32 x 32 lanes per cycle x 2.4 GHz (a wave64
# instruction issues over 2 cycles, MI355X_MICROARCH.md), in lane-ops/s
VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12

# BASELINE.json configs[1..4]: C2 4,096 sites on one GPU (weak scaling: per GPU);
# C3 1 M chains, C4 16,384 sites, C5 65,536 sites for the node (strong scaling)
DEFAULT_CHAINS = {"c2": 4096, "c3": 1048576, "c4": 16384, "c5": 65536}
STRONG = ("c3", "c4", "c5")


def rank_chains(workload, chains, rank, world):
    """This rank's chains: (chain0 of its shard within one batch, n_local, n_node, scaling).

    Weak (c2): every rank has `chains` of its own, rank r's ids start at r * chains.
    Strong (c3 / c4 / c5): `chains` is the node total, split into contiguous shards
    (dist.shard: sizes differ by at most one)."""
    from tmhpvsim_amd.dist import shard
    if workload in STRONG:
        c0, n = shard(chains, rank, world)
        return c0, n, chains, "strong"
    return rank * chains, chains, chains * world, "weak"


def launch_ranks(n, argv, script=None):
    """`bench.py --gpus N` started without a launcher: N child ranks of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, one GPU each), started before this
    process imports torch.cuda or touches the GPU; this process only waits and
    returns the worst exit status (it never execs).  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    if os.environ.get("TMH_BENCH_SHARE_GPU") != "1":
        visible = _visible_gpus()
        if visible < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {visible} "
                  f"(TMH_BENCH_SHARE_GPU=1 runs every rank on device 0, rehearsal only)", file=sys.stderr)
            return 2
    with socket.socket() as s:   # a free rendezvous port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:   # one rank failed: the others would wait in a collective
                    rc = r
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc if rc >= 0 else 128 - rc


def _visible_gpus():
    """GPUs this process may use, without initialising HIP (torch.cuda.device_count
    reads the device list only on this image)."""
    import torch
    return torch.cuda.device_count()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2: the headline (BASELINE.json configs[1]); c3: 1,048,576 chains x 1 day, stats, two "
                         "batches in flight (74 GB of scratch each); c4: 16,384 chains x the year 2019 "
                         "(Europe/Berlin wall clock, stats, day windows); c5: the lat/lon sweep (65,536 sites x 1 "
                         "week, markov cc with per-site tables, per-site PV geometry, stats mode, day windows)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chains", type=int, default=None,
                    help="c2: chains per GPU (4096, weak scaling); c3 / c4 / c5: chains of the whole node, "
                         "sharded over the GPUs (1048576 / 16384 / 65536, strong scaling)")
    ap.add_argument("--seconds", type=int, default=None, help="c2: 86400, c5: 604800")
    ap.add_argument("--window", type=int, default=None, help="steps per tmh_step window (c2: all, c5: 86400)")
    ap.add_argument("--cc", default=None, choices=["faithful", "markov"],
                    help="hourly cloud-cover mode (c2: faithful, the reference's; c5: markov, whose low-cover "
                         "AssertionError (cloud_cover_binary.py:91) ends most chains within days)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--mode", default=None, choices=["trace", "stats"], help="c2: trace, c5: stats")
    ap.add_argument("--start", default=None, help="c2/c5: 2019-09-05 00:00:00, c4: 2019-01-01 00:00:00")
    ap.add_argument("--cpu-sample-chains", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", default="auto", choices=["auto", "sequential", "time_parallel"])
    ap.add_argument("--build-on", default=None, choices=["expand", "walk"],
                    help="stream of each batch's construction, plan and draws: in order on the expansion "
                         "stream, or ahead of its walk on the walk stream (default: walk for c2, else expand)")
    ap.add_argument("--no-stagger", dest="stagger", action="store_false",
                    help="issue each batch as one tmh_step (batches then run in lockstep across streams)")
    ap.add_argument("--walk-priority", default=None, choices=["high", "normal"],
                    help="HIP stream priority of the construction + segment walk (pipelined batches; "
                         "default: normal for c2, where construction shares the walk stream, else high)")
    ap.add_argument("--expand-priority", default="normal", choices=["high", "normal"],
                    help="HIP stream priority of the expansion stream (pipelined batches)")
    ap.add_argument("--schedule", default="gated", choices=["gated", "stagger"],
                    help="pipelined one-window batches: 'gated' releases the expansion of batch k, the walk of "
                         "k + 1 and the construction of k + 2 together when walk k ends; 'stagger' is round 1's")
    ap.add_argument("--walks", type=int, default=None,
                    help="gated schedule: segment walks in flight on their own streams (each batch's walk "
                         "overlaps the next one's; use with --walk-cpr > 1 so they share the CUs' walk slots)")
    ap.add_argument("--walk-cpr", type=int, default=1,
                    help="chains per walk row (tmh_set_walk_chains_per_row): the walk launches n / cpr rows "
                         "that take the next chain when theirs is done")
    ap.add_argument("--walk-lanes", type=int, default=0,
                    help="lanes per chain in the segment walk (tmh_set_walk_lanes: 4, 8 or 16; 0 = by batch size: 16 up to 8,192 chains, else 4)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; 0 = leave the environment's). "
                         "HIP maps streams round-robin onto that many hardware queues and a queue runs its "
                         "packets in order across the streams sharing it: with HIP's default 4 the expansion "
                         "stream shares a queue with another pipeline stream and waits for its kernels (same "
                         "box: 1.74-1.76 ms per C2 batch with 4 queues, 1.49-1.51 with 8, 1.47-1.51 with 16)")
    ap.add_argument("--secondary", default=None,
                    help="after the headline measurement (one GPU only), run the other configurations in child "
                         "processes and add their lines under 'secondary': all | none | a comma list of "
                         "c2_fp64,c3,c4,c5 (default: all for the C2 fp32 run with its CPU baseline, else none)")
    ap.add_argument("--timeline", action="store_true",
                    help="gated schedule: time each batch's build, walk and expansion with HIP events and add the "
                         "expansion stream's idle gaps (and what it waited for) to the JSON line")
    ap.add_argument("--walk-order", type=int, default=1,
                    help="walk rows windiest chain first (tmh_set_walk_order, 1) or in chain order (0)")
    ap.add_argument("--walk-cus", type=int, default=0,
                    help="gated schedule: run the segment walks on CU-mask bits 0 .. K-1 only (a CU-masked HIP "
                         "stream, tmh_stream_create_cus; 0 = all CUs)")
    ap.add_argument("--other-cus", default="all", choices=["all", "rest"],
                    help="with --walk-cus: the expansion, construction and commit streams on all CUs or on the "
                         "CUs the walks do not use")
    ap.add_argument("--build-ahead", type=int, default=None,
                    help="gated schedule: when the walk of batch k ends, the construction of batch k + A is "
                         "released (default A = walks + 2 with two or more walks, else walks + 1; needs --pipeline >= A + 1)")
    ap.add_argument("--build-priority", default="normal", choices=["high", "normal"],
                    help="gated schedule: HIP stream priority of the construction stream")
    ap.add_argument("--minutes-ahead", type=int, default=None,
                    help="gated schedule: build each batch's minute table with its construction (1) instead of "
                         "before its expansion on the expansion stream (0, the default)")
    ap.add_argument("--commit-stream", type=int, default=None,
                    help="gated schedule: each batch's fixup + commit on a stream of their own beside the next "
                         "expansion (1) or after its expansion on the expansion stream (0, the default)")
    ap.add_argument("--compact", type=int, default=None,
                    help="multi-window stats workloads: run each window after the first on the chains still "
                         "live (faulted chains, e.g. C5's markov AssertionError, drop out); default 1 for c5")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="batches in flight on separate HIP streams (1 = no overlap): the segment walks of the "
                         "next batches (latency-bound, one wave per SIMD) run beside this batch's expansion")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    c5, c4 = a.workload == "c5", a.workload == "c4"
    a.chains = a.chains or DEFAULT_CHAINS[a.workload]
    a.seconds = a.seconds or {"c2": 86400, "c3": 86400, "c4": 365 * 86400, "c5": 604800}[a.workload]
    if a.compact is None:
        a.compact = int(c5)
    # C2: two walks in flight (r02, same-box A/B: 1.71-1.72 ms per batch against 1.81 with one)
    a.walks = a.walks if a.walks is not None else (2 if a.workload == "c2" else 1)
    # C5's compacted windows walk and expand in turn (latency-bound walk): 16 lanes per
    # chain (1.76e10 against 1.73e10 with the batch-size default, r02 same box)
    a.walk_lanes = a.walk_lanes or (16 if c5 else 0)
    # construction released walks + 2 batches ahead (round 3, 16 queues, same box, 3 reps:
    # 1.41-1.44 ms per C2 batch at 4, 5 or 6 ahead against 1.48-1.55 at 3, 1.86-1.90 at 2)
    a.build_ahead = a.build_ahead or max(1, a.walks) + (2 if a.walks > 1 else 1)
    # c3: two 1 M-chain batches in flight (2 x 83 GB of state + scratch): +3 % over one (r02)
    a.pipeline = a.pipeline or (2 if a.workload == "c3" else a.build_ahead + 1)
    # round 3, 16 hardware queues, same box, 3 reps: the minute table before its expansion
    # and the fixup + commit after it, both on the expansion stream, 1.485-1.490 ms per C2
    # batch against 1.528-1.552 with both on streams of their own (round 2's choice, made
    # when 4 queues serialised the streams anyway); either one alone 1.49-1.52
    if a.minutes_ahead is None:
        a.minutes_ahead = 0
    if a.commit_stream is None:
        a.commit_stream = 0
    a.mode = a.mode or ("trace" if a.workload == "c2" else "stats")
    if a.secondary is None:
        # the full report (the default C2 run with its CPU baseline) carries them; quick runs do not
        a.secondary = "all" if (a.workload == "c2" and a.precision == "fp32" and not a.no_cpu_baseline) else "none"
    a.cc = a.cc or ("markov" if c5 else "faithful")
    a.window = min(a.window or (86400 if (c5 or c4) else a.seconds), a.seconds)
    a.start = a.start or ("2019-01-01 00:00:00" if c4 else "2019-09-05 00:00:00")
    # C2 (same-box A/B, r01): construction on the walk stream at normal priority
    # 1.94e11 chain-s/s vs 1.82e11 on the expansion stream with high-priority walks
    a.build_on = a.build_on or ("walk" if a.workload == "c2" else "expand")
    a.walk_priority = a.walk_priority or ("normal" if a.workload == "c2" else "high")
    return a


SECONDARY = {   # --secondary: the other BASELINE.json configs, each in a child process of its own
    "c2_fp64": ["--precision", "fp64", "--steps", "10", "--warmup", "3"],
    "c3": ["--workload", "c3", "--steps", "4", "--warmup", "1"],
    "c4": ["--workload", "c4", "--steps", "2", "--warmup", "1"],
    "c5": ["--workload", "c5", "--steps", "2", "--warmup", "1"],
}


def secondary_lines(args):
    """The fp64 C2 line (the reference's precision) and the C3 / C4 / C5 stats-mode lines,
    each a fresh bench.py process on this GPU after the headline measurement, so the
    default run reports every configuration's rate and roofline.  A failed one reports
    its error; the headline line is printed either way."""
    import subprocess
    out = {}
    for name, extra in SECONDARY.items():
        if args.secondary != "all" and name not in args.secondary.split(","):
            continue
        cmd = [sys.executable, os.path.abspath(__file__), "--no-cpu-baseline", "--secondary", "none",
               "--hw-queues", str(args.hw_queues)] + extra
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            roof = d.get("roofline", {})
            out[name] = {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
                         "steps": d["steps"], "dtype": d["dtype"], "workload": d["config"]["workload"],
                         "roofline": {k: roof.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                               "kernel_ms")},
                         "roofline_alone": roof.get("alone"), "faulted_chains": d.get("faulted_chains"),
                         "chain_seconds_live": d.get("chain_seconds_live")}
        except Exception as e:   # noqa: BLE001 - report, never lose the headline line
            out[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
    return out


def cpu_baseline(args, kw):
    """The C oracle on a bounded sample of the same workload (same site(s)/day/modes, fp64):
    OpenMP over the box's CPU share (<= 16 threads) and one thread on a smaller sample."""
    from oracle import oracle as O
    from tmhpvsim_amd.params import CC_MARKOV, ModelParams
    nproc = os.cpu_count() or 1
    threads = max(1, min(16, nproc))
    c5 = args.workload == "c5"
    mp = ModelParams(cc_mode=CC_MARKOV if args.cc == "markov" else 0)
    secs = min(args.seconds, 86400)

    def timed(n, nt):
        extra = {}
        if c5:   # the first n sites of the sweep, their tables; geometry per chain-second like the GPU path
            extra = dict(tables=tuple(x[:n] for x in kw["shape_tables"]), sites=kw["sites"][:n])
        t = time.perf_counter()
        O.run(mp, 10 ** 9, n, secs, args.start, tz="Europe/Berlin", n_threads=nt, outputs=("residual",), **extra)
        return time.perf_counter() - t

    O.run(mp, 0, 2, 600, args.start, tz="Europe/Berlin", n_threads=1)   # load + warm
    n = args.cpu_sample_chains if not c5 else min(args.cpu_sample_chains // 16, args.chains)
    dt = timed(n, threads)
    n1 = max(1, n // 16)
    dt1 = timed(n1, 1)
    what = 'C5 sites/tables, ' + args.cc if c5 else 'C2 site/day'
    return {"value": n * secs / dt, "unit": "chain-seconds/s", "cores": threads, "kind": "port",
            "sample": f"{n} chains x {secs} s ({what}, fp64 C oracle, {threads} OpenMP threads = the GPU box's CPU "
                      f"share for one GPU (nproc={nproc} counts the whole machine), {dt:.1f} s wall)",
            "single_thread": {"value": n1 * secs / dt1, "cores": 1,
                              "sample": f"{n1} chains x {secs} s, 1 thread, {dt1:.1f} s wall"},
            "reference_python_per_core": {"value": 4.0e4, "source": "BASELINE.md (timed in the build container; "
                                                                    "the reference cannot run on the GPU box)"}}


def pmc_record(args, n, launch_secs):
    """The committed PMC record of the dominant kernel on this workload
    (profiles/pmc_kernels.json, written by scripts/pmc_summary.py from the
    rocprofv3 --pmc passes of scripts/pmc_workload.sh): per-launch VALU / SALU
    wave-instructions and HBM bytes.  None when that workload was not measured
    with this build of the library (the record's build_stamp: a hash of the
    sources and compile flags), so a kernel change cannot reuse stale counters."""
    from tmhpvsim_amd.build import build_stamp
    path = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    try:
        recs = json.load(open(path))["records"]
    except (OSError, ValueError, KeyError):
        return None
    stamp = build_stamp()
    recs = [r for r in recs if r.get("build_stamp") == stamp]
    want = dict(workload=args.workload, chains=n, launch_seconds=launch_secs, precision=args.precision,
                mode=args.mode, cc=args.cc)
    compact = int(bool(args.compact and args.mode == "stats" and args.seconds > launch_secs))
    for r in recs:   # a compacted run's launches hold fewer chains: its own record
        if all(r.get(k) == v for k, v in want.items()) and int(r.get("compact", 0)) == compact:
            return r
    return None


def main():
    args = parse()
    if args.hw_queues:   # before anything starts the HIP runtime (it reads this once)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # TMH_BENCH_SHARE_GPU=1 (rehearsal only): every rank on device 0 over gloo, so
        # the N > 1 path runs on a one-GPU box; the scaling runs use one GPU per rank, RCCL
        if os.environ.get("TMH_BENCH_SHARE_GPU") == "1":
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if world > 1:   # the process group's own count, not the flag
        world = dist.get_world_size()
        rank = dist.get_rank()

    from tmhpvsim_amd import _lib
    from tmhpvsim_amd.engine import BatchedSim
    from tmhpvsim_amd.params import CC_MARKOV, ModelParams, site_grid, site_shape_tables

    from tmhpvsim_amd.dist import all_reduce_stats

    L = _lib.load()
    shard0, n, n_node, scaling = rank_chains(args.workload, args.chains, rank, world)
    secs, win = args.seconds, args.window

    def batch_chain0(k):   # global id of this rank's first chain in batch k: fresh chains every batch
        return k * n_node + shard0

    c5 = args.workload == "c5"
    kw = {}
    if c5:   # the node's 256 x 256 lat/lon grid (or chains / 256 rows); this rank's shard of it
        grid = site_grid(max(1, (args.chains + 255) // 256), 256)
        kw = dict(shape_tables=site_shape_tables(n, site0=shard0), sites=grid[shard0:shard0 + n])
    sim = BatchedSim(n, args.start, tz="Europe/Berlin", params=ModelParams(cc_mode=CC_MARKOV if args.cc == "markov" else 0),
                     precision=args.precision, chain0=shard0, device=dev, horizon=secs, kernel_path=args.path, **kw)
    real = sim.real
    if args.walk_cpr != 1:
        _lib.check(L.tmh_set_walk_chains_per_row(sim._eng, args.walk_cpr))
    if args.walk_lanes:
        _lib.check(L.tmh_set_walk_lanes(sim._eng, args.walk_lanes))
    if hasattr(L, "tmh_set_walk_order"):
        _lib.check(L.tmh_set_walk_order(sim._eng, args.walk_order))

    nwin = (secs + win - 1) // win
    prio_lo, prio_hi = torch.cuda.Stream.priority_range()

    class Ctx:   # one batch in flight: its own state, plan, scratch, outputs and HIP streams
        # The context's own streams are created on first use: the gated schedule runs on
        # shared streams, and every extra stream shares one of HIP's few hardware queues
        # with a busy one (a queue runs its packets in order, across streams).
        @property
        def stream(self):
            if self._stream is None:
                self._stream = torch.cuda.Stream(dev)
            return self._stream

        @property
        def sptr(self):
            return C.c_void_p(self.stream.cuda_stream)

        @property
        def wstream(self):   # the walk runs on a stream of its own, high priority by default
            if self._wstream is None:
                self._wstream = torch.cuda.Stream(dev, priority=prio_hi if args.walk_priority == "high" else prio_lo)
            return self._wstream

        @property
        def wptr(self):
            return C.c_void_p(self.wstream.cuda_stream)

        def __init__(self):
            self._stream = self._wstream = None
            self.walked = torch.cuda.Event()
            self.done = torch.cuda.Event()
            self.kernel_done = torch.cuda.Event()
            self.expanded = None   # recorded after this context's last expansion
            self.state = torch.zeros(L.tmh_state_bytes(n), dtype=torch.uint8, device=dev)
            self.plan = torch.empty(L.tmh_plan_bytes(win), dtype=torch.uint8, device=dev)
            self.scratch = torch.empty(L.tmh_engine_scratch_bytes(sim._eng, n, win), dtype=torch.uint8, device=dev)
            if args.compact and args.mode == "stats" and nwin > 1:   # compacted windows: a working state
                self.work = torch.empty_like(self.state)
                self.ids = torch.empty(n, dtype=torch.int32, device=dev)
                self.nlive = torch.zeros(1, dtype=torch.int32, device=dev)
            if nwin > 1:   # second plan + scratch: window w+1's walk beside window w's expansion
                self.plan2 = torch.empty_like(self.plan)
                self.scratch2 = torch.empty_like(self.scratch)
                self.wev = [torch.cuda.Event(), torch.cuda.Event()]
                self.eev = [torch.cuda.Event(), torch.cuda.Event()]
            self.trace = {f: torch.empty(win, n, dtype=real, device=dev) for f in ("pv", "meter", "residual")} \
                if args.mode == "trace" else {}
            self.tr = _lib.Trace(None, None, *(self.trace[f].data_ptr() if f in self.trace else None
                                               for f in ("pv", "meter", "residual")), n)
            self.st = None
            if args.mode == "stats":
                self.hist = torch.zeros(4096, dtype=torch.int64, device=dev)
                self.acc = torch.zeros(4, n, dtype=torch.float64, device=dev)
                self.acc[3].fill_(-float("inf"))
                self.st = _lib.Stats(self.hist.data_ptr(), 4096, 0, -300.0, 9000.0, self.acc.data_ptr())

    ctxs = [Ctx() for _ in range(max(1, args.pipeline))]
    # one stream for every batch's expansion: expansions run back to back, in order
    # (they fill the chip on their own), while the walks of the next batches run on
    # their contexts' high-priority streams beside them
    estream = torch.cuda.Stream(dev, priority=prio_hi if args.expand_priority == "high" else prio_lo)
    eptr = C.c_void_p(estream.cuda_stream)
    torch.cuda.synchronize()
    L.tmh_profile_enable(sim._eng, 1)

    def one_step(k):   # a whole batch on its context's streams
        cx = ctxs[k % len(ctxs)]
        chain0 = batch_chain0(k)                          # fresh global chains every batch
        _lib.check(L.tmh_init(sim._eng, C.c_void_p(cx.state.data_ptr()), chain0, n, None, cx.sptr))
        if nwin == 1 or sim.path != "time_parallel":
            for s0 in range(0, secs, win):   # windows: a trace window is overwritten by the next
                w = min(win, secs - s0)
                _lib.check(L.tmh_plan(sim._eng, s0, w, C.c_void_p(cx.plan.data_ptr()), cx.sptr))
                _lib.check(L.tmh_step(sim._eng, C.c_void_p(cx.state.data_ptr()), chain0, n, s0, w, None,
                                      C.byref(cx.tr), C.byref(cx.st) if cx.st is not None else None,
                                      C.c_void_p(cx.plan.data_ptr()), C.c_void_p(cx.scratch.data_ptr()),
                                      cx.scratch.numel(), cx.sptr))
            return
        if args.compact and args.mode == "stats":   # windows in order, the live chains of each only
            sp = C.c_void_p(cx.state.data_ptr())
            for s0 in range(0, secs, win):
                w = min(win, secs - s0)
                nl, cur = n, cx.state
                if s0 > 0:
                    _lib.check(L.tmh_live_chains(sim._eng, sp, n, None, C.c_void_p(cx.ids.data_ptr()),
                                                 C.c_void_p(cx.nlive.data_ptr()), cx.sptr))
                    cx.stream.synchronize()                # n_live was written on the batch's stream
                    nl = int(cx.nlive.item())
                    if nl < n:
                        cur = cx.work
                        if nl:
                            _lib.check(L.tmh_state_move(sim._eng, sp, n, C.c_void_p(cx.work.data_ptr()), nl,
                                                        C.c_void_p(cx.ids.data_ptr()), C.c_void_p(cx.nlive.data_ptr()),
                                                        nl, 0, cx.sptr))
                            _lib.check(L.tmh_set_chain_ids(sim._eng, C.c_void_p(cx.ids.data_ptr()), n))
                if nl:
                    _lib.check(L.tmh_plan(sim._eng, s0, w, C.c_void_p(cx.plan.data_ptr()), cx.sptr))
                    _lib.check(L.tmh_step(sim._eng, C.c_void_p(cur.data_ptr()), chain0, nl, s0, w, None,
                                          C.byref(cx.tr), C.byref(cx.st), C.c_void_p(cx.plan.data_ptr()),
                                          C.c_void_p(cx.scratch.data_ptr()), cx.scratch.numel(), cx.sptr))
                if nl and cur is cx.work:
                    _lib.check(L.tmh_state_move(sim._eng, C.c_void_p(cx.work.data_ptr()), nl, sp, n,
                                                C.c_void_p(cx.ids.data_ptr()), C.c_void_p(cx.nlive.data_ptr()),
                                                nl, 1, cx.sptr))
                _lib.check(L.tmh_set_chain_ids(sim._eng, None, 0))
            return
        # multi-window: the segment walk of window w+1 (high-priority stream) beside the
        # expansion of window w; plans and draws on the expansion's stream (as BatchedSim.run)
        bufs = [(cx.plan, cx.scratch), (cx.plan2, cx.scratch2)]
        wins = [(s0, min(win, secs - s0)) for s0 in range(0, secs, win)]
        sp = C.c_void_p(cx.state.data_ptr())

        def views(w):
            return tuple(C.c_void_p(t.data_ptr()) for t in bufs[w & 1])

        def prev_of(w):
            return (views(w - 1)[1], wins[w - 1][1]) if w > 0 else (None, 0)

        def draws(w):
            pl, sc = views(w)
            _lib.check(L.tmh_plan(sim._eng, wins[w][0], wins[w][1], pl, cx.sptr))
            _lib.check(L.tmh_walk_part(sim._eng, sp, chain0, n, wins[w][0], wins[w][1], pl, sc, cx.scratch.numel(),
                                       *prev_of(w), _lib.WALK_DRAWS, cx.sptr))
            cx.wev[w & 1].record(cx.stream)

        def segments(w):
            pl, sc = views(w)
            cx.wstream.wait_event(cx.wev[w & 1])
            _lib.check(L.tmh_walk_part(sim._eng, sp, chain0, n, wins[w][0], wins[w][1], pl, sc, cx.scratch.numel(),
                                       *prev_of(w), _lib.WALK_SEGMENTS, cx.wptr))
            cx.eev[w & 1].record(cx.wstream)

        draws(0)
        segments(0)
        for w in range(len(wins)):
            cx.stream.wait_event(cx.eev[w & 1])
            if w + 1 < len(wins):
                draws(w + 1)
                segments(w + 1)
            pl, sc = views(w)
            _lib.check(L.tmh_expand(sim._eng, sp, chain0, n, wins[w][0], wins[w][1], None,
                                    C.byref(cx.tr), C.byref(cx.st) if cx.st is not None else None, pl, sc,
                                    cx.scratch.numel(), cx.sptr))

    def build(k):      # construction of batch k's chains, its plan and draws
        cx = ctxs[k % len(ctxs)]
        cx.chain0 = batch_chain0(k)
        if args.build_on == "walk":   # on the batch's walk stream, after the expansion
            bs, bp = cx.wstream, cx.wptr   # that last used this context: beside the running expansion
            if cx.expanded is not None:
                bs.wait_event(cx.expanded)
        else:                          # in order on the expansion stream
            bs, bp = estream, eptr
        _lib.check(L.tmh_init(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, None, bp))
        _lib.check(L.tmh_plan(sim._eng, 0, secs, C.c_void_p(cx.plan.data_ptr()), bp))
        _lib.check(L.tmh_walk_part(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs,
                                   C.c_void_p(cx.plan.data_ptr()), C.c_void_p(cx.scratch.data_ptr()),
                                   cx.scratch.numel(), None, 0, _lib.WALK_DRAWS, bp))
        cx.done.record(bs)

    def start(k):      # the segment walk of batch k, on its context's walk stream
        cx = ctxs[k % len(ctxs)]
        cx.wstream.wait_event(cx.done)
        _lib.check(L.tmh_walk_part(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs,
                                   C.c_void_p(cx.plan.data_ptr()), C.c_void_p(cx.scratch.data_ptr()),
                                   cx.scratch.numel(), None, 0, _lib.WALK_SEGMENTS, cx.wptr))
        cx.walked.record(cx.wstream)

    def finish(k):     # second half: the expansion (trace / stats) on the expansion stream, then its
        cx = ctxs[k % len(ctxs)]   # commit (fp32 guard-band fixup + state) on the batch's walk stream,
        estream.wait_event(cx.walked)   # beside the next batch's expansion (tmh_expand_part)
        args_ = (sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs, None, C.byref(cx.tr),
                 C.byref(cx.st) if cx.st is not None else None, C.c_void_p(cx.plan.data_ptr()),
                 C.c_void_p(cx.scratch.data_ptr()), cx.scratch.numel())
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL, eptr))
        cx.kernel_done.record(estream)
        cx.wstream.wait_event(cx.kernel_done)
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, cx.wptr))
        if cx.expanded is None:
            cx.expanded = torch.cuda.Event()
        cx.expanded.record(cx.wstream)

    # gated schedule: one walk stream and one construction stream for all batches.
    # When the walk of batch k ends, three streams are released together: the
    # expansion of k, the walk of k + 1 and the construction of k + 2.  Their
    # workgroups are then dispatched interleaved, so the walk (one long-lived wave
    # per SIMD) and the construction kernels are resident beside the expansion
    # instead of queueing behind its 10,800 workgroups (a kernel launched while an
    # expansion fills the CUs waits for its tail: the walks then ran three at a time,
    # between expansions, rocprofv3 kernel trace r02).
    W = max(1, args.walks)
    wsts = [torch.cuda.Stream(dev, priority=prio_hi if args.walk_priority == "high" else prio_lo) for _ in range(W)]
    bst = torch.cuda.Stream(dev, priority=prio_hi if args.build_priority == "high" else prio_lo)
    cst = torch.cuda.Stream(dev)
    if args.walk_cus:   # the walks on a share of every XCD's CUs (CU-masked streams)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        wsts = [_lib.cu_stream(0, args.walk_cus, dev) for _ in range(W)]
        if args.other_cus == "rest":
            bst, cst = (_lib.cu_stream(args.walk_cus, ncu - args.walk_cus, dev) for _ in range(2))
            estream = _lib.cu_stream(args.walk_cus, ncu - args.walk_cus, dev)
            eptr = C.c_void_p(estream.cuda_stream)
    bst_p = C.c_void_p(bst.cuda_stream)
    A = args.build_ahead

    def expand_args(cx):
        return (sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs, None, C.byref(cx.tr),
                C.byref(cx.st) if cx.st is not None else None, C.c_void_p(cx.plan.data_ptr()),
                C.c_void_p(cx.scratch.data_ptr()), cx.scratch.numel())

    def g_build(j, gate):
        cx = ctxs[j % len(ctxs)]
        cx.chain0 = batch_chain0(j)
        if gate is not None:
            bst.wait_event(gate)
        if cx.expanded is not None:                        # the context's previous batch is committed
            bst.wait_event(cx.expanded)
        _lib.check(L.tmh_init(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, None, bst_p))
        _lib.check(L.tmh_plan(sim._eng, 0, secs, C.c_void_p(cx.plan.data_ptr()), bst_p))
        _lib.check(L.tmh_walk_part(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs,
                                   C.c_void_p(cx.plan.data_ptr()), C.c_void_p(cx.scratch.data_ptr()),
                                   cx.scratch.numel(), None, 0, _lib.WALK_DRAWS, bst_p))
        if args.minutes_ahead:   # the minute table needs the draws, not the walk
            _lib.check(L.tmh_expand_part(*expand_args(cx), _lib.EXPAND_MINUTES, bst_p))
        cx.done.record(bst)
        tl_mark("built", j, bst)

    tl = {}   # --timeline: per-batch HIP timing events (build done, walk start / end, expansion start / end)

    def tl_mark(key, j, stream):
        if args.timeline:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            tl.setdefault(key, {})[j] = e

    def g_walk(j):
        cx = ctxs[j % len(ctxs)]
        wst = wsts[j % W]
        wst.wait_event(cx.done)
        tl_mark("walk0", j, wst)
        _lib.check(L.tmh_walk_part(sim._eng, C.c_void_p(cx.state.data_ptr()), cx.chain0, n, 0, secs,
                                   C.c_void_p(cx.plan.data_ptr()), C.c_void_p(cx.scratch.data_ptr()),
                                   cx.scratch.numel(), None, 0, _lib.WALK_SEGMENTS, C.c_void_p(wst.cuda_stream)))
        cx.walked.record(wst)
        tl_mark("walk1", j, wst)

    def g_expand(j):
        cx = ctxs[j % len(ctxs)]
        es, ep = estream, eptr
        es.wait_event(cx.walked)
        args_ = expand_args(cx)
        tl_mark("exp0", j, es)
        _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_KERNEL | (_lib.EXPAND_NO_MINUTES if args.minutes_ahead else 0),
                                     ep))
        tl_mark("exp1", j, es)
        if cx.expanded is None:
            cx.expanded = torch.cuda.Event()
        if args.commit_stream:   # fixup + commit beside the next expansion
            cx.kernel_done.record(es)
            cst.wait_event(cx.kernel_done)
            _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, C.c_void_p(cst.cuda_stream)))
            cx.expanded.record(cst)
        else:
            _lib.check(L.tmh_expand_part(*args_, _lib.EXPAND_COMMIT, ep))
            cx.expanded.record(es)

    def run_gated(k0, cnt):
        """W walks in flight (W + 2 contexts): when the walk of batch k ends, the
        expansion of k, the walk of k + W (on k's walk stream) and the construction
        of k + W + 1 are released together."""
        end = k0 + cnt
        for j in range(k0, min(k0 + A, end)):
            # the run's first walk is the pipeline's fill latency (its expansion waits for it with
            # nothing else to do): chain order, whose windiest wavefront is shorter than the wind
            # order's (four windy chains); the wind order for the rest, which run beside expansions
            if args.walk_order and hasattr(L, "tmh_set_walk_order"):
                _lib.check(L.tmh_set_walk_order(sim._eng, 0 if (j == k0 and W > 1) else 1))
            g_build(j, None)
        for j in range(k0, min(k0 + W, end)):
            g_walk(j)
        for k in range(k0, end):
            gate = ctxs[k % len(ctxs)].walked
            if k + A < end:
                g_build(k + A, gate)
            if k + W < end:
                g_walk(k + W)
            g_expand(k)

    def run_batches(k0, cnt):
        """Batches k0 .. k0 + cnt - 1.  One-window batches are software-pipelined:
        construction + plan and the expansions run in order on one stream, the
        segment walks of the next (depth - 1) batches on high-priority streams beside
        them, so the one-wave-per-SIMD walks overlap the expansion instead of running
        in lockstep with it (separate per-batch streams drift into lockstep: every
        expansion then shares the chip with the others and with every walk)."""
        if nwin > 1 or not args.stagger:
            for k in range(k0, k0 + cnt):
                one_step(k)
            return
        if args.schedule == "gated" and len(ctxs) >= max(A + 1, W + 2):
            run_gated(k0, cnt)
            return
        D = len(ctxs)
        ahead = D - 1
        for k in range(k0, min(k0 + D, k0 + cnt)):
            build(k)
        for k in range(k0, min(k0 + ahead, k0 + cnt)):
            start(k)
        for k in range(k0, k0 + cnt):
            if k + ahead < k0 + cnt:
                start(k + ahead)
            finish(k)
            if k + D < k0 + cnt:
                build(k + D)

    def exchange():
        """stats mode: the one cross-GPU step, an RCCL all-reduce of the aggregate statistics"""
        torch.cuda.synchronize()
        for cx in ctxs:   # (streams a schedule never created have nothing to wait for)
            for st_ in (cx._stream, cx._wstream):
                if st_ is not None:
                    st_.synchronize()
        hist = sum(cx.hist for cx in ctxs)
        acc = torch.stack([cx.acc for cx in ctxs])
        tot = dict(energy_pv=acc[:, 0].sum(), energy_meter=acc[:, 1].sum(), energy_residual=acc[:, 2].sum(),
                   peak_residual=acc[:, 3].max(), hist=hist)
        return all_reduce_stats(tot)

    run_batches(0, args.warmup)
    if args.mode == "stats":
        exchange()                                         # loads torch's reduction kernels outside the timing
        for cx in ctxs:
            cx.hist.zero_()
            cx.acc[:3].zero_()
            cx.acc[3].fill_(-float("inf"))
    torch.cuda.synchronize()
    for kk in (_lib.K_EXPAND, _lib.K_SEGMENTS, _lib.K_CANDIDATES, _lib.K_STEP):
        _lib.profile_read(sim._eng, kk)                    # drop the warmup launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_batches(args.warmup, args.steps)
    tot = exchange() if args.mode == "stats" else None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    phases = {}
    for name, kk in (("expand", _lib.K_EXPAND), ("segments", _lib.K_SEGMENTS),
                     ("candidates", _lib.K_CANDIDATES), ("tmh_step", _lib.K_STEP)):
        ms, cnt = _lib.profile_read(sim._eng, kk)
        phases[name] = ms / cnt if cnt else None
    # the dominant kernel alone: one more batch with nothing beside it (after the timed
    # region, not part of `value`): its duration without the pipelined walks sharing the CUs
    one_step(args.warmup + args.steps)
    torch.cuda.synchronize()
    alone_ms, alone_n = _lib.profile_read(sim._eng, _lib.K_EXPAND)
    alone_ms = alone_ms / alone_n if alone_n else float("nan")
    alone_ms *= 1 if nwin == 1 else nwin
    for kk in (_lib.K_SEGMENTS, _lib.K_CANDIDATES, _lib.K_STEP):
        _lib.profile_read(sim._eng, kk)
    bad = 0
    for cx in ctxs:
        sim.state = cx.state
        bad += int((sim.status() != 0).sum())
    for name in phases:                                    # per batch (all windows)
        if phases[name] is not None:
            phases[name] *= nwin
    kmean = phases["expand"] if phases["expand"] else float("nan")
    if world > 1:
        t = torch.tensor([elapsed, kmean], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmean = float(t[0]), float(t[1])
        b = torch.tensor([bad], device=dev, dtype=torch.int64)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        bad = int(b[0])
    chain_seconds = n_node * secs * args.steps                 # every rank's chains (C2: n per rank)
    # stats mode: the chain-seconds actually simulated = the histogram's count (a chain
    # that faults, e.g. the reference's AssertionError in markov mode, freezes and
    # records nothing more; edge bins absorb out-of-range residuals)
    live = int(tot["hist"].sum()) if tot is not None else None
    value = (live if live is not None else chain_seconds) / elapsed
    TB = TRACE_BYTES * (2 if args.precision == "fp64" else 1)
    achieved = TB * n * secs / (kmean / 1e3) / 1e9
    launch_secs = min(win, secs)
    rec = pmc_record(args, n, launch_secs)
    kms_launch = kmean / nwin                              # one expand launch (one window)

    def valu(ms):
        if rec is None or not ms or ms != ms:
            return None
        a = rec["valu_insts_per_launch"] * 64 / (ms / 1e3) / 1e12
        return {"achieved": a, "peak": VALU_PEAK_TLANE, "unit": "T lane-ops/s", "frac": a / VALU_PEAK_TLANE,
                "valu_per_chain_second": rec["valu_insts_per_launch"] * 64 / (n * launch_secs),
                "salu_per_chain_second": rec["salu_insts_per_launch"] * 64 / (n * launch_secs)}

    if args.mode == "trace":
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": rec["traffic_bytes_per_launch"] if rec else None,
                "kernel": "expand_kernel (P2, " + sim.path + ")", "kernel_ms": kmean,
                "bytes_per_launch": TB * n * secs,
                # the same launch with no other batch in flight (one extra batch after the timed region)
                "alone": {"kernel_ms": alone_ms, "achieved": TB * n * secs / (alone_ms / 1e3) / 1e9,
                          "frac": TB * n * secs / (alone_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
                "valu": valu(kms_launch)}
    else:
        v = valu(kms_launch) or {}
        va = valu(alone_ms / nwin) or {}   # the same launch with no other batch in flight
        roof = {"bound": "valu", "achieved": v.get("achieved"), "peak": VALU_PEAK_TLANE, "unit": "T lane-ops/s",
                "frac": v.get("frac"), "traffic": rec["traffic_bytes_per_launch"] if rec else None,
                "alone": {"kernel_ms": alone_ms / nwin, "achieved": va.get("achieved"), "frac": va.get("frac")},
                "kernel": "expand_kernel (P2, " + sim.path + ")", "kernel_ms": kms_launch,
                "launches_per_batch": nwin, "chain_seconds_per_launch": n * launch_secs,
                "valu_per_chain_second": v.get("valu_per_chain_second"),
                "salu_per_chain_second": v.get("salu_per_chain_second"),
                "source": "VALU lane-ops = SQ_INSTS_VALU x 64 per launch (profiles/pmc_kernels.json) / HIP-event "
                          "launch time" if rec else "no PMC record of this build for this workload in "
                                                    "profiles/pmc_kernels.json"}
    line = {
        "metric": "simulated chain-seconds/sec (node) at 1/2/4/8 GPUs + % HBM roofline",
        "value": value, "unit": "chain-seconds/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": args.precision, "data": "synthetic (keyed Philox)",
        "config": {"workload": (f"{args.workload.upper()}: {n_node} chains"
                                + (f" ({n} per GPU)" if scaling == "weak" else f" on {world} GPU(s)")
                                + f" x {secs} s at 1 s, Munich, Europe/Berlin, "
                                + (f"{win} s windows, " if nwin > 1 else "") if not c5 else
                                f"C5: {n_node} sites on a lat/lon grid (35-60 N, 10 W-30 E, {world} GPU(s)) x {secs} s, "
                                f"{args.cc} cc with per-site tables, per-site PV geometry, {win} s windows, Europe/Berlin, ")
                               + f"{args.start[:10]}, {args.mode} mode ("
                               + (f"meter+pv+residual {args.precision} trace" if args.mode == "trace" else f"on-GPU {args.precision} stats")
                               + ")",
                   "chains_node": n_node, "chains_per_gpu": n, "seconds": secs,
                   "parallelism": f"chains sharded over {world} GPU(s), {scaling} scaling",
                   "batches_in_flight": len(ctxs), "staggered": bool(args.stagger and nwin == 1),
                   "construction_on": args.build_on, "walk_priority": args.walk_priority,
                   "schedule": args.schedule if (args.stagger and nwin == 1 and len(ctxs) >= 3) else None,
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "walks_in_flight": W, "walk_order": bool(args.walk_order), "walk_cus": args.walk_cus or "all", "other_cus": args.other_cus if args.walk_cus else "all",
                   "walk_chains_per_row": args.walk_cpr, "walk_lanes": args.walk_lanes or "auto", "build_ahead": A,
                   "minutes_ahead": bool(args.minutes_ahead), "commit_stream": bool(args.commit_stream),
                   "compacted_windows": bool(args.compact and args.mode == "stats" and nwin > 1)},
        "roofline": roof,
        "chain_seconds_total": chain_seconds, "chain_seconds_live": live,
        "phases_ms": phases,
        # whole-pipeline rate: trace bytes of all batches / wall time (kernels overlap across batches)
        "effective_trace_gbs": (TB * n * secs / (elapsed / args.steps) / 1e9) if args.mode == "trace" else None,
        "faulted_chains": bad,
    }
    if args.timeline and "exp0" in tl:
        ks = sorted(k for k in tl["exp0"] if k >= args.warmup and k in tl["exp1"] and k + 1 in tl.get("exp0", {}))
        gaps = [tl["exp1"][k].elapsed_time(tl["exp0"][k + 1]) for k in ks]
        late = [tl["exp1"][k].elapsed_time(tl["walk1"][k + 1]) for k in ks if k + 1 in tl.get("walk1", {})]
        wdur = [tl["walk0"][k].elapsed_time(tl["walk1"][k]) for k in ks if k in tl.get("walk0", {})]
        bwait = [tl["built"][k].elapsed_time(tl["walk0"][k]) for k in ks if k in tl.get("built", {}) and k in tl.get("walk0", {})]
        line["timeline"] = {"expansion_gap_ms": gaps, "walk_end_after_prev_expansion_ms": late,
                            "walk_ms": wdur, "walk_start_after_build_ms": bwait}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, kw)
    if rank == 0 and world == 1 and args.secondary != "none":
        del ctxs   # the children need the memory
        torch.cuda.empty_cache()
        line["secondary"] = secondary_lines(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
