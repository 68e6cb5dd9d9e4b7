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
# Issue cycles per wave64 VALU instruction by rocprofv3 class, from the dependent-free
# ("distinct") loops of profiles/r03_isa_rate.txt: fp32 add / mul / fma 2.2, integer
# add and bit ops 2.3-2.8, fp64 add / mul / fma, cvt, 64-bit integer mad 4.1-4.3,
# fp32 transcendentals 8.4, fp64 reciprocal 16.  Instructions in no class (compares,
# selects, min / max / med3, DPP moves: 4.1-4.2; plain moves 2.2) are weighed at 4.
VALU_CYCLES = {"ADD_F32": 2, "MUL_F32": 2, "FMA_F32": 2, "INT32": 2.5, "TRANS_F32": 8,
               "ADD_F64": 4, "MUL_F64": 4, "FMA_F64": 4, "INT64": 4, "CVT": 4, "TRANS_F64": 16}
VALU_OTHER_CYCLES = 4
SIMD_CYCLES_PER_S = 256 * 4 * 2.4e9   # SIMDs x nominal clock


def valu_busy(rec, ms):
    """Cycle-weighted VALU-busy fraction of one launch of `ms` milliseconds: the
    per-class wave-instruction counts x their issue cycles over the SIMDs' cycles.
    The instruction-count 'frac' beside it prices every instruction at the 2-cycle
    fp32 rate.  (SQ_ACTIVE_INST_VALU, kept in the PMC record, counts each wave's VALU
    cycles with the waves of a SIMD overlapping -- C3 reads 1.01 of the SIMD cycles --
    so it is not a busy fraction.)"""
    out = {}
    denom = SIMD_CYCLES_PER_S * ms / 1e3
    mix = rec.get("valu_mix")
    if mix:
        known = sum(mix.get(k, 0.0) for k in VALU_CYCLES)
        other = max(0.0, rec["valu_insts_per_launch"] - known)
        cyc = sum(mix.get(k, 0.0) * w for k, w in VALU_CYCLES.items()) + other * VALU_OTHER_CYCLES
        out.update(busy_frac_weighted=cyc / denom, valu_cycles_per_launch=cyc,
                   valu_other_insts_per_launch=other)
    return out

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
                         "batches in flight (~33 GB of state + scratch each); c4: 16,384 chains x the year 2019 "
                         "(Europe/Berlin wall clock, stats, 30-day windows); c5: the lat/lon sweep (65,536 sites x 1 "
                         "week, markov cc with per-site tables, per-site PV geometry, stats mode, day windows)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=150.0,
                    help="C2: untimed batches of other fresh chains for at least this long before the W warm-up "
                         "steps (the GPU leaves idle; 0 = off); reported as prewarm_batches")
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
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; 0 = leave the environment's). "
                         "HIP maps streams round-robin onto that many hardware queues and a queue runs its "
                         "packets in order across the streams sharing it: with HIP's default 4 the expansion "
                         "stream shares a queue with another pipeline stream and waits for its kernels (same "
                         "box: 1.74-1.76 ms per C2 batch with 4 queues, 1.49-1.51 with 8, 1.47-1.51 with 16); "
                         "default 16, 32 for c4 / c5 (three streams per batch in flight, up to 8 batches)")
    ap.add_argument("--queues", default="dedicated", choices=["dedicated", "shared"],
                    help="pipeline streams on hardware queues of their own (dedicated: CU-masked over every CU, "
                         "independent of GPU_MAX_HW_QUEUES) or plain streams sharing HIP's queue pool (shared)")
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
    ap.add_argument("--drain-order", type=int, default=None,
                    help="gated schedule: the run's last N walks in chain order (default 1; 0: wind order)")
    ap.add_argument("--plan-stream", type=int, default=None,
                    help="gated schedule: each construction's plan on a stream of its own beside its chains' init (1)")
    ap.add_argument("--build-streams", type=int, default=None,
                    help="gated schedule: the constructions on this many streams in turn (consecutive batches' "
                         "constructions may then overlap)")
    ap.add_argument("--build-priority", default="normal", choices=["high", "normal"],
                    help="gated schedule: HIP stream priority of the construction stream")
    ap.add_argument("--commit-stream", type=int, default=None,
                    help="gated schedule: each batch's fixup + commit on a stream of their own beside the next "
                         "expansion (1) or after its expansion on the expansion stream (0, the default)")
    ap.add_argument("--first-split", type=int, default=None,
                    help="gated schedule: the run's first batch in this many consecutive windows of whole hours, "
                         "so the first expansion waits for a part of the first walk only (the pipeline's fill); "
                         "default 1 (off; 2 measured slower for c2, DESIGN.md round 5)")
    ap.add_argument("--compact", type=int, default=None,
                    help="multi-window stats workloads: run each window after the first on the chains still "
                         "live (faulted chains, e.g. C5's markov AssertionError, drop out); default 1 for c5")
    ap.add_argument("--proxy-world", type=int, default=1,
                    help="one-GPU proxy of an N-GPU strong-scaled run (c3 / c4 / c5): time rank 0's shard of "
                         "N GPUs (chains / N) alone on this GPU; `value` is then that rank's rate and "
                         "`projected_node_value` N times it. Not a scaling measurement: the RCCL exchange and "
                         "the other ranks are absent")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="batches in flight on separate HIP streams (1 = no overlap): the segment walks of the "
                         "next batches (latency-bound, one wave per SIMD) run beside this batch's expansion")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.proxy_world > 1 and (a.gpus > 1 or a.workload not in STRONG):
        ap.error("--proxy-world: a one-GPU proxy of a strong-scaled workload (c3 / c4 / c5)")
    from tmhpvsim_amd.pipeline import pipeline_defaults
    c5, c4 = a.workload == "c5", a.workload == "c4"
    a.chains = a.chains or DEFAULT_CHAINS[a.workload]
    a.seconds = a.seconds or {"c2": 86400, "c3": 86400, "c4": 365 * 86400, "c5": 604800}[a.workload]
    # the schedule (contexts, walks in flight, construction ahead, streams): the measured-best
    # defaults of each workload, shared with the tests that run the timed schedule
    # the chains of one batch on one GPU: C2 per GPU; C3 / C4 / C5 the node total / N (the proxy's N)
    a.chains = a.chains or DEFAULT_CHAINS[a.workload]
    per_gpu = a.chains if a.workload not in STRONG else -(-a.chains // (a.gpus * max(1, a.proxy_world)))
    a.cfg = pipeline_defaults(a.workload, a.precision, chains=per_gpu, seconds=a.seconds, window=a.window, walks=a.walks,
                              build_ahead=a.build_ahead, pipeline=a.pipeline, compact=a.compact, mode=a.mode,
                              stagger=a.stagger, schedule=a.schedule, build_on=a.build_on,
                              walk_priority=a.walk_priority, expand_priority=a.expand_priority,
                              build_priority=a.build_priority,
                              commit_stream=None if a.commit_stream is None else bool(a.commit_stream),
                              walk_order=bool(a.walk_order), walk_cus=a.walk_cus, other_cus=a.other_cus,
                              timeline=a.timeline, queues=a.queues, first_split=a.first_split,
                              build_streams=a.build_streams,
                              plan_stream=None if a.plan_stream is None else bool(a.plan_stream),
                              drain_order=a.drain_order)
    for k in ("mode", "window", "pipeline", "walks", "build_ahead", "build_streams", "build_on", "walk_priority",
              "compact", "commit_stream"):
        setattr(a, k, getattr(a.cfg, k))
    # C5's compacted windows walk and expand in turn (latency-bound walk): 16 lanes per
    # chain (1.76e10 against 1.73e10 with the batch-size default, r02 same box)
    # C3 / C4 batches above 8,192 chains: 8 lanes per chain (round 4, same box, twice: C3
    # 2.95 -> 2.99e11, C4 2.81-2.82 -> 2.86e11 against the library's batch-size default of 4);
    # smaller shards keep the default 16 (the C4 N = 8 shard: 2.50 against 2.46e11 with 8)
    a.walk_lanes = a.walk_lanes or (16 if c5 else (8 if a.workload in ("c3", "c4") and per_gpu > 8192 else 0))
    if a.secondary is None:
        # the full report (the default C2 run with its CPU baseline) carries them; quick runs do not
        a.secondary = "all" if (a.workload == "c2" and a.precision == "fp32" and not a.no_cpu_baseline) else "none"
    a.cc = a.cc or ("markov" if c5 else "faithful")
    a.hw_queues_given = a.hw_queues is not None   # secondaries pick their own default otherwise
    if a.hw_queues is None:
        a.hw_queues = 32 if (c4 or c5) else 16
    a.start = a.start or ("2019-01-01 00:00:00" if c4 else "2019-09-05 00:00:00")
    return a


SECONDARY = {   # --secondary: the other BASELINE.json configs, each in a child process of its own
    "c2_fp64": ["--precision", "fp64", "--steps", "20", "--warmup", "5"],
    # the headline at HIP's default of 4 hardware queues (the pipelines' streams have queues of
    # their own, PipelineConfig.queues = "dedicated": no result depends on GPU_MAX_HW_QUEUES)
    "c2_q4": ["--hw-queues", "4", "--steps", "20", "--warmup", "5"],
    "c3": ["--workload", "c3", "--steps", "4", "--warmup", "1"],
    # C4 / C5 at N = 1 keep 3 / 5 batches in flight: whole rounds of them (6 / 5 timed batches)
    "c4": ["--workload", "c4", "--steps", "6", "--warmup", "1"],
    "c5": ["--workload", "c5", "--steps", "5", "--warmup", "1"],
    # one-GPU proxies of the strong-scaled configurations at N = 8 (and C4 at 2, 4): rank 0's
    # shard timed alone (8 batches in flight for C4 / C5 shards, pipeline_defaults);
    # `projected_efficiency` = T_1 / (N T_N) = its (rank) rate / the N = 1 rate above
    "c3_proxy8": ["--workload", "c3", "--proxy-world", "8", "--steps", "6", "--warmup", "2"],
    "c4_proxy2": ["--workload", "c4", "--proxy-world", "2", "--steps", "6", "--warmup", "1"],
    "c4_proxy4": ["--workload", "c4", "--proxy-world", "4", "--steps", "8", "--warmup", "1"],
    "c4_proxy8": ["--workload", "c4", "--proxy-world", "8", "--steps", "8", "--warmup", "1"],
    "c5_proxy8": ["--workload", "c5", "--proxy-world", "8", "--steps", "8", "--warmup", "1"],
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
        cmd = [sys.executable, os.path.abspath(__file__), "--no-cpu-baseline", "--secondary", "none"] + extra
        if getattr(args, "hw_queues_given", False) and "--hw-queues" not in extra:
            cmd += ["--hw-queues", str(args.hw_queues)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            roof = d.get("roofline", {})
            out[name] = {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
                         "steps": d["steps"], "dtype": d["dtype"], "workload": d["config"]["workload"],
                         "roofline": {k: roof.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                               "kernel_ms", "busy_frac_weighted", "aggregate", "per_launch")},
                         "roofline_alone": roof.get("alone"), "faulted_chains": d.get("faulted_chains"),
                         "chain_seconds_live": d.get("chain_seconds_live")}
            if d.get("proxy_world"):
                out[name].update(proxy_world=d["proxy_world"], projected_node_value=d["projected_node_value"],
                                 proxy_note=d["proxy_note"])
        except Exception as e:   # noqa: BLE001 - report, never lose the headline line
            out[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
    for name, d in out.items():   # strong-scaling readiness on one GPU: T_1 / (N T_N) = rank rate / N = 1 rate
        base = out.get(name.split("_proxy")[0], {})
        if d.get("proxy_world") and base.get("value"):
            d["projected_efficiency"] = d["value"] / base["value"]
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
    proxy = args.proxy_world if world == 1 else 1
    shard0, n, n_node, scaling = rank_chains(args.workload, args.chains, rank, world * proxy)
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
    if args.walk_cpr != 1:
        _lib.check(L.tmh_set_walk_chains_per_row(sim._eng, args.walk_cpr))
    if args.walk_lanes:
        _lib.check(L.tmh_set_walk_lanes(sim._eng, args.walk_lanes))
    if hasattr(L, "tmh_set_walk_order"):
        _lib.check(L.tmh_set_walk_order(sim._eng, args.walk_order))

    from tmhpvsim_amd.pipeline import BatchPipeline
    pipe = BatchPipeline(sim, n, secs, args.cfg, batch_chain0, dev)
    nwin = pipe.nwin
    torch.cuda.synchronize()
    L.tmh_profile_enable(sim._eng, 1)
    run_batches, one_step = pipe.run, pipe.one_step

    def exchange():
        """stats mode: the one cross-GPU step, an RCCL all-reduce of the aggregate statistics"""
        pipe.sync()
        return all_reduce_stats(pipe.totals())

    # GPU warm-up before the W warm-up steps (C2 only, untimed): batches of other fresh chains for
    # at least --prewarm-ms, so the timed steps do not start on a GPU that has just left idle (a
    # 300-step timeline from a fresh process: the first 20 expansions 1.20 ms, the rest 1.13-1.15)
    prewarm = 0
    if args.workload == "c2" and args.prewarm_ms > 0:
        tp = time.perf_counter()
        kp0 = args.warmup + args.steps + 1   # batch ids past the timed ones and the `alone` batch
        while (time.perf_counter() - tp) * 1e3 < args.prewarm_ms:
            run_batches(kp0 + prewarm, max(1, args.warmup))
            pipe.sync()
            prewarm += max(1, args.warmup)
    run_batches(0, args.warmup)
    if args.mode == "stats":
        exchange()                                         # loads torch's reduction kernels outside the timing
        pipe.reset_stats()
    torch.cuda.synchronize()
    for kk in (_lib.K_EXPAND, _lib.K_SEGMENTS, _lib.K_CANDIDATES, _lib.K_STEP):
        _lib.profile_read(sim._eng, kk)                    # drop the warmup launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t0ev = None
    if args.timeline:   # the timed region's start on the GPU clock (the pipeline fill is measured from it)
        t0ev = torch.cuda.Event(enable_timing=True)
        t0ev.record()
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
        # per launch, below made per batch (x windows).  One-window batches: the total over
        # the batches, since the gated schedule's first batch runs as first_split windows
        phases[name] = (ms / cnt if nwin > 1 else ms / args.steps) if cnt else None
    # the dominant kernel alone: one more batch with nothing beside it (after the timed
    # region, not part of `value`): its duration without the pipelined walks sharing the CUs
    one_step(args.warmup + args.steps)
    torch.cuda.synchronize()
    alone_ms, alone_n = _lib.profile_read(sim._eng, _lib.K_EXPAND)
    alone_ms = alone_ms / alone_n if alone_n else float("nan")
    alone_ms *= 1 if nwin == 1 else nwin
    for kk in (_lib.K_SEGMENTS, _lib.K_CANDIDATES, _lib.K_STEP):
        _lib.profile_read(sim._eng, kk)
    bad = pipe.faulted()
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
    chain_seconds = (n if proxy > 1 else n_node) * secs * args.steps   # every rank's chains (C2: n per rank)
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
                "salu_per_chain_second": rec["salu_insts_per_launch"] * 64 / (n * launch_secs),
                **valu_busy(rec, ms)}

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
        agg = rec["valu_insts_per_launch"] * 64 * nwin * args.steps / elapsed / 1e12 if rec else None
        agg_w = valu_busy(rec, elapsed * 1e3 / (args.steps * nwin)).get("busy_frac_weighted") if rec else None
        # `achieved` / `frac`: the expansion lane-ops of the whole timed region over its wall
        # time.  With several batches' expansions overlapping (C4 / C5 contexts, C3's two
        # batches) a launch's HIP-event span also covers its neighbours' work, so the
        # per-launch figure (`per_launch`) understates the chip's VALU use there
        roof = {"bound": "valu", "achieved": agg, "peak": VALU_PEAK_TLANE, "unit": "T lane-ops/s",
                "frac": agg / VALU_PEAK_TLANE if agg else None,
                "traffic": rec["traffic_bytes_per_launch"] if rec else None,
                "busy_frac_weighted": agg_w,
                "per_launch": {"kernel_ms": kms_launch, "achieved": v.get("achieved"), "frac": v.get("frac"),
                               "busy_frac_weighted": v.get("busy_frac_weighted")},
                "alone": {"kernel_ms": alone_ms / nwin, "achieved": va.get("achieved"), "frac": va.get("frac"),
                          "busy_frac_weighted": va.get("busy_frac_weighted")},
                "aggregate": ({"achieved": agg, "frac": agg / VALU_PEAK_TLANE, "busy_frac_weighted": agg_w}
                              if rec else None),
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
        "warmup": args.warmup, "prewarm_batches": prewarm, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
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
                   "batches_in_flight": len(pipe.ctxs), "staggered": bool(args.stagger and nwin == 1),
                   "construction_on": args.build_on, "walk_priority": args.walk_priority,
                   "schedule": args.schedule if pipe.gated() else None,
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "walks_in_flight": pipe.W, "walk_order": bool(args.walk_order), "walk_cus": args.walk_cus or "all", "other_cus": args.other_cus if args.walk_cus else "all",
                   "walk_chains_per_row": args.walk_cpr, "queues": args.queues, "walk_lanes": args.walk_lanes or "auto", "build_ahead": pipe.A, "build_streams": args.build_streams,
                   "commit_stream": bool(args.commit_stream),
                   "first_batch_windows": len(pipe.split) if (pipe.split and pipe.gated()) else 1,
                   "compacted_windows": bool(args.compact and args.mode == "stats" and nwin > 1)},
        "roofline": roof,
        "chain_seconds_total": chain_seconds, "chain_seconds_live": live,
        "phases_ms": phases,
        # whole-pipeline rate: trace bytes of all batches / wall time (kernels overlap across batches)
        "effective_trace_gbs": (TB * n * secs / (elapsed / args.steps) / 1e9) if args.mode == "trace" else None,
        "faulted_chains": bad,
        # the loaded library's build stamp (tmh_build_stamp; _lib.load refuses a stale in-tree library)
        "lib_stamp": _lib.loaded_stamp(),
    }
    if proxy > 1:
        line["proxy_world"] = proxy
        line["projected_node_value"] = value * proxy
        line["proxy_note"] = (f"one-GPU proxy: rank 0's shard of {proxy} GPUs ({n} of {n_node} chains) timed alone on one "
                              "GPU; value = that rank's rate, projected_node_value = value x N (equal shards, no "
                              "exchange cost); not a scaling measurement")
    tl = pipe.tl
    if args.timeline and "exp0" in tl:
        ks = sorted(k for k in tl["exp0"] if k >= args.warmup and k in tl["exp1"] and k + 1 in tl.get("exp0", {}))
        gaps = [tl["exp1"][k].elapsed_time(tl["exp0"][k + 1]) for k in ks]
        late = [tl["exp1"][k].elapsed_time(tl["walk1"][k + 1]) for k in ks if k + 1 in tl.get("walk1", {})]
        wdur = [tl["walk0"][k].elapsed_time(tl["walk1"][k]) for k in ks if k in tl.get("walk0", {})]
        bwait = [tl["built"][k].elapsed_time(tl["walk0"][k]) for k in ks if k in tl.get("built", {}) and k in tl.get("walk0", {})]
        k0 = args.warmup
        fill = {}
        for key, name in (("built", "first_build_done_ms"), ("walk0", "first_walk_start_ms"),
                          ("walk1", "first_walk_end_ms"), ("exp0", "first_expansion_start_ms"),
                          ("exp1", "first_expansion_end_ms")):
            if k0 in tl.get(key, {}):
                fill[name] = t0ev.elapsed_time(tl[key][k0])
        line["timeline"] = {"fill": fill, "expansion_gap_ms": gaps, "walk_end_after_prev_expansion_ms": late,
                            "walk_ms": wdur, "walk_start_after_build_ms": bwait,
                            # every batch's marks from the timed region's start (ms): built, walk start /
                            # end, expansion start / end
                            "marks_ms": {key: [round(t0ev.elapsed_time(ev[k]), 4) if k in ev else None
                                               for k in range(k0, k0 + args.steps)]
                                         for key, ev in tl.items()}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, kw)
    pipe.close()   # drain and release the pipeline's dedicated streams
    if rank == 0 and world == 1 and args.secondary != "none":
        del pipe, run_batches, one_step   # the children need the memory
        torch.cuda.empty_cache()
        line["secondary"] = secondary_lines(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
