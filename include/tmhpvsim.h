/*
 * tmhpvsim.h — C-ABI of the MI355X batched simulator for tmhpvsim's
 * clear-sky-index chain + PV model (libtmhpvsim.so, gfx950).
 *
 * The reference (coroa/tmhpvsim) is pure Python; its per-step operator API is
 *   ClearskyindexModel(time).next(time) -> float   tmhpvsim/clearskyindexmodel.py:57,128
 *   PVModel(time).next(time) -> float              tmhpvsim/pvmodel.py:12,82
 *   get_meter_value() -> float                     tmhpvsim/metersim.py:49
 *   residual = meter - pv                          tmhpvsim/pvsim.py:83
 * The Python package tmhpvsim_amd keeps those classes and signatures and binds
 * this library with ctypes (tmhpvsim_amd/_lib.py); INTEGRATION.md shows the
 * ctypes stub a reference maintainer would add.  Every entry point below
 * replaces a batch of those per-step calls: one call advances N chains
 * (chain = site x scenario) over a window of consecutive seconds.
 *
 * Conventions
 *  - plain pointers and sizes only; every device buffer is allocated by the
 *    caller (PyTorch-ROCm in tmhpvsim_amd) and passed as a raw device pointer.
 *    The library allocates nothing persistent on the device.
 *  - return 0 on success or a negative TMH_E_* code; never aborts; the last
 *    error message of the calling thread is available from tmh_last_error().
 *  - model faults that the reference raises as Python exceptions are reported
 *    per chain in the state's status word (TMH_CHAIN_*); a faulted chain is
 *    frozen and emits NaN (covered = 255) from the faulting step on.
 *  - `stream` is a hipStream_t (NULL = default stream); all work is enqueued
 *    asynchronously on it.  One engine per device; not re-entrant per engine.
 */
#ifndef TMHPVSIM_H
#define TMHPVSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMH_ABI_VERSION 1

/* ---- error codes ---- */
#define TMH_OK 0
#define TMH_E_INVAL (-1)
#define TMH_E_HIP (-2)
#define TMH_E_NOMEM (-3)
#define TMH_E_STATE (-4)

/* ---- per-chain status (the reference's exceptions) ---- */
#define TMH_CHAIN_OK 0
#define TMH_CHAIN_NAMEERROR_INIT 1  /* clearskyindexmodel.py:72-80 (undefined x, cc in [0.75,0.875)) */
#define TMH_CHAIN_ASSERT_BINARY 2   /* cloud_cover_binary.py:90-98 (assert not recurse) */
#define TMH_CHAIN_SIGMA_OVERFLOW 3  /* sigma arrays exceed TMH_SIGMA_CAP (no reference analogue) */
#define TMH_CHAIN_U_EXHAUSTED 4     /* injected uniform stream ran out */
#define TMH_CHAIN_SEGMENT_OVERFLOW 5 /* more than cap + 2,048 cloud segments in one window, where the row
                                         cap = (n_steps/135 + 16) rounded up to 16 (656 a day: ~1.7x the
                                         mean 386 calls, exceeded by ~0.3 % of the chain-days); or more
                                         than cap while the batch's demand exceeds the window's shared
                                         overflow pool (n/16 + 8 chunks of 256): then every such chain
                                         faults at its first record past the row (deterministic;
                                         time-parallel path) */
#define TMH_CHAIN_GUARD_OVERFLOW 6   /* fp32 guard-band records of the batch exceeded their room (never observed; time-parallel path) */

/* ---- modes ---- */
#define TMH_CC_FAITHFUL 0  /* reference: a fresh get_cloud_cover generator per hourly draw */
#define TMH_CC_MARKOV 1    /* persistent 6-bin hourly Markov chain (cloud_cover_hourly.py:290-316) */
#define TMH_RNG_KEYED 0    /* counter-based Philox4x32-10 keyed by (chain, step, draw family) */
#define TMH_RNG_INJECTED 1 /* per-chain uniform stream, consumed in reference order */
#define TMH_FP32 0         /* per-second CSI/PV/meter arithmetic in fp32 (Markov state stays fp64) */
#define TMH_FP64 1         /* everything in fp64 */
#define TMH_PATH_AUTO 0          /* time-parallel when possible (keyed + faithful), else sequential */
#define TMH_PATH_SEQUENTIAL 1    /* one work-item per chain, seconds in order */
#define TMH_PATH_TIME_PARALLEL 2 /* segment pass + (chain x 128 s block) expansion */

#define TMH_SIGMA_CAP 512  /* capacity of sigma_cloud / sigma_clear per chain (max seen: 132) */
#define TMH_GEOM_FIELDS 22 /* doubles per step in the clock/geometry table (DESIGN.md "Data layout") */

/* ---- SAPM module parameter order (tmh_params.module) ---- */
enum {
    TMH_MOD_A0 = 0, TMH_MOD_A4 = 4, TMH_MOD_B0 = 5, TMH_MOD_B5 = 10, TMH_MOD_FD = 11,
    TMH_MOD_IMPO = 12, TMH_MOD_VMPO = 13, TMH_MOD_AIMP = 14, TMH_MOD_C0 = 15, TMH_MOD_C1 = 16,
    TMH_MOD_C2 = 17, TMH_MOD_C3 = 18, TMH_MOD_BVMPO = 19, TMH_MOD_MBVMP = 20, TMH_MOD_N = 21,
    TMH_MOD_NS = 22, TMH_MOD_TEMP_A = 23, TMH_MOD_TEMP_B = 24, TMH_MOD_TEMP_DT = 25,
    TMH_MOD_COUNT = 26
};
/* ---- Sandia inverter order (tmh_params.inverter): Paco Pdco Vdco Pso C0 C1 C2 C3 Pnt ---- */
#define TMH_INV_COUNT 9

typedef struct tmh_params {
    int32_t cc_mode;          /* TMH_CC_* */
    int32_t rng_mode;         /* TMH_RNG_* */
    int32_t precision;        /* TMH_FP32 / TMH_FP64 */
    int32_t with_pv;          /* 0: pv = 0 (CSI-only runs, as ClearskyindexModel) */
    int32_t kernel_path;      /* TMH_PATH_* */
    int32_t reserved;
    uint64_t seed;            /* keyed Philox seed (the meter always draws keyed) */
    double shapes[6][4];      /* loc, scale, kappa, df per cloud-cover bin (mc_dist_shapes.csv) */
    int32_t shape_is_t[6];    /* 1: Student-t bin, 0: asymmetric Laplace */
    double edges[6];          /* right edges of the bins */
    double site[8];           /* lat, lon, altitude, tilt, surface azimuth, albedo, temp_air, wind */
    double linke[12];         /* monthly Linke turbidity */
    double module[TMH_MOD_COUNT];
    double inverter[TMH_INV_COUNT];
} tmh_params;

/* Wall clock of a run.  Step s is the (s+1)-th call of ClearskyindexModel.next;
 * the engine is constructed at the time of step 0 (clearskyindexmodel.py:57). */
typedef struct tmh_clock {
    int64_t utc0;            /* unix seconds of step 0 (solar geometry) */
    int64_t local0;          /* local wall-clock seconds of step 0, counted from 1970-01-01 00:00 local */
    int32_t n_shifts;        /* DST changes within the horizon (<= 8) */
    int32_t reserved;
    int64_t shift_step[8];   /* from this step on ... */
    int32_t shift_delta[8];  /* ... local time is shifted by this many seconds (e.g. -3600) */
} tmh_clock;

/* Injected uniform streams: chain i (0-based within the call) reads
 * u[i * stride + k] for its k-th draw, k < len.  Device pointer. */
typedef struct tmh_ustream {
    const double* u;
    uint64_t stride;
    uint64_t len;
} tmh_ustream;

/* Per-second traces, time-major: element (step j of the call, chain i) lives at
 * [j * ld + i].  Real = float (TMH_FP32) or double (TMH_FP64).  Any may be NULL. */
typedef struct tmh_trace {
    void* csi;          /* clear-sky index (ClearskyindexModel.next) */
    uint8_t* covered;   /* CloudCoverBinary bit (1 = the "covered" branch), 255 on fault */
    void* pv;           /* AC power, W (PVModel.next) */
    void* meter;        /* 9000 * U, W (get_meter_value) */
    void* residual;     /* meter - pv, W (pvsim.py:83) */
    uint64_t ld;        /* >= n_chains */
} tmh_trace;

/* On-GPU statistics, accumulated over calls (caller zero-initialises).  Device pointers. */
typedef struct tmh_stats {
    uint64_t* hist;     /* [n_bins] residual histogram, edge bins absorb out-of-range; NULL = off */
    uint32_t n_bins;
    uint32_t reserved;
    double lo, hi;      /* histogram range, W */
    double* chain_acc;  /* [4][n_chains] sum pv, sum meter, sum residual (W*s), max residual */
} tmh_stats;

int tmh_abi_version(void);
const char* tmh_last_error(void);
/* Provenance: "TMHSTAMP:" + the 16-hex-digit hash of the sources and compile flags
 * this library was built from (tmhpvsim_amd/build.py build_stamp; "unstamped" for a
 * build outside it).  The Python loader refuses an in-tree library whose stamp differs
 * from its sources, so a stale binary is never tested or benchmarked. */
const char* tmh_build_stamp(void);

/* Chain state (structure of arrays, one element per chain per field). */
size_t tmh_state_bytes(uint32_t n_chains);
/* byte offsets of the TMH_STATE_NFIELDS fields (order documented in DESIGN.md) */
#define TMH_STATE_NFIELDS 24
int tmh_state_offsets(uint32_t n_chains, uint64_t* offsets);

/* Device buffers a window needs:
 *  plan    (chain-independent): clock/geometry table, boundary events, block descriptors;
 *  scratch (time-parallel path): segment records, window-end state, stats partials;
 *  workspace = plan + scratch (tmh_run builds the plan itself). */
size_t tmh_plan_bytes(uint32_t n_steps);
size_t tmh_scratch_bytes(uint32_t n_chains, uint32_t n_steps);
size_t tmh_workspace_bytes(uint32_t n_chains, uint32_t n_steps);
/* The scratch this engine's time-parallel path needs (its precision sizes the minute
 * table: fp32 engines need less than tmh_scratch_bytes, which fits any engine). */
size_t tmh_engine_scratch_bytes(const struct tmh_engine* eng, uint32_t n_chains, uint32_t n_steps);
/* The segment walk's rows (16 lanes each, four per wavefront) per chain: with
 * chains_per_row = k the walk launches ceil(n / k) rows, each row starting with one
 * chain and taking the next unstarted chain of the window's queue when its chain
 * is done.  The walk's duration is set by the longest chain either way; k > 1
 * shrinks its footprint on the CUs (for callers that run several batches' walks
 * beside other kernels).  Results do not depend on k.  0 or 1 = one chain per row
 * (default); at most 64. */
int tmh_set_walk_chains_per_row(struct tmh_engine* eng, uint32_t chains_per_row);
/* Lanes per chain in the segment walk: 16 (four chains per wavefront), 8 or 4
 * (sixteen chains per wavefront, four times the sigma entries per lane); 0 = by
 * batch size (the default: 16 up to 8,192 chains, where the walk is latency-bound,
 * else 4).  Fewer lanes per chain: fewer instructions and registers per chain-call,
 * a longer chain of work per call.  Results do not depend on it. */
int tmh_set_walk_lanes(struct tmh_engine* eng, uint32_t lanes);
/* Walk rows in the order of the chains' wind over the window, windiest first (on
 * by default): the chains of one walk wavefront then make similar numbers of
 * next_cloud calls.  Set it before a window's draws (TMH_WALK_DRAWS: they compute the
 * order and store the candidate table by it).  Results do not depend on it. */
int tmh_set_walk_order(struct tmh_engine* eng, int on);
/* A HIP stream whose kernels run on a range of compute units only (no reference
 * counterpart: a scheduling helper for callers that pipeline batches).  CU-mask
 * bits cu_first .. cu_first + cu_count - 1 of the current device; the driver
 * spreads consecutive mask bits over the XCDs, so a range is an even share of
 * every XCD.  cu_count == 0: all CUs (a plain stream).  A range of every CU runs
 * anywhere like a plain stream but, being CU-masked, on a hardware queue of its own
 * (plain streams share GPU_MAX_HW_QUEUES queues round-robin, a queue running its
 * packets in order across them): the pipelines' streams (tmhpvsim_amd.pipeline).
 * *stream receives the hipStream_t; release it with tmh_stream_destroy.  The stream
 * belongs to the calling thread's current device (hipSetDevice first).  A CU-masked
 * stream is a blocking stream (it synchronises with the legacy null stream, as
 * hipStreamCreate's default does); cu_count == 0 gives a non-blocking one. */
int tmh_stream_create_cus(uint32_t cu_first, uint32_t cu_count, void** stream);
int tmh_stream_destroy(void* stream);
/* Compaction (batches whose chains fault, e.g. the reference's markov-mode
 * AssertionError, cloud_cover_binary.py:91): run later windows on the live chains
 * only.  A launch slot then holds chain ids[slot] of a full batch of n_full chains:
 * the slot's keyed draws are that chain's (chain0 + ids[slot]), and it reads row
 * ids[slot] of the per-chain shape tables and sites and accumulates into column
 * ids[slot] of tmh_stats.chain_acc ([4][n_full]).  State, scratch and traces stay
 * per slot.  ids == NULL: slot i is chain i (the default).  Results per chain do
 * not depend on the compaction. */
int tmh_set_chain_ids(struct tmh_engine* eng, const uint32_t* ids, uint32_t n_full);
/* the ids (ids_in[slot], or the slot itself when ids_in == NULL) of the slots of
 * `state` (n_chains slots) whose status is 0, in slot order, into ids_out
 * (device, n_chains entries); their count into *n_live (device uint32). */
int tmh_live_chains(struct tmh_engine* eng, const void* state, uint32_t n_chains, const uint32_t* ids_in,
                    uint32_t* ids_out, uint32_t* n_live, void* stream);
/* move chains between two state buffers: gather (scatter = 0) dst slot i <- src
 * slot map[i], scatter (1) dst slot map[i] <- src slot i, for i < min(*count, cap)
 * (count: device uint32, e.g. tmh_live_chains' n_live). */
int tmh_state_move(struct tmh_engine* eng, const void* src, uint32_t n_src, void* dst, uint32_t n_dst,
                   const uint32_t* map, const uint32_t* count, uint32_t cap, int scatter, void* stream);
/* Tests only: segment records kept per chain (a multiple of 16; 0 = the default
 * (n_steps/135 + 16) rounded up to 16) and the overflow pool's chunks (0 = n_chains/16 + 8), for
 * every later tmh_scratch_bytes / launch in this process.  Exercises the
 * overflow path, which the default sizes reach only on the windiest days. */
int tmh_test_set_segment_capacity(uint32_t cap, uint32_t pool_chunks);

int tmh_engine_create(const tmh_params* params, const tmh_clock* clock, int device,
                      struct tmh_engine** out);
int tmh_engine_destroy(struct tmh_engine* eng);
/* Replace the engine's wall clock for later plans (a rolling DST table: the
 * shift table holds 8 changes, so open-ended runs roll it forward).  Steps keep
 * their numbering (same utc0); the new clock must describe every step still to
 * be run plus the one before the first (boundary detection compares with it).
 * tmh_init keeps using the step-0 time of the creation clock. */
int tmh_set_clock(struct tmh_engine* eng, const tmh_clock* clock);
/* the kernel path the engine resolved (TMH_PATH_SEQUENTIAL or TMH_PATH_TIME_PARALLEL) */
int tmh_engine_path(const struct tmh_engine* eng);

/* Per-chain hourly cloud-cover shape tables (a lat/lon sweep with one table per
 * site).  Replaces, for every chain, the single table of
 * tmh_params.shapes / shape_is_t that get_distributions_from_shapes_file loads
 * (cloud_cover_hourly.py:269-288) and get_cloud_cover draws from (:290-316);
 * the bin edges stay tmh_params.edges.  shapes: device [n_chains][6][4] fp64
 * (loc, scale, kappa, df per bin), is_t: device [n_chains][6] int32 or NULL
 * (then tmh_params.shape_is_t).  Row i serves the chain at index i of the
 * tmh_init / tmh_run batch (chain0 + i), so n_chains must cover the batch.
 * The buffers are read by every later launch and must outlive them; shapes ==
 * NULL restores the single table; shapes must be 16-byte aligned (the markov
 * kernel stages each workgroup's rows in LDS with 16-B loads; TMH_E_INVAL
 * otherwise).  Both cc modes and both kernel paths. */
int tmh_set_shape_tables(struct tmh_engine* eng, const double* shapes, const int32_t* is_t,
                         uint32_t n_chains);

/* Per-chain PV sites (the lat/lon sweep of SURVEY C5; the reference builds one
 * PVModel per site, pvmodel.py:19-30).  sites: device [n_chains][8] fp64 rows in
 * tmh_params.site order; columns 0-5 (latitude, longitude, altitude, tilt,
 * surface azimuth, albedo) are per chain, temp_air and wind stay tmh_params'
 * (pvmodel.py:69-70 fixes them).  linke: device [n_chains][12] monthly Linke
 * turbidity or NULL (tmh_params.linke).  The clock, the boundary schedule and
 * the sun's place stay in the shared plan; solar position, clear-sky GHI,
 * DISC, POA and the SAPM factors are then evaluated per chain-second.  Row i
 * serves the chain at index i of the batch; buffers must outlive the
 * launches; sites == NULL restores the engine's single site. */
int tmh_set_sites(struct tmh_engine* eng, const double* sites, const double* linke, uint32_t n_chains);

/* ClearskyindexModel.__init__ for chains [chain0, chain0 + n_chains): the 14+
 * constructor draws and CloudCoverBinary's first cloud.  `inj` may be NULL
 * (keyed mode). */
int tmh_init(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains,
             const tmh_ustream* inj, void* stream);

/* Advance the chains over steps [step0, step0 + n_steps): per second the
 * hourly/daily/minute resampling, the cloud-cover binary, the clear-sky index,
 * the PV chain, the meter draw and the residual, fused.  Writes traces and/or
 * accumulates statistics.  = tmh_plan + tmh_step on `workspace`
 * (tmh_workspace_bytes(n_chains, n_steps) bytes). */
int tmh_run(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains,
            int64_t step0, uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace,
            const tmh_stats* stats, void* workspace, size_t workspace_bytes, void* stream);

/* Build the chain-independent plan of the window [step0, step0 + n_steps) into
 * `plan` (tmh_plan_bytes(n_steps) bytes).  The first TMH_GEOM_FIELDS * n_steps
 * doubles are the clock/geometry table (row layout in DESIGN.md).  One plan
 * serves every chain batch of the same site and window. */
int tmh_plan(struct tmh_engine* eng, int64_t step0, uint32_t n_steps, void* plan, void* stream);

/* tmh_run on a plan built by tmh_plan(step0, n_steps) for this engine. */
int tmh_step(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains,
             int64_t step0, uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace,
             const tmh_stats* stats, const void* plan, void* scratch, size_t scratch_bytes,
             void* stream);

/* tmh_step in its two halves, for callers that overlap independent batches
 * (bench.py: the latency-bound segment walks of the next batches run beside
 * this batch's expansion).  tmh_walk: boundary draws, candidate cloud lengths
 * and the P1 segment walk into `scratch`; tmh_expand: the P2 expansion
 * (traces / statistics) and the state commit from that scratch.  Call them in
 * this order on the same plan, scratch and state (the same stream, or with the
 * caller ordering them); tmh_step == tmh_walk + tmh_expand.  On the sequential
 * path tmh_walk does nothing and tmh_expand runs the whole step. */
int tmh_walk(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
             uint32_t n_steps, const void* plan, void* scratch, size_t scratch_bytes, void* stream);
int tmh_expand(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
               uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
               const void* plan, void* scratch, size_t scratch_bytes, void* stream);

/* The walk in parts and across windows (time-parallel path).
 * parts: TMH_WALK_DRAWS = boundary draws, markov hourly cover, candidate cloud
 * lengths and the window's minute draws (many small workgroups); TMH_WALK_SEGMENTS = the P1 segment walk (one
 * wave per SIMD, long-lived).  Small grids issued beside a running expansion
 * wait for CU slots, so a pipelining caller puts the draws on the expansion's
 * stream and only the segment walk on a second, high-priority stream.
 * prev_scratch (nullable): the scratch (laid out for prev_n_steps) of the previous
 * window of these chains; the window-start status, cloud-cover and wind pairs then
 * come from that window's walk instead of the state, so this walk may run while
 * the previous window's expansion and commit are in flight.  Order: draws(w+1)
 * after segments(w); segments(w+1) after draws(w+1); expand(w+1) after
 * segments(w+1) and expand(w); any part of w+2 after expand(w), the last reader
 * of the buffers w+2 reuses (BatchedSim.run, bench.py).  Same bits as tmh_step
 * window by window. */
#define TMH_WALK_DRAWS 1
#define TMH_WALK_SEGMENTS 2
int tmh_walk_part(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
                  uint32_t n_steps, const void* plan, void* scratch, size_t scratch_bytes,
                  const void* prev_scratch, uint32_t prev_n_steps, int parts, void* stream);

/* tmh_expand in its two halves, for callers that overlap independent batches
 * (bench.py): TMH_EXPAND_KERNEL = the P2 expansion (traces / statistics);
 * TMH_EXPAND_COMMIT = the fp32 guard-band recomputation (fixup) and the state /
 * statistics commit.  The commit half is latency-bound (a few waves); on a second
 * stream, after an event recorded behind the kernel half, it runs beside the next
 * batch's expansion.  Order: KERNEL then COMMIT on the same buffers; the traces and
 * statistics are final after COMMIT.  tmh_expand == KERNEL | COMMIT.  The window's
 * minute draws are part of TMH_WALK_DRAWS (one launch with the candidate lengths,
 * built with the construction, off the expansion's stream); TMH_EXPAND_MINUTES and
 * TMH_EXPAND_NO_MINUTES (round 3's split of them) are accepted and do nothing. */
#define TMH_EXPAND_KERNEL 1
#define TMH_EXPAND_COMMIT 2
#define TMH_EXPAND_MINUTES 4
#define TMH_EXPAND_NO_MINUTES 8
int tmh_expand_part(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
                    uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
                    const void* plan, void* scratch, size_t scratch_bytes, int parts, void* stream);

/* Kernel timing (measurement only).  While enabled, tmh_step records HIP
 * events, on the stream each kernel runs on, around the kernels of the
 * time-parallel path; tmh_profile_read waits for them and returns the summed
 * milliseconds and launch count of one kernel since the last read, then resets
 * it.  kernel: TMH_K_EXPAND (P2 trace/stats expansion), TMH_K_SEGMENTS (P1
 * segment walk), TMH_K_CANDIDATES (P1's candidate table), TMH_K_STEP (the
 * whole tmh_step). */
enum { TMH_K_EXPAND = 0, TMH_K_SEGMENTS = 1, TMH_K_CANDIDATES = 2, TMH_K_STEP = 3, TMH_K_COUNT = 4 };
int tmh_profile_enable(struct tmh_engine* eng, int on);
int tmh_profile_read(struct tmh_engine* eng, int kernel, double* total_ms, int* launches);

/* The expansion variant the engine's last tmh_step / tmh_expand(_part) launched
 * (tests and measurement: which kernel instantiation produced a line or a trace):
 * TMH_OUT_ANY (any trace fields and/or statistics), TMH_OUT_TRACE3 (exactly pv,
 * meter, residual, no statistics: the trace-mode hot path), TMH_OUT_STATS
 * (statistics only), plus TMH_OUT_SITES with per-chain sites and TMH_OUT_FP64 in
 * fp64; -1 before the first expansion (and on the sequential path, whose one
 * kernel serves every output). */
#define TMH_OUT_ANY 0
#define TMH_OUT_TRACE3 1
#define TMH_OUT_STATS 2
#define TMH_OUT_SITES 16
#define TMH_OUT_FP64 32
int tmh_engine_last_expand(const struct tmh_engine* eng);

/* Device math probes for parity tests: out[i] = f(a, x[i]) with
 * f = 0 ndtri, 1 gammaincinv, 2 stdtrit, 3 al_ppf, 4 ndtri (fp32 path),
 * 8 ocml's ndtri (the fp64 noise quantile's tails), 9 / 10 the fp32 PV chain's
 * v_med3_f32 clamps med3(x, 0, a) / med3(x, -inf, a), and the fp64 PV chain's
 * table functions: 11 the noise quantile of the 32-bit word x[i], 12 log, 13 exp. */
int tmh_probe(int fn, double a, const double* x, double* out, uint32_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TMHPVSIM_H */
