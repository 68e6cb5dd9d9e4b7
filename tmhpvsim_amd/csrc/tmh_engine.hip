// libtmhpvsim — MI355X (gfx950) batched simulator of tmhpvsim's clear-sky-index
// chain + PV model behind the C-ABI of include/tmhpvsim.h.
//
// Two execution paths over the same model code (tmh_model.h):
//
//  * sequential (chain_kernel): one work-item per chain runs the seconds of a
//    window in order, exactly like ClearskyindexModel.next.  Used for injected
//    uniform streams (the reference's consumption order is data dependent).
//
//  * time-parallel (keyed Philox, both cloud-cover modes): the only sequential
//    processes are CloudCoverBinary's cloud/clear segment sequence and, in
//    markov mode, the hour-to-hour cloud cover.
//      draws: event_draws_kernel (day/hour boundary draws), markov_cc_kernel
//         (markov mode), draws_tail_kernel (the next calls' try-0 lengths and the
//         window's minute draws).
//      P1 segments_kernel: four chains per wavefront, one per 16-lane row, walk
//         from segment end to segment end (next_cloud with the sigma scan spread
//         over the row, DPP argmin and shift) and record each segment as
//         (first clear step, next call step).
//      P2 expand_kernel: one work-item per (chain, block of 128 seconds)
//         rebuilds the sampler state at the block start from the keyed draws
//         of the last boundary events (block descriptors), then runs the fused
//         per-second body.  Every draw is keyed by (chain, step or call number),
//         so P2's outputs are bit-identical to the sequential kernel's.
//
// Per-window, chain-independent work (wall-clock fractions, boundary flags,
// solar geometry, clear-sky irradiance, SAPM spectral/AOI factors, the boundary
// event list and block descriptors) is built once by the plan kernels and read
// by the chain kernels with wave-uniform loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

// min waves per SIMD of the construction kernels (init, variates, geometry, boundary draws), i.e.
// their VGPR bound: beside the expansion (72-VGPR waves) a wave that needs more registers than
// one expansion wave frees waits for several to retire (A/B builds)
#ifndef TMH_BUILD_WAVES
#define TMH_BUILD_WAVES 4   // geom_kernel 146 -> 128 VGPRs (38 spilled): C2 +0.9 % over three pairs, round 6
#endif
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "tmh_math.h"
#include "tmh_model.h"
#include "tmhpvsim.h"

using namespace tmh;
static_assert(OUT_ANY == TMH_OUT_ANY && OUT_TRACE3 == TMH_OUT_TRACE3 && OUT_STATS == TMH_OUT_STATS,
              "expansion variants: tmh_model.h and include/tmhpvsim.h agree");

namespace {

constexpr int BLOCK_STEPS = 128;   // seconds per P2 work-item
static_assert(BLOCK_STEPS <= 128, "FixRec holds a 128-bit mask of a block's seconds");

struct BlockDesc {                 // as of the step before the block start; -1 = none in the window
    int32_t q0, q1;                // minute-draw indices of the last two minute boundaries
    int32_t h0, h1;                // event indices of the last two hour boundaries
    int32_t cd0, cd1;              // last two clear_day pushes: event index * 2 + (0 day | 1 hour push)
    int32_t evi;                   // first event index at or after the block start
    int32_t h2;                    // event index of the third-last hour boundary
};

// Segment records: a chain's first `cap` records sit in its row of `rec`; records
// past that go to 256-record chunks of a shared overflow pool, allocated by the
// walk (atomic counter) and listed per chain in `ovf` (OVF_SLOTS chunks).  cap =
// (n_steps/135 + 16) rounded up to 16 (seg_cap: 656 a day, ~1.7x the mean 386 calls per
// window; ~0.3 % of the chain-days spill past it), so the pool serves the windy tail.  TMH_CHAIN_SEGMENT_OVERFLOW is deterministic: a chain
// past cap + 256 OVF_SLOTS records faults at that record (a property of the chain
// alone); and when the batch's demand exceeds the pool (some claim failed: the
// total demand, not the claim order, decides that), overflow_settle_kernel faults
// EVERY chain that reached the pool, at its first record past the row
// (`ovf_first`), whichever claims the atomic counter happened to grant.
constexpr int OVF_SLOTS = 8, OVF_CHUNK = 256;
struct SegView {                   // P1 -> P2 scratch
    int2* rec;                     // [n][cap] (first uncovered step, next call step), global steps
    uint32_t cap;                  // a multiple of 16 (the walk flushes records in groups of 16)
    int32_t* ovf;                  // [n][OVF_SLOTS] pool chunk of the chain's records cap + 256 k ..
    int2* pool;                    // [pool_cap][OVF_CHUNK]
    uint32_t pool_cap;
    uint32_t* pool_n;              // chunks handed out (zeroed by the draws phase)
    uint32_t* walk_q;              // the walk's chain queue: chains taken past the first `rows` (zeroed likewise)
    uint32_t* pool_short;          // some chain found the pool exhausted (zeroed likewise)
    uint32_t* order;               // [n] walk row -> chain (windiest first, walk_order_kernel; the identity without walk order)
    uint32_t* rank;                // [n] chain -> walk row (the inverse; cand is stored by row)
    int32_t* ovf_first;            // [n] window-relative step of the chain's record `cap` (INT_MAX: none)
    uint32_t* count;               // [n]
    int32_t* fault;                // [n] window-relative fault step (INT_MAX = none)
    uint32_t* status;              // [n] status after the window
    double* end_p1;                // [4][n] cc before/after, ws before/after at window end
    uint32_t nblk;
    double* evd;                   // [ev_cap][4][n] per boundary event: cc, ws, clear_day (day), clear_day (hour)
    uint32_t evcap;
    double* cand;                  // [kcap][n] try-0 cloud lengths (before / ws) of the window's next kcap calls
    uint32_t kcap;
    void* mtab;                    // [nmin][2][n] R: the _next_min draws (cloudy, clear noise) of every minute boundary
    uint32_t nmin;
    double* mend;                  // [4][n] fp64 draws of the window end's minute boundaries q1, q0 (cloudy, clear; fp32 engines)
    struct FixRec* fix;            // [fixcap] fp32 guard-band seconds for fixup_kernel
    uint32_t fixcap;
    uint32_t* nfix;                // records appended (> fixcap: some were lost, see commit_kernel)
    double* corr;                  // [2][n] exact pv / residual sum corrections of the fixed seconds
    // The window's per-chain statistics, summed over its 128-s blocks by integer atomics:
    // sums of pv, meter, residual in fixed point (units of 1 / fx_scale W s; integer
    // addition is associative, so the totals do not depend on the order the blocks
    // finish in) and the peak residual as an order-preserving int64 key (max_key).
    long long* acc_fx;             // [3][n], zeroed with nfix / corr before each expansion
    long long* acc_mx;             // [n]
    double fx_scale, fx_inv;       // 2^k with 9,001 W x n_steps x 2^k < 2^62
    uint32_t* brec;                // [nblk][n] the record holding each block's start (block_rec_kernel)
};

// double <-> int64 key with the same order (max of keys = key of the max)
__device__ __forceinline__ long long max_key(double v)
{
    const long long b = __double_as_longlong(v);
    return b >= 0 ? b : b ^ 0x7FFFFFFFFFFFFFFFll;
}
__device__ __forceinline__ double max_unkey(long long k)
{
    return __longlong_as_double(k >= 0 ? k : k ^ 0x7FFFFFFFFFFFFFFFll);
}

// A (chain, 128-s block) of the fp32 expansion with a second in a guard band of
// the PV chain's discontinuities (pv_power_f): fixup_kernel recomputes it.
struct FixRec {
    uint32_t c;                    // chain index in the batch
    uint32_t b;                    // block
    uint32_t jr;                   // segment record index at the block's last step
    uint32_t pad;
    uint4 mask;                    // bit i: second b * 128 + i lies in a guard band
    uint4 cov;                     // bit i: second b * 128 + i is covered (the tile's covered bits)
};

// The window-start values a walk takes from the PREVIOUS window's walk instead of
// the state (tmh_walk_next): status and the (before, after) cloud-cover and wind
// pairs at that window's end, so a walk can run while the previous window's
// expansion and commit are still in flight.  status == NULL: read the state.
struct PrevView {
    const uint32_t* status;
    const double* end_p1;   // [4][n]: cc before/after, ws before/after
};

// record i of chain c (its row, or its overflow chunks)
__device__ __forceinline__ int2 rec_at(const SegView& sg, uint32_t c, uint32_t i)
{
    if (i < sg.cap) return sg.rec[(size_t)c * sg.cap + i];
    const uint32_t o = i - sg.cap;
    const int32_t ch = sg.ovf[(size_t)c * OVF_SLOTS + o / OVF_CHUNK];
    return sg.pool[(size_t)ch * OVF_CHUNK + o % OVF_CHUNK];
}


// ------------------------------------------------------------ state I/O
__device__ __forceinline__ void load_chain(const StateView& st, uint32_t c, Chain& ch)
{
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        ch.s.b[k] = st.sb[k][c];
        ch.s.a[k] = st.sa[k][c];
    }
    ch.cl = st.cl[c];
    ch.clr = st.clr[c];
    ch.mstate = st.mstate[c];
    ch.sec = st.sec[c];
    ch.L = st.L[c];
    ch.pos = st.pos[c];
    ch.status = st.status[c];
    ch.ncalls = st.ncalls[c];
    ch.t1 = ceil_thr(ch.cl);
    ch.t2 = ceil_thr(ch.cl + ch.clr);
}

__device__ __forceinline__ void store_chain(const StateView& st, uint32_t c, const Chain& ch)
{
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        st.sb[k][c] = ch.s.b[k];
        st.sa[k][c] = ch.s.a[k];
    }
    st.cl[c] = ch.cl;
    st.clr[c] = ch.clr;
    st.mstate[c] = ch.mstate;
    st.sec[c] = ch.sec;
    st.L[c] = ch.L;
    st.pos[c] = ch.pos;
    st.status[c] = ch.status;
    st.ncalls[c] = ch.ncalls;
}

// ------------------------------------------------------------ init kernel
// The constructor's variates 2..11 (clear-day pair, cloudy-hour pair, the four
// minute noises, the wind-speed pair: fp64 ndtri / gammaincinv, the bulk of the
// constructor's time) one work-item per (chain, variate) instead of twelve in a
// row per chain (keyed mode).  Parked in the chain's sigma row, entries
// CAP-12.., which the constructor's next_cloud never reaches.
constexpr int INIT_SLOT = CAP - 12;

__device__ __forceinline__ void init_cc_pair(const KParams& kp, uint32_t c, const double* u, double& b, double& a)
{
    Chain ch;
    ch.mstate = 1.0;
    b = draw_cc(kp, gid(kp.ids, c), ch, u[0]);
    a = draw_cc(kp, gid(kp.ids, c), ch, u[1]);
}

__global__ __launch_bounds__(256, TMH_BUILD_WAVES) void init_variates_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                            double hf)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = 2 + (int)blockIdx.y;   // variate 2..11
    if (c >= n) return;
    const uint64_t chain = chain0 + gid(kp.ids, c);
    const U4 blk = keyed_block(kp.seed, chain, 0, TAG_INIT, (uint32_t)(j >> 1));
    const double u = (j & 1) ? u52(blk.z, blk.w) : u52(blk.x, blk.y);
    double v;
    if (j <= 3) {
        v = normal(u, 0.99, 0.08);
    } else if (j >= 10) {
        v = 2.14 * gammaincinv(2.69, u);
    } else {
        const U4 b0 = keyed_block(kp.seed, chain, 0, TAG_INIT, 0);
        const double u01[2] = {u52(b0.x, b0.y), u52(b0.z, b0.w)};
        double ccb, cca;
        init_cc_pair(kp, c, u01, ccb, cca);
        const double cc = interp(ccb, cca, hf);
        if (j <= 5) {   // clearskyindexmodel.py:68-82; 6/8 <= cc < 7/8 is the NameError
            v = cc < 6.0 / 8 ? normal(u, 0.6784, 0.2046) : (cc < 7.0 / 8 ? NAN : gammaincinv(3.5624, u) * 0.0867 + 0.0);
        } else {
            v = j <= 7 ? scaled_noise(kp, u, 0.01, 0.003, cc) : scaled_noise(kp, u, 0.001, 0.0015, cc);
        }
    }
    sig_c(st, c)[INIT_SLOT + j] = v;
}

// ClearskyindexModel.__init__ (clearskyindexmodel.py:57-99)
template <int RNG>
__global__ __launch_bounds__(256, TMH_BUILD_WAVES) void init_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                   double hf, InjView inj)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    Chain ch;
    for (int k = 0; k < 6; ++k) ch.s.b[k] = ch.s.a[k] = NAN;
    ch.cl = ch.clr = NAN;
    ch.mstate = 1.0;
    ch.sec = 0;
    ch.L = 0;
    ch.t1 = ch.t2 = 0;
    ch.pos = 0;
    ch.status = 0;
    ch.ncalls = 0;
    Draw<RNG> dr;
    if constexpr (RNG == TMH_RNG_KEYED) {
        dr.seed = kp.seed;
        dr.chain = chain0 + gid(kp.ids, c);
    } else {
        dr.u = inj.u + (size_t)c * inj.stride;
        dr.len = inj.len;
    }
    const double* pre = sig_c(st, c) + INIT_SLOT;   // keyed: variates 2..11 from init_variates_kernel
    double u[12];
    if constexpr (RNG == TMH_RNG_KEYED) {
        dr.two(ch, 0, TAG_INIT, 0, u[0], u[1]);
    } else {
        for (int d = 0; d < 12; d += 2) dr.two(ch, 0, TAG_INIT, (uint32_t)(d >> 1), u[d], u[d + 1]);
    }
    ch.s.b[S_CC] = draw_cc(kp, gid(kp.ids, c), ch, u[0]);
    ch.s.a[S_CC] = draw_cc(kp, gid(kp.ids, c), ch, u[1]);
    if constexpr (RNG == TMH_RNG_KEYED) {
        ch.s.b[S_CLEAR_DAY] = pre[2];
        ch.s.a[S_CLEAR_DAY] = pre[3];
    } else {
        ch.s.b[S_CLEAR_DAY] = normal(u[2], 0.99, 0.08);
        ch.s.a[S_CLEAR_DAY] = normal(u[3], 0.99, 0.08);
    }
    bool name_error = false;
    for (int j = 0; j < 2; ++j) {   // :68-82
        const double cc = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
        double v;
        if (cc < 6.0 / 8) v = RNG == TMH_RNG_KEYED ? pre[4 + j] : normal(u[4 + j], 0.6784, 0.2046);
        else if (cc < 7.0 / 8) {
            name_error = true;       // gamma.pdf(x, ...) with x undefined (:80)
            break;
        } else v = RNG == TMH_RNG_KEYED ? pre[4 + j] : gammaincinv(3.5624, u[4 + j]) * 0.0867 + 0.0;
        if (j == 0) ch.s.b[S_CLOUDY_HOUR] = v;
        else ch.s.a[S_CLOUDY_HOUR] = v;
    }
    if (name_error) {
        if constexpr (RNG == TMH_RNG_INJECTED) ch.pos = ch.pos < 4 ? ch.pos : 4;   // raised after 4 draws
        ch.status = TMH_CHAIN_NAMEERROR_INIT;
        store_chain(st, c, ch);
        return;
    }
    if constexpr (RNG == TMH_RNG_KEYED) {
        ch.s.b[S_CLOUDY_NOISE] = pre[6];
        ch.s.a[S_CLOUDY_NOISE] = pre[7];
        ch.s.b[S_CLEAR_NOISE] = pre[8];
        ch.s.a[S_CLEAR_NOISE] = pre[9];
        ch.s.b[S_WS] = pre[10];
        ch.s.a[S_WS] = pre[11];
    } else {
        const double cch = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
        ch.s.b[S_CLOUDY_NOISE] = scaled_noise(kp, u[6], 0.01, 0.003, cch);
        ch.s.a[S_CLOUDY_NOISE] = scaled_noise(kp, u[7], 0.01, 0.003, cch);
        ch.s.b[S_CLEAR_NOISE] = scaled_noise(kp, u[8], 0.001, 0.0015, cch);
        ch.s.a[S_CLEAR_NOISE] = scaled_noise(kp, u[9], 0.001, 0.0015, cch);
        ch.s.b[S_WS] = 2.14 * gammaincinv(2.69, u[10]);
        ch.s.a[S_WS] = 2.14 * gammaincinv(2.69, u[11]);
    }
    // CloudCoverBinary(cc.interpolate(0), ws.interpolate(0)) (:98-99)
    const double h0 = interp(ch.s.b[S_CC], ch.s.a[S_CC], 0.0);
    const double h = 0.95 < h0 ? 0.95 : h0;
    const double ws = interp(ch.s.b[S_WS], ch.s.a[S_WS], 0.0);
    double* sc = sig_c(st, c);
    double* sl = sig_l(st, c);
    const uint32_t f = next_cloud_fresh<RNG>(kp, sc, sl, ch, dr, h, ws, TAG_INIT_CLOUD);   // reset_sigma + next_cloud
    if (!f) {
        const double us = dr.one(ch, 0, TAG_INIT_SEC, 0, 0);
        ch.sec = (int32_t)((ch.cl + ch.clr) * us);   // cloud_cover_binary.py:68
    }
    if (f && !ch.status) ch.status = f;
    store_chain(st, c, ch);
    // the fp32 kernels' noise pairs start as the constructor's draws rounded
    st.fn[0][c] = make_float2((float)ch.s.b[S_CLOUDY_NOISE], (float)ch.s.a[S_CLOUDY_NOISE]);
    st.fn[1][c] = make_float2((float)ch.s.b[S_CLEAR_NOISE], (float)ch.s.a[S_CLEAR_NOISE]);
}

// ------------------------------------------------------------ plan kernels
__global__ __launch_bounds__(256, TMH_BUILD_WAVES) void geom_kernel(GParams gp, int64_t step0, uint32_t n, double* tab64,
                                                   float* tab32, double* sun)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const tmh_clock& ck = gp.clock;
    const int64_t s = step0 + j;
    const int64_t lt = local_at(ck, s), lp = local_at(ck, s > 0 ? s - 1 : 0);
    const int64_t dn = floordiv(lt, 86400), dp = floordiv(lp, 86400);
    const int64_t sod = lt - dn * 86400, sodp = lp - dp * 86400;
    const int hour = (int)(sod / 3600), minute = (int)((sod / 60) % 60), second = (int)(sod % 60);
    const int hourp = (int)(sodp / 3600), minutep = (int)((sodp / 60) % 60);
    double g[ROW];
    for (int i = 0; i < ROW; ++i) g[i] = 0.0;
    clock_fractions(hour, minute, second, g[G_MINF], g[G_HOURF], g[G_DAYF]);   // clearskyindexmodel.py:114-116
    uint32_t fl = 0;
    if (dn != dp) fl |= FL_DAY;           // :121 prev.day != day
    if (hour != hourp) fl |= FL_HOUR;     // :123
    if (minute != minutep) fl |= FL_MIN;  // :125
    // ---- PV geometry (pvmodel.py:50-76; pvlib 0.6.3 model choices) ----
    int doy, leap;
    civil_doy(dn, doy, leap);
    double sn[SUN_W];
    sun_at(ck.utc0 + s, doy, leap, gp.linke, sn);
    {   // the hour angle's advance since the step's 128-s block start (lane_row's rotation)
        const uint32_t jb = j / BLOCK_STEPS * BLOCK_STEPS;
        double sb[SUN_W];
        if (jb == j) {
            sb[SUN_MIN] = sn[SUN_MIN];
            sb[SUN_EOT] = sn[SUN_EOT];
        } else {
            const int64_t ltb = local_at(ck, step0 + jb);
            int doyb, leapb;
            civil_doy(floordiv(ltb, 86400), doyb, leapb);
            sun_at(ck.utc0 + step0 + jb, doyb, leapb, nullptr, sb);
        }
        const double dh = rad(((sn[SUN_MIN] + sn[SUN_EOT]) - (sb[SUN_MIN] + sb[SUN_EOT])) / 4.0);
        sincos(dh, &sn[SUN_SDH], &sn[SUN_CDH]);
    }
    for (int i = 0; i < SUN_W; ++i) sun[(size_t)j * SUN_W + i] = sn[i];
    site_geom<true>(site_k(gp.site), sn, sn[SUN_TL], gp.module, g);
    if (g[G_GHICS] == 0.0) fl |= FL_NIGHT;   // ghi_cs = 0 -> pv = 0 whatever the csi
    if (g[G_DISCOK] != 0.0) fl |= FL_DISCOK;
    g[G_FLAGS] = (double)fl;
    double* o64 = tab64 + (size_t)j * ROW;
    float* o32 = tab32 + (size_t)j * ROW32;
    for (int i = 0; i < ROW; ++i) o64[i] = g[i];
    const int fr[3] = {G_MINF, G_HOURF, G_DAYF}, fc[3] = {G32_MINF_C, G32_HOURF_C, G32_DAYF_C};
    for (int i = 0; i < 3; ++i) {   // (1 - f, f) pairs, 1 - f rounded in fp32 as the kernels computed it
        const float f = (float)g[fr[i]];
        o32[fc[i]] = 1.0f - f;
        o32[fc[i] + 1] = f;
    }
    for (int i = G_COSZ; i <= G_LAST; ++i) o32[i + G32] = (float)g[i];
    o32[G_FLAGS + G32] = __uint_as_float(fl);
    o32[G_I0H + G32] = (float)(1.0 / g[G_I0H]);   // fp32 path multiplies by reciprocals
    o32[G_DNIEXTRA + G32] = (float)(1.0 / g[G_DNIEXTRA]);
    o32[G_AM + G32] = (float)(g[G_AM] * LOG2E);   // exp(c am) = exp2(c * am log2 e)
    o32[G_F1 + G32] = (float)(g[G_F1] * 1e-3);    // Ee = F1 (...) / 1000 with the division folded in
    o32[G_RB + G32] = (float)(g[G_RB] - g[G_TERM2]);   // sky = dhi (term2 + AI (Rb - term2))
}

// The kind of each four-step group (first row j with (step0 + j) % 4 == 0, j + 3 < n) of a
// window on the four-step grid, ORed into its first fp32 row's flags: FL_G_NIGHT (four night
// seconds), FL_G_DAY (four daylight seconds with DISC valid); either only when seconds 1-3
// carry no boundary event.  Other windows and partial groups get neither bit.
__global__ __launch_bounds__(256) void group_kind_kernel(int64_t step0, uint32_t n, float* tab32, double* tab64)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, j = 4 * g;
    if ((step0 & 3) != 0 || j + 3 >= n) return;
    uint32_t f[4], ev = 0, all = ~0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        f[q] = __float_as_uint(tab32[(size_t)(j + q) * ROW32 + G_FLAGS + G32]);
        all &= f[q];
        if (q > 0) ev |= f[q] & (FL_DAY | FL_HOUR | FL_MIN);
    }
    const uint32_t anyn = (f[0] | f[1] | f[2] | f[3]) & FL_NIGHT;
    uint32_t k = 0;
    if (!ev && (all & FL_NIGHT)) k = FL_G_NIGHT;
    else if (!ev && !anyn && (all & FL_DISCOK)) k = FL_G_DAY;
    if (k) {   // both rows: the fp32 and the fp64 single-site expansions read it
        tab32[(size_t)j * ROW32 + G_FLAGS + G32] = __uint_as_float(f[0] | k);
        tab64[(size_t)j * ROW + G_FLAGS] = (double)(f[0] | k);
    }
}

// The window's 128-s blocks in the order the single-site expansion takes its tiles (round 6):
// blocks with a daylight second first, then the all-night blocks, each class in time order
// (a stable partition; one workgroup).  A night tile costs a tenth of a daylight one, so the
// expansion's last tiles are short ones and its tail no longer waits for late daylight tiles.
// A block is all night when every four-step group of it carries FL_G_NIGHT; windows off the
// four-step grid (no group kinds) keep the time order.
__global__ __launch_bounds__(1024) void block_order_kernel(const float* __restrict__ tab32, int64_t step0, uint32_t n,
                                                           uint32_t* __restrict__ perm)
{
    __shared__ uint32_t cnt[1024];
    const uint32_t t = threadIdx.x, nb = (n + BLOCK_STEPS - 1) / BLOCK_STEPS;
    const uint32_t chunk = (nb + 1023) / 1024, lo = min(t * chunk, nb), hi = min(lo + chunk, nb);
    auto night = [&](uint32_t b) {
        if ((step0 & 3) != 0) return false;
        const uint32_t j0 = b * BLOCK_STEPS, j1 = min(j0 + (uint32_t)BLOCK_STEPS, n);
        if (j1 - j0 < BLOCK_STEPS) return false;   // a short last block: its tail groups carry no kind
        for (uint32_t j = j0; j < j1; j += 4)
            if (!(__float_as_uint(tab32[(size_t)j * ROW32 + G_FLAGS + G32]) & FL_G_NIGHT)) return false;
        return true;
    };
    uint32_t d = 0;
    for (uint32_t b = lo; b < hi; ++b) d += night(b) ? 0u : 1u;
    cnt[t] = d;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // inclusive scan of the daylight counts
        const uint32_t v = t >= off ? cnt[t - off] : 0;
        __syncthreads();
        cnt[t] += v;
        __syncthreads();
    }
    const uint32_t nday = cnt[1023];
    uint32_t od = cnt[t] - d, on = nday + (lo - od);   // this range's first daylight / night slots
    for (uint32_t b = lo; b < hi; ++b) perm[night(b) ? on++ : od++] = b;
}

// Compact the window's day/hour boundary steps, in order (one workgroup).
// Every such boundary is also a minute boundary (local second 0 = UTC second 0
// for whole-minute offsets), so only one row per minute is inspected.
__global__ __launch_bounds__(1024) void events_kernel(const float* __restrict__ tab32, int64_t step0, uint32_t n,
                                                      int64_t utc0, int2* events, uint32_t cap, uint32_t* n_events)
{
    __shared__ uint32_t cnt[1024];
    const uint32_t t = threadIdx.x;
    const int64_t first = (60 - (((utc0 + step0) % 60) + 60) % 60) % 60;   // first candidate (window-relative)
    const uint32_t ncand = first < (int64_t)n ? (uint32_t)((n - 1 - first) / 60 + 1) : 0;
    const uint32_t chunk = (ncand + 1023) / 1024;
    const uint32_t lo = t * chunk, hi = min(lo + chunk, ncand);
    uint32_t c = 0;
    for (uint32_t q = lo; q < hi; ++q) {
        const uint64_t j = (uint64_t)(first + 60 * (int64_t)q);
        if (__float_as_uint(tab32[j * ROW32 + G_FLAGS + G32]) & (FL_DAY | FL_HOUR)) ++c;
    }
    cnt[t] = c;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // inclusive scan
        const uint32_t v = t >= off ? cnt[t - off] : 0;
        __syncthreads();
        cnt[t] += v;
        __syncthreads();
    }
    uint32_t o = cnt[t] - c;
    for (uint32_t q = lo; q < hi; ++q) {
        const uint64_t j = (uint64_t)(first + 60 * (int64_t)q);
        const uint32_t fl = __float_as_uint(tab32[j * ROW32 + G_FLAGS + G32]) & (FL_DAY | FL_HOUR);
        if (fl) {
            if (o < cap) events[o] = make_int2((int)(step0 + (int64_t)j), (int)fl);
            ++o;
        }
    }
    if (t == 1023) *n_events = cnt[1023];
}

// Room for a window's day / hour boundary events: a local hour boundary every 3,600 s
// (a day boundary is one of them) plus one per clock shift (<= 8), so n / 3600 + 10 at most
__device__ __forceinline__ uint32_t ev_cap_dev(uint32_t n_steps) { return n_steps / 3600 + 16; }

__host__ __device__ __forceinline__ int64_t first_minute(int64_t utc0, int64_t W0)
{   // window-relative step of the first candidate minute boundary (UTC second 0)
    return (60 - (((utc0 + W0) % 60) + 60) % 60) % 60;
}
inline int64_t first_minute_host(int64_t utc0, int64_t W0) { return first_minute(utc0, W0); }

// Descriptor of the sampler state after step p (window [step0, step0 + n), p >=
// step0): the last two minute draws, hour and clear-day events at or before p.
__device__ BlockDesc desc_for(int64_t step0, uint32_t n, int64_t utc0, const int2* __restrict__ events, int ne,
                              int64_t p)
{
    BlockDesc d{-1, -1, -1, -1, -1, -1, 0, -1};
    {
        const int64_t lo = step0 > 1 ? step0 : 1;          // step 0 is the constructor time
        const int64_t fm = first_minute(utc0, step0);
        const int64_t m0 = p - (((utc0 + p) % 60) + 60) % 60;
        if (m0 >= lo) d.q0 = (int32_t)((m0 - step0 - fm) / 60);
        if (m0 - 60 >= lo) d.q1 = (int32_t)((m0 - 60 - step0 - fm) / 60);
        int a = 0, z = ne;                                  // last event <= p
        while (a < z) {
            const int mid = (a + z) / 2;
            if (events[mid].x <= p) a = mid + 1;
            else z = mid;
        }
        d.evi = a;
        int nh = 0, ncd = 0;
        for (int i = a - 1; i >= 0 && (nh < 3 || ncd < 2); --i) {
            const int fl = events[i].y;
            if (fl & FL_HOUR) {
                if (nh == 0) d.h0 = i;
                else if (nh == 1) d.h1 = i;
                else if (nh == 2) d.h2 = i;
                ++nh;
                if (ncd < 2) {            // the hour push of clear_day follows its day push
                    if (ncd == 0) d.cd0 = 2 * i + 1;
                    else d.cd1 = 2 * i + 1;
                    ++ncd;
                }
            }
            if ((fl & FL_DAY) && ncd < 2) {
                if (ncd == 0) d.cd0 = 2 * i;
                else d.cd1 = 2 * i;
                ++ncd;
            }
        }
    }
    return d;
}

// desc_for(p) from an earlier descriptor d (of some step before p, evi = its first
// event after it): the window's events up to p applied forward (clear_day's day
// push before its hour push), the minute indices taken at p
__device__ __forceinline__ BlockDesc desc_advance(BlockDesc d, int64_t step0, int64_t utc0,
                                                  const int2* __restrict__ events, int ne, int64_t p)
{
    int i = d.evi;
    for (; i < ne && (int64_t)events[i].x <= p; ++i) {
        const int fl = events[i].y;
        if (fl & FL_DAY) {
            d.cd1 = d.cd0;
            d.cd0 = 2 * i;
        }
        if (fl & FL_HOUR) {
            d.h2 = d.h1;
            d.h1 = d.h0;
            d.h0 = i;
            d.cd1 = d.cd0;
            d.cd0 = 2 * i + 1;
        }
    }
    d.evi = i;
    const int64_t lo = step0 > 1 ? step0 : 1, fm = first_minute(utc0, step0);
    const int64_t m0 = p - (((utc0 + p) % 60) + 60) % 60;
    d.q0 = m0 >= lo ? (int32_t)((m0 - step0 - fm) / 60) : -1;
    d.q1 = m0 - 60 >= lo ? (int32_t)((m0 - 60 - step0 - fm) / 60) : -1;
    return d;
}

// Descriptor of the sampler state after step W0 + min(b * BLOCK_STEPS, n) - 1,
// for b = 0 .. nblk (the last one describes the window end).
__global__ __launch_bounds__(256) void desc_kernel(int64_t step0, uint32_t n, int64_t utc0,
                                                   const int2* __restrict__ events,
                                                   const uint32_t* __restrict__ n_events, BlockDesc* desc,
                                                   uint32_t nblk)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nblk) return;
    const int64_t jb = min((int64_t)b * BLOCK_STEPS, (int64_t)n);
    desc[b] = jb > 0 ? desc_for(step0, n, utc0, events, (int)min(*n_events, ev_cap_dev(n)), step0 + jb - 1)
                     : BlockDesc{-1, -1, -1, -1, -1, -1, 0, -1};
}

// ------------------------------------------------------------ boundary draws
// markov mode: the first Student-t bin of chain slot c's shape table (the reference's table has
// one, bin 2: cloud_cover_hourly.py:282-288,314) and its degrees of freedom; -1 when none
__device__ __forceinline__ int first_t_bin(const KParams& kp, uint32_t c, double& df)
{
    const uint32_t r = gid(kp.ids, c);   // the table row of the slot's chain
    for (int b = 0; b < 6; ++b) {
        const int t = kp.tab && kp.tab_t ? kp.tab_t[(size_t)r * 6 + b] : kp.is_t[b];
        if (t) {
            df = kp.tab ? kp.tab[(size_t)r * 24 + 4 * b + 3] : kp.shapes[b][3];
            return b;
        }
    }
    df = 0.0;
    return -1;
}

// _next_day / _next_hour draws of every (event, chain): clearskyindexmodel.py:101-107.
// Markov mode (round 6): the hour's Student-t quantile of the chain's first t bin,
// stdtrit(df, u) of the hour's uniform, into the cc slot (evd[e][0]): it does not depend on the
// hour-to-hour state, so it is drawn here for every (hour, chain) at full occupancy, and
// markov_cc_kernel's one-lane-per-chain walk takes it when the state's bin is that bin (the same
// function of the same values, so bit for bit what it computed in line).  Only for batches of at
// most the engine's mk_pre_max chains (the walk is latency-bound there: C5's N = 8 shard, 8,192
// chains, 3.13 -> 4.14e10 live chain-s/s); a full C5 batch (65,536) computes the quantile in the
// walk, only for the hours whose state sits in the t bin (precomputed: 5.36 -> 4.96e10).  mk_pre:
// this launch precomputes (markov_cc_kernel's tb = -1 otherwise).
__global__ __launch_bounds__(256, TMH_BUILD_WAVES) void event_draws_kernel(DrawParams dp, KParams kp, bool mk_pre, uint64_t chain0,
                                                          uint32_t n, uint32_t nsteps, const int2* __restrict__ events,
                                                          const uint32_t* __restrict__ n_events, double* evd,
                                                          uint32_t* identity_order, uint32_t* identity_rank)
{
    const uint32_t c = blockIdx.y * blockDim.x + threadIdx.x;
    const uint32_t e = blockIdx.x;
    if (identity_order && e == 0 && c < n) {   // walk rows in chain order (tmh_set_walk_order off)
        identity_order[c] = c;
        identity_rank[c] = c;
    }
    if (c >= n || e >= min(*n_events, ev_cap_dev(nsteps))) return;
    const uint64_t chain = chain0 + gid(dp.ids, c), step = (uint64_t)events[e].x;
    const int fl = events[e].y;
    double* o = evd + (size_t)e * 4 * n + c;
    if (fl & FL_DAY) {
        const U4 u = keyed_block(dp.seed, chain, step, TAG_BOUNDARY, 0);
        o[2 * (size_t)n] = normal(u52(u.x, u.y), 0.99, 0.08);
        o[(size_t)n] = 2.14 * gammaincinv(2.69, u52(u.z, u.w));
    }
    if (fl & FL_HOUR) {
        const U4 u = keyed_block(dp.seed, chain, step, TAG_BOUNDARY, 1);
        if (!dp.markov) {
            o[0] = cc_faithful(dp, gid(dp.ids, c), u52(u.x, u.y));
        } else if (mk_pre) {
            double df;
            const int tb = first_t_bin(kp, c, df);
            o[0] = tb >= 0 ? stdtrit(df, u52(u.x, u.y)) : 0.0;
        }
        o[3 * (size_t)n] = normal(u52(u.z, u.w), 0.99, 0.08);
    }
}

// markov-mode hourly cloud cover (cloud_cover_hourly.py:309-316 as one long-lived
// generator per chain): the only sequential dependence in the window is the
// hour-to-hour cc state, 24 draws a day, so one lane per chain walks the
// window's hour events in order and fills evd[e][0] for the time-parallel
// kernels.  The state is the last drawn cc, i.e. sa[S_CC] (init and every
// _next_hour push the markov state), so nothing extra is carried over.
//
// Per-chain tables (C5's lat/lon sweep): the workgroup's 256 rows of shape
// parameters ([256][6][4] fp64 + [256][6] Student-t flags, 54 KB, one contiguous
// range of the caller's table) are staged in LDS once with coalesced 16-B loads,
// so each hourly draw reads its bin's four parameters from LDS instead of a
// scattered 32-B global read per chain-hour.  The bin select (np.searchsorted on
// the shared right edges, :309) is branch-free per lane, and the two quantile
// families are taken as wave-uniform branches on a wave64 ballot of the lanes'
// Student-t flags (bin 2 of the reference's table, cloud_cover_hourly.py:314),
// so a wave whose lanes all sit in AL bins never enters stdtrit.
constexpr int MK_BLOCK = 256;
__global__ __launch_bounds__(MK_BLOCK) void markov_cc_kernel(KParams kp, bool mk_pre, StateView st, uint64_t chain0, uint32_t n,
                                                        uint32_t nsteps, const int2* __restrict__ events,
                                                        const uint32_t* __restrict__ n_events, double* evd,
                                                        PrevView prev)
{
    __shared__ double2 tab_s[MK_BLOCK * 12];   // [chain][bin][4] fp64, as double2 pairs
    __shared__ int32_t tabt_s[MK_BLOCK * 6];
    const uint32_t cb0 = blockIdx.x * MK_BLOCK;
    const uint32_t nb = min((uint32_t)MK_BLOCK, n - cb0);
    if (kp.tab && !kp.ids) {   // the block's rows are one contiguous range: coalesced 16-B loads
        const double2* src = reinterpret_cast<const double2*>(kp.tab + (size_t)cb0 * 24);
        for (uint32_t i = threadIdx.x; i < nb * 12; i += MK_BLOCK) tab_s[i] = src[i];
        for (uint32_t i = threadIdx.x; i < nb * 6; i += MK_BLOCK)
            tabt_s[i] = kp.tab_t ? kp.tab_t[(size_t)cb0 * 6 + i] : kp.is_t[i % 6];
    } else if (kp.tab) {   // a compacted batch: each slot's row of its chain (12 x 16 B)
        for (uint32_t i = threadIdx.x; i < nb * 12; i += MK_BLOCK) {
            const uint32_t g = kp.ids[cb0 + i / 12];
            tab_s[i] = reinterpret_cast<const double2*>(kp.tab + (size_t)g * 24)[i % 12];
        }
        for (uint32_t i = threadIdx.x; i < nb * 6; i += MK_BLOCK)
            tabt_s[i] = kp.tab_t ? kp.tab_t[(size_t)kp.ids[cb0 + i / 6] * 6 + i % 6] : kp.is_t[i % 6];
    }
    __syncthreads();
    const uint32_t c = cb0 + threadIdx.x;
    if (c >= n) return;
    const uint64_t chain = chain0 + gid(kp.ids, c);
    const uint32_t ne = min(*n_events, ev_cap_dev(nsteps));
    const double* row = kp.tab ? reinterpret_cast<const double*>(tab_s) + threadIdx.x * 24 : nullptr;
    const int32_t* rowt = tabt_s + threadIdx.x * 6;
    double state = prev.status ? prev.end_p1[(size_t)n + c] : st.mstate[c];   // the last hourly draw
    // the first Student-t bin, whose quantile event_draws_kernel left in the hour's cc slot
    int tb = -1;
    if (mk_pre)
        for (int b = 5; b >= 0; --b)
            if (row ? rowt[b] : kp.is_t[b]) tb = b;
    for (uint32_t e = 0; e < ne; ++e) {
        const int2 ev = events[e];
        if (!(ev.y & FL_HOUR)) continue;
        const double qt = mk_pre ? evd[(size_t)e * 4 * n + c] : 0.0;   // stdtrit(df of bin tb, u): event_draws_kernel
        const U4 u4 = keyed_block(kp.seed, chain, (uint64_t)ev.x, TAG_BOUNDARY, 1);
        const double u = u52(u4.x, u4.y);
        int bin = 5;   // np.searchsorted(bins, state): the first bin whose right edge is >= state
#pragma unroll
        for (int k = 4; k >= 0; --k) bin = kp.edges[k] < state ? bin : k;
        double loc, scale, kappa, df;
        int is_t;
        if (row) {
            const double* sh = row + 4 * bin;
            loc = sh[0];
            scale = sh[1];
            kappa = sh[2];
            df = sh[3];
            is_t = rowt[bin];
        } else {
            loc = kp.shapes[bin][0];
            scale = kp.shapes[bin][1];
            kappa = kp.shapes[bin][2];
            df = kp.shapes[bin][3];
            is_t = kp.is_t[bin];
        }
        // a t bin other than tb (none in the reference's table) draws its quantile here
        const bool t_here = is_t && bin != tb;
        const uint64_t tl = __builtin_amdgcn_ballot_w64(t_here);
        const uint64_t al = __builtin_amdgcn_ballot_w64(is_t == 0);
        double v = is_t ? qt : 0.0;
        if (tl && t_here) v = stdtrit(df, u);
        if (al && !is_t) v = al_ppf(u, kappa);
        v = v * scale + loc;                              // scipy rvs: vals * scale + loc
        const double x = state + v;
        state = x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);      // np.clip(., 0, 1)
        evd[(size_t)e * 4 * n + c] = state;
    }
}

// _next_min draws of every (minute boundary, chain): clearskyindexmodel.py:86-95,109-111
// the two _next_min draws of the minute boundary at window step j (keyed by step):
// fp64 (minute_noise) or the fp32 kernels' copies (minute_noise_fast)
template <typename R>
__device__ __forceinline__ void minute_draws(const DrawParams& dp, uint64_t chain, int64_t step, double cc,
                                             double& cloudy, double& clear)
{
    const U4 u = keyed_block(dp.seed, chain, (uint64_t)step, TAG_BOUNDARY, 2);
    if constexpr (sizeof(R) == 8) {
        cloudy = minute_noise<R>(u52(u.x, u.y), 0.01, 0.003, cc, dp.sqrt09);
        clear = minute_noise<R>(u52(u.z, u.w), 0.001, 0.0015, cc, dp.sqrt09);
    } else {
        cloudy = minute_noise_fast(u52(u.x, u.y), 0.01, 0.003, cc, dp.sqrt09);
        clear = minute_noise_fast(u52(u.z, u.w), 0.001, 0.0015, cc, dp.sqrt09);
    }
}

// the cloud cover in force at the minute boundary at window step jm (the last
// two hourly draws at or before it, or the window-start pair: the state's, or the
// previous window's walk's end pair when the window is chained to it), interpolated
__device__ __forceinline__ double minute_cc(const StateView& st, const PrevView& prev, const SegView& sg, uint32_t n,
                                            uint32_t c, int64_t W0, int64_t jm, const int2* __restrict__ events, int ne,
                                            const double* __restrict__ tab64)
{
    const int64_t step = W0 + jm;
    int lo = 0, hi = ne;   // h0 = number of boundary events at or before the step, minus one
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)events[mid].x <= step) lo = mid + 1;
        else hi = mid;
    }
    const int h0 = lo - 1, h1 = lo - 2;
    const double* evd = sg.evd;
    const double sb = prev.status ? prev.end_p1[c] : st.sb[S_CC][c];
    const double sa = prev.status ? prev.end_p1[(size_t)n + c] : st.sa[S_CC][c];
    double pb, pa;
    if (h0 < 0) {
        pb = sb;
        pa = sa;
    } else {
        pa = evd[(size_t)h0 * 4 * n + c];
        pb = h1 < 0 ? sa : evd[(size_t)h1 * 4 * n + c];
    }
    return interp(pb, pa, tab64[(size_t)jm * ROW + G_HOURF]);
}

// The window's per-chain draws that need the boundary-event draws but not the segment
// walk: one launch after event_draws_kernel (+ markov_cc_kernel, walk_order_kernel).
//  * rows y < kcap: the try-0 candidate lengths pow(alpha + delta u, expo) of each
//    chain's next kcap next_cloud calls (cloud_cover_binary.py:35-40; keyed by (chain,
//    call number) only, so drawn here at full occupancy instead of one wave-redundant
//    Philox + pow per call in the walk), stored by walk row;
//  * rows kcap + m: the _next_min draws (clearskyindexmodel.py:86-95,109-111) of the
//    window's minute boundary m (window step fm + 60 m) of every chain, which the
//    expansion's per-second loop, its block-start reconstruction and the commit read
//    instead of drawing.  R = float: the fp32 kernels' copies, plus the fp64 draws of
//    the window's last two minute boundaries (the state's noise samplers at the window
//    end, which commit_kernel stores) in `mend`;
//  * row 0 also resets the walk's pool / queue counters and the expansion's guard-band
//    records and statistics accumulators.
// Chained to the previous window's walk (prev), the window-start status and cloud-cover
// pair come from that walk, so these draws may run before that window's expansion and
// commit (tmh_walk_part).  Built with the construction (TMH_WALK_DRAWS), the minute
// table is off the expansion's stream.
// rows y of the launch: y < kcap the try-0 candidate of the chain's call ncalls + y;
// y = kcap + m the draws of the window's minute boundary m.  Grid-stride over y (ny
// rows, gridDim.y <= 65,535), so no window length is bounded by the grid.
template <typename R>
__global__ __launch_bounds__(256) void draws_tail_kernel(DrawParams dp, StateView st, uint64_t chain0, uint32_t n,
                                                         int64_t W0, uint32_t nsteps, int64_t fm, uint32_t ny,
                                                         const double* __restrict__ tab64,
                                                         const int2* __restrict__ events,
                                                         const uint32_t* __restrict__ n_events,
                                                         const BlockDesc* __restrict__ desc_end, SegView sg,
                                                         PrevView prev)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.y == 0) {
        if (c == 0) {   // the walk that follows hands out overflow chunks and queued chains
            *sg.pool_n = 0;
            *sg.walk_q = 0;
            *sg.pool_short = 0;
            *sg.nfix = 0;
        }
        if (c < n) {    // the expansion's guard-band corrections and fixed-point statistics
            sg.corr[c] = 0.0;
            sg.corr[(size_t)n + c] = 0.0;
            for (int k = 0; k < 3; ++k) sg.acc_fx[(size_t)k * n + c] = 0;
            sg.acc_mx[c] = max_key(-INFINITY);
        }
    }
    if (c >= n) return;
    const uint64_t chain = chain0 + gid(dp.ids, c);
    const bool live = (prev.status ? prev.status[c] : st.status[c]) == 0;
    const int ne = (int)min(*n_events, ev_cap_dev(nsteps));
    for (uint32_t y = blockIdx.y; y < ny; y += gridDim.y) {
        if (y < sg.kcap) {
            if (!live) continue;
            const U4 b = keyed_block(dp.seed, chain, (uint64_t)(st.ncalls[c] + y), TAG_CLOUD, 0);
            // stored by walk row: the chains of a walk wavefront read adjacent words
            sg.cand[(size_t)y * n + (sg.rank ? sg.rank[c] : c)] = pow_d(dp.alpha + dp.delta * u52(b.x, b.y), dp.expo);
            continue;
        }
        const uint32_t m = y - sg.kcap;
        const int64_t jm = fm + 60 * (int64_t)m;
        if (jm >= (int64_t)nsteps) continue;
        const double cc = minute_cc(st, prev, sg, n, c, W0, jm, events, ne, tab64);
        double cloudy, clear;
        minute_draws<R>(dp, chain, W0 + jm, cc, cloudy, clear);
        R* t = reinterpret_cast<R*>(sg.mtab);
        t[(size_t)(2 * m) * n + c] = (R)cloudy;
        t[(size_t)(2 * m + 1) * n + c] = (R)clear;
        if constexpr (sizeof(R) == 4) {   // the window end's last two minute boundaries, in fp64
            const BlockDesc de = *desc_end;
            const int q = (int32_t)m == de.q0 ? 1 : ((int32_t)m == de.q1 ? 0 : -1);
            if (q >= 0) {
                minute_draws<double>(dp, chain, W0 + jm, cc, cloudy, clear);
                sg.mend[(size_t)(2 * q) * n + c] = cloudy;
                sg.mend[(size_t)(2 * q + 1) * n + c] = clear;
            }
        }
    }
}

// cc / clear_day / noise pairs described by `d`, from the draw tables (start = window start)
// what the minute draws of a block start / window end need
struct MinuteCtx {
    DrawParams dp;
    uint64_t chain;
    int64_t W0, fm;
    const int2* events;
    int ne;
    const double* tab64;
};

// R = float: the noise pairs are the fp32 copies (the caller starts them from StateView::fn)
template <typename R>
__device__ __forceinline__ void samplers_at(const BlockDesc& d, const SegView& sg, uint32_t n, uint32_t c, Samp& s,
                                            const MinuteCtx& mc, const StateView& st)
{
    const double* evd = sg.evd;
    if (d.h0 >= 0) {
        const double na = evd[(size_t)d.h0 * 4 * n + c];
        s.b[S_CC] = d.h1 >= 0 ? evd[(size_t)d.h1 * 4 * n + c] : s.a[S_CC];
        s.a[S_CC] = na;
    }
    if (d.cd0 >= 0) {
        auto cdv = [&](int32_t key) { return evd[((size_t)(key >> 1) * 4 + ((key & 1) ? 3 : 2)) * n + c]; };
        const double na = cdv(d.cd0);
        s.b[S_CLEAR_DAY] = d.cd1 >= 0 ? cdv(d.cd1) : s.a[S_CLEAR_DAY];
        s.a[S_CLEAR_DAY] = na;
    }
    if (d.q0 >= 0) {   // the last two minute boundaries: their draws from the minute table
        const R* t = reinterpret_cast<const R*>(sg.mtab);
        if (d.q1 >= 0) {
            s.b[S_CLOUDY_NOISE] = (double)t[(size_t)(2 * d.q1) * n + c];
            s.b[S_CLEAR_NOISE] = (double)t[(size_t)(2 * d.q1 + 1) * n + c];
        } else {
            s.b[S_CLOUDY_NOISE] = s.a[S_CLOUDY_NOISE];
            s.b[S_CLEAR_NOISE] = s.a[S_CLEAR_NOISE];
        }
        s.a[S_CLOUDY_NOISE] = (double)t[(size_t)(2 * d.q0) * n + c];
        s.a[S_CLEAR_NOISE] = (double)t[(size_t)(2 * d.q0 + 1) * n + c];
    }
}

// the cloud cover in force after descriptor d's step (back = 1: before its last
// hour push), interpolated at hour fraction hf
__device__ __forceinline__ double desc_cc(const BlockDesc& d, int back, const StateView& st, const SegView& sg,
                                          uint32_t n, uint32_t c, double hf)
{
    const int h0 = back ? d.h1 : d.h0, h1 = back ? d.h2 : d.h1;
    double pb, pa;
    if (h0 < 0) {
        pb = st.sb[S_CC][c];
        pa = st.sa[S_CC][c];
    } else {
        pa = sg.evd[(size_t)h0 * 4 * n + c];
        pb = h1 < 0 ? st.sa[S_CC][c] : sg.evd[(size_t)h1 * 4 * n + c];
    }
    return interp(pb, pa, hf);
}

// fp32 mode: the fp64 noise pairs described by `d` (s starts from the state's
// fp64 pairs): the minute draws of d.q0 / d.q1 computed again in fp64 (the fp32
// minute table holds the fast copies only).  Every hour event at or before d's
// step is at or before minute q0 (hour boundaries are minute boundaries), so q0
// draws with d's cloud-cover pair, q1 with the pair before an hour push at q0.
__device__ __forceinline__ void exact_noise_at(const BlockDesc& d, const DrawParams& dp, const StateView& st,
                                               const SegView& sg, uint32_t n, uint32_t c, uint64_t chain0,
                                               int64_t W0, int64_t fm, const int2* events, const double* tab64,
                                               Samp& s)
{
    if (d.q0 < 0) return;
    const int64_t jm0 = fm + 60 * (int64_t)d.q0;
    double cl, cr;
    if (d.q1 >= 0) {
        const int64_t jm1 = jm0 - 60;
        const int back = (d.h0 >= 0 && (int64_t)events[d.h0].x == W0 + jm0) ? 1 : 0;
        minute_draws<double>(dp, chain0 + gid(dp.ids, c), W0 + jm1, desc_cc(d, back, st, sg, n, c, tab64[(size_t)jm1 * ROW + G_HOURF]),
                             cl, cr);
        s.b[S_CLOUDY_NOISE] = cl;
        s.b[S_CLEAR_NOISE] = cr;
    } else {
        s.b[S_CLOUDY_NOISE] = s.a[S_CLOUDY_NOISE];
        s.b[S_CLEAR_NOISE] = s.a[S_CLEAR_NOISE];
    }
    minute_draws<double>(dp, chain0 + gid(dp.ids, c), W0 + jm0, desc_cc(d, 0, st, sg, n, c, tab64[(size_t)jm0 * ROW + G_HOURF]), cl,
                         cr);
    s.a[S_CLOUDY_NOISE] = cl;
    s.a[S_CLEAR_NOISE] = cr;
}

// the fp32 state's fast noise pairs into a Samp about to be rounded to float
__device__ __forceinline__ void load_fast_noise(const StateView& st, uint32_t c, Samp& s)
{
    const float2 a = st.fn[0][c], b = st.fn[1][c];
    s.b[S_CLOUDY_NOISE] = a.x;
    s.a[S_CLOUDY_NOISE] = a.y;
    s.b[S_CLEAR_NOISE] = b.x;
    s.a[S_CLEAR_NOISE] = b.y;
}

// One second of a chain at window step j, rebuilt outside the expansion: the
// sampler state (window-start state + desc_for(j) over the fp64 draw tables, as
// a block start does), the covered bit (the tile's, from its FixRec) and the step's
// Philox words.  fixup_kernel uses it for the fp32 expansion's guard-band seconds
// (pv_power_f: DISC's kt = 0.6 split, the inverter's Pso cut-in): `pv32` is the
// second as the fp32 expansion emitted it (the same fp32 arithmetic on the same
// values), `pv64` the fp64 kernel's second, whose branch falls as in the fp64
// reference.  need32 = false (no statistics to correct): the fp32 second is not
// recomputed, since a recorded second is a guard-band second by construction (the
// expansion's `held` is this `risky`), and the meter comes from its Philox word alone.
template <bool SITES>
__device__ __forceinline__ bool redo_second(const KParams& kp, const DrawParams& dp, const StateView& st,
                                            const SegView& sg, uint32_t n, uint32_t c, uint64_t chain0, int64_t W0,
                                            int64_t utc0, uint32_t j, const BlockDesc& db, bool covered, bool need32,
                                            const int2* events, int ne, const double* tab64, const float* tab32,
                                            const double* sun, float& pv32, float& meter32, float& pv64)
{   // returns whether the fp32 second lies in a guard band (then pv64 is set)
    double row64[ROW];   // issued first: independent of the samplers' chain of loads
#pragma unroll
    for (int i = 0; i < ROW; ++i) row64[i] = tab64[(size_t)j * ROW + i];
    const int64_t step = W0 + (int64_t)j;
    const BlockDesc d = desc_advance(db, W0, utc0, events, ne, step);   // db: the block's descriptor
    Samp s;   // the fp32 kernels' samplers: fast noise copies
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        s.b[k] = st.sb[k][c];
        s.a[k] = st.sa[k][c];
    }
    load_fast_noise(st, c, s);
    const MinuteCtx mc{};
    samplers_at<float>(d, sg, n, c, s, mc, st);
    Samp sx = s;   // the fp64 samplers: the state's fp64 noise pairs + the fp64 minute draws
    sx.b[S_CLOUDY_NOISE] = st.sb[S_CLOUDY_NOISE][c];
    sx.a[S_CLOUDY_NOISE] = st.sa[S_CLOUDY_NOISE][c];
    sx.b[S_CLEAR_NOISE] = st.sb[S_CLEAR_NOISE][c];
    sx.a[S_CLEAR_NOISE] = st.sa[S_CLEAR_NOISE][c];
    exact_noise_at(d, dp, st, sg, n, c, chain0, W0, first_minute(utc0, W0), events, tab64, sx);
    const uint64_t gch = chain0 + gid(kp.ids, c);   // the step's noise and meter words (TAG_NOISE4 / TAG_METER4)
    const uint32_t wn = word_of(keyed_block(kp.seed, gch, (uint64_t)step >> 2, TAG_NOISE4, 0), (uint32_t)step & 3u);
    const uint32_t wm = word_of(keyed_block(kp.seed, gch, (uint64_t)step >> 2, TAG_METER4, 0), (uint32_t)step & 3u);
    LaneSite ls{};
    if constexpr (SITES) {
        ls.k = site_k(kp.sites + (size_t)gid(kp.ids, c) * 8);
        ls.linke = kp.site_linke ? kp.site_linke + (size_t)gid(kp.ids, c) * 12 : nullptr;
        ls.tl_doy = -1;
        lane_anchor(ls, sun + (size_t)(j / BLOCK_STEPS * BLOCK_STEPS) * SUN_W);
    }
    bool risky = true;
    if (need32) {   // fp32, as expand_kernel<float>
        FSamp<float> f;
        to_real(f, s);
        float row[ROW32];
#pragma unroll
        for (int i = 0; i < ROW32; ++i) row[i] = tab32[(size_t)j * ROW32 + i];
        float csi, m, r;
        const uint32_t fl = __float_as_uint(row[G_FLAGS + G32]) & ~(uint32_t)FL_NIGHT;
        uint32_t flp = __float_as_uint(row[G_FLAGS + G32]);
        if constexpr (SITES) flp = lane_flags(fl, lane_row<float>(ls, sun + (size_t)j * SUN_W, kp.module, row), row);
        second_body<float>(kp, kp.pvf, row, flp, f, covered, noise_z<float>(wn), meter_w<float>(wm), csi, pv32, m, r,
                           risky);
        meter32 = m;
        if (!risky) return false;
    } else {
        meter32 = meter_w<float>(wm);   // second_body's meter
        pv32 = 0.0f;
    }
    {   // fp64, as expand_kernel<double>
        FSamp<double> f;
        to_real(f, sx);
        if constexpr (SITES) lane_row<double>(ls, sun + (size_t)j * SUN_W, kp.module, row64);
        double csi, pv, m, r;
        second_body<double>(kp, kp.pvf, row64, 0u, f, covered, noise_z<double>(wn), 0.0, csi, pv, m, r,
                            risky);
        pv64 = (float)pv;
    }
    return true;
}

// ------------------------------------------------------------ sequential kernel
// Advance chains [0, n) over steps [step0, step0 + nsteps), one lane per chain.
template <typename R, int RNG>
__global__ __launch_bounds__(256) void chain_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                    int64_t step0, uint32_t nsteps,
                                                    const double* __restrict__ tab64,
                                                    const float* __restrict__ tab32,
                                                    const double* __restrict__ sun, InjView inj, TraceView tr,
                                                    StatsView sv)
{
    extern __shared__ uint32_t lds_hist[];
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = c < n;
    if (sv.hist) {
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x) lds_hist[i] = 0;
        __syncthreads();
    }
    Chain ch;
    if (live) load_chain(st, c, ch);
    else ch.status = 0xFFFFFFFFu;
    Draw<RNG> dr;
    if constexpr (RNG == TMH_RNG_KEYED) {
        dr.seed = kp.seed;
        dr.chain = chain0 + gid(kp.ids, c);
    } else {
        dr.u = inj.u + (size_t)c * inj.stride;
        dr.len = inj.len;
    }
    const uint64_t chain = chain0 + gid(kp.ids, c);
    double* sc = live ? sig_c(st, c) : nullptr;
    double* sl = live ? sig_l(st, c) : nullptr;
    FSamp<R> fs;
    to_real(fs, ch.s);
    float2 fnc{0.f, 0.f}, fnl{0.f, 0.f};   // fp32: the fast noise pairs (StateView::fn) the fp32 second samples
    if constexpr (sizeof(R) == 4) {
        if (live) {
            fnc = st.fn[0][c];
            fnl = st.fn[1][c];
        }
        set_fast_noise(fs, fnc, fnl);
    }
    Acc acc{0.0, 0.0, 0.0, -INFINITY};
    LaneSite ls{};   // per-chain sites (tmh_set_sites)
    uint32_t ls_block = ~0u;   // the block whose start anchors ls's hour angle
    if (kp.sites) {
        ls.k = site_k(kp.sites + (size_t)(live ? gid(kp.ids, c) : 0) * 8);
        ls.linke = kp.site_linke ? kp.site_linke + (size_t)(live ? gid(kp.ids, c) : 0) * 12 : nullptr;
        ls.tl_doy = -1;
    }
    uint64_t grp = ~0ull;   // the per-second draws' current four-step group and its two blocks
    U4 bn{0u, 0u, 0u, 0u}, bm{0u, 0u, 0u, 0u};
    for (uint32_t j = 0; j < nsteps; ++j) {
        const uint64_t step = (uint64_t)(step0 + j);
        const float* r32 = tab32 + (size_t)j * ROW32;
        const double* r64 = tab64 + (size_t)j * ROW;
        const uint32_t fl = __float_as_uint(r32[G_FLAGS + G32]);
        R row[row_w<R>()];
#pragma unroll
        for (int i = 0; i < row_w<R>(); ++i) row[i] = sizeof(R) == 8 ? (R)r64[i] : (R)r32[i];
        R csi = R(NAN), pv = R(NAN), meter = R(NAN), res = R(NAN);
        uint8_t cov = 255;
        bool ok = false;
        if (ch.status == 0) {
            if (fl & (FL_DAY | FL_HOUR | FL_MIN)) {   // _set_time boundaries (:120-126)
                const double hf = r64[G_HOURF];
                double u0, u1;
                if (fl & FL_DAY) {                     // _next_day
                    dr.two(ch, step, TAG_BOUNDARY, 0, u0, u1);
                    push(ch.s, S_CLEAR_DAY, normal(u0, 0.99, 0.08));
                    push(ch.s, S_WS, 2.14 * gammaincinv(2.69, u1));
                }
                if (fl & FL_HOUR) {                    // _next_hour (advances clear_day)
                    dr.two(ch, step, TAG_BOUNDARY, 1, u0, u1);
                    push(ch.s, S_CC, draw_cc(kp, gid(kp.ids, c), ch, u0));
                    push(ch.s, S_CLEAR_DAY, normal(u1, 0.99, 0.08));
                }
                if (fl & FL_MIN) {                     // _next_min
                    dr.two(ch, step, TAG_BOUNDARY, 2, u0, u1);
                    const double cc = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
                    push(ch.s, S_CLOUDY_NOISE, minute_noise<R>(u0, 0.01, 0.003, cc, kp.sqrt09));
                    push(ch.s, S_CLEAR_NOISE, minute_noise<R>(u1, 0.001, 0.0015, cc, kp.sqrt09));
                    if constexpr (sizeof(R) == 4) {
                        fnc = make_float2(fnc.y, minute_noise_fast(u0, 0.01, 0.003, cc, kp.sqrt09));
                        fnl = make_float2(fnl.y, minute_noise_fast(u1, 0.001, 0.0015, cc, kp.sqrt09));
                    }
                }
                to_real(fs, ch.s);
                if constexpr (sizeof(R) == 4) set_fast_noise(fs, fnc, fnl);
            }
            ch.sec += 1;                                 // CloudCoverBinary.__next__
            while (ch.sec >= ch.t2 && ch.status == 0) {  // segment over: next_cloud(); next(self)
                const double hh = interp(ch.s.b[S_CC], ch.s.a[S_CC], r64[G_HOURF]);
                const double h = 0.95 < hh ? 0.95 : hh;  // update_parameters
                const double ws = interp(ch.s.b[S_WS], ch.s.a[S_WS], r64[G_DAYF]);
                const uint32_t f = next_cloud<RNG>(kp, sc, sl, ch, dr, h, ws, TAG_CLOUD);
                if (f) ch.status = f;
                else ch.sec += 1;
            }
            if (ch.status == 0) {
                // keyed: the noise's and the meter's streams, one Philox block per four
                // steps each, 32-bit words; the meter is its own process in the
                // reference: always keyed.  Drawn again when the step's group changes.
                if ((uint64_t)step >> 2 != grp) {
                    grp = (uint64_t)step >> 2;
                    bn = keyed_block(kp.seed, chain, grp, TAG_NOISE4, 0);
                    bm = keyed_block(kp.seed, chain, grp, TAG_METER4, 0);
                }
                const uint32_t wn = word_of(bn, (uint32_t)step & 3u);
                R z = noise_z<R>(wn);
                double z64 = 0.0;   // fp32: the fp64 quantile for the guard-band recomputation
                const R mtr = meter_w<R>(word_of(bm, (uint32_t)step & 3u));
                if constexpr (RNG == TMH_RNG_INJECTED) {
                    const double ue = dr.one(ch, step, TAG_STEP, 0, 0);
                    if constexpr (sizeof(R) == 8) z = ndtri(ue);
                    else {
                        z = ndtri_f(ue);
                        z64 = ue;   // quantile taken on the rare path only
                    }
                }
                if (ch.status == 0) {
                    const bool covered = ch.sec < ch.t1;
                    cov = covered ? 1 : 0;
                    uint32_t flp = fl;
                    if (kp.sites) {   // this chain's own site (hour angle anchored at the 128-s block start)
                        const uint32_t jb = j / BLOCK_STEPS * BLOCK_STEPS;
                        if (jb != ls_block) {
                            lane_anchor(ls, sun + (size_t)jb * SUN_W);
                            ls_block = jb;
                        }
                        flp = lane_flags(fl, lane_row<R>(ls, sun + (size_t)j * SUN_W, kp.module, row), row);
                    }
                    bool risky;
                    second_body<R>(kp, kp.pvf, row, flp, fs, covered, z, mtr, csi, pv, meter, res, risky);
                    if constexpr (sizeof(R) == 4) {
                        if (risky) {   // guard band of a PV discontinuity: the fp64 second (pv_fp64_tp)
                            FSamp<double> f64;
                            to_real(f64, ch.s);
                            double row64[ROW];
                            for (int i = 0; i < ROW; ++i) row64[i] = r64[i];
                            if (kp.sites) lane_row<double>(ls, sun + (size_t)j * SUN_W, kp.module, row64);
                            const double zz = RNG == TMH_RNG_INJECTED ? ndtri(z64) : noise_z<double>(wn);
                            double c64, p64, m64, r64s;
                            bool rk;
                            second_body<double>(kp, kp.pvf, row64, flp, f64, covered, zz, 0.0, c64, p64, m64, r64s, rk);
                            pv = (float)p64;
                            res = meter - pv;
                        }
                    }
                    ok = true;
                }
            }
        }
        if (live) emit<R, OUT_ANY | OUT_BRT>(tr, sv, lds_hist, (uint64_t)j * tr.ld + c, cov, csi, pv, meter, res, acc, ok);
    }
    if (live) {
        store_chain(st, c, ch);
        if constexpr (sizeof(R) == 4) {
            st.fn[0][c] = fnc;
            st.fn[1][c] = fnl;
        }
        if (sv.acc) {
            const uint32_t g = gid(kp.ids, c);
            const size_t an = kp.ids ? kp.ids_n : n;   // acc rows: the full batch
            sv.acc[g] += acc.pv;
            sv.acc[an + g] += acc.m;
            sv.acc[2 * an + g] += acc.r;
            sv.acc[3 * an + g] = fmax(sv.acc[3 * an + g], acc.max());
        }
    }
    if (sv.hist) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x)
            if (lds_hist[i]) atomicAdd((unsigned long long*)&sv.hist[i], (unsigned long long)lds_hist[i]);
    }
}

// ------------------------------------------------------------ P1: segments
// hour / day fractions of step s (clearskyindexmodel.py:114-116) from the window's
// local second-of-day at W0: 32-bit arithmetic, shift table in registers
struct WinClock {
    int32_t sod0;                 // local second of day at W0
    int32_t shifts;               // clock shifts inside or after the window (0: skip the table)
    int32_t step[8], delta[8];    // window-relative shift steps (INT_MAX = unused) and sizes
};

__device__ __forceinline__ WinClock win_clock(const tmh_clock& ck, int64_t W0)
{
    WinClock w;
    const int64_t l0 = local_at(ck, W0);
    w.sod0 = (int32_t)(l0 - floordiv(l0, 86400) * 86400);
    w.shifts = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const bool use = i < ck.n_shifts && ck.shift_step[i] > W0;
        w.step[i] = use ? (int32_t)(ck.shift_step[i] - W0) : INT_MAX;
        w.delta[i] = use ? ck.shift_delta[i] : 0;
        w.shifts += use ? 1 : 0;
    }
    return w;
}

// hour_f for every second of an hour (minute 60 + second): the walk's table in LDS
constexpr int HOUR_S = 3600;
__device__ __forceinline__ void hour_fractions(double* tab)
{
    for (int i = threadIdx.x; i < HOUR_S; i += blockDim.x) {
        double mf, hf, df;
        clock_fractions(0, i / 60, i % 60, mf, hf, df);   // hour_f depends on (minute, second) only
        tab[i] = hf;
    }
    __syncthreads();
}

// hour_f from the table (hf_tab, hour_fractions; TAB), day_f = div_exact(hour + hour_f, 24)
// as clock_fractions computes it: the same bits, without the minute / second split and
// the first two exact divisions per call.  Without TAB, clock_fractions itself.
template <bool TAB>
__device__ __forceinline__ void fractions_at(const WinClock& w, int32_t j, const double* hf_tab, double& hour_f,
                                             double& day_f)
{
    int32_t sod = w.sod0 + j;
    if (w.shifts) {   // wave-uniform: most windows (no DST change ahead) skip the shift table
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (j >= w.step[i]) sod += w.delta[i];
    }
    sod %= 86400;
    if (sod < 0) sod += 86400;
    if constexpr (TAB) {
        const int hour = sod / HOUR_S;
        hour_f = hf_tab[sod - HOUR_S * hour];
        day_f = div_exact(hour + hour_f, 24.0, 1.0 / 24.0);
    } else {
        double min_f;
        clock_fractions(sod / 3600, (sod / 60) % 60, sod % 60, min_f, hour_f, day_f);
    }
}

// Walk rows ordered by the chain's wind over the window, windiest first.  A chain's
// next_cloud calls per window grow with its wind speed (the cloud lengths are x / ws;
// correlation 0.84 between calls and the window-start wind pair's sum over 4,096 oracle
// chain-days), and a walk wavefront runs as many iterations as the busiest of its 4
// (16) chains: grouping chains of similar wind cuts the wavefronts' iterations by 11 %
// (17 % at 16 chains per wavefront), and the busiest wavefronts are dispatched first.
// Faulted chains last.  Bitonic sort of (key, chain) per tile of ORDER_TILE rows in LDS
// (walk_order_kernel), or for small batches a rank sort (walk_rank_kernel, the same permutation).
// The walk's results do not depend on the order (each group walks its own chain).  The
// try-0 candidate table is stored by walk row (draws_tail_kernel writes row rank[c]), so
// a wavefront's candidate loads stay on shared cache lines as in chain order (read by
// chain, the scattered rows made the 16-chain C3 walk 3.7x slower).
constexpr uint32_t ORDER_TILE = 4096;
constexpr uint32_t ORDER_EPB = 64;   // walk_rank_kernel: tile entries ranked per workgroup (4 waves: a quarter of the tile each)
constexpr uint32_t WALK_RANK_TILES = 4;   // up to this many tiles the rank sort (O(tile^2) compares per tile, 64 workgroups)
__global__ __launch_bounds__(1024) void walk_order_kernel(StateView st, uint32_t n, SegView sg, PrevView prev)
{
    __shared__ unsigned long long v[ORDER_TILE];
    const uint32_t t0 = blockIdx.x * ORDER_TILE;
    for (uint32_t i = threadIdx.x; i < ORDER_TILE; i += blockDim.x) {
        const uint32_t c = t0 + i;
        uint32_t kb = 0;   // positive floats order as their bit patterns; 0 = faulted or padding
        if (c < n) {
            const bool ok = (prev.status ? prev.status[c] : st.status[c]) == 0;
            const double w = prev.status ? prev.end_p1[2 * (size_t)n + c] + prev.end_p1[3 * (size_t)n + c]
                                         : st.sb[S_WS][c] + st.sa[S_WS][c];
            kb = ok && w > 0.0 ? __float_as_uint((float)w) : 0u;
        }
        // ascending order of the complement: larger key first, then the lower chain
        v[i] = ~(((unsigned long long)kb << 32) | (0xFFFFFFFFu - c));
    }
    __syncthreads();
    for (uint32_t k = 2; k <= ORDER_TILE; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < ORDER_TILE; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const unsigned long long a = v[i], b = v[l];
                    if (((i & k) == 0) ? a > b : a < b) {
                        v[i] = b;
                        v[l] = a;
                    }
                }
            }
            __syncthreads();
        }
    // the tile's real chains sort ahead of its padding (key 0, chain ids >= n)
    for (uint32_t i = threadIdx.x; i < ORDER_TILE && t0 + i < n; i += blockDim.x) {
        const uint32_t c = 0xFFFFFFFFu - (uint32_t)~v[i];
        sg.order[t0 + i] = c;
        sg.rank[c] = t0 + i;
    }
}

// Batches of at most WALK_RANK_TILES tiles (C2, C4): the same permutation by a rank sort.
__global__ __launch_bounds__(256) void walk_rank_kernel(StateView st, uint32_t n, SegView sg, PrevView prev)
{
    // round 6: a rank sort.  Every workgroup loads its tile's keys into LDS and ranks 64 of them
    // (each wave counts the smaller keys in a quarter of the tile, broadcast LDS reads); the
    // rank of a key among the tile's is its place in the ascending order, so the permutation is
    // the bitonic sort's of round 2 bit for bit (keys are unique: the chain id is in the low word),
    // in 64 workgroups per tile instead of one workgroup's 78 barrier stages (79 us per C2 batch).
    __shared__ unsigned long long v[ORDER_TILE];
    __shared__ uint32_t part[4][ORDER_EPB];
    constexpr uint32_t SUBS = ORDER_TILE / ORDER_EPB;
    const uint32_t t0 = (blockIdx.x / SUBS) * ORDER_TILE;
    const uint32_t m = min(ORDER_TILE, n - t0);   // the tile's chains (a partial last tile has no padding keys)
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) {
        const uint32_t c = t0 + i;
        const bool ok = (prev.status ? prev.status[c] : st.status[c]) == 0;
        const double w = prev.status ? prev.end_p1[2 * (size_t)n + c] + prev.end_p1[3 * (size_t)n + c]
                                     : st.sb[S_WS][c] + st.sa[S_WS][c];
        const uint32_t kb = ok && w > 0.0 ? __float_as_uint((float)w) : 0u;   // positive floats order as their bits
        // ascending order of the complement: larger key first, then the lower chain
        v[i] = ~(((unsigned long long)kb << 32) | (0xFFFFFFFFu - c));
    }
    __syncthreads();
    const uint32_t e = (blockIdx.x % SUBS) * ORDER_EPB + (threadIdx.x & (ORDER_EPB - 1));   // entry in the tile
    const uint32_t q = threadIdx.x / ORDER_EPB;                                               // quarter (wave)
    uint32_t cnt = 0;
    if (e < m) {
        const unsigned long long me = v[e];
        const uint32_t j1 = min((q + 1) * (ORDER_TILE / 4), m);
#pragma unroll 8
        for (uint32_t j = q * (ORDER_TILE / 4); j < j1; ++j) cnt += v[j] < me ? 1u : 0u;
    }
    part[q][threadIdx.x & (ORDER_EPB - 1)] = cnt;
    __syncthreads();
    if (q == 0 && e < m) {
        const uint32_t r = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
        const uint32_t c = t0 + e;
        sg.order[t0 + r] = c;
        sg.rank[c] = t0 + r;
    }
}

// ---- lane-group primitives (DPP inside groups of G = 4, 8 or 16 lanes: one chain per group)
// a double moved across lanes by DPP without an `old` operand: lanes whose source lies
// outside the row read 0 (bound_ctrl), so no register is initialised for them first
template <int CTRL>
__device__ __forceinline__ double mov_dpp_f64(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

template <int G>
__device__ __forceinline__ int grp_min_i32(int v);

template <int G>
__device__ __forceinline__ uint32_t grp_min_u32(uint32_t v)
{
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
    if constexpr (G >= 8) v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
    if constexpr (G >= 16) v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
    return v;
}

// np.argmin's first-index rule over the group's lanes (round 6): each lane holds its best
// distance d >= 0 (or +inf) and that entry's index k.  The high words of non-negative
// doubles order like the doubles, so the group minimum of the high words (32-bit DPP minima,
// one instruction a step) leaves the candidates that share it; the minimum of their low
// words leaves the lanes whose d equals the true minimum bit for bit, and the lowest k among
// those is the argmin.  Returns the index, or -1 when no lane has a finite d (no possible
// entry): the same result as an fp64 group minimum followed by the minimum index at it, with
// 32-bit reductions only.
template <int G>
__device__ __forceinline__ int grp_argmin_f64(double bd, int bk, uint32_t mh)
{
    const uint64_t bits = (uint64_t)__double_as_longlong(bd);
    const uint32_t hi = (uint32_t)(bits >> 32), lo = (uint32_t)bits;
    if (mh >= 0x7FF00000u) return -1;   // group-uniform: every lane +inf
    const bool cand = hi == mh;
    const uint32_t ml = grp_min_u32<G>(cand ? lo : 0xFFFFFFFFu);
    return grp_min_i32<G>(cand && lo == ml ? bk : INT_MAX);
}

template <int G>
__device__ __forceinline__ int grp_min_i32(int v)
{
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));
    if constexpr (G >= 8) v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));
    if constexpr (G >= 16) v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));
    return v;
}

// max over the wave of a group-uniform value (wave-uniform result, SGPR).  Every
// lane must be active: the DPP steps fold the groups of a row together first
// (row_half_mirror pairs the quads of a half row, row_mirror the halves).
template <int G>
__device__ __forceinline__ int wave_max_grp(int v)
{
    if constexpr (G <= 4) v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));
    if constexpr (G <= 8) v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}

__device__ __forceinline__ double bperm_f64(int src_lane, double v)
{
    const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

// Batch size up to which the automatic choice walks with 16 lanes per chain: up to 2
// waves per SIMD the walk is latency-bound (C2: 4,096 chains, 1,024 waves) and the
// short per-call chain of 16 lanes wins; past it the walk is throughput-bound and 4
// lanes per chain (37 % fewer instructions, 14 instead of 36 VGPRs per chain) win
// (r02, same box: C3 2.48 -> 2.69e11, C4 2.24 -> 2.36e11 chain-s/s).
constexpr uint32_t WALK_AUTO_SMALL = 8192;
constexpr int WALK_REG = 64;   // sigma entries held in VGPRs per chain (entries past them: the chain's global row)
// TP: the 8-lane walk of a throughput-bound batch (rows >= the engine's walk_tp_rows, 65,536 by
// default: C3's 1 M chains, 131,072 waves): 32 register entries and at least 4 waves per SIMD (128
// VGPRs, 27 spilled) instead of 64 entries at 180 VGPRs (2 waves).  Round 6, same box: C3 3.06
// against 2.96e11; a latency-bound batch (C4's 16,384 chains, 2 waves per SIMD) keeps the
// unspilled walk (the TP walk: C4 3.01 against 3.09e11).
// (a 4-lane TP walk, 16 entries at 3 or 4 waves per SIMD: C3 2.90 / 2.72e11, round 6)
// the 16-lane walk (latency-bound batches: C2, C5) -- A/B builds: its register entries and minimum
// waves per SIMD (its VGPRs decide how many expansion waves fit beside two walk waves)
#ifndef TMH_WALK16_REG
#define TMH_WALK16_REG WALK_REG
#endif
#ifndef TMH_WALK16_WAVES
#define TMH_WALK16_WAVES 1
#endif
template <int G, bool TP>
constexpr int walk_reg()
{
    return TP ? 32 : (G == 16 ? TMH_WALK16_REG : WALK_REG);
}
template <int G, bool TP>
constexpr int walk_waves()
{
    return TP ? 4 : (G == 16 ? TMH_WALK16_WAVES : 1);
}
constexpr int WALK_FIX = 16;   // entries scanned unconditionally (one chunk at G = 16); the rest only when some chain of the wave needs them
static_assert(WALK_FIX >= 12, "reset_sigma writes up to 11 entries into the unconditional chunks");
constexpr int WALK_CAND = 32;   // try-0 candidates per LDS refill of a chain (one exposed load per 32 calls)

// P1: segment walk.  64 / G chains per wavefront, one per group of G lanes
// (G = 16 / 8 / 4, tmh_set_walk_lanes); entry k of a chain's sigma arrays lives
// in register chunk k / G, lane k % G of its group (entries WALK_REG.. stay
// in the chain's global sigma row).  Each loop iteration is one
// CloudCoverBinary.next_cloud call (cloud_cover_binary.py:80-107) of every group
// that still has a call inside the window; the per-call scalar work (clock
// fractions, update_parameters, the two divisions) is shared by the G lanes of a
// chain, the argmin is a DPP group reduction with np.argmin's first-index rule,
// the r_[cl, nsc[:last+1]] shift is row_shr:1 plus row_shl:G-1 for the carry
// between chunks.  Smaller G: fewer lanes (and issue slots) per chain-call,
// more chunks per lane.  Output per chain: segment records (first uncovered
// step, next call step) and the window-end binary state.
#ifdef TMH_WALK_PROF
// Diagnostic build only (-DTMH_WALK_PROF, scripts/walk_prof.py): per-lane cycles of the
// walk loop's sections (s_memtime stamps) over the iterations the lane took part in, its
// iteration count and total, read back with tmh_debug_walk_prof.  The lanes of a wave's
// busiest group see every iteration.  Not compiled into the product library.
constexpr int WPROF_N = 6, WPROF_WAVES = 1 << 18;   // (threads)
__device__ unsigned long long g_walk_prof[WPROF_WAVES][WPROF_N + 2];
#define WPROF(i)                                                    \
    do {                                                            \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();           \
        wp[i] += t_ - wpt;                                          \
        wpt = t_;                                                   \
    } while (0)
#else
#define WPROF(i) \
    do {         \
    } while (0)
#endif

template <bool QUEUE, int G, bool TP = false>
__global__ __launch_bounds__(256, (walk_waves<G, TP>())) void segments_kernel(DrawParams dp, StateView st, uint64_t chain0, uint32_t n,
                                                          int64_t W0, uint32_t nsteps, tmh_clock ck,
                                                          const int2* __restrict__ events,
                                                          const uint32_t* __restrict__ n_events, SegView sg,
                                                          PrevView prev)
{
    static_assert(G == 4 || G == 8 || G == 16, "lanes per chain");
#ifdef TMH_WALK_SETPRIO
    __builtin_amdgcn_s_setprio(TMH_WALK_SETPRIO);   // A/B builds: the walk's waves issue first on their SIMD
#endif
    constexpr int NCH = walk_reg<G, TP>() / G;                     // register chunks
    constexpr int NFIX = (WALK_FIX + G - 1) / G < NCH ? (WALK_FIX + G - 1) / G : NCH;
    static_assert(NCH * G == walk_reg<G, TP>() && NCH * G >= 12, "register entries: a multiple of G, >= 12 (reset_sigma)");
    constexpr int GSH = G == 4 ? 2 : G == 8 ? 3 : 4;
    constexpr int CARRY = 0x100 | (G - 1);                        // row_shl:G-1: group lane 0 <- group lane G-1
    extern __shared__ double walk_lds[];                           // [groups of the workgroup][WALK_CAND]
    const int lane = threadIdx.x & 63, p = lane & (G - 1), row0 = lane & ~(G - 1);
    double* const cbuf = walk_lds + (threadIdx.x >> GSH) * WALK_CAND;
    const int64_t W1 = W0 + nsteps;
    const uint32_t nev = min(*n_events, ev_cap_dev(nsteps));
    const WinClock wck = win_clock(ck, W0);
    // the calls' hour fractions by table (28.8 KB of LDS) in the 16-lane walk, whose 256-thread
    // workgroups are one per CU or two; the 4- and 8-lane walks run one-wave workgroups, many
    // per CU (C3: 262,144 waves), where the table's LDS would cap the waves per CU (walk
    // 62 -> 114 ms per 1 M-chain day): they compute the fractions
    constexpr bool HTAB = G == 16;
    __shared__ double hf_tab[HTAB ? HOUR_S : 1];
    if constexpr (HTAB) hour_fractions(hf_tab);
    // Groups take chains: group r starts with chain r, and a group whose chain is done
    // takes the next unstarted one from the window's queue (chains groups.. n - 1), so
    // with fewer groups than chains the walk's waves stay busy instead of idling
    // behind the windiest chain of their wave (its duration is the longest chain's
    // call count either way; its footprint on the CUs shrinks).  Everything below
    // is the group's current chain, group-uniform.
    const uint32_t* order = sg.order;   // walk row -> chain (walk_order_kernel), or the identity
    uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> GSH;   // the group's walk row
    bool live = r < n;
    uint32_t c = live && order ? order[r] : r;
    uint32_t status = 0xFFFFFFFFu;
    double ccb = 0.0, cca = 0.0, wsb = 0.0, wsa = 0.0;   // window-start cloud-cover and wind pairs
    int32_t fault = INT_MAX;
    uint32_t nrec = 0;
    double cl = 0.0, clr = 0.0;
    int L = 0;
    double* gsc = nullptr;
    double* gsl = nullptr;
    double vc[NCH], vl[NCH];
    int64_t s_start = 0, e = 0;
    // No global load or store sits on the per-call path: records and boundary
    // events move through G-entry lane-distributed buffers (lane p of a group =
    // entry p), flushed / refilled once per G uses and read back with
    // ds_bpermute; the try-0 candidates through the group's LDS slots, refilled
    // once per WALK_CAND calls from registers loaded one refill ahead.  (A per-call
    // load behind a per-call store makes every call wait for the store's round
    // trip: vmcnt counts both.)
    int2* rec = nullptr;
    int rb_x = 0, rb_y = 0;       // record buffer: lane p = record rbase + p
    uint32_t rbase = 0;
    int32_t chunk = 0;            // the overflow chunk of records >= cap (group-uniform)
    auto group_at = [&](uint32_t b) {   // where the record group starting at b goes
        return b < sg.cap ? rec + b : sg.pool + (size_t)chunk * OVF_CHUNK + (b - sg.cap) % OVF_CHUNK;
    };
    auto put_rec = [&](uint32_t i, int x, int y) {
        const uint32_t slot = i - rbase;
        const bool mine = (uint32_t)p == slot;
        rb_x = mine ? x : rb_x;
        rb_y = mine ? y : rb_y;
        if (slot == G - 1) {
            group_at(rbase)[p] = make_int2(rb_x, rb_y);
            rbase += G;
        }
    };
    uint32_t ev = 0, evb = 0;
    int eb_step = INT_MAX, eb_fl = 0;   // event buffer: lane p = event evb + p
    double eb_cc = 0.0, eb_ws = 0.0;
    auto load_events = [&]() {
        const uint32_t i = evb + p;
        eb_step = INT_MAX;
        if (i < nev) {
            const int2 r = events[i];
            eb_step = r.x;
            eb_fl = r.y;
            eb_cc = sg.evd[(size_t)i * 4 * n + c];
            eb_ws = sg.evd[((size_t)i * 4 + 1) * n + c];
        }
    };
    int64_t next_ev = INT64_MAX;
    int ev_fl = 0;
    double ev_cc = 0.0, ev_ws = 0.0;
    auto fetch_event = [&]() {   // event `ev` out of the buffer
        if (ev - evb >= G) {
            evb = ev;
            load_events();
        }
        const int src = row0 | (int)(ev - evb);
        const int es = __builtin_amdgcn_ds_bpermute(src << 2, eb_step);
        next_ev = es == INT_MAX ? INT64_MAX : (int64_t)es;
        ev_fl = __builtin_amdgcn_ds_bpermute(src << 2, eb_fl);
        ev_cc = bperm_f64(src, eb_cc);
        ev_ws = bperm_f64(src, eb_ws);
    };
    uint32_t ncall0 = 0, ncall = 0;
    // call ncall0 + k's try-0 length: the table, or past it (the windiest chains) drawn here,
    // one per lane of the group per refill, as draws_tail_kernel would have
    auto cand_at = [&](uint32_t k) {
        if (k < sg.kcap) return sg.cand[(size_t)k * n + r];   // stored by walk row
        const U4 b = keyed_block(dp.seed, chain0 + gid(dp.ids, c), (uint64_t)(ncall0 + k), TAG_CLOUD, 0);
        return pow_d(dp.alpha + dp.delta * u52(b.x, b.y), dp.expo);
    };
    uint32_t kb = 0;                                     // cbuf holds the try-0 lengths of calls kb .. kb + WALK_CAND - 1
    double cn[WALK_CAND / G];                            // lane p: calls kb + WALK_CAND + j G + p (the next refill)
    auto cand_fill = [&]() {   // cn -> cbuf, then load the refill after it
#pragma unroll
        for (int j = 0; j < WALK_CAND / G; ++j) cbuf[j * G + p] = cn[j];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < WALK_CAND / G; ++j) cn[j] = cand_at(kb + 2 * WALK_CAND + j * G + p);
    };
    bool active = false;
    auto start_chain = [&]() {   // the group's chain c (< n) at the window start
        const uint32_t cs = c;
        status = prev.status ? prev.status[cs] : st.status[cs];
        if (prev.status) {
            ccb = prev.end_p1[cs];
            cca = prev.end_p1[(size_t)n + cs];
            wsb = prev.end_p1[2 * (size_t)n + cs];
            wsa = prev.end_p1[3 * (size_t)n + cs];
        } else {
            ccb = st.sb[S_CC][cs];
            cca = st.sa[S_CC][cs];
            wsb = st.sb[S_WS][cs];
            wsa = st.sa[S_WS][cs];
        }
        fault = INT_MAX;
        cl = st.cl[cs];
        clr = st.clr[cs];
        L = st.L[cs];
        const int32_t sec0 = st.sec[cs];
        gsc = sig_c(st, cs);
        gsl = sig_l(st, cs);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int k = ch * G + p;
            vc[ch] = k < L ? gsc[k] : 0.0;
            vl[ch] = k < L ? gsl[k] : 0.0;
        }
        s_start = W0 - sec0;   // step at which sec was 1
        e = s_start + ceil_thr(cl + clr) - 1;
        rec = sg.rec + (size_t)cs * sg.cap;
        rb_x = rb_y = 0;
        rbase = 0;
        chunk = 0;
        put_rec(0, (int)(s_start + ceil_thr(cl) - 1), (int)e);
        nrec = 1;
        ev = evb = 0;
        load_events();
        fetch_event();
        ncall0 = ncall = st.ncalls[cs];
#pragma unroll
        for (int j = 0; j < WALK_CAND / G; ++j) cn[j] = cand_at(j * G + p);
        kb = -(uint32_t)WALK_CAND;   // cand_fill: cbuf <- calls 0.., cn <- calls WALK_CAND..
        cand_fill();
        kb = 0;
        active = status == 0;
    };
    auto finish_chain = [&]() {   // the group's chain at the window end: records, state, walk outputs
        if ((uint32_t)p < nrec - rbase) group_at(rbase)[p] = make_int2(rb_x, rb_y);   // partial record group
        if (status == 0) {
            while (next_ev <= W1 - 1) {   // remaining boundaries of the window
                if (ev_fl & FL_DAY) {
                    wsb = wsa;
                    wsa = ev_ws;
                }
                if (ev_fl & FL_HOUR) {
                    ccb = cca;
                    cca = ev_cc;
                }
                ++ev;
                fetch_event();
            }
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {   // register chunks back to the state row
                const int k = ch * G + p;
                if (k < L) {
                    gsc[k] = vc[ch];
                    gsl[k] = vl[ch];
                }
            }
            if (p == 0) {
                st.sec[c] = (int32_t)(W1 - s_start);   // sec after step W1 - 1
                st.cl[c] = cl;
                st.clr[c] = clr;
                st.L[c] = L;
                st.ncalls[c] = ncall;
            }
        }
        if (p == 0) {
            sg.count[c] = nrec;
            if (nrec <= sg.cap) sg.ovf_first[c] = INT_MAX;   // never reached the pool
            sg.fault[c] = fault;
            sg.status[c] = status;
            sg.end_p1[c] = ccb;
            sg.end_p1[(size_t)n + c] = cca;
            sg.end_p1[2 * (size_t)n + c] = wsb;
            sg.end_p1[3 * (size_t)n + c] = wsa;
        }
    };
    const uint32_t groups = gridDim.x * blockDim.x / G;
    if (live) start_chain();
#ifdef TMH_WALK_PROF
    uint64_t wp[WPROF_N] = {0, 0, 0, 0, 0, 0}, wpt = __builtin_amdgcn_s_memtime(), wit = 0;
    const uint64_t wt0 = wpt;
#endif
    for (;;) {
        if constexpr (QUEUE) {
            while (live && !(active && e < W1)) {   // group-uniform: the group's chain is done, take the next one
                finish_chain();
                int v = 0;
                if (p == 0) v = (int)atomicAdd(sg.walk_q, 1u);
                r = groups + (uint32_t)__builtin_amdgcn_ds_bpermute(row0 << 2, v);   // the whole group is active here
                live = r < n;
                c = live && order ? order[r] : r;
                if (live) start_chain();
            }
        }
        const bool run = active && e < W1;
        if (__builtin_amdgcn_ballot_w64(run) == 0) break;
        // wave-uniform bound on the sigma lengths: the gated chunk loops branch on SGPRs only.
        // Every chunk an array of the wave reaches (and, for the shift, the one past it:
        // (last + 1) / G <= L / G) is processed; a reset (L <= 11) stays in the NFIX chunks.
        const int Lmax = wave_max_grp<G>(run ? L : 0);
        WPROF(0);
        if (!run) continue;
#ifdef TMH_WALK_PROF
        ++wit;
#endif
        while (next_ev <= e) {   // _next_day / _next_hour at steps <= e
            if (ev_fl & FL_DAY) {
                wsb = wsa;
                wsa = ev_ws;
            }
            if (ev_fl & FL_HOUR) {
                ccb = cca;
                cca = ev_cc;
            }
            ++ev;
            fetch_event();
        }
        double hf, df;
        fractions_at<HTAB>(wck, (int32_t)(e - W0), hf_tab, hf, df);
        const double hh = interp(ccb, cca, hf);
        const double h = 0.95 < hh ? 0.95 : hh;   // update_parameters
        const double ws = interp(wsb, wsa, df);
        // f = 1 / h - 1: in faithful mode the hourly cover sits above 0.95 in ~98 % of the hours
        // (cloud_cover_hourly.py's bin-5 draw), so h = 0.95 and f is the constant F95 (the same
        // division, rounded at compile time); the fp64 division runs only when some chain of the
        // wave is below the cap (round 6: one division off the walk's latency chain)
        constexpr double F95 = 1.0 / 0.95 - 1.0;
        const double f = __builtin_amdgcn_ballot_w64(!(hh >= 0.95)) == 0 ? F95 : 1.0 / h - 1.0;
        const uint32_t rel = ncall - ncall0;
        if (rel - kb >= WALK_CAND) {   // refill once per WALK_CAND calls (loaded one refill ahead)
            cand_fill();
            kb += WALK_CAND;
        }
        const double x0 = cbuf[rel - kb];
        WPROF(1);
        // ---- next_cloud: tries (cloud_cover_binary.py:82-98).  Try 0 (its length from the
        // candidate table) is straight-line code; the retries (8 % of the calls: tries 1..39,
        // reset_sigma before try 20, the AssertionError after try 39) loop only for the groups
        // whose try 0 found no possible entry.
        int tries = 0, last = -1;
        double ncl = 0.0, bdl = 0.0, bd = INFINITY;
        int bk = INT_MAX;
        auto attempt = [&](double x) __attribute__((always_inline)) {   // one try: scan + group minimum
            ncl = x / ws;
            bd = INFINITY;
            bk = INT_MAX;
            auto scan = [&](int k, double sc, double sl) {   // :83-88, branch-free
                const double nsc = ncl + sc;
                const double nsl = f * nsc;
                const double tot = nsc + nsl;
                const double dl = nsl - sl;   // the new clear length if k is picked (:103)
                const bool ok = (k < L) & (dl > 0.0) & (tot < 5400.0);
                const double d = fabs(tot - 3600.0);
                const bool take = ok & (d < bd);   // ascending k: ties keep the lower k (bd starts at +inf)
                bd = take ? d : bd;
                bk = take ? k : bk;
                bdl = take ? dl : bdl;
            };
#pragma unroll
            for (int ch = 0; ch < NFIX; ++ch) scan(ch * G + p, vc[ch], vl[ch]);
#pragma unroll
            for (int ch = NFIX; ch < NCH; ++ch)
                if (Lmax > G * ch) scan(ch * G + p, vc[ch], vl[ch]);   // wave-uniform
            for (int k0 = NCH * G; k0 < L; k0 += G) {   // rare: entries WALK_REG..
                const int k = k0 + p;
                if (k < L) scan(k, gsc[k], gsl[k]);
            }
            // the group's minimum high word of the distances (grp_argmin_f64); >= +inf's: no entry possible
            return grp_min_u32<G>((uint32_t)((uint64_t)__double_as_longlong(bd) >> 32));
        };
        auto draw = [&](int t) {   // try t's cloud length, keyed by (chain, call number, try)
            return pow_d(dp.alpha + dp.delta * keyed_u(dp.seed, chain0 + gid(dp.ids, c), ncall, TAG_CLOUD,
                                                       (uint32_t)(t >> 1), t & 1),
                         dp.expo);
        };
        uint32_t mh = attempt(x0 >= 0.0 ? x0 : draw(0));
        if (mh >= 0x7FF00000u) {   // group-uniform: no possible entry
            for (;;) {
                ++tries;
                if (tries == 20) {   // reset_sigma (cloud_cover_binary.py:76-78); 300 (k+1) is exact
                    const int nl = (int)(h * 12);
#pragma unroll
                    for (int ch = 0; ch * G < 12; ++ch) {
                        vc[ch] = 300.0 * (ch * G + p + 1);
                        vl[ch] = f * vc[ch];
                    }
                    L = nl;
                }
                if (tries == 40) break;
                mh = attempt(draw(tries));
                if (mh < 0x7FF00000u) break;
            }
        }
        last = grp_argmin_f64<G>(bd, bk, mh);
        ++ncall;
        WPROF(2);
        if (last < 0) {   // assert not recurse (:91)
            status = TMH_CHAIN_ASSERT_BINARY;
            fault = (int32_t)(e - W0);
            active = false;
            continue;
        }
        if (last + 2 > CAP) {
            status = TMH_CHAIN_SIGMA_OVERFLOW;
            fault = (int32_t)(e - W0);
            active = false;
            continue;
        }
        // sigma_cloud = r_[cl, nsc[:last+1]], sigma_clear = r_[clr, nsl[:last+1]] (:101-105);
        // clr = nsl[last] - sigma_clear[last] is the scan's dl of entry `last`, held by
        // the lane that owns it (its best is `last`)
        const double nclr = bperm_f64(row0 | (last & (G - 1)), bdl);
        const int top = (last + 1) / G;   // highest chunk written
        // entry G NCH - 1 (register chunk NCH - 1, group lane G - 1) for lane 0 of the first
        // global chunk: the DPP runs with the whole group active
        const double carry_g = mov_dpp_f64<CARRY>(vc[NCH - 1]);
        for (int ch = top; ch >= NCH; --ch) {   // rare, descending: reads before writes
            const int k = ch * G + p;
            const double prv = (ch == NCH && p == 0) ? carry_g : gsc[k - 1];
            const double nsc = ncl + prv;
            gsc[k] = nsc;
            gsl[k] = f * nsc;
        }
        // chunks a longer array of the wave needs are rewritten for every group: entries >= the new L, harmless
#pragma unroll
        for (int ch = NCH - 1; ch >= 0; --ch) {
            if (ch < NFIX || Lmax >= G * ch) {   // wave-uniform
                const double sh = mov_dpp_f64<0x111>(vc[ch]);                               // row_shr:1
                const double carry = ch > 0 ? mov_dpp_f64<CARRY>(vc[ch > 0 ? ch - 1 : 0]) : 0.0;   // row_shl:G-1
                const double prv = p == 0 ? carry : sh;
                const double nsc = ncl + prv;
                const bool first = ch == 0 && p == 0;
                vc[ch] = first ? ncl : nsc;
                vl[ch] = first ? nclr : f * nsc;
            }
        }
        WPROF(3);
        L = last + 2;
        cl = ncl;
        clr = nclr;
        s_start = e;
        e = s_start + ceil_thr(cl + clr) - 1;
        if (nrec >= sg.cap && (nrec - sg.cap) % OVF_CHUNK == 0) {   // a new overflow chunk (windy tail)
            const uint32_t k = (nrec - sg.cap) / OVF_CHUNK;
            if (k == 0 && p == 0) sg.ovf_first[c] = (int32_t)(s_start - W0);   // record `cap`: this call's
            int got = -1;
            if (k < OVF_SLOTS) {
                int v = 0;
                if (p == 0) v = (int)atomicAdd(sg.pool_n, 1u);
                got = __builtin_amdgcn_ds_bpermute(row0 << 2, v);   // the whole group is active here
                if ((uint32_t)got >= sg.pool_cap) {
                    got = -1;
                    if (p == 0) atomicOr(sg.pool_short, 1u);   // the batch's demand exceeds the pool
                } else if (p == 0) sg.ovf[(size_t)c * OVF_SLOTS + k] = got;
            }
            if (got < 0) {
                status = TMH_CHAIN_SEGMENT_OVERFLOW;
                fault = (int32_t)(s_start - W0);
                active = false;
                continue;
            }
            chunk = got;
        }
        put_rec(nrec, (int)(s_start + ceil_thr(cl) - 1), (int)e);
        ++nrec;
        WPROF(4);
    }
#ifdef TMH_WALK_PROF
    {
        const uint32_t wave = blockIdx.x * blockDim.x + threadIdx.x;
        if (wave < (uint32_t)WPROF_WAVES) {
            for (int i = 0; i < WPROF_N; ++i) g_walk_prof[wave][i] = wp[i];
            g_walk_prof[wave][WPROF_N] = wit;
            g_walk_prof[wave][WPROF_N + 1] = __builtin_amdgcn_s_memtime() - wt0;
        }
    }
#endif
    if constexpr (!QUEUE)   // one chain per group
        if (live) finish_chain();
}

// The pool ran short (overflow_settle, SegView): every chain that reached it faults
// at its first record past the row, so which chains fault does not depend on the
// order in which the walk's waves claimed chunks.  The chain's records below the
// row cover every step before that fault; count is cut to them.
__global__ __launch_bounds__(256) void overflow_settle_kernel(uint32_t n, SegView sg)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n || *sg.pool_short == 0) return;
    const int32_t f = sg.ovf_first[c];
    if (f == INT_MAX) return;
    sg.status[c] = TMH_CHAIN_SEGMENT_OVERFLOW;
    sg.fault[c] = f;
    sg.count[c] = min(sg.count[c], sg.cap);
}

// The record holding each block's start, for the expansion's tiles (a tile reads one
// coalesced word instead of a binary search of ~9 dependent, lane-scattered record loads
// at its start): the first record whose next-call step lies past the block start, or the
// chain's last record (expand_tile's rule).  One work-item per (chain, BREC_G blocks): a
// binary search for the first block, then a forward scan, the records' next-call steps
// being nondecreasing.  After the walk, on its stream (so the expansion's wait for the walk
// includes it): 32 blocks per work-item took 122 us per C2 batch, a latency chain of ~60
// dependent loads; 8 blocks, ~23.
constexpr uint32_t BREC_G = 8;
__global__ __launch_bounds__(256) void block_rec_kernel(uint32_t n, int64_t W0, SegView sg)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint32_t b0 = blockIdx.y * BREC_G, b1 = min(b0 + BREC_G, sg.nblk);
    const int last = (int)sg.count[c] - 1;
    const int32_t s00 = (int32_t)(W0 + (int64_t)b0 * BLOCK_STEPS);
    int lo = 0, hi = last;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rec_at(sg, c, mid).y > s00) hi = mid;
        else lo = mid + 1;
    }
    int32_t y = lo < last ? rec_at(sg, c, lo).y : 0;
    for (uint32_t b = b0; b < b1; ++b) {
        const int32_t s0 = (int32_t)(W0 + (int64_t)b * BLOCK_STEPS);
        while (lo < last && y <= s0) y = rec_at(sg, c, ++lo).y;
        sg.brec[(size_t)b * n + c] = (uint32_t)lo;
    }
}

// ------------------------------------------------------------ P2: expand
// one trace store: a buffer resource on a wave-uniform base (SGPRs) plus the lane's
// 32-bit byte offset, non-temporal (the trace is written once); no per-lane 64-bit
// address arithmetic.  0x00020000: gfx9 raw-buffer dword 3.  Offsets past
// num_records are dropped by the range check (lanes past the last chain)
// a non-temporal trace store at lane byte offset `off` (range-checked) plus the row's
// wave-uniform offset `soff` (the store's scalar offset)
template <typename R>
__device__ __forceinline__ void row_store(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t soff, R v)
{
    if constexpr (sizeof(R) == 8)
    {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const uint64_t u = (uint64_t)__double_as_longlong(v);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)u, (uint32_t)(u >> 32)}, rs, (int)off, (int)soff, 2 /* nt */);
    }
    else
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)off, (int)soff, 2 /* nt */);
}

// One work-item per (chain, block of 128 seconds).  The boundary draws come
// from the draw tables, so the per-second loop holds only the R copies of the
// sampler pairs and does no fp64 work in fp32 mode.
// 256-thread workgroups: one-wave workgroups (so the SIMDs take expansion waves
// independently of a walk wave's footprint) measured +5 % alone, no gain beside the walks
// statistics workgroups of 512 chains (C3 / C4): one histogram flush per 65,536
// chain-seconds instead of 32,768 (32-bit LDS bins, 16 KB); round 4, same box: C4
// 2.41 -> 2.51e11 chain-s/s, C3 2.87e11 either way (its expansion 240 -> 235 ms alone)
#ifndef TMH_EXP_WG_STATS
#define TMH_EXP_WG_STATS 512
#endif
#ifndef TMH_HELD_OR
#define TMH_HELD_OR 0   // fp32 expansion: the guard-band bit as an unconditional LDS or (A/B builds; DESIGN round 6)
#endif
#ifndef TMH_DISC_LDS
#define TMH_DISC_LDS 0   // fp32 single-site expansion: DISC's coefficient sets from an LDS table (disc_row; A/B builds)
#endif
#ifndef TMH_ROW_LDS
#define TMH_ROW_LDS 0   // fp32 single-site expansion: the tile's geometry rows staged in LDS (A/B builds)
#endif
#ifndef TMH_ROW_LDS_WAVES
#define TMH_ROW_LDS_WAVES 6
#endif
// expand_kernel's tile order: 0 launch order, 1 / 2 XCD-aware (below).  Order 1 for the
// per-site kernels (C5: 4.20 against 3.995e10 live chain-s/s, same box), launch order for
// the rest (C2: order 1 2.17 against 2.39e11); TMH_EXP_TILE_ORDER sets one order for every
// instantiation (A/B builds).
template <typename R, int OUT, bool SITES>
constexpr int exp_tile_order()
{
#ifdef TMH_EXP_TILE_ORDER
    return TMH_EXP_TILE_ORDER;
#else
    return SITES ? 1 : 0;
#endif
}
template <typename R, int OUT, bool SITES>
constexpr int exp_wg()
{
    return out_base(OUT) == OUT_STATS && !SITES ? TMH_EXP_WG_STATS : 256;
}
// the LDS histogram as 16-bit bin pairs when one tile (WG chains x 128 s) cannot fill a
// 16-bit bin, else one 32-bit word per bin
// time blocks per workgroup: the statistics-only single-site expansion (C3, C4) may loop over
// TMH_STATS_TPW consecutive blocks, one histogram flush for all of them (A/B builds)
#ifndef TMH_STATS_TPW
#define TMH_STATS_TPW 1
#endif
template <typename R, int OUT, bool SITES>
constexpr int exp_tpw()
{
    return out_base(OUT) == OUT_STATS && !SITES ? TMH_STATS_TPW : 1;
}
template <typename R, int OUT, bool SITES>
constexpr bool exp_hist_pack()
{
    return exp_wg<R, OUT, SITES>() * BLOCK_STEPS * exp_tpw<R, OUT, SITES>() <= 32768;
}
#ifndef TMH_PVF_VGPR
#define TMH_PVF_VGPR 0
#endif
constexpr int PVF_VGPR = TMH_PVF_VGPR;   // leading PVF fields pinned in VGPRs in the fp32 single-site expansion
#ifndef TMH_EXP_WAVES_TRACE
#define TMH_EXP_WAVES_TRACE 7
#endif
// min waves per SIMD (__launch_bounds__) of each expansion instantiation:
//  fp32 single-site trace (C2): 7 = at most 72 VGPRs (alone -4 % vs 6, no VGPR spills);
//  fp32 statistics / other outputs (C3, C4): 6 = 80 VGPRs (the 16-bit-pair LDS histogram,
//    8 KB, + 12 KB staging: 8 workgroups per CU; +6 % over 5 waves);
//  fp64 single-site: 4 = at most 128 VGPRs (the trace kernel takes 110, no VGPR spills since the
//    round-4 PV-constant and table changes; 5 waves = 96 VGPRs spill 14 and run 6 % slower, round 5);
//  per-chain sites (C5): 3 = at most 168 VGPRs (12-18 spilled): C5 5.36 against 4.47e10 at 2 (206 VGPRs,
//    round 6, same box) and 4.37e10 at 4 (79 spilled); 2 was 35 % faster than 1 (round 2)
template <typename R, int OUT, bool SITES>
constexpr int exp_waves()
{
#ifndef TMH_EXP_WAVES_F64
#define TMH_EXP_WAVES_F64 4
#endif
#ifndef TMH_EXP_WAVES_STATS
#define TMH_EXP_WAVES_STATS 6
#endif
#ifndef TMH_EXP_WAVES_SITES
#define TMH_EXP_WAVES_SITES 3
#endif
    return SITES ? TMH_EXP_WAVES_SITES : (sizeof(R) == 8 ? TMH_EXP_WAVES_F64 : (out_base(OUT) == OUT_TRACE3 ? (TMH_ROW_LDS ? TMH_ROW_LDS_WAVES : TMH_EXP_WAVES_TRACE) : TMH_EXP_WAVES_STATS));
}
// One (128-second block b, chain block cblk) tile of the expansion: one work-item per
// chain of the block (the expansion's unit of work, below).  The LDS staging areas are
// the kernel's (one column per thread, so consecutive tiles need no barrier between them).
template <typename R, int OUT, bool SITES, int WGT>
__device__ __forceinline__ void expand_tile(uint32_t b, uint32_t cblk, const KParams& kp, const DrawParams& dp,
                                            const StateView& st, uint64_t chain0, uint32_t n, int64_t W0,
                                            uint32_t nsteps, int64_t utc0, const double* __restrict__ tab64,
                                            const float* __restrict__ tab32, const double* __restrict__ sun,
                                            const int2* __restrict__ events, const uint32_t* __restrict__ n_events,
                                            const BlockDesc* __restrict__ desc, const SegView& sg,
                                            const TraceView& tr, const StatsView& sv, uint32_t* lds_hist,
                                            uint32_t (*cov_lds)[WGT], R (*min_lds)[WGT], uint4* held_lds,
                                            const PV64* pv_lds, const double* pv_lds_tab, float* row_lds,
                                            const float4* nd_lds)
{
    // TMH_ROW_LDS: the tile's fp32 geometry rows copied to LDS once (coalesced vector loads),
    // read back per second with broadcast ds_reads instead of per-second scalar loads
    constexpr bool ROWL = TMH_ROW_LDS && sizeof(R) == 4 && !SITES;
    // fp32: DISC's coefficient sets from the LDS table after the quantile's (the single-site
    // second bodies; TMH_DISC_LDS=0 builds the constant-coefficient branches instead, for A/B)
    const float4* disc_lds = sizeof(R) == 4 && TMH_DISC_LDS ? nd_lds + ND32_N : nullptr;
    const uint32_t c = cblk * blockDim.x + threadIdx.x;
    const bool live = c < n;
    const uint32_t j0 = b * BLOCK_STEPS, j1 = min(j0 + (uint32_t)BLOCK_STEPS, nsteps);
    const uint64_t chain = chain0 + gid(kp.ids, c);
    const int64_t fm = first_minute(utc0, W0);
    // the fp32 PV constants as per-lane registers (VGPRs): held in SGPRs across
    // the loop they are spilled to VGPR lanes and read back by v_readlane each step
    PVF pkv = kp.pvf;
    if constexpr (sizeof(R) == 4 && !SITES) {
        float* f = reinterpret_cast<float*>(&pkv);
#pragma unroll
        for (int i = 0; i < PVF_VGPR; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(f[i]) : "s"(f[i]));
    }
    Acc acc{0.0, 0.0, 0.0, -INFINITY};
    bool alive = false;
    int32_t fault = INT_MAX;
    uint32_t jr = 0, evi = 0;
    FSamp<R> fs;
    const MinuteCtx mc{dp, chain, W0, fm, events, (int)min(*n_events, ev_cap_dev(nsteps)), tab64};
    LaneSite ls{};   // per-chain sites (C5): this chain's site constants
    bool blk_night = false;
    if constexpr (SITES) {
        static_assert(BLOCK_STEPS <= 128, "site_block_night's bound assumes blocks of <= 128 s");
        ls.k = site_k(kp.sites + (size_t)(live ? gid(kp.ids, c) : 0) * 8);
        ls.linke = kp.site_linke ? kp.site_linke + (size_t)(live ? gid(kp.ids, c) : 0) * 12 : nullptr;
        ls.tl_doy = -1;
        blk_night = site_block_night(ls.k, sun + (size_t)(b * BLOCK_STEPS) * SUN_W);
        if (!blk_night) lane_anchor(ls, sun + (size_t)(b * BLOCK_STEPS) * SUN_W);
    }
    if (live) {
        alive = st.status[c] == 0;
        fault = sg.fault[c];
        Samp s;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            s.b[k] = st.sb[k][c];
            s.a[k] = st.sa[k][c];
        }
        if constexpr (sizeof(R) == 4) load_fast_noise(st, c, s);
        const BlockDesc d = desc[b];
        evi = (uint32_t)d.evi;
        if (alive && b > 0) samplers_at<R>(d, sg, n, c, s, mc, st);
        to_real(fs, s);
    }
    // The block's covered bits and its minute draws staged in LDS before the loop:
    // the per-second loop then issues no vector loads, so no s_waitcnt vmcnt in it
    // waits behind the trace stores (gfx9's vmcnt counts loads and stores alike;
    // per-second record loads cost 42 % of the waves' cycles in such waits, PMC
    // SQ_WAIT_ANY).  Word-major: lane-consecutive dwords, no bank conflicts.
    const int32_t s0i = (int32_t)(W0 + j0), s1i = (int32_t)(W0 + j1);
    const int32_t mA = (int32_t)j0 <= (int32_t)fm ? 0 : ((int32_t)j0 - (int32_t)fm + 59) / 60;
    {
        uint32_t cw[4] = {0u, 0u, 0u, 0u};
        if (alive) {   // segment containing the block start: first record with next-call step > start
            int lo = (int)sg.brec[(size_t)b * n + c];   // block_rec_kernel
            const int last = (int)sg.count[c] - 1;
            // covered iff step < x of the segment holding it: [start, min(x, y)) per segment
            int2 r = rec_at(sg, c, lo);
            int32_t a = s0i;
            for (;;) {
                const int32_t e = min(min(r.x, r.y), s1i);
                if (e > a) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const int32_t wl = max(a - s0i - 32 * w, 0), wh = min(e - s0i - 32 * w, 32);
                        if (wh > wl) cw[w] |= (wh - wl == 32 ? ~0u : ((1u << (wh - wl)) - 1u)) << wl;
                    }
                }
                if (r.y >= s1i || lo >= last) break;
                a = max(a, r.y);
                r = rec_at(sg, c, ++lo);
            }
            jr = (uint32_t)lo;   // the segment of the block's last step (fixup_kernel walks back from it)
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) cov_lds[w][threadIdx.x] = cw[w];
        const R* mt = reinterpret_cast<const R*>(sg.mtab);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int32_t m = mA + k;
            const bool in = live && (int32_t)fm + 60 * m < (int32_t)j1;
            min_lds[2 * k][threadIdx.x] = in ? mt[(size_t)(2 * m) * n + c] : R(0);
            min_lds[2 * k + 1][threadIdx.x] = in ? mt[(size_t)(2 * m + 1) * n + c] : R(0);
        }
    }
    uint32_t cov_w = 0;
    const double* evd = sg.evd + c;
    // the guard-band seconds of the lane's block, a bit each, in LDS: no register carried through the loop
    held_lds[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
    // Trace stores: one buffer resource per output for the block's rows (built here,
    // not per store) and one running per-lane byte offset; lanes past the last chain
    // start at 2^31, out of the resource's range, so the stores need no exec mask.
    // (The host keeps a block's rows under 2 GiB: tmh_expand checks the trace's ld.)
    constexpr int RW = sizeof(R) == 8 ? ROW : ROW32;   // geometry row: wave-uniform, scalar loads
    const R* rowp = (sizeof(R) == 8 ? reinterpret_cast<const R*>(tab64) : reinterpret_cast<const R*>(tab32)) +
                    (size_t)j0 * RW;
    if constexpr (ROWL) {
        const uint32_t nw = (j1 - j0) * ROW32;
        const float* src = tab32 + (size_t)j0 * ROW32;
        for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) row_lds[i] = src[i];
        __syncthreads();
    }
    __amdgpu_buffer_rsrc_t rs_pv, rs_m, rs_r;
    // the lane's byte offset in a trace row (lanes past the last chain at 2^31: outside the
    // resource's range, so their stores are dropped without an exec mask); the row's offset
    // within the block goes in the stores' scalar offset (range checks use the lane offset
    // only), so a second's stores cost no VALU for addressing
    const uint32_t voff = live ? c * (uint32_t)sizeof(R) : 0x80000000u;
    const uint32_t rowb = (uint32_t)(tr.ld * sizeof(R));
    if constexpr (out_base(OUT) == OUT_TRACE3) {
        const size_t bo = (size_t)j0 * tr.ld * sizeof(R);
        const int nb = (int)((j1 - j0) * rowb);
        rs_pv = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(tr.pv) + bo, 0, nb, 0x00020000);
        rs_m = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(tr.meter) + bo, 0, nb, 0x00020000);
        rs_r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(tr.residual) + bo, 0, nb, 0x00020000);
    }
    const int32_t fault_eff = alive ? fault : 0;   // ok = j < fault_eff: one compare, no branch
    // One second.  Every lane computes it; a lane whose chain is faulted (or not
    // alive) emits NaN / no statistics.  un, um: the step's Philox words (noise, meter).
    // wave_ok: no lane of the wave has a fault before the block's end (the common case),
    // so a scalar branch skips the per-second NaN selects.
    // lanes past the last chain store out of range (voff) and emit nothing: they never fault the wave
    // The loops are instantiated twice: FF (fault-free, wave_ok) with ok = true and no
    // NaN selects at all (if-converted, they cost a compare and three selects per second
    // even when wave_ok holds), and the general one (below).
    const bool wave_ok = __builtin_amdgcn_ballot_w64(live && fault_eff < (int32_t)j1) == 0;
    // per-chain sites: some lane's site sees daylight in this block (else every second of the
    // wave is night: no noise block, no geometry)
    const bool wave_day = !SITES || __builtin_amdgcn_ballot_w64(live && !blk_night) != 0;
    // _next_day / _next_hour / _next_min at step j (flags fl): the pushes of the day and hour
    // draws (event table) and of the block's staged minute draws
    auto apply_events = [&](uint32_t j, uint32_t fl) __attribute__((always_inline)) {
        if (fl & (FL_DAY | FL_HOUR)) {            // _next_day, _next_hour (rare: loads waited here)
            const size_t eo = (size_t)evi * 4 * n;
            if (live) {
                if (fl & FL_DAY) fpush(fs, S_CLEAR_DAY, (R)evd[eo + 2 * (size_t)n]);
                if (fl & FL_HOUR) {
                    fpush(fs, S_CC, (R)evd[eo]);
                    fpush(fs, S_CLEAR_DAY, (R)evd[eo + 3 * (size_t)n]);
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            ++evi;
        }
        if (fl & FL_MIN) {                         // _next_min: staged minute draws
            const int32_t mi = ((int32_t)j - (int32_t)fm) / 60;
            const int32_t k = mi - mA;   // wave-uniform
            const int32_t kk = min(k, 1);
            R ncl = min_lds[2 * kk][threadIdx.x], ncr = min_lds[2 * kk + 1][threadIdx.x];
            if (k >= 2) {   // a third boundary in the block (its first within 8 s of the start): rare
                if (live) {
                    const R* mt = reinterpret_cast<const R*>(sg.mtab) + (size_t)(2 * mi) * n + c;
                    ncl = mt[0];
                    ncr = mt[n];
                }
                __builtin_amdgcn_s_waitcnt(0);   // wait here, not at the join every minute
            }
            fpush(fs, S_CLOUDY_NOISE, ncl);
            fpush(fs, S_CLEAR_NOISE, ncr);
        }
    };
    // the second's outputs: NaN on a faulted lane, the guard-band bit, the trace stores or
    // the statistics (jb = j - j0, wave-uniform)
    auto finish = [&](uint32_t j, uint32_t jb, bool covered, R csi, R pv, R meter, R res, bool held, auto ff)
        __attribute__((always_inline)) {
        constexpr bool FF = decltype(ff)::value;
        const bool ok = FF || (int32_t)j < fault_eff;
        held = held && ok && live;   // lanes past the last chain run on uninitialised samplers: never held
        if constexpr (sizeof(R) == 4) {
            // jb is wave-uniform: the word and the bit are scalars.  TMH_HELD_OR: every lane ors
            // its bit or 0 into its word (one ds_or, no exec-mask branch around a rare store)
            uint32_t* hw = reinterpret_cast<uint32_t*>(&held_lds[threadIdx.x]) + (jb >> 5);
            if constexpr (TMH_HELD_OR)
                __hip_atomic_fetch_or(hw, held ? 1u << (jb & 31) : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else if (held)
                *hw |= 1u << (jb & 31);
        }
        if constexpr (!FF) {
            csi = ok ? csi : R(NAN);
            pv = ok ? pv : R(NAN);
            meter = ok ? meter : R(NAN);
            res = ok ? res : R(NAN);
        }
        const uint8_t cov = ok ? (covered ? 1 : 0) : 255;
        if constexpr (out_base(OUT) == OUT_TRACE3) {
            const uint32_t so = jb * rowb;
            row_store(rs_pv, voff, so, pv);
            row_store(rs_m, voff, so, meter);
            row_store(rs_r, voff, so, res);
        } else if (live) {
            emit<R, OUT, exp_hist_pack<R, OUT, SITES>()>(tr, sv, lds_hist, (uint64_t)j * tr.ld + c, cov, csi, pv, meter,
                                                         res, acc, ok, held);
        }
    };
    auto second = [&](uint32_t j, uint32_t un, uint32_t um, auto ff) __attribute__((always_inline)) {
        R row[row_w<R>()];
        uint32_t fl;
        if constexpr (ROWL) {
            const float* lr = row_lds + (j - j0) * ROW32;
#pragma unroll
            for (int i = 0; i < ROW32; ++i) row[i] = lr[i];
            fl = __builtin_amdgcn_readfirstlane(__float_as_uint(row[G_FLAGS + G32]));
        } else {
#pragma unroll
            for (int i = 0; i < row_w<R>(); ++i) row[i] = rowp[i];
            rowp += RW;
            fl = sizeof(R) == 8 ? (uint32_t)(double)rowp[G_FLAGS - RW] : __float_as_uint(row[G_FLAGS + G32]);
        }
        apply_events(j, fl);
        const uint32_t jb = j - j0;   // wave-uniform
        if ((jb & 31) == 0) cov_w = cov_lds[jb >> 5][threadIdx.x];
        const bool covered = (cov_w >> (jb & 31)) & 1u;
        uint32_t flp = fl;
        if constexpr (SITES) {   // this chain's own site: geometry per chain-second (none in a night block)
            flp = lane_flags(fl, blk_night || lane_row<R>(ls, sun + (size_t)j * SUN_W, kp.module, row,
                                                          (LdsD*)pv_lds_tab), row);
        }
        R csi, pv, meter, res;
        bool held = false;   // fp32: PV in a guard band, recomputed in fp64 by fixup_kernel
        if (out_base(OUT) != OUT_ANY && (!kp.with_pv || (flp & FL_NIGHT))) {
            // the CSI is not an output (trace of pv / meter / residual, or statistics) and
            // pv = 0 whatever it is (second_body: night, or no PV): no noise quantile, no
            // samplers, no PV chain; the same values.  Wave-uniform for a single site.
            csi = R(0);
            pv = R(0);
            meter = meter_w<R>(um);
            res = meter - pv;
        } else {
            if constexpr (sizeof(R) == 8 && !SITES) {
                // the PV constants re-read from LDS each second (ds_read, no VALU) through an
                // address the compiler cannot see is loop-invariant: hoisted, they would sit
                // in SGPRs across the loop, be spilled to VGPR lanes and cost two v_readlane
                // each per use (a sixth of the loop's VALU)
                uint32_t pa = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) PV64*)pv_lds;
                asm volatile("" : "+v"(pa));
                const __attribute__((address_space(3))) PV64* p = (const __attribute__((address_space(3))) PV64*)(uintptr_t)pa;
                second_body<R>(kp, pkv, row, flp, fs, covered, ndtri64(un, (LdsD*)pv_lds_tab), meter_w<R>(um), csi, pv,
                               meter, res, held, p, (LdsD*)pv_lds_tab);
            } else {
                second_body<R, !SITES && !ROWL>(kp, pkv, row, flp, fs, covered, noise_lds<R>(un, nd_lds), meter_w<R>(um),
                                                csi, pv, meter, res, held, nullptr, nullptr, disc_lds);
            }
        }
        finish(j, jb, covered, csi, pv, meter, res, held, ff);
    };
    // fp32 single-site kernels (C2 trace, C3 / C4 statistics): four-second groups whose kind the
    // plan gives on the group's first row (geom_kernel: FL_G_NIGHT, FL_G_DAY -- every second
    // night, or every second daylight with DISC valid, and no boundary event after the first
    // second; a window start on the four-step grid makes every minute, hour and day boundary
    // a group's first second).  Such a group applies its first second's events once and runs
    // four straight-line seconds with no flag tests; a night second is its meter alone (no
    // row loads).  Other groups (sunrise, sunset, DISC's zenith limit) take the per-second path.
    constexpr bool FASTG = !SITES && !ROWL && out_base(OUT) != OUT_ANY;
    // TMH_ISA_MARKS (analysis builds only, scripts/isa_loop.py --groups): comment markers around
    // the four-second group bodies, so the listing's instructions per group can be counted
#ifdef TMH_ISA_MARKS
#define TMH_MARK(s) asm volatile("; TMH_MARK " s)
#else
#define TMH_MARK(s) \
    do {        \
    } while (0)
#endif
    auto night4 = [&](uint32_t j, const U4& pm, auto ff) __attribute__((always_inline)) {
        const uint32_t w[4] = {pm.x, pm.y, pm.z, pm.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const R meter = meter_w<R>(w[q]);
            finish(j + q, j + q - j0, false, R(0), R(0), meter, meter, false, ff);
        }
    };
    auto day4 = [&](uint32_t j, const U4& pn, const U4& pm, auto ff) __attribute__((always_inline)) {
        const uint32_t wn[4] = {pn.x, pn.y, pn.z, pn.w}, wm[4] = {pm.x, pm.y, pm.z, pm.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            R row[row_w<R>()];
#pragma unroll
            for (int i = 0; i < row_w<R>(); ++i) row[i] = rowp[i];
            rowp += RW;
            const uint32_t jb = j + q - j0;
            const bool covered = (cov_w >> (jb & 31)) & 1u;
            R csi, pv, meter, res;
            bool held = false;
            if constexpr (sizeof(R) == 8) {   // the PV constants from LDS (see second), the table quantile
                uint32_t pa = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) PV64*)pv_lds;
                asm volatile("" : "+v"(pa));
                const __attribute__((address_space(3))) PV64* p = (const __attribute__((address_space(3))) PV64*)(uintptr_t)pa;
                second_body<R>(kp, pkv, row, FL_DISCOK, fs, covered, ndtri64(wn[q], (LdsD*)pv_lds_tab),
                               meter_w<R>(wm[q]), csi, pv, meter, res, held, p, (LdsD*)pv_lds_tab);
            } else {
                second_body<R, true>(kp, pkv, row, FL_DISCOK, fs, covered, noise_lds<R>(wn[q], nd_lds),
                                     meter_w<R>(wm[q]), csi, pv, meter, res, held, nullptr, nullptr, disc_lds);
            }
            finish(j + q, jb, covered, csi, pv, meter, res, held, ff);
        }
    };
    // The per-second draws: the meter's and the noise's streams, one Philox block per four
    // steps each (word step & 3).  A four-second group draws its noise block only when
    // one of its seconds needs the noise (the CSI is an output, per-chain sites, or a
    // daylight second with PV: the rows' night bits, wave-uniform), so a night second
    // costs a quarter of a block instead of half.
    auto loops = [&](auto ff) __attribute__((always_inline)) {
        uint32_t j = j0;
        if (((W0 + j0) & 3) == 0) {
            for (; j + 4 <= j1; j += 4) {
                const uint64_t g = (uint64_t)(W0 + j) >> 2;
                TMH_MARK("meter begin");
                const U4 pm = keyed_block(kp.seed, chain, g, TAG_METER4, 0);
                TMH_MARK("meter end");
                if constexpr (FASTG) {
                    const uint32_t fl0 = sizeof(R) == 8 ? (uint32_t)(double)rowp[G_FLAGS]   // the group's first row
                                                        : __float_as_uint((float)rowp[G_FLAGS + G32]);
                    if (!kp.with_pv || (fl0 & FL_G_NIGHT)) {
                        apply_events(j, fl0);
                        if (((j - j0) & 31) == 0) cov_w = cov_lds[(j - j0) >> 5][threadIdx.x];
                        rowp += 4 * RW;
                        TMH_MARK("night4 begin");
                        night4(j, pm, ff);
                        TMH_MARK("night4 end");
                        continue;
                    }
                    if (fl0 & FL_G_DAY) {
                        TMH_MARK("noise begin");
                        const U4 pn = keyed_block(kp.seed, chain, g, TAG_NOISE4, 0);
                        TMH_MARK("noise end");
                        apply_events(j, fl0);
                        if (((j - j0) & 31) == 0) cov_w = cov_lds[(j - j0) >> 5][threadIdx.x];
                        TMH_MARK("day4 begin");
                        day4(j, pn, pm, ff);
                        TMH_MARK("day4 end");
                        continue;
                    }
                }
                bool need = out_base(OUT) == OUT_ANY || !kp.with_pv || (SITES && wave_day);
                if (!need && !SITES) {   // any daylight second among the four (scalar loads of their flags)
                    uint32_t nf = FL_NIGHT;
                    if constexpr (ROWL) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) nf &= __float_as_uint(row_lds[(j - j0 + q) * ROW32 + G_FLAGS + G32]);
                        nf = __builtin_amdgcn_readfirstlane(nf);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            nf &= sizeof(R) == 8 ? (uint32_t)(double)rowp[q * RW + G_FLAGS]
                                                 : __float_as_uint((float)rowp[q * RW + G_FLAGS + G32]);
                    }
                    need = nf == 0;
                }
                U4 pn{0u, 0u, 0u, 0u};
                if (need) pn = keyed_block(kp.seed, chain, g, TAG_NOISE4, 0);
                second(j, pn.x, pm.x, ff);
                second(j + 1, pn.y, pm.y, ff);
                second(j + 2, pn.z, pm.z, ff);
                second(j + 3, pn.w, pm.w, ff);
            }
        }
        for (; j < j1; ++j) {   // a window start off the four-step grid, or a short last block (rare)
            const uint64_t g = (uint64_t)(W0 + j) >> 2;
            const uint32_t q = (uint32_t)(W0 + j) & 3u;
            second(j, word_of(keyed_block(kp.seed, chain, g, TAG_NOISE4, 0), q),
                   word_of(keyed_block(kp.seed, chain, g, TAG_METER4, 0), q), ff);
        }
    };
    // (fp32 single-site only: in the fp64 and per-site kernels, which sit at their
    // register bounds, the second copy adds spills)
#ifndef TMH_EXP_FF_F64
#define TMH_EXP_FF_F64 0   // the fault-free loop copy for the fp64 single-site kernels too (A/B builds)
#endif
    if ((sizeof(R) == 4 || (TMH_EXP_FF_F64 && out_base(OUT) == OUT_TRACE3)) && !SITES && wave_ok) loops(std::true_type{});
    else loops(std::false_type{});
    if constexpr (sizeof(R) == 4) {
        const uint4 hm = held_lds[threadIdx.x];
        const bool held_any = (hm.x | hm.y | hm.z | hm.w) != 0;
        if (live && held_any) {   // (chain, block, seconds) for fixup_kernel (outside the loop: no registers held across it)
            const uint32_t k = atomicAdd(sg.nfix, 1u);
            if (k < sg.fixcap)
                sg.fix[k] = FixRec{c, b, jr, 0u, hm,
                                   make_uint4(cov_lds[0][threadIdx.x], cov_lds[1][threadIdx.x], cov_lds[2][threadIdx.x],
                                              cov_lds[3][threadIdx.x])};
        }
    }
    if (live && sv.acc) {   // the block's sums into the chain's fixed-point window totals (order-free)
        unsigned long long* fx = reinterpret_cast<unsigned long long*>(sg.acc_fx);
        atomicAdd(fx + c, (unsigned long long)llrint(acc.pv * sg.fx_scale));
        atomicAdd(fx + (size_t)n + c, (unsigned long long)llrint(acc.m * sg.fx_scale));
        atomicAdd(fx + 2 * (size_t)n + c, (unsigned long long)llrint(acc.r * sg.fx_scale));
        __hip_atomic_fetch_max(sg.acc_mx + c, max_key(acc.max()), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}


// Statistics: one tile per workgroup, its LDS histogram flushed to the device histogram
// by 64-bit atomics at the end.  Round 4 measured workgroups looping over several tiles
// (one flush per workgroup): a persistent grid 8-40 % slower on C3 / C4, four tiles per
// workgroup 13 % slower on C3 (the inlined tile loop spills 45 VGPRs instead of 4).
template <typename R, int OUT, bool SITES>
__global__ __launch_bounds__((exp_wg<R, OUT, SITES>()), (exp_waves<R, OUT, SITES>())) void expand_kernel(KParams kp, DrawParams dp, StateView st, uint64_t chain0,
                                                     uint32_t n, int64_t W0, uint32_t nsteps, int64_t utc0,
                                                     const double* __restrict__ tab64,
                                                     const float* __restrict__ tab32,
                                                     const double* __restrict__ sun,
                                                     const int2* __restrict__ events,
                                                     const uint32_t* __restrict__ n_events,
                                                     const BlockDesc* __restrict__ desc, SegView sg, TraceView tr,
                                                     StatsView sv, const uint32_t* __restrict__ bperm)
{
    extern __shared__ uint32_t lds_hist[];
    constexpr int WGT = exp_wg<R, OUT, SITES>();   // threads per workgroup
    __shared__ uint32_t cov_lds[4][WGT];
    __shared__ R min_lds[4][WGT];   // minute boundaries mA, mA + 1 of the block: cloudy, clear noise
    __shared__ uint4 held_lds[WGT];
    // fp64: the PV constants; fp64 and per-chain sites: the log / exp table (one copy per workgroup)
    __shared__ PV64 pv_lds[1];   // (176 + 16 bytes in the fp32 kernels: unused)
    __shared__ __attribute__((aligned(16))) double pv_tab[sizeof(R) == 8 || SITES ? PV_TAB : 2];
    __shared__ __attribute__((aligned(16))) float row_lds[TMH_ROW_LDS && sizeof(R) == 4 && !SITES ? BLOCK_STEPS * ROW32 : 1];
    // fp32: the noise quantile's table (ndtri_t), 8 KB, copied once per workgroup
    // (with TMH_DISC_LDS, DISC's coefficient sets after it: disc_row)
    __shared__ float4 nd_tab[sizeof(R) == 4 ? ND32_N + (TMH_DISC_LDS ? DISC_TAB : 0) : 1];
    if constexpr (sizeof(R) == 8 || SITES) {
        if (threadIdx.x < PV64_N) reinterpret_cast<double*>(pv_lds)[threadIdx.x] = reinterpret_cast<const double*>(&kp.pv64)[threadIdx.x];
        for (uint32_t i = threadIdx.x; i < PV_TAB; i += blockDim.x) pv_tab[i] = g_pv_tab[i];
    }
    if constexpr (sizeof(R) == 4)
    {
        for (uint32_t i = threadIdx.x; i < ND32_N; i += blockDim.x) nd_tab[i] = g_nd32_tab[i];
        if (TMH_DISC_LDS && threadIdx.x < DISC_TAB) nd_tab[ND32_N + threadIdx.x] = disc_row(threadIdx.x);
    }
    __syncthreads();
    constexpr bool PACK = exp_hist_pack<R, OUT, SITES>();
    const uint32_t nw = PACK ? (sv.n_bins + 1) / 2 : sv.n_bins;   // 16-bit bin pairs, or bins
    if (sv.hist) {
        for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) lds_hist[i] = 0;
        __syncthreads();
    }
    auto tile = [&](uint32_t b, uint32_t cblk) __attribute__((always_inline)) {
        expand_tile<R, OUT, SITES, WGT>(b, cblk, kp, dp, st, chain0, n, W0, nsteps, utc0, tab64, tab32, sun, events,
                                        n_events, desc, sg, tr, sv, lds_hist, cov_lds, min_lds, held_lds, pv_lds, pv_tab,
                                        row_lds, nd_tab);
    };
    {   // grid: x = time block, y = chain block; XCD-aware tile order (speed only): the
        // hardware deals workgroups round-robin over the 8 XCDs in launch order (x fastest),
        // so workgroup L runs on XCD L % 8.  XCD x takes the x-th contiguous range of tiles in
        // the order (time block m of a stride-8 permutation of the blocks, chain block): its
        // workgroups then read the geometry rows (scalar loads) of ~every 8th 128-s block
        // only, 1/8 of the window's rows (C2 fp32: 0.95 of 7.6 MB) in its 4 MB L2, each time
        // block by all its chain blocks in a row, and every XCD still gets an even share of
        // day and night blocks.  Bijections for any grid: XCD x has q + (x < r) workgroups
        // (N = 8 q + r), and the permutation lists the blocks b = x mod 8 for x = 0..7.
        const uint32_t T = gridDim.x, CB = gridDim.y, N = T * CB;
        const uint32_t L = blockIdx.x + T * blockIdx.y, x = L & 7u, q = N >> 3, r = N & 7u;
        const uint32_t k = x * q + min(x, r) + (L >> 3);
        const uint32_t m = k / CB, qt = T >> 3, rt = T & 7u, big = rt * (qt + 1);
        const uint32_t xm = m < big ? m / (qt + 1) : rt + (m - big) / max(qt, 1u);
        const uint32_t b = xm + 8u * (m - (xm * qt + min(xm, rt)));
        constexpr int ORD = exp_tile_order<R, OUT, SITES>();
        uint32_t bs, cs;
        if constexpr (ORD == 0) {   // launch order
            bs = blockIdx.x;
            cs = blockIdx.y;
            (void)b;
            if (exp_tpw<R, OUT, SITES>() == 1 && bperm) {
                // cost order (round 6): the tiles in chunks of TCH blocks of the plan's order
                // (daylight blocks first), each chunk's tiles chain block by chain block, time
                // block fastest -- so concurrent workgroups still write different trace rows, as
                // in launch order, but the day tiles are all dealt before the night ones
                constexpr uint32_t TCH = 16;
                const uint32_t per = TCH * CB, ch = L / per, rr = L - ch * per;
                const uint32_t cc = min(TCH, T - ch * TCH), y = rr / cc;
                bs = bperm[ch * TCH + (rr - y * cc)];
                cs = y;
            }
        } else if constexpr (ORD == 2) {
            // order 2: the tiles listed class by class (time blocks b = x mod 8), chain block major
            // inside a class (consecutive workgroups of an XCD: different time blocks, as in launch
            // order, so the trace rows written at a time spread over the HBM channels); XCD x's
            // contiguous range of that list is (nearly) class x: 1/8 of the rows per L2
            const uint32_t kbig = big * CB;   // tiles of the rt classes with qt + 1 blocks
            const uint32_t x2 = k < kbig ? k / (CB * (qt + 1)) : rt + (k - kbig) / max(CB * qt, 1u);
            const uint32_t cum = x2 <= rt ? x2 * CB * (qt + 1) : kbig + (x2 - rt) * CB * qt;
            const uint32_t nbx = qt + (x2 < rt ? 1u : 0u), i2 = k - cum;
            bs = __builtin_amdgcn_readfirstlane(x2 + 8u * (i2 % nbx));
            cs = __builtin_amdgcn_readfirstlane(i2 / nbx);
            (void)b;
        } else {
            // (uniform, but computed by VALU integer division: readfirstlane keeps them in SGPRs, so
            // the row pointer and the tile's block loads stay scalar)
            bs = __builtin_amdgcn_readfirstlane(b);
            cs = __builtin_amdgcn_readfirstlane(k % CB);
        }
        constexpr int TPW = exp_tpw<R, OUT, SITES>();
        if constexpr (TPW == 1) tile(bs, cs);
        else {   // time blocks bs TPW .. bs TPW + TPW - 1 (x counts super-blocks of TPW blocks)
            for (int t = 0; t < TPW; ++t) {
                // laundered per tile: nothing of a tile is hoisted out of the loop and held in
                // registers across it (the per-chain loads are repeated instead)
                uint32_t bb = bs * TPW + t, cc = cs;
                asm volatile("" : "+s"(bb), "+s"(cc));
                if (bb < sg.nblk) tile(bb, cc);
            }
        }
    }
    if (sv.hist) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) {
            const uint32_t w = lds_hist[i];
            if constexpr (PACK) {
                const uint32_t lo = w & 0xFFFFu, hi = w >> 16;
                if (lo) atomicAdd((unsigned long long*)&sv.hist[2 * i], (unsigned long long)lo);
                if (hi) atomicAdd((unsigned long long*)&sv.hist[2 * i + 1], (unsigned long long)hi);   // hi = 0 past n_bins
            } else if (w) {
                atomicAdd((unsigned long long*)&sv.hist[i], (unsigned long long)w);
            }
        }
    }
}

// ------------------------------------------------------------ compaction
// Batches whose chains fault (the reference's AssertionError in markov mode ends
// most C5 chains within the week) keep only their live chains in the launches:
// live_chains_kernel lists the slots with status 0 (in slot order, one
// workgroup, deterministic), state_move_kernel gathers those slots into a dense
// working state and scatters them back after the window.  Keyed draws, tables,
// sites and statistics follow the chain, not the slot (KParams::ids).
__global__ __launch_bounds__(1024) void live_chains_kernel(StateView st, uint32_t n, const uint32_t* __restrict__ ids_in,
                                                           uint32_t* __restrict__ ids_out, uint32_t* __restrict__ n_out)
{
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t c0 = 0; c0 < n; c0 += 1024) {
        const uint32_t c = c0 + threadIdx.x;
        const bool live = c < n && st.status[c] == 0;
        const uint64_t bal = __builtin_amdgcn_ballot_w64(live);
        const uint32_t below = (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = (uint32_t)__builtin_popcountll(bal);
        __syncthreads();
        uint32_t off = base;
        for (uint32_t k = 0; k < w; ++k) off += wsum[k];
        if (live) ids_out[off + below] = ids_in ? ids_in[c] : c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (uint32_t k = 0; k < 16; ++k) t += wsum[k];
            base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_out = base;
}

// dst slot i <- src slot map[i] (gather) or dst slot map[i] <- src slot i
// (scatter), for i < *count; the sigma rows up to the chain's length only
__global__ __launch_bounds__(256) void state_move_kernel(StateView src, StateView dst, const uint32_t* __restrict__ map,
                                                         const uint32_t* __restrict__ count, uint32_t cap, int scatter)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(*count, cap)) return;
    const uint32_t a = scatter ? i : map[i], b = scatter ? map[i] : i;   // src slot a -> dst slot b
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        dst.sb[k][b] = src.sb[k][a];
        dst.sa[k][b] = src.sa[k][a];
    }
    dst.cl[b] = src.cl[a];
    dst.clr[b] = src.clr[a];
    dst.mstate[b] = src.mstate[a];
    dst.sec[b] = src.sec[a];
    const int L = src.L[a];
    dst.L[b] = L;
    dst.pos[b] = src.pos[a];
    dst.status[b] = src.status[a];
    dst.ncalls[b] = src.ncalls[a];
    dst.fn[0][b] = src.fn[0][a];
    dst.fn[1][b] = src.fn[1][a];
    const double* sc = src.sc + (size_t)a * CAP;
    const double* sl = src.sl + (size_t)a * CAP;
    double* dc = dst.sc + (size_t)b * CAP;
    double* dl = dst.sl + (size_t)b * CAP;
    for (int k = 0; k < min(L, CAP); ++k) {
        dc[k] = sc[k];
        dl[k] = sl[k];
    }
}

// The fp32 expansion's guard-band seconds (the blocks FixRec lists), recomputed
// in fp64 (redo_second) after the expansion and before the commit: the trace's pv and
// residual are overwritten; the statistics get the exact differences of the
// sums (fp32 values in fp64 differ exactly, so the corrections add up in any
// order), the final residual's maximum and histogram count (the expansion left
// these seconds out of both).  One wave per FIX_RPW records (one mask word per lane):
// the wave compacts their set bits (a prefix sum of the words' popcounts) and runs one
// flagged second per lane, so the kernel's duration is one second's recomputation (a
// latency-bound fp64 chain) and the waves that run it are full.  (Round 4 gave every
// (record, second) a work-item: ~1 flagged second in 20 per wave, 95 us per C2 batch.)
// Grid-stride over the record groups.
constexpr uint32_t FIX_RPW = 16;
#ifndef TMH_FIX_WAVES_SITES
#define TMH_FIX_WAVES_SITES 1   // min waves per SIMD of the per-site fixup (its fp64 redo recomputes the site's geometry)
#endif
template <bool SITES>
__global__ __launch_bounds__(64, (SITES ? TMH_FIX_WAVES_SITES : 1)) void fixup_kernel(KParams kp, DrawParams dp, StateView st, uint64_t chain0, uint32_t n,
                                                    int64_t W0, uint32_t nsteps, int64_t utc0,
                                                    const double* __restrict__ tab64, const float* __restrict__ tab32,
                                                    const double* __restrict__ sun,
                                                    const int2* __restrict__ events,
                                                    const uint32_t* __restrict__ n_events,
                                                    const BlockDesc* __restrict__ desc, SegView sg, TraceView tr,
                                                    StatsView sv)
{
    const uint32_t nrec = min(*sg.nfix, sg.fixcap);
    const int ne = (int)min(*n_events, ev_cap_dev(nsteps));
    const uint32_t lane = threadIdx.x;   // one wave per workgroup
    for (uint32_t r0 = blockIdx.x * FIX_RPW; r0 < nrec; r0 += gridDim.x * FIX_RPW) {   // wave-uniform
        const uint32_t rw = r0 + (lane >> 2);
        uint32_t word = 0;
        if (rw < nrec) {
            const uint4 m = sg.fix[rw].mask;
            const uint32_t w = lane & 3;
            word = w == 0 ? m.x : (w == 1 ? m.y : (w == 2 ? m.z : m.w));
        }
        uint32_t cum = __popc(word);   // inclusive prefix sum over the wave's words
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(cum, d, 64);
            if (lane >= (uint32_t)d) cum += u;
        }
        const uint32_t total = __builtin_amdgcn_readfirstlane(__shfl(cum, 63, 64));
        for (uint32_t k0 = 0; k0 < total; k0 += 64) {   // wave-uniform
            const uint32_t k = k0 + lane;
            // the word holding flagged second k: the first q with cum[q] > k (every lane
            // takes part in the shuffles; lanes past the total search for nothing)
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t h = 32; h; h >>= 1)
                if (__shfl(cum, (int)(lo + h - 1), 64) <= k) lo += h;
            const uint32_t wq = __shfl(word, (int)lo, 64);
            const uint32_t cq = __shfl(cum, (int)lo, 64);
            if (k >= total) continue;
            uint32_t m = wq;
            for (uint32_t rank = k - (cq - __popc(wq)); rank; --rank) m &= m - 1;   // drop the lower set bits
            const uint32_t i = (lo & 3) * 32 + (uint32_t)(__ffs(m) - 1);   // second of the record's block
            const FixRec& fr = sg.fix[r0 + (lo >> 2)];
            const uint32_t c = fr.c;
            if (c >= n || fr.b >= sg.nblk) continue;   // (never appended: the expansion records live chains only)
            const BlockDesc db = desc[fr.b];
            const uint32_t j = fr.b * BLOCK_STEPS + i;
            const uint32_t cw = (lo & 3) == 0 ? fr.cov.x : ((lo & 3) == 1 ? fr.cov.y : ((lo & 3) == 2 ? fr.cov.z : fr.cov.w));
            const bool covered = (cw >> (i & 31)) & 1u;
            float pv32, meter, pv;
            if (!redo_second<SITES>(kp, dp, st, sg, n, c, chain0, W0, utc0, j, db, covered, sv.acc != nullptr, events, ne,
                                    tab64, tab32, sun, pv32, meter, pv))
                continue;
            const float res = meter - pv, res32 = meter - pv32;   // second_body's residual
            const size_t o = (size_t)j * tr.ld + c;
            if (tr.pv) reinterpret_cast<float*>(tr.pv)[o] = pv;
            if (tr.residual) reinterpret_cast<float*>(tr.residual)[o] = res;
            if (sv.acc) {
                atomicAdd(&sg.corr[c], (double)pv - (double)pv32);
                atomicAdd(&sg.corr[(size_t)n + c], (double)res - (double)res32);
                __hip_atomic_fetch_max(sg.acc_mx + c, max_key((double)res), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (sv.hist) {
                atomicAdd((unsigned long long*)&sv.hist[hist_bin_rt<float>(sv, res)], 1ull);
            }
        }
    }
}

// The window's end, one work-item per chain, after the expansion (and the fixup):
//  * statistics (sv.acc): the window's fixed-point block sums + the fixup's exact
//    corrections into the caller's fp64 accumulators (every input is order-free, so
//    the result is deterministic);
//  * state: the window-end sampler pairs (the last hour / clear-day events from the
//    draw tables, the last two minute draws: fp32 engines take the fast copies from the
//    minute table and the fp64 ones from `mend`), the walk's wind pair and status.
template <typename R>
__global__ __launch_bounds__(256) void commit_kernel(StateView st, uint32_t n, SegView sg, StatsView sv, MinuteCtx mc0,
                                                     const uint32_t* __restrict__ n_events,
                                                     const BlockDesc* __restrict__ desc_end, int markov,
                                                     const uint32_t* __restrict__ ids, uint32_t acc_n)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    if (sv.acc) {
        const double p = (double)sg.acc_fx[c] * sg.fx_inv + sg.corr[c];
        const double m = (double)sg.acc_fx[(size_t)n + c] * sg.fx_inv;
        const double r = (double)sg.acc_fx[2 * (size_t)n + c] * sg.fx_inv + sg.corr[(size_t)n + c];
        const double mx = max_unkey(sg.acc_mx[c]);
        const uint32_t g = gid(ids, c);
        const size_t an = acc_n ? acc_n : n;   // acc rows: the full batch
        sv.acc[g] += p;
        sv.acc[an + g] += m;
        sv.acc[2 * an + g] += r;
        sv.acc[3 * an + g] = fmax(sv.acc[3 * an + g], mx);
    }
    if (st.status[c] != 0) return;
    // records lost (never observed: room for ~100x the measured rate): the batch's
    // chains are marked, as it is not known whose seconds were not recomputed
    st.status[c] = *sg.nfix > sg.fixcap ? TMH_CHAIN_GUARD_OVERFLOW : sg.status[c];
    if (st.status[c] != 0) return;
    Samp sp;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        sp.b[k] = st.sb[k][c];
        sp.a[k] = st.sa[k][c];
    }
    MinuteCtx mc = mc0;
    mc.chain += gid(mc.dp.ids, c);
    mc.ne = (int)min(*n_events, sg.evcap);
    const BlockDesc de = *desc_end;
    if constexpr (sizeof(R) == 4) {   // the fast noise copies from the fp32 table, the fp64 pairs from mend
        Samp sf = sp;
        load_fast_noise(st, c, sf);
        samplers_at<float>(de, sg, n, c, sf, mc, st);
        st.fn[0][c] = make_float2((float)sf.b[S_CLOUDY_NOISE], (float)sf.a[S_CLOUDY_NOISE]);
        st.fn[1][c] = make_float2((float)sf.b[S_CLEAR_NOISE], (float)sf.a[S_CLEAR_NOISE]);
        if (de.q0 >= 0) {   // as exact_noise_at: q1's draws (or the pair's after value), then q0's
            if (de.q1 >= 0) {
                sp.b[S_CLOUDY_NOISE] = sg.mend[c];
                sp.b[S_CLEAR_NOISE] = sg.mend[(size_t)n + c];
            } else {
                sp.b[S_CLOUDY_NOISE] = sp.a[S_CLOUDY_NOISE];
                sp.b[S_CLEAR_NOISE] = sp.a[S_CLEAR_NOISE];
            }
            sp.a[S_CLOUDY_NOISE] = sg.mend[2 * (size_t)n + c];
            sp.a[S_CLEAR_NOISE] = sg.mend[3 * (size_t)n + c];
        }
        for (int k : {S_CC, S_CLEAR_DAY}) {
            sp.b[k] = sf.b[k];
            sp.a[k] = sf.a[k];
        }
    } else {
        samplers_at<R>(de, sg, n, c, sp, mc, st);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {   // cc, clear_day, cloudy_hour (unchanged), noises
        st.sb[k][c] = sp.b[k];
        st.sa[k][c] = sp.a[k];
    }
    st.sb[S_WS][c] = sg.end_p1[2 * (size_t)n + c];
    st.sa[S_WS][c] = sg.end_p1[3 * (size_t)n + c];
    if (markov) st.mstate[c] = sp.a[S_CC];   // the markov state is the last hourly draw
}

__global__ void probe_kernel(int fn, double a, const double* x, double* out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = 0.0;
    switch (fn) {
        case 0: v = ndtri(x[i]); break;
        case 1: v = gammaincinv(a, x[i]); break;
        case 2: v = stdtrit(a, x[i]); break;
        case 3: v = al_ppf(x[i], a); break;
        case 4: v = (double)ndtri_f(x[i]); break;
        case 8: v = normcdfinv(x[i]); break;   // the fp64 per-second noise quantile
        case 5: {   // wavefront argmin (first index on ties) of x[wave lanes]; needs full waves
            double dm;
            int km;
            argmin_first(x[i], (int)(i & 63), dm, km);
            v = (double)km;
            break;
        }
        case 6: v = dpp_f64<0x138>(a, x[i]); break;            // wave_shr:1, lane 0 <- a
        case 7: v = readlane_f64(x[i], 63); break;
        case 9: v = (double)__builtin_amdgcn_fmed3f((float)x[i], 0.0f, (float)a); break;   // pv_power_f's final clamp
        case 10: v = (double)__builtin_amdgcn_fmed3f((float)x[i], -INFINITY, (float)a); break;   // its min(csi, csimax)
        // the fp64 PV chain's table functions (g_pv_tab): the noise quantile of a 32-bit word, log, exp
        case 11: v = ndtri64((uint32_t)x[i], (const double*)g_pv_tab); break;
        case 12: v = log_tab(x[i], (const double*)g_pv_tab); break;
        case 13: v = exp_tab(x[i], (const double*)g_pv_tab); break;
        // the fp32 per-second noise quantile of a 32-bit word: the table form the kernels use
        // (ndtri_t, g_nd32_tab) and round 5's log form (ndtri_w)
        case 14: v = (double)ndtri_t((uint32_t)x[i], (const float4*)g_nd32_tab); break;
        case 15: v = (double)ndtri_w((uint32_t)x[i]); break;
        case 16: {   // pv_power_f<true>'s min(csi, csimax): v_min_f32 with the bound in an SGPR
            float c;
            const float b = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint((float)a)));
            asm("v_min_f32 %0, %1, %2" : "=v"(c) : "s"(b), "v"((float)x[i]));
            v = (double)c;
            break;
        }
        default: v = NAN;
    }
    out[i] = v;
}

// ------------------------------------------------------------ host side
thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_check(hipError_t e, const char* what)
{
    if (e == hipSuccess) return TMH_OK;
    return fail(TMH_E_HIP, "%s: %s", what, hipGetErrorString(e));
}

constexpr size_t ALIGN = 256;
size_t align_up(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

// state field order: sb[6], sa[6], cl, clr, mstate, sec, L, pos, status, ncalls, sigma_cloud, sigma_clear,
// fn cloudy, fn clear
void state_layout(uint32_t n, uint64_t* off, size_t* total)
{
    size_t o = 0;
    const size_t d = (size_t)n * 8, w = (size_t)n * 4;
    for (int f = 0; f < TMH_STATE_NFIELDS; ++f) {
        off[f] = o;
        size_t bytes = 0;
        if (f < 15) bytes = d;
        else if (f < 20) bytes = w;
        else if (f < 22) bytes = d * CAP;
        else bytes = d;   // fn pairs (float2)
        o += align_up(bytes);
    }
    *total = o;
}

StateView make_view(void* base, uint32_t n)
{
    uint64_t off[TMH_STATE_NFIELDS];
    size_t total;
    state_layout(n, off, &total);
    char* b = (char*)base;
    StateView v;
    for (int k = 0; k < 6; ++k) {
        v.sb[k] = (double*)(b + off[k]);
        v.sa[k] = (double*)(b + off[6 + k]);
    }
    v.cl = (double*)(b + off[12]);
    v.clr = (double*)(b + off[13]);
    v.mstate = (double*)(b + off[14]);
    v.sec = (int32_t*)(b + off[15]);
    v.L = (int32_t*)(b + off[16]);
    v.pos = (uint32_t*)(b + off[17]);
    v.status = (uint32_t*)(b + off[18]);
    v.ncalls = (uint32_t*)(b + off[19]);
    v.sc = (double*)(b + off[20]);
    v.sl = (double*)(b + off[21]);
    v.fn[0] = (float2*)(b + off[22]);
    v.fn[1] = (float2*)(b + off[23]);
    v.n = n;
    return v;
}

// plan: tab64 | tab32 | events | n_events | block descriptors
uint32_t ev_cap(uint32_t n_steps) { return n_steps / 3600 + 16; }   // = ev_cap_dev
uint32_t nblk_of(uint32_t n_steps) { return (n_steps + BLOCK_STEPS - 1) / BLOCK_STEPS; }
// next_cloud calls a chain makes per day window (the oracle, 4,096 chain-days): mean 386,
// p99 620, p99.9 692, max 744; n / 150 + 32 covers 608 a day (~98.5 %); calls past the
// table are drawn in the walk
uint32_t cand_cap(uint32_t n_steps) { return n_steps / 150 + 32; }

struct PlanView {
    double* tab64;
    float* tab32;
    int2* events;
    uint32_t* n_events;
    BlockDesc* desc;
    double* sun;   // [n_steps][SUN_W]: the sun's place per step (per-chain sites)
    uint32_t* bperm;   // [nblk]: the 128-s blocks, daylight blocks first (block_order_kernel)
};

size_t plan_layout(uint32_t n_steps, void* base, PlanView* v)
{
    size_t o = 0;
    char* b = (char*)base;
    if (v) v->tab64 = (double*)(b + o);
    o += align_up((size_t)n_steps * ROW * 8);
    if (v) v->tab32 = (float*)(b + o);
    o += align_up((size_t)n_steps * ROW32 * 4);
    if (v) v->events = (int2*)(b + o);
    o += align_up((size_t)ev_cap(n_steps) * 8);
    if (v) v->n_events = (uint32_t*)(b + o);
    o += ALIGN;
    if (v) v->desc = (BlockDesc*)(b + o);
    o += align_up((size_t)(nblk_of(n_steps) + 1) * sizeof(BlockDesc));
    if (v) v->sun = (double*)(b + o);
    o += align_up((size_t)n_steps * SUN_W * 8);
    if (v) v->bperm = (uint32_t*)(b + o);
    o += align_up((size_t)nblk_of(n_steps) * 4);
    return o;
}

// segment records (one per call + the window-start one): 656 a day, a multiple of 16,
// exceeded by ~0.3 % of the chain-days (above); the pool (one 256-record chunk per 16
// chains) takes that tail
uint32_t g_cap_override = 0, g_pool_override = 0;   // tmh_test_set_segment_capacity (tests only)
uint32_t seg_cap(uint32_t n_steps) { return g_cap_override ? g_cap_override : (n_steps / 135 + 16 + 15) & ~15u; }
uint32_t pool_chunks(uint32_t n) { return g_pool_override ? g_pool_override : n / 16 + 8; }
// (chain, block)s with a guard-band second of the fp32 PV chain: ~1e-5 of the
// chain-seconds are such seconds, ~1.3e-3 of the blocks; room for 1/64
uint32_t fix_cap(uint32_t n, uint32_t n_steps) { return (uint32_t)((uint64_t)n * nblk_of(n_steps) / 64) + 1024; }

// rbytes: bytes per minute-table entry, the engine's real (4 in fp32 mode, 8 in fp64)
size_t scratch_layout(uint32_t n, uint32_t n_steps, void* base, SegView* v, size_t rbytes)
{
    size_t o = 0;
    char* b = (char*)base;
    const uint32_t nblk = nblk_of(n_steps);
    if (v) {
        v->cap = seg_cap(n_steps);
        v->nblk = nblk;
        v->rec = (int2*)(b + o);
    }
    o += align_up((size_t)n * seg_cap(n_steps) * 8);
    if (v) {
        v->ovf = (int32_t*)(b + o);
        v->pool_cap = pool_chunks(n);
    }
    o += align_up((size_t)n * OVF_SLOTS * 4);
    if (v) v->pool = (int2*)(b + o);
    o += align_up((size_t)pool_chunks(n) * OVF_CHUNK * 8);
    if (v) {
        v->pool_n = (uint32_t*)(b + o);
        v->walk_q = v->pool_n + 1;
        v->pool_short = v->pool_n + 2;
    }
    o += ALIGN;
    if (v) v->order = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->rank = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->ovf_first = (int32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->count = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->fault = (int32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->status = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->end_p1 = (double*)(b + o);
    o += align_up((size_t)n * 4 * 8);
    const uint32_t evc = ev_cap(n_steps);
    if (v) {
        v->evcap = evc;
        v->evd = (double*)(b + o);
    }
    o += align_up((size_t)n * evc * 4 * 8);
    const uint32_t kc = cand_cap(n_steps);
    if (v) {
        v->kcap = kc;
        v->cand = (double*)(b + o);
    }
    o += align_up((size_t)n * kc * 8);
    const uint32_t nmin = n_steps / 60 + 2;
    if (v) {
        v->nmin = nmin;
        v->mtab = (void*)(b + o);
    }
    o += align_up((size_t)n * nmin * 2 * rbytes);
    if (v) v->mend = (double*)(b + o);
    o += align_up((size_t)n * 4 * 8);
    const uint32_t fc = fix_cap(n, n_steps);
    if (v) {
        v->fixcap = fc;
        v->fix = (FixRec*)(b + o);
    }
    o += align_up((size_t)fc * sizeof(FixRec));
    if (v) v->nfix = (uint32_t*)(b + o);   // nfix | corr[2][n] | acc_fx | acc_mx: reset before each expansion
    o += ALIGN;
    if (v) v->corr = (double*)(b + o);
    o += align_up((size_t)n * 2 * 8);
    if (v) v->acc_fx = (long long*)(b + o);
    o += align_up((size_t)n * 3 * 8);
    if (v) v->acc_mx = (long long*)(b + o);
    o += align_up((size_t)n * 8);
    if (v) v->brec = (uint32_t*)(b + o);
    o += align_up((size_t)nblk * n * 4);
    return o;
}

}  // namespace

struct tmh_engine {
    KParams kp;
    DrawParams dp;
    GParams gp;
    int device;
    int path;          // resolved kernel path: 1 sequential, 2 time-parallel
    int64_t local_step0 = 0;   // local wall-clock seconds of step 0 (the constructors' time), kept across tmh_set_clock
    uint32_t n_tab = 0;     // rows of the per-chain shape tables (0: none)
    uint32_t n_sites = 0;   // rows of the per-chain sites (0: the engine's one site)
    uint32_t walk_cpr = 1;  // chains per walk row (tmh_set_walk_chains_per_row)
    uint32_t walk_lanes = 0;  // lanes per chain in the walk (tmh_set_walk_lanes; 0: by batch size)
    bool walk_order = true;   // walk rows windiest chain first (tmh_set_walk_order)
    int last_expand = -1;     // TMH_OUT_* of the last expansion launched (tmh_engine_last_expand)
    // expansion tiles daylight blocks first (env TMH_EXP_COST_ORDER=1, A/B; measured slower in the C2
    // pipeline, round 6: 1.55 against 1.42-1.45 ms per step, same box -- launch order mixes the
    // store-bound night tiles with the VALU-bound day tiles over the launch)
    bool cost_order = false;
    uint32_t walk_tp_rows = 65536;   // 8-lane walks of this many rows or more: segments_kernel's TP variant
    uint32_t mk_pre_max = 16384;     // markov batches of at most this many chains: hour quantiles precomputed
    // kernel timing (tmh_profile_*): event pairs per kernel, read and recycled
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof[TMH_K_COUNT];
    std::vector<hipEvent_t> pool;
    hipEvent_t event()
    {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        // timing only: no system-scope fence (an L2 writeback + invalidate at every record,
        // which the kernels beside the timed one would pay for too)
        hipEvent_t e = nullptr;
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
        return e;
    }
    // returns the start event of a timed region (nullptr when not profiling)
    hipEvent_t mark(hipStream_t s)
    {
        if (!profiling) return nullptr;
        hipEvent_t a = event();
        (void)hipEventRecord(a, s);
        return a;
    }
    void close(int k, hipEvent_t a, hipStream_t s)
    {
        if (!a) return;
        hipEvent_t b = event();
        (void)hipEventRecord(b, s);
        prof[k].emplace_back(a, b);
    }
    ~tmh_engine()
    {
        for (auto& v : prof)
            for (auto& p : v) {
                (void)hipEventDestroy(p.first);
                (void)hipEventDestroy(p.second);
            }
        for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    }
};

static bool whole_minutes(const tmh_clock& ck)
{
    bool m = ((ck.local0 - ck.utc0) % 60) == 0;
    for (int i = 0; i < ck.n_shifts; ++i) m = m && (ck.shift_delta[i] % 60) == 0;
    return m;
}

extern "C" {

int tmh_abi_version(void) { return TMH_ABI_VERSION; }

#ifndef TMH_BUILD_STAMP
#define TMH_BUILD_STAMP "unstamped"   // tmhpvsim_amd/build.py defines "TMHSTAMP:<hash of the sources + flags>"
#endif
const char* tmh_build_stamp(void) { return TMH_BUILD_STAMP; }

const char* tmh_last_error(void) { return g_err.c_str(); }

size_t tmh_state_bytes(uint32_t n_chains)
{
    uint64_t off[TMH_STATE_NFIELDS];
    size_t total;
    state_layout(n_chains, off, &total);
    return total;
}

int tmh_state_offsets(uint32_t n_chains, uint64_t* offsets)
{
    if (!offsets) return fail(TMH_E_INVAL, "offsets is NULL");
    size_t total;
    state_layout(n_chains, offsets, &total);
    return TMH_OK;
}

size_t tmh_plan_bytes(uint32_t n_steps) { return plan_layout(n_steps, nullptr, nullptr); }

size_t tmh_scratch_bytes(uint32_t n_chains, uint32_t n_steps)
{
    return scratch_layout(n_chains, n_steps, nullptr, nullptr, 8);   // any engine (fp64 minute table)
}

size_t tmh_workspace_bytes(uint32_t n_chains, uint32_t n_steps)
{
    return tmh_plan_bytes(n_steps) + tmh_scratch_bytes(n_chains, n_steps);
}

static size_t tmh_engine_scratch_rbytes(const struct tmh_engine* eng)
{
    return eng->kp.precision == TMH_FP64 ? 8 : 4;   // the minute table's real
}

size_t tmh_engine_scratch_bytes(const struct tmh_engine* eng, uint32_t n_chains, uint32_t n_steps)
{
    if (!eng) return tmh_scratch_bytes(n_chains, n_steps);
    return scratch_layout(n_chains, n_steps, nullptr, nullptr, tmh_engine_scratch_rbytes(eng));
}

// fp64 standard normal quantile on the host, lower half (p <= 0.5): Acklam's rational
// approximation (1.2e-9 relative) polished by two Halley steps on libm's erfc (to ~1 ulp);
// only the fp32 noise table is built from it
static double host_ndtri_lower(double p)
{
    static const double a[6] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                                1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
    static const double b[5] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                                6.680131188771972e+01, -1.328068155288572e+01};
    static const double c[6] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                                -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
    static const double d[4] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                                3.754408661907416e+00};
    double x;
    if (p < 0.02425) {
        const double q = std::sqrt(-2.0 * std::log(p));
        x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
            ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0);
    } else {
        const double q = p - 0.5, r = q * q;
        x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
            (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0);
    }
    for (int it = 0; it < 2; ++it) {
        const double e = 0.5 * std::erfc(-x * 0.70710678118654752440) - p;
        const double u = e * 2.50662827463100050242 * std::exp(0.5 * x * x);
        x = x - u / (1.0 + 0.5 * x * u);
    }
    return x;
}

// g_nd32_tab (ndtri_t): per segment (exponent e, top ND32_S mantissa bits) the cubic in the
// low ND32_SHIFT bits r that interpolates the fp64 quantile at the four Chebyshev nodes of
// the segment, solved in x = r 2^-18 (well conditioned) and scaled to r exactly (powers of
// two), then rounded to fp32.  Deterministic host arithmetic: every engine and process
// uploads the same bits.
static int nd32_tab_upload()
{
    std::vector<float> t(4 * (size_t)ND32_N, 0.0f);
    const double PI = 3.14159265358979323846;
    for (int i = 0; i < ND32_N; ++i) {
        const int e = ND32_EMIN + (i >> ND32_S), top = i & ((1 << ND32_S) - 1);
        if (e >= 126) continue;   // uf >= 0.5 (rounded up): z = 0
        double xk[4], yk[4];
        for (int k = 0; k < 4; ++k) {
            xk[k] = 0.5 * (1.0 + std::cos(PI * (2 * k + 1) / 8.0));
            const double m = (double)top * (double)(1 << ND32_SHIFT) + xk[k] * (double)(1 << ND32_SHIFT);
            yk[k] = host_ndtri_lower(std::ldexp(1.0 + m * 0x1p-23, e - 127));
        }
        double A[4][5];   // Vandermonde in x, Gaussian elimination with partial pivoting
        for (int k = 0; k < 4; ++k) {
            double v = 1.0;
            for (int j = 0; j < 4; ++j) {
                A[k][j] = v;
                v *= xk[k];
            }
            A[k][4] = yk[k];
        }
        for (int col = 0; col < 4; ++col) {
            int piv = col;
            for (int r = col + 1; r < 4; ++r)
                if (std::fabs(A[r][col]) > std::fabs(A[piv][col])) piv = r;
            for (int j = 0; j < 5; ++j) std::swap(A[col][j], A[piv][j]);
            for (int r = 0; r < 4; ++r) {
                if (r == col) continue;
                const double f = A[r][col] / A[col][col];
                for (int j = col; j < 5; ++j) A[r][j] -= f * A[col][j];
            }
        }
        for (int j = 0; j < 4; ++j) t[4 * (size_t)i + j] = (float)std::ldexp(A[j][4] / A[j][j], -ND32_SHIFT * j);
    }
    return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_nd32_tab), t.data(), t.size() * sizeof(float)),
                     "hipMemcpyToSymbol(g_nd32_tab)");
}

// the table of log_tab / exp_tab / ndtri64 (g_pv_tab) on `device`: the same host values
// for every engine and process, so every kernel's fp64 PV agrees bit for bit
static int pv_tab_upload(int device)
{
    double lt[PV_TAB];
    for (int i = 0; i < LOG_TAB; ++i) {
        const double c = 1.0 + (i + 0.5) * (1.0 / LOG_TAB);
        lt[2 * i] = 1.0 / c;
        lt[2 * i + 1] = std::log(c);
    }
    for (int i = 0; i < EXP_TAB; ++i) lt[EXP_OFF + i] = std::exp2(i * (1.0 / EXP_TAB));
    for (int q = 0; q < NDTRI_PIECES; ++q) {
        lt[NDTRI_OFF + NDTRI_STRIDE * q] = NDTRI_CENTER[q];
        for (int i = 0; i <= NDTRI_DEG; ++i) lt[NDTRI_OFF + NDTRI_STRIDE * q + 1 + i] = NDTRI_COEF[q][i];
    }
    if (int rc = hip_check(hipSetDevice(device), "hipSetDevice")) return rc;
    if (int rc = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_pv_tab), lt, sizeof lt), "hipMemcpyToSymbol(g_pv_tab)")) return rc;
    return nd32_tab_upload();
}

int tmh_engine_create(const tmh_params* p, const tmh_clock* clock, int device, struct tmh_engine** out)
{
    if (!p || !clock || !out) return fail(TMH_E_INVAL, "NULL argument to tmh_engine_create");
    if (p->cc_mode != TMH_CC_FAITHFUL && p->cc_mode != TMH_CC_MARKOV)
        return fail(TMH_E_INVAL, "bad cc_mode %d", p->cc_mode);
    if (p->rng_mode != TMH_RNG_KEYED && p->rng_mode != TMH_RNG_INJECTED)
        return fail(TMH_E_INVAL, "bad rng_mode %d", p->rng_mode);
    if (p->precision != TMH_FP32 && p->precision != TMH_FP64)
        return fail(TMH_E_INVAL, "bad precision %d", p->precision);
    if (p->kernel_path < TMH_PATH_AUTO || p->kernel_path > TMH_PATH_TIME_PARALLEL)
        return fail(TMH_E_INVAL, "bad kernel_path %d", p->kernel_path);
    if (clock->n_shifts < 0 || clock->n_shifts > 8) return fail(TMH_E_INVAL, "bad n_shifts %d", clock->n_shifts);
    // the time-parallel path needs every draw keyed by step, the reference's
    // memoryless (faithful) hourly draw, and whole-minute UTC offsets
    const bool tp_ok = p->rng_mode == TMH_RNG_KEYED && whole_minutes(*clock);
    int path = p->kernel_path == TMH_PATH_AUTO ? (tp_ok ? TMH_PATH_TIME_PARALLEL : TMH_PATH_SEQUENTIAL)
                                               : p->kernel_path;
    if (path == TMH_PATH_TIME_PARALLEL && !tp_ok)
        return fail(TMH_E_INVAL, "kernel_path time-parallel needs keyed rng and whole-minute offsets");
    int ndev = 0;
    if (int rc = hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return rc;
    if (device < 0 || device >= ndev) return fail(TMH_E_INVAL, "device %d out of range (%d devices)", device, ndev);
    tmh_engine* e = new (std::nothrow) tmh_engine;
    if (!e) return fail(TMH_E_NOMEM, "out of host memory");
    if (const char* co = std::getenv("TMH_EXP_COST_ORDER")) e->cost_order = std::atoi(co) != 0;
    // the 8-lane walk's throughput variant from this many walk rows (tests force it on small batches)
    if (const char* tp = std::getenv("TMH_WALK_TP_ROWS")) e->walk_tp_rows = (uint32_t)std::strtoul(tp, nullptr, 10);
    // the markov walk's precomputed Student-t quantiles up to this batch size (tests force either path)
    if (const char* mp = std::getenv("TMH_MK_PRE_MAX")) e->mk_pre_max = (uint32_t)std::strtoul(mp, nullptr, 10);
    KParams& k = e->kp;
    memset(&k, 0, sizeof k);
    k.cc_mode = p->cc_mode;
    k.rng_mode = p->rng_mode;
    k.with_pv = p->with_pv;
    k.precision = p->precision;
    k.seed = p->seed;
    memcpy(k.shapes, p->shapes, sizeof k.shapes);
    memcpy(k.is_t, p->shape_is_t, sizeof k.is_t);
    memcpy(k.edges, p->edges, sizeof k.edges);
    memcpy(k.module, p->module, sizeof k.module);
    memcpy(k.inverter, p->inverter, sizeof k.inverter);
    // cloud_cover_binary.py:35-40 — Python-float constants, bit-exact (host libm pow == CPython's)
    const double omb = 1.0 - 1.66;
    k.alpha = pow(1e6, omb);
    k.delta = pow(0.1e3, omb) - k.alpha;
    k.expo = 1.0 / omb;
    k.sqrt09 = sqrt(0.9);
    k.sqrt6 = sqrt(0.1 * 60);
    k.temp_air = p->site[6];
    k.wind = p->site[7];
    k.tmod_k = std::exp(k.module[TMH_MOD_TEMP_A] + k.module[TMH_MOD_TEMP_B] * k.wind);   // sapm_celltemp factor
    {   // fp32 constants of the PV chain (pv_power_f)
        PVF& f = k.pvf;
        const double* m = k.module;
        const double* iv = k.inverter;
        const double nkq = m[TMH_MOD_N] * (1.38066e-23 / 1.60218e-19) * 0.693147180559945309;   // x ln 2: log2(Ee)
        const double vdco = iv[2];
        const double a1 = iv[1] * iv[5], a0 = iv[1] * (1.0 - iv[5] * vdco);   // A = Pdco (1 + C1 (vmp - Vdco))
        const double b1 = iv[3] * iv[6], b0 = iv[3] * (1.0 - iv[6] * vdco);   // B = Pso (1 + C2 (vmp - Vdco))
        const double c1 = iv[4] * iv[7], c0 = iv[4] * (1.0 - iv[7] * vdco);   // C = C0 (1 + C3 (vmp - Vdco))
        f.tk = (float)(k.tmod_k + m[TMH_MOD_TEMP_DT] * 1e-3);
        f.temp_air = (float)k.temp_air;
        f.fd = (float)m[TMH_MOD_FD];
        f.nmbvmp = (float)(-m[TMH_MOD_MBVMP]);
        f.bvmpo1 = (float)(m[TMH_MOD_BVMPO] + m[TMH_MOD_MBVMP]);
        f.nkq = (float)nkq;
        f.nkq273 = (float)(nkq * 273.15);
        f.impo_c0 = (float)(m[TMH_MOD_IMPO] * m[TMH_MOD_C0]);
        f.impo_c1 = (float)(m[TMH_MOD_IMPO] * m[TMH_MOD_C1]);
        f.aimp = (float)m[TMH_MOD_AIMP];
        f.vmpo = (float)m[TMH_MOD_VMPO];
        f.c2ns = (float)(m[TMH_MOD_C2] * m[TMH_MOD_NS]);
        f.c3ns = (float)(m[TMH_MOD_C3] * m[TMH_MOD_NS]);
        f.paco = (float)iv[0];
        f.pso = (float)iv[3];
        f.ab1 = (float)(a1 - b1);
        f.ab0 = (float)(a0 - b0);
        f.b1 = (float)b1;
        f.b0 = (float)b0;
        f.c1 = (float)c1;
        f.c0 = (float)c0;
        f.pacoc = (float)(iv[0] > 0.0 ? iv[0] : 0.0);
        f.eps0 = (float)(k.sqrt6 * 0.001);
        f.eps1 = (float)(k.sqrt6 * (0.0015 * 8));
        if (f.eps0 != EPS0F || f.eps1 != EPS1F) {   // the fp32 kernels' literals (second_body)
            delete e;
            return fail(TMH_E_INVAL, "fp32 noise-scale literals differ from the host's (%a, %a)", (double)f.eps0,
                        (double)f.eps1);
        }
        PV64& d = k.pv64;   // the same forms in fp64 (ln, not log2: pv_power_d's log is natural)
        d.tk = k.tmod_k + m[TMH_MOD_TEMP_DT] * 1e-3;
        d.temp_air = k.temp_air;
        d.fd = m[TMH_MOD_FD];
        d.nmbvmp = -m[TMH_MOD_MBVMP];
        d.bvmpo1 = m[TMH_MOD_BVMPO] + m[TMH_MOD_MBVMP];
        d.nkq = m[TMH_MOD_N] * 1.38066e-23 / 1.60218e-19;
        d.impo_c0 = m[TMH_MOD_IMPO] * m[TMH_MOD_C0];
        d.impo_c1 = m[TMH_MOD_IMPO] * m[TMH_MOD_C1];
        d.aimp0 = 1.0 - 25.0 * m[TMH_MOD_AIMP];
        d.aimp = m[TMH_MOD_AIMP];
        d.vmpo = m[TMH_MOD_VMPO];
        d.c2ns = m[TMH_MOD_C2] * m[TMH_MOD_NS];
        d.c3ns = m[TMH_MOD_C3] * m[TMH_MOD_NS];
        d.paco = iv[0];
        d.pso = iv[3];
        d.ab1 = a1 - b1;
        d.ab0 = a0 - b0;
        d.b1 = b1;
        d.b0 = b0;
        d.c1 = c1;
        d.c0 = c0;
        d.pnt = -fabs(iv[8]);
    }
    memcpy(e->gp.site, p->site, sizeof e->gp.site);
    memcpy(e->gp.linke, p->linke, sizeof e->gp.linke);
    memcpy(e->gp.module, p->module, sizeof e->gp.module);
    e->gp.clock = *clock;
    DrawParams& d = e->dp;
    memset(&d, 0, sizeof d);
    d.seed = k.seed;
    d.alpha = k.alpha;
    d.delta = k.delta;
    d.expo = k.expo;
    d.sqrt09 = k.sqrt09;
    {   // the candidates' cloud-length range (x at u = 1 and u = 0), for the walk's doomed-call test
        const double xa = pow(k.alpha, k.expo), xb = pow(k.alpha + k.delta, k.expo);
        d.x_lo = std::min(xa, xb);
        d.x_hi = std::max(xa, xb);
    }
    int fb = 0;   // bin of a fresh generator: searchsorted(edges, 1.0)
    while (fb < 5 && p->edges[fb] < 1.0) ++fb;
    d.fb_is_t = p->shape_is_t[fb];
    d.fb_k = d.fb_is_t ? p->shapes[fb][3] : p->shapes[fb][2];
    d.fb_scale = p->shapes[fb][1];
    d.fb_loc = p->shapes[fb][0];
    d.fb_bin = fb;
    d.markov = p->cc_mode == TMH_CC_MARKOV;
    if (int rc = pv_tab_upload(device)) {
        delete e;
        return rc;
    }
    e->device = device;
    e->path = path;
    e->local_step0 = clock->local0;
    for (int i = 0; i < clock->n_shifts; ++i)
        if (clock->shift_step[i] <= 0) e->local_step0 += clock->shift_delta[i];
    *out = e;
    return TMH_OK;
}

int tmh_set_clock(struct tmh_engine* eng, const tmh_clock* clock)
{
    if (!eng || !clock) return fail(TMH_E_INVAL, "NULL engine/clock");
    if (clock->n_shifts < 0 || clock->n_shifts > 8) return fail(TMH_E_INVAL, "bad n_shifts %d", clock->n_shifts);
    if (clock->utc0 != eng->gp.clock.utc0) return fail(TMH_E_INVAL, "tmh_set_clock: utc0 differs (steps renumbered)");
    if (eng->path == TMH_PATH_TIME_PARALLEL && !whole_minutes(*clock))
        return fail(TMH_E_INVAL, "tmh_set_clock: the time-parallel path needs whole-minute offsets");
    eng->gp.clock = *clock;
    return TMH_OK;
}

int tmh_engine_destroy(struct tmh_engine* eng)
{
    delete eng;
    return TMH_OK;
}

int tmh_engine_path(const struct tmh_engine* eng) { return eng ? eng->path : TMH_E_INVAL; }

int tmh_engine_last_expand(const struct tmh_engine* eng) { return eng ? eng->last_expand : TMH_E_INVAL; }

int tmh_set_shape_tables(struct tmh_engine* eng, const double* shapes, const int32_t* is_t, uint32_t n_chains)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    if (shapes && n_chains == 0) return fail(TMH_E_INVAL, "per-chain shape tables with n_chains 0");
    if ((uintptr_t)shapes & 15) return fail(TMH_E_INVAL, "shape tables must be 16-byte aligned (staged as 16-B loads)");
    eng->kp.tab = eng->dp.tab = shapes;
    eng->kp.tab_t = eng->dp.tab_t = shapes ? is_t : nullptr;
    eng->n_tab = shapes ? n_chains : 0;
    return TMH_OK;
}

int tmh_set_sites(struct tmh_engine* eng, const double* sites, const double* linke, uint32_t n_chains)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    if (sites && n_chains == 0) return fail(TMH_E_INVAL, "per-chain sites with n_chains 0");
    eng->kp.sites = sites;
    eng->kp.site_linke = sites ? linke : nullptr;
    eng->n_sites = sites ? n_chains : 0;
    return TMH_OK;
}

static int check_tables(const tmh_engine* eng, uint32_t n_chains)
{
    if (eng->kp.ids) n_chains = std::max(n_chains, eng->kp.ids_n);
    if (eng->kp.tab && n_chains > eng->n_tab)
        return fail(TMH_E_INVAL, "batch of %u chains exceeds the %u per-chain shape tables", n_chains, eng->n_tab);
    if (eng->kp.sites && n_chains > eng->n_sites)
        return fail(TMH_E_INVAL, "batch of %u chains exceeds the %u per-chain sites", n_chains, eng->n_sites);
    return TMH_OK;
}

int tmh_set_walk_chains_per_row(struct tmh_engine* eng, uint32_t chains_per_row)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    if (chains_per_row > 64) return fail(TMH_E_INVAL, "chains_per_row %u > 64", chains_per_row);
    eng->walk_cpr = chains_per_row ? chains_per_row : 1;
    return TMH_OK;
}

int tmh_set_walk_lanes(struct tmh_engine* eng, uint32_t lanes)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    if (lanes != 0 && lanes != 4 && lanes != 8 && lanes != 16) return fail(TMH_E_INVAL, "walk lanes %u: 4, 8 or 16", lanes);
    eng->walk_lanes = lanes;
    return TMH_OK;
}

int tmh_set_walk_order(struct tmh_engine* eng, int on)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    eng->walk_order = on != 0;
    return TMH_OK;
}

int tmh_stream_create_cus(uint32_t cu_first, uint32_t cu_count, void** stream)
{
    if (!stream) return fail(TMH_E_INVAL, "NULL stream out");
    *stream = nullptr;
    hipStream_t s = nullptr;
    if (cu_count == 0) {
        if (int rc = hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate")) return rc;
        *stream = s;
        return TMH_OK;
    }
    int dev = 0, ncu = 0;
    if (int rc = hip_check(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (int rc = hip_check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "CU count")) return rc;
    if ((uint64_t)cu_first + cu_count > (uint64_t)ncu)
        return fail(TMH_E_INVAL, "CU range %u + %u past the device's %d CUs", cu_first, cu_count, ncu);
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (uint32_t i = cu_first; i < cu_first + cu_count; ++i) mask[i >> 5] |= 1u << (i & 31);
    if (int rc = hip_check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask"))
        return rc;
    *stream = s;
    return TMH_OK;
}

int tmh_stream_destroy(void* stream)
{
    if (!stream) return TMH_OK;
    return hip_check(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
}

int tmh_set_chain_ids(struct tmh_engine* eng, const uint32_t* ids, uint32_t n_full)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    if (ids && n_full == 0) return fail(TMH_E_INVAL, "chain ids with n_full 0");
    eng->kp.ids = eng->dp.ids = ids;
    eng->kp.ids_n = ids ? n_full : 0;
    return TMH_OK;
}

int tmh_live_chains(struct tmh_engine* eng, const void* state, uint32_t n_chains, const uint32_t* ids_in,
                    uint32_t* ids_out, uint32_t* n_live, void* stream)
{
    if (!eng || !state || !ids_out || !n_live) return fail(TMH_E_INVAL, "NULL engine/state/ids_out/n_live");
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    hipLaunchKernelGGL(live_chains_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                       make_view(const_cast<void*>(state), n_chains), n_chains, ids_in, ids_out, n_live);
    return hip_check(hipGetLastError(), "live_chains_kernel launch");
}

int tmh_state_move(struct tmh_engine* eng, const void* src, uint32_t n_src, void* dst, uint32_t n_dst,
                   const uint32_t* map, const uint32_t* count, uint32_t cap, int scatter, void* stream)
{
    if (!eng || !src || !dst || !map || !count) return fail(TMH_E_INVAL, "NULL engine/src/dst/map/count");
    if (cap > (scatter ? n_src : n_dst)) return fail(TMH_E_INVAL, "cap %u exceeds the moved-to/from slots", cap);
    if (cap == 0) return TMH_OK;
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    hipLaunchKernelGGL(state_move_kernel, dim3((cap + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       make_view(const_cast<void*>(src), n_src), make_view(dst, n_dst), map, count, cap, scatter);
    return hip_check(hipGetLastError(), "state_move_kernel launch");
}

int tmh_test_set_segment_capacity(uint32_t cap, uint32_t pool_chunks)
{
    if (cap % 16) return fail(TMH_E_INVAL, "segment capacity %u is not a multiple of 16", cap);
    g_cap_override = cap;
    g_pool_override = pool_chunks;
    return TMH_OK;
}

int tmh_profile_enable(struct tmh_engine* eng, int on)
{
    if (!eng) return fail(TMH_E_INVAL, "NULL engine");
    eng->profiling = on != 0;
    return TMH_OK;
}

int tmh_profile_read(struct tmh_engine* eng, int kernel, double* total_ms, int* launches)
{
    if (!eng || !total_ms || kernel < 0 || kernel >= TMH_K_COUNT) return fail(TMH_E_INVAL, "bad profile_read args");
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    double t = 0.0;
    int n = 0;
    for (auto& p : eng->prof[kernel]) {
        if (int rc = hip_check(hipEventSynchronize(p.second), "hipEventSynchronize")) return rc;
        float ms = 0.f;
        if (int rc = hip_check(hipEventElapsedTime(&ms, p.first, p.second), "hipEventElapsedTime")) return rc;
        t += ms;
        ++n;
        eng->pool.push_back(p.first);
        eng->pool.push_back(p.second);
    }
    eng->prof[kernel].clear();
    *total_ms = t;
    if (launches) *launches = n;
    return TMH_OK;
}

int tmh_init(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, const tmh_ustream* inj,
             void* stream)
{
    if (!eng || !state) return fail(TMH_E_INVAL, "NULL engine/state");
    if (n_chains == 0) return TMH_OK;
    if (eng->kp.rng_mode == TMH_RNG_INJECTED && (!inj || !inj->u || inj->stride < inj->len))
        return fail(TMH_E_INVAL, "injected mode needs a stream with stride >= len");
    if (int rc = check_tables(eng, n_chains)) return rc;
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    int64_t sod = eng->local_step0 % 86400;   // the constructor time (step 0)
    if (sod < 0) sod += 86400;
    const double hf = ((int)((sod / 60) % 60) + (int)(sod % 60) / 60.0) / 60.0;
    StateView v = make_view(state, n_chains);
    InjView iv{inj ? inj->u : nullptr, inj ? inj->stride : 0, inj ? inj->len : 0};
    dim3 grid((n_chains + 255) / 256), block(256);
    hipStream_t s = (hipStream_t)stream;
    if (eng->kp.rng_mode == TMH_RNG_KEYED)
    {
        hipLaunchKernelGGL(init_variates_kernel, dim3(grid.x, 10), block, 0, s, eng->kp, v, chain0, n_chains, hf);
        hipLaunchKernelGGL(init_kernel<TMH_RNG_KEYED>, grid, block, 0, s, eng->kp, v, chain0, n_chains, hf, iv);
    }
    else
        hipLaunchKernelGGL(init_kernel<TMH_RNG_INJECTED>, grid, block, 0, s, eng->kp, v, chain0, n_chains, hf, iv);
    return hip_check(hipGetLastError(), "init_kernel launch");
}

int tmh_plan(struct tmh_engine* eng, int64_t step0, uint32_t n_steps, void* plan, void* stream)
{
    if (!eng || !plan) return fail(TMH_E_INVAL, "NULL engine/plan");
    if (n_steps == 0) return TMH_OK;
    if (step0 < 0 || step0 + (int64_t)n_steps > (int64_t)INT_MAX - (1 << 20))
        return fail(TMH_E_INVAL, "step window [%lld, +%u) outside [0, 2^31 - 2^20)", (long long)step0, n_steps);
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    PlanView pv;
    plan_layout(n_steps, plan, &pv);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(geom_kernel, dim3((n_steps + 255) / 256), dim3(256), 0, s, eng->gp, step0, n_steps, pv.tab64,
                       pv.tab32, pv.sun);
    hipLaunchKernelGGL(group_kind_kernel, dim3((n_steps / 4 + 255) / 256 + 1), dim3(256), 0, s, step0, n_steps, pv.tab32,
                       pv.tab64);
    if (eng->cost_order)   // the expansion reads the tile order only then
        hipLaunchKernelGGL(block_order_kernel, dim3(1), dim3(1024), 0, s, pv.tab32, step0, n_steps, pv.bperm);
    hipLaunchKernelGGL(events_kernel, dim3(1), dim3(1024), 0, s, pv.tab32, step0, n_steps, eng->gp.clock.utc0,
                       pv.events, ev_cap(n_steps), pv.n_events);
    const uint32_t nb = nblk_of(n_steps);
    hipLaunchKernelGGL(desc_kernel, dim3((nb + 1 + 255) / 256), dim3(256), 0, s, step0, n_steps, eng->gp.clock.utc0,
                       pv.events, pv.n_events, pv.desc, nb);
    return hip_check(hipGetLastError(), "plan kernels launch");
}

enum { PH_DRAWS = 1, PH_SEGMENTS = 4, PH_WALK = PH_DRAWS | PH_SEGMENTS, PH_EXPAND = 2, PH_COMMIT = 8, PH_ALL = 15,
       PH_MINUTES = 16, PH_NO_MINUTES = 32 };

static int step_phases(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
                       uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
                       const void* plan, void* scratch, size_t scratch_bytes, void* stream, int phases,
                       PrevView prev = PrevView{nullptr, nullptr})
{
    if (!eng || !state || !plan) return fail(TMH_E_INVAL, "NULL engine/state/plan");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    if (step0 < 0 || step0 + (int64_t)n_steps > (int64_t)INT_MAX - (1 << 20))
        return fail(TMH_E_INVAL, "step window [%lld, +%u) outside [0, 2^31 - 2^20)", (long long)step0, n_steps);
    if ((n_chains + 255) / 256 > 65535) return fail(TMH_E_INVAL, "n_chains %u > 16,776,960 per call", n_chains);
    if ((phases & PH_EXPAND) && eng->kp.rng_mode == TMH_RNG_INJECTED && (!inj || !inj->u || inj->stride < inj->len))
        return fail(TMH_E_INVAL, "injected mode needs a stream with stride >= len");
    if (trace && (trace->csi || trace->pv || trace->meter || trace->residual || trace->covered) &&
        trace->ld < n_chains)
        return fail(TMH_E_INVAL, "trace ld %llu < n_chains %u", (unsigned long long)trace->ld, n_chains);
    if (stats && stats->hist && (stats->n_bins == 0 || stats->n_bins > 16384 || !(stats->hi > stats->lo)))
        return fail(TMH_E_INVAL, "bad histogram spec (n_bins %u in [1,16384], hi > lo)", stats->n_bins);
    if (int rc = check_tables(eng, n_chains)) return rc;
    const bool tp = eng->path == TMH_PATH_TIME_PARALLEL;
    if (tp && (!scratch || scratch_bytes < tmh_engine_scratch_bytes(eng, n_chains, n_steps)))
        return fail(TMH_E_INVAL, "scratch too small: %zu < %zu", scratch_bytes, tmh_engine_scratch_bytes(eng, n_chains, n_steps));
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    PlanView pv;
    plan_layout(n_steps, (void*)plan, &pv);
    StateView v = make_view(state, n_chains);
    InjView iv{inj ? inj->u : nullptr, inj ? inj->stride : 0, inj ? inj->len : 0};
    TraceView tv{};
    if (trace) tv = TraceView{trace->csi, trace->pv, trace->meter, trace->residual, trace->covered, trace->ld};
    StatsView sv{};
    size_t lds = 0;
    if (stats) {
        sv.hist = stats->hist;
        sv.n_bins = stats->hist ? stats->n_bins : 0;
        sv.lo = stats->lo;
        sv.scale = stats->hist ? stats->n_bins / (stats->hi - stats->lo) : 0.0;
        sv.scale_f = (float)sv.scale;
        sv.off_f = (float)(-sv.lo * sv.scale);
        if (stats->hist) {   // hist_bin: the fp32 bin position's error bound, in bins
            const double rmax = std::max({9001.0 + std::fabs(eng->kp.inverter[0]), std::fabs(stats->lo), std::fabs(stats->hi)});
            const double err = std::ldexp(sv.scale * (2.0 * rmax + std::fabs(stats->lo)) + stats->n_bins, -24);
            sv.bin64 = err > 1e-3 ? 1u : 0u;
        }
        sv.acc = stats->chain_acc;
        lds = stats->hist ? (size_t)stats->n_bins * 4 : 0;
    }
    hipStream_t s = (hipStream_t)stream;
    const bool f64 = eng->kp.precision == TMH_FP64, keyed = eng->kp.rng_mode == TMH_RNG_KEYED;
    if (!tp) {   // sequential path: one kernel, run by the expand phase
        if (!(phases & PH_EXPAND)) return TMH_OK;
        dim3 grid((n_chains + 255) / 256), block(256);
#define LAUNCH(R, M)                                                                                                 \
    hipLaunchKernelGGL((chain_kernel<R, M>), grid, block, lds, s, eng->kp, v, chain0, n_chains, step0, n_steps,      \
                       pv.tab64, pv.tab32, pv.sun, iv, tv, sv)
        if (f64 && keyed) LAUNCH(double, TMH_RNG_KEYED);
        else if (f64) LAUNCH(double, TMH_RNG_INJECTED);
        else if (keyed) LAUNCH(float, TMH_RNG_KEYED);
        else LAUNCH(float, TMH_RNG_INJECTED);
#undef LAUNCH
        return hip_check(hipGetLastError(), "chain_kernel launch");
    }
    SegView sg;
    scratch_layout(n_chains, n_steps, scratch, &sg, f64 ? 8 : 4);
    {   // fixed-point scale of the statistics: |a window's sum| <= (9,000 + max(Paco, 0)) W x n_steps < 2^62 / 2^k
        const double bound = (9000.0 + std::max(eng->kp.inverter[0], 0.0) + 1.0) * (double)n_steps;
        const int k = 62 - (int)std::ceil(std::log2(bound));
        sg.fx_scale = std::ldexp(1.0, k);
        sg.fx_inv = std::ldexp(1.0, -k);
    }
    const uint32_t cb = (n_chains + 255) / 256;
    const int64_t utc0 = eng->gp.clock.utc0;
    hipEvent_t t_step = phases == PH_ALL ? eng->mark(s) : nullptr;
    if (phases & PH_DRAWS) {
        // the walk rows' order, read by the candidate table's layout and by the walk: computed
        // here (tmh_set_walk_order before a window's draws), so the walk uses the order its
        // window's draws were made with whatever the engine's flag says when it runs
        const bool mk_pre = eng->dp.markov && n_chains <= eng->mk_pre_max;
        hipLaunchKernelGGL(event_draws_kernel, dim3(sg.evcap, cb), dim3(256), 0, s, eng->dp, eng->kp, mk_pre, chain0, n_chains, n_steps,
                           pv.events, pv.n_events, sg.evd, eng->walk_order ? nullptr : sg.order,
                           eng->walk_order ? nullptr : sg.rank);
        if (eng->dp.markov)
            hipLaunchKernelGGL(markov_cc_kernel, dim3(cb), dim3(256), 0, s, eng->kp, mk_pre, v, chain0, n_chains, n_steps,
                               pv.events, pv.n_events, sg.evd, prev);
        if (eng->walk_order)
        {
            const uint32_t tiles = (n_chains + ORDER_TILE - 1) / ORDER_TILE;
            if (tiles <= WALK_RANK_TILES)   // small batches (latency-bound on the construction stream): the rank sort
                hipLaunchKernelGGL(walk_rank_kernel, dim3(tiles * (ORDER_TILE / ORDER_EPB)), dim3(256), 0, s, v, n_chains,
                                   sg, prev);
            else
                hipLaunchKernelGGL(walk_order_kernel, dim3(tiles), dim3(1024), 0, s, v, n_chains, sg, prev);
        }
        hipEvent_t t_cand = eng->mark(s);
        {   // candidates + the window's minute draws (+ counter resets), one launch
            const int64_t fmh = first_minute_host(utc0, step0);
            const uint32_t nm = fmh < (int64_t)n_steps ? (uint32_t)((n_steps - 1 - fmh) / 60 + 1) : 0;
            const uint32_t ny = sg.kcap + nm;   // rows; the kernel strides over y past 65,535 (long windows)
            const dim3 grid(cb, std::min(ny, 65535u));
            const BlockDesc* de = pv.desc + nblk_of(n_steps);
            if (f64)
                hipLaunchKernelGGL(draws_tail_kernel<double>, grid, dim3(256), 0, s, eng->dp, v, chain0, n_chains, step0,
                                   n_steps, fmh, ny, pv.tab64, pv.events, pv.n_events, de, sg, prev);
            else
                hipLaunchKernelGGL(draws_tail_kernel<float>, grid, dim3(256), 0, s, eng->dp, v, chain0, n_chains, step0,
                                   n_steps, fmh, ny, pv.tab64, pv.events, pv.n_events, de, sg, prev);
        }
        eng->close(TMH_K_CANDIDATES, t_cand, s);
        if (int rc = hip_check(hipGetLastError(), "draws kernels launch")) return rc;
    }
    if (phases & PH_SEGMENTS) {
    hipEvent_t t_seg = eng->mark(s);
    // groups of walk_lanes lanes, 16 per workgroup (16 G threads, 16 x WALK_CAND candidate slots in LDS)
    const uint32_t rows = (uint32_t)(((uint64_t)n_chains + eng->walk_cpr - 1) / eng->walk_cpr);
    const uint32_t G = eng->walk_lanes ? eng->walk_lanes : (n_chains > WALK_AUTO_SMALL ? 4u : 16u);
    const uint32_t gpw = 16;   // groups (chains) per workgroup
    const dim3 wg((rows + gpw - 1) / gpw), wt(gpw * G);
    const size_t wlds = gpw * WALK_CAND * sizeof(double);
#define WALK(Q, GG, ...)                                                                                          \
    hipLaunchKernelGGL((segments_kernel<Q, GG, ##__VA_ARGS__>), wg, wt, wlds, s, eng->dp, v, chain0, n_chains, step0, \
                       n_steps, eng->gp.clock, pv.events, pv.n_events, sg, prev)
    const bool q = rows < n_chains;   // groups take queued chains
    if (G == 4) { if (q) WALK(true, 4); else WALK(false, 4); }
    else if (G == 8) { if (q) WALK(true, 8); else if (rows >= eng->walk_tp_rows) WALK(false, 8, true); else WALK(false, 8); }
    else { if (q) WALK(true, 16); else WALK(false, 16); }
#undef WALK
    hipLaunchKernelGGL(overflow_settle_kernel, dim3(cb), dim3(256), 0, s, n_chains, sg);
    hipLaunchKernelGGL(block_rec_kernel, dim3(cb, (sg.nblk + BREC_G - 1) / BREC_G), dim3(256), 0, s, n_chains, step0, sg);
    eng->close(TMH_K_SEGMENTS, t_seg, s);
    if (int rc = hip_check(hipGetLastError(), "segments kernel launch")) return rc;
    }
    if (phases & PH_EXPAND) {
    hipEvent_t t_exp = eng->mark(s);
    const bool no_stats = !sv.hist && !sv.acc;
    int out = (no_stats && tv.pv && tv.meter && tv.residual && !tv.csi && !tv.covered) ? OUT_TRACE3
                    : (!tv.pv && !tv.meter && !tv.residual && !tv.csi && !tv.covered) ? OUT_STATS
                                                                                      : OUT_ANY;
    const size_t hist_bins = stats && stats->hist ? stats->n_bins : 0;
    // x = time blocks, y = chain blocks; LDS: the histogram (16-bit bin pairs or bins)
    auto exp_grid = [&](uint32_t wg, uint32_t tpw) { return dim3((sg.nblk + tpw - 1) / tpw, (n_chains + wg - 1) / wg); };
    // the tiles in cost order (block_order_kernel's plan permutation; TMH_EXP_COST_ORDER=1, A/B only)
    const uint32_t* bperm = eng->cost_order ? pv.bperm : nullptr;
    auto exp_lds = [&](bool pack) { return pack ? (hist_bins + 1) / 2 * 4 : hist_bins * 4; };
    if (out == OUT_TRACE3 && tv.ld * (f64 ? 8u : 4u) * BLOCK_STEPS >= (1ull << 31))   // one block's rows: one buffer range
        return fail(TMH_E_INVAL, "trace ld %llu too large (a 128-step block of rows must stay under 2 GiB)",
                    (unsigned long long)tv.ld);
#define LAUNCH(R, O, S)                                                                                            \
    hipLaunchKernelGGL((expand_kernel<R, O, S>),                                                                   \
                       exp_grid(exp_wg<R, O, S>(), exp_tpw<R, O, S>()), dim3(exp_wg<R, O, S>()),                 \
                       exp_lds(exp_hist_pack<R, O, S>()), s,                                                      \
                       eng->kp, eng->dp, v, chain0, n_chains, step0, n_steps,   \
                       utc0, pv.tab64, pv.tab32, pv.sun, pv.events, pv.n_events, pv.desc, sg, tv, sv, bperm)
#ifndef TMH_SITES_STATS
#define TMH_SITES_STATS 1   // per-chain sites: the statistics-only instantiation (0: OUT_ANY for every output, A/B)
#endif
    // fp32 kernels and a histogram spec their fp32 binning cannot resolve (StatsView::bin64):
    // the OUT_B64 instantiations bin in fp64 (no per-second branch in the others)
    const bool b64 = !f64 && sv.hist && sv.bin64;
    if (eng->kp.sites) {   // per-chain sites: statistics only (C5), or any output
        if (!TMH_SITES_STATS && out == OUT_STATS) out = OUT_ANY;
        if (f64) {
            if (out == OUT_STATS) LAUNCH(double, OUT_STATS, true);
            else LAUNCH(double, OUT_ANY, true);
        } else if (b64) {
            if (out == OUT_STATS) LAUNCH(float, OUT_STATS | OUT_B64, true);
            else LAUNCH(float, OUT_ANY | OUT_B64, true);
        } else {
            if (out == OUT_STATS) LAUNCH(float, OUT_STATS, true);
            else LAUNCH(float, OUT_ANY, true);
        }
    } else if (f64) {
        if (out == OUT_TRACE3) LAUNCH(double, OUT_TRACE3, false);
        else if (out == OUT_STATS) LAUNCH(double, OUT_STATS, false);
        else LAUNCH(double, OUT_ANY, false);
    } else if (b64) {
        if (out == OUT_STATS) LAUNCH(float, OUT_STATS | OUT_B64, false);
        else LAUNCH(float, OUT_ANY | OUT_B64, false);
    } else {
        if (out == OUT_TRACE3) LAUNCH(float, OUT_TRACE3, false);
        else if (out == OUT_STATS) LAUNCH(float, OUT_STATS, false);
        else LAUNCH(float, OUT_ANY, false);
    }
#undef LAUNCH
    eng->last_expand = (eng->kp.sites ? ((out == OUT_STATS ? TMH_OUT_STATS : TMH_OUT_ANY) | TMH_OUT_SITES) : out) |
                       (f64 ? TMH_OUT_FP64 : 0);
    eng->close(TMH_K_EXPAND, t_exp, s);
    if (int rc = hip_check(hipGetLastError(), "expand_kernel launch")) return rc;
    }
    if (!(phases & PH_COMMIT)) return TMH_OK;
    if (!f64 && eng->kp.with_pv) {   // the fp32 guard-band seconds, in fp64
        // one wave per FIX_RPW records, one workgroup per group of the record capacity (up to
        // 65,535, grid-stride past it: C3): the groups past the count exit at once.  (A grid
        // sized for ~1.3e-3 records per (chain, block) left a quarter of the C2 workgroups two
        // groups in a row -- 2.0e-3 are recorded, ~1 flagged second each, diagnostic run r05 --
        // and the kernel two redo latencies long.)
        const uint32_t gx = (uint32_t)std::min<uint64_t>(65535, ((uint64_t)sg.fixcap + FIX_RPW - 1) / FIX_RPW);
        if (eng->kp.sites)
            hipLaunchKernelGGL(fixup_kernel<true>, dim3(gx), dim3(64), 0, s, eng->kp, eng->dp, v, chain0, n_chains, step0,
                               n_steps, utc0, pv.tab64, pv.tab32, pv.sun, pv.events, pv.n_events, pv.desc, sg, tv, sv);
        else
            hipLaunchKernelGGL(fixup_kernel<false>, dim3(gx), dim3(64), 0, s, eng->kp, eng->dp, v, chain0, n_chains, step0,
                               n_steps, utc0, pv.tab64, pv.tab32, pv.sun, pv.events, pv.n_events, pv.desc, sg, tv, sv);
        if (int rc = hip_check(hipGetLastError(), "fixup_kernel launch")) return rc;
    }
    const MinuteCtx mc{eng->dp, chain0, step0, first_minute_host(utc0, step0), pv.events, 0, pv.tab64};
    const uint32_t acc_n = eng->kp.ids ? eng->kp.ids_n : 0u;
    if (f64)
        hipLaunchKernelGGL(commit_kernel<double>, dim3(cb), dim3(256), 0, s, v, n_chains, sg, sv, mc, pv.n_events,
                           pv.desc + nblk_of(n_steps), eng->dp.markov, eng->dp.ids, acc_n);
    else
        hipLaunchKernelGGL(commit_kernel<float>, dim3(cb), dim3(256), 0, s, v, n_chains, sg, sv, mc, pv.n_events,
                           pv.desc + nblk_of(n_steps), eng->dp.markov, eng->dp.ids, acc_n);
    eng->close(TMH_K_STEP, t_step, s);
    return hip_check(hipGetLastError(), "commit_kernel launch");
}

int tmh_step(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
             uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
             const void* plan, void* scratch, size_t scratch_bytes, void* stream)
{
    return step_phases(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, plan, scratch, scratch_bytes,
                       stream, PH_ALL);
}

int tmh_walk(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
             uint32_t n_steps, const void* plan, void* scratch, size_t scratch_bytes, void* stream)
{
    return step_phases(eng, state, chain0, n_chains, step0, n_steps, nullptr, nullptr, nullptr, plan, scratch,
                       scratch_bytes, stream, PH_WALK);
}

int tmh_walk_part(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
                  uint32_t n_steps, const void* plan, void* scratch, size_t scratch_bytes, const void* prev_scratch,
                  uint32_t prev_n_steps, int parts, void* stream)
{
    if (parts & ~(TMH_WALK_DRAWS | TMH_WALK_SEGMENTS)) return fail(TMH_E_INVAL, "bad walk parts %d", parts);
    if (eng && eng->path != TMH_PATH_TIME_PARALLEL) return fail(TMH_E_INVAL, "tmh_walk_part needs the time-parallel path");
    PrevView prev{nullptr, nullptr};
    if (prev_scratch) {
        SegView ps;
        scratch_layout(n_chains, prev_n_steps, const_cast<void*>(prev_scratch), &ps, tmh_engine_scratch_rbytes(eng));
        prev = PrevView{ps.status, ps.end_p1};
    }
    const int ph = ((parts & TMH_WALK_DRAWS) ? PH_DRAWS : 0) | ((parts & TMH_WALK_SEGMENTS) ? PH_SEGMENTS : 0);
    return step_phases(eng, state, chain0, n_chains, step0, n_steps, nullptr, nullptr, nullptr, plan, scratch,
                       scratch_bytes, stream, ph, prev);
}

int tmh_expand(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
               uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
               const void* plan, void* scratch, size_t scratch_bytes, void* stream)
{
    return step_phases(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, plan, scratch, scratch_bytes,
                       stream, PH_EXPAND | PH_COMMIT);
}

int tmh_expand_part(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
                    uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
                    const void* plan, void* scratch, size_t scratch_bytes, int parts, void* stream)
{
    if (parts & ~(TMH_EXPAND_KERNEL | TMH_EXPAND_COMMIT | TMH_EXPAND_MINUTES | TMH_EXPAND_NO_MINUTES))
        return fail(TMH_E_INVAL, "bad expand parts %d", parts);
    if (eng && eng->path != TMH_PATH_TIME_PARALLEL && parts != (TMH_EXPAND_KERNEL | TMH_EXPAND_COMMIT))
        return fail(TMH_E_INVAL, "tmh_expand_part in parts needs the time-parallel path");
    const int ph = ((parts & TMH_EXPAND_KERNEL) ? PH_EXPAND : 0) | ((parts & TMH_EXPAND_COMMIT) ? PH_COMMIT : 0) |
                   ((parts & TMH_EXPAND_MINUTES) ? PH_MINUTES : 0) | ((parts & TMH_EXPAND_NO_MINUTES) ? PH_NO_MINUTES : 0);
    return step_phases(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, plan, scratch, scratch_bytes,
                       stream, ph);
}

int tmh_run(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
            uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
            void* workspace, size_t workspace_bytes, void* stream)
{
    if (!eng || !state) return fail(TMH_E_INVAL, "NULL engine/state");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    const size_t pb = tmh_plan_bytes(n_steps);
    const size_t need = eng->path == TMH_PATH_TIME_PARALLEL ? pb + tmh_engine_scratch_bytes(eng, n_chains, n_steps) : pb;
    if (!workspace || workspace_bytes < need)
        return fail(TMH_E_INVAL, "workspace too small: %zu < %zu", workspace_bytes, need);
    if (int rc = tmh_plan(eng, step0, n_steps, workspace, stream)) return rc;
    return tmh_step(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, workspace,
                    (char*)workspace + pb, workspace_bytes - pb, stream);
}

#ifdef TMH_WALK_PROF
// diagnostic build only: the walk's per-wave section cycles (see g_walk_prof)
int tmh_debug_walk_prof(unsigned long long* host, uint32_t waves)
{
    if (waves > (uint32_t)WPROF_WAVES) waves = WPROF_WAVES;
    return hip_check(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_walk_prof), (size_t)waves * (WPROF_N + 2) * 8, 0,
                                         hipMemcpyDeviceToHost), "walk prof");
}
#endif

int tmh_probe(int fn, double a, const double* x, double* out, uint32_t n, void* stream)
{
    if (fn >= 11 && fn <= 14) {   // the table functions need the tables on the current device
        int dev = 0;
        if (int rc = hip_check(hipGetDevice(&dev), "hipGetDevice")) return rc;
        if (int rc = pv_tab_upload(dev)) return rc;
    }
    if (!x || !out) return fail(TMH_E_INVAL, "NULL probe buffers");
    if (n == 0) return TMH_OK;
    hipLaunchKernelGGL(probe_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, a, x, out, n);
    return hip_check(hipGetLastError(), "probe_kernel launch");
}

}  // extern "C"
