// libtmhpvsim — MI355X (gfx950) batched simulator of tmhpvsim's clear-sky-index
// chain + PV model behind the C-ABI of include/tmhpvsim.h.
//
// Two execution paths over the same model code (tmh_model.h):
//
//  * sequential (chain_kernel): one work-item per chain runs the seconds of a
//    window in order, exactly like ClearskyindexModel.next.  Used for injected
//    uniform streams (the reference's consumption order is data dependent) and
//    for the markov cloud-cover mode.
//
//  * time-parallel (keyed Philox, faithful mode): the only data-dependent
//    sequential process is CloudCoverBinary's cloud/clear segment sequence.
//      P1 segments_kernel: one wavefront per chain walks from segment end to
//         segment end (next_cloud with the sigma scan spread over 64 lanes and
//         a butterfly argmin) and records each segment as (first clear step,
//         next call step).
//      P2 expand_kernel: one work-item per (chain, block of 256 seconds)
//         rebuilds the sampler state at the block start from the keyed draws
//         of the last boundary events (block descriptors), then runs the fused
//         per-second body.  Every draw is keyed by (chain, step), so P2's
//         outputs are bit-identical to the sequential kernel's.
//
// Per-window, chain-independent work (wall-clock fractions, boundary flags,
// solar geometry, clear-sky irradiance, SAPM spectral/AOI factors, the boundary
// event list and block descriptors) is built once by the plan kernels and read
// by the chain kernels with wave-uniform loads.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "tmh_math.h"
#include "tmh_model.h"
#include "tmhpvsim.h"

using namespace tmh;

namespace {

constexpr int BLOCK_STEPS = 256;   // seconds per P2 work-item

struct BlockDesc {                 // as of the step before the block start; -1 = none in the window
    int32_t q0, q1;                // minute-draw indices of the last two minute boundaries
    int32_t h0, h1;                // event indices of the last two hour boundaries
    int32_t cd0, cd1;              // last two clear_day pushes: event index * 2 + (0 day | 1 hour push)
    int32_t evi;                   // first event index at or after the block start
    int32_t pad;
};

struct SegView {                   // P1 -> P2 scratch
    int2* rec;                     // [n][cap] (first uncovered step, next call step), global steps
    uint32_t cap;
    uint32_t* count;               // [n]
    int32_t* fault;                // [n] window-relative fault step (INT_MAX = none)
    uint32_t* status;              // [n] status after the window
    double* end_p1;                // [4][n] cc before/after, ws before/after at window end
    double* end_p2;                // [6][n] clear_day, cloudy_noise, clear_noise pairs at window end
    double* part;                  // [4][nblk][n] stats partials
    uint32_t nblk;
    double* evd;                   // [ev_cap][4][n] per boundary event: cc, ws, clear_day (day), clear_day (hour)
    double* mind;                  // [nmin][2][n] per minute boundary: cloudy noise, clear noise
    uint32_t evcap, nmin;
};

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
// ClearskyindexModel.__init__ (clearskyindexmodel.py:57-99)
template <int RNG>
__global__ __launch_bounds__(256) void init_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
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
        dr.chain = chain0 + c;
    } else {
        dr.u = inj.u + (size_t)c * inj.stride;
        dr.len = inj.len;
    }
    double u[12];
    for (int d = 0; d < 12; ++d) u[d] = dr.one(ch, 0, TAG_INIT, (uint32_t)(d >> 1), d & 1);
    ch.s.b[S_CC] = draw_cc(kp, ch, u[0]);
    ch.s.a[S_CC] = draw_cc(kp, ch, u[1]);
    ch.s.b[S_CLEAR_DAY] = normal(u[2], 0.99, 0.08);
    ch.s.a[S_CLEAR_DAY] = normal(u[3], 0.99, 0.08);
    bool name_error = false;
    for (int j = 0; j < 2; ++j) {   // :68-82
        const double cc = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
        double v;
        if (cc < 6.0 / 8) v = normal(u[4 + j], 0.6784, 0.2046);
        else if (cc < 7.0 / 8) {
            name_error = true;       // gamma.pdf(x, ...) with x undefined (:80)
            break;
        } else v = gammaincinv(3.5624, u[4 + j]) * 0.0867 + 0.0;
        if (j == 0) ch.s.b[S_CLOUDY_HOUR] = v;
        else ch.s.a[S_CLOUDY_HOUR] = v;
    }
    if (name_error) {
        if constexpr (RNG == TMH_RNG_INJECTED) ch.pos = ch.pos < 4 ? ch.pos : 4;   // raised after 4 draws
        ch.status = TMH_CHAIN_NAMEERROR_INIT;
        store_chain(st, c, ch);
        return;
    }
    const double cch = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
    ch.s.b[S_CLOUDY_NOISE] = scaled_noise(kp, u[6], 0.01, 0.003, cch);
    ch.s.a[S_CLOUDY_NOISE] = scaled_noise(kp, u[7], 0.01, 0.003, cch);
    ch.s.b[S_CLEAR_NOISE] = scaled_noise(kp, u[8], 0.001, 0.0015, cch);
    ch.s.a[S_CLEAR_NOISE] = scaled_noise(kp, u[9], 0.001, 0.0015, cch);
    ch.s.b[S_WS] = 2.14 * gammaincinv(2.69, u[10]);
    ch.s.a[S_WS] = 2.14 * gammaincinv(2.69, u[11]);
    // CloudCoverBinary(cc.interpolate(0), ws.interpolate(0)) (:98-99)
    const double h0 = interp(ch.s.b[S_CC], ch.s.a[S_CC], 0.0);
    const double h = 0.95 < h0 ? 0.95 : h0;
    const double ws = interp(ch.s.b[S_WS], ch.s.a[S_WS], 0.0);
    double* sc = sig_c(st, c);
    double* sl = sig_l(st, c);
    reset_sigma(sc, sl, ch, h);
    const uint32_t f = next_cloud<RNG>(kp, sc, sl, ch, dr, h, ws, TAG_INIT_CLOUD);
    if (!f) {
        const double us = dr.one(ch, 0, TAG_INIT_SEC, 0, 0);
        ch.sec = (int32_t)((ch.cl + ch.clr) * us);   // cloud_cover_binary.py:68
    }
    if (f && !ch.status) ch.status = f;
    store_chain(st, c, ch);
}

// ------------------------------------------------------------ plan kernels
__global__ __launch_bounds__(256) void geom_kernel(GParams gp, int64_t step0, uint32_t n, double* tab64,
                                                   float* tab32)
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
    const double lat = gp.site[0], lon = gp.site[1], alt = gp.site[2], tilt = gp.site[3], saz = gp.site[4],
                 albedo = gp.site[5];
    int doy, leap;
    civil_doy(dn, doy, leap);
    const double pres = 100.0 * pow((44331.514 - alt) / 11880.516, 1.0 / 0.1902632);   // alt2pres
    double zen, azen, az;
    solpos(ck.utc0 + s, lat, lon, pres, 12.0, zen, azen, az);
    const double ct = cos(rad(zen));
    g[G_COSZ] = ct;
    g[G_CSIMAX] = 27.21 * exp(-114 * ct) + 1.665 * exp(-4.494 * ct) + 1.08;
    const double dni_extra = extra_rad(doy, 1366.1);
    const double am_rel =
        azen <= 90.0 ? 1.0 / (cos(rad(azen)) + 0.50572 * pow(6.07995 + (90.0 - azen), -1.6364)) : NAN;
    const double am_abs = am_rel * pres / 101325.0;
    const double tl = linke_at(gp.linke, doy, leap);
    const double fh1 = exp(-alt / 8000.0), fh2 = exp(-alt / 1250.0);
    const double cg1 = 5.09e-05 * alt + 0.868, cg2 = 3.92e-05 * alt + 0.0387;
    double cz = cosd(azen);
    cz = cz > 0.0 ? cz : 0.0;
    const double gexp = exp(-cg2 * am_abs * (fh1 + fh2 * (tl - 1.0)));
    const double gmax = isnan(gexp) ? 0.0 : (gexp > 0.0 ? gexp : 0.0);
    g[G_GHICS] = cg1 * dni_extra * cz * tl / tl * gmax;
    const double I0 = extra_rad(doy, 1370.0);
    const double czd = cosd(zen);
    g[G_I0] = I0;
    g[G_I0H] = I0 * (czd > 0.065 ? czd : 0.065);
    double amd = zen <= 90.0 ? 1.0 / (cos(rad(zen)) + 0.15 * pow(93.885 - zen, -1.253)) : NAN;
    amd = amd * 101325.0 / 101325.0;
    amd = amd < 12.0 ? amd : (isnan(amd) ? amd : 12.0);
    g[G_AM] = amd;
    g[G_KNC] = 0.866 - 0.122 * amd + 0.0121 * (amd * amd) - 0.000653 * pow(amd, 3.0) + 0.000014 * pow(amd, 4.0);
    g[G_DISCOK] = zen > 87.0 ? 0.0 : 1.0;
    double proj = cosd(tilt) * cosd(azen) + sind(tilt) * sind(azen) * cosd(az - saz);
    proj = proj > 1.0 ? 1.0 : (proj < -1.0 ? -1.0 : proj);
    const double cos_tt = proj > 0.0 ? proj : 0.0;
    const double czs = cosd(azen);
    g[G_RB] = cos_tt / (czs > 0.01745 ? czs : 0.01745);
    g[G_DNIEXTRA] = dni_extra;
    g[G_TERM2] = 0.5 * (1.0 + cosd(tilt));
    g[G_GFAC] = albedo * (1.0 - cos(rad(tilt))) * 0.5;
    const double aoi = deg(acos(proj));
    g[G_COSAOI] = cos(rad(aoi));
    const double* m = gp.module;
    double f1 = (((m[4] * am_abs + m[3]) * am_abs + m[2]) * am_abs + m[1]) * am_abs + m[0];
    f1 = isnan(f1) ? 0.0 : f1;
    g[G_F1] = f1 > 0.0 ? f1 : 0.0;
    double f2 = ((((m[10] * aoi + m[9]) * aoi + m[8]) * aoi + m[7]) * aoi + m[6]) * aoi + m[5];
    f2 = f2 > 0.0 ? f2 : 0.0;
    if (aoi < 0.0) f2 = 0.0;
    g[G_F2] = f2;
    if (g[G_GHICS] == 0.0) fl |= FL_NIGHT;   // ghi_cs = 0 -> pv = 0 whatever the csi
    g[G_FLAGS] = (double)fl;
    double* o64 = tab64 + (size_t)j * ROW;
    float* o32 = tab32 + (size_t)j * ROW;
    for (int i = 0; i < ROW; ++i) {
        o64[i] = g[i];
        o32[i] = (float)g[i];
    }
    o32[G_FLAGS] = __uint_as_float(fl);
    o32[G_I0H] = (float)(1.0 / g[G_I0H]);   // fp32 path multiplies by reciprocals
    o32[G_DNIEXTRA] = (float)(1.0 / g[G_DNIEXTRA]);
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
        if (__float_as_uint(tab32[j * ROW + G_FLAGS]) & (FL_DAY | FL_HOUR)) ++c;
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
        const uint32_t fl = __float_as_uint(tab32[j * ROW + G_FLAGS]) & (FL_DAY | FL_HOUR);
        if (fl) {
            if (o < cap) events[o] = make_int2((int)(step0 + (int64_t)j), (int)fl);
            ++o;
        }
    }
    if (t == 1023) *n_events = cnt[1023];
}

__device__ __forceinline__ uint32_t ev_cap_dev(uint32_t n_steps) { return n_steps / 1800 + 64; }

__device__ __forceinline__ int64_t first_minute(int64_t utc0, int64_t W0)
{   // window-relative step of the first candidate minute boundary (UTC second 0)
    return (60 - (((utc0 + W0) % 60) + 60) % 60) % 60;
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
    BlockDesc d{-1, -1, -1, -1, -1, -1, 0, 0};
    const int64_t jb = min((int64_t)b * BLOCK_STEPS, (int64_t)n);
    if (jb > 0) {
        const int64_t p = step0 + jb - 1;                  // last step before the block
        const int64_t lo = step0 > 1 ? step0 : 1;          // step 0 is the constructor time
        const int64_t fm = first_minute(utc0, step0);
        const int64_t m0 = p - (((utc0 + p) % 60) + 60) % 60;
        if (m0 >= lo) d.q0 = (int32_t)((m0 - step0 - fm) / 60);
        if (m0 - 60 >= lo) d.q1 = (int32_t)((m0 - 60 - step0 - fm) / 60);
        const int ne = (int)min(*n_events, ev_cap_dev(n));
        int a = 0, z = ne;                                  // last event <= p
        while (a < z) {
            const int mid = (a + z) / 2;
            if (events[mid].x <= p) a = mid + 1;
            else z = mid;
        }
        d.evi = a;
        int nh = 0, ncd = 0;
        for (int i = a - 1; i >= 0 && (nh < 2 || ncd < 2); --i) {
            const int fl = events[i].y;
            if (fl & FL_HOUR) {
                if (nh == 0) d.h0 = i;
                else if (nh == 1) d.h1 = i;
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
    desc[b] = d;
}

// ------------------------------------------------------------ boundary draws
// _next_day / _next_hour draws of every (event, chain): clearskyindexmodel.py:101-107
__global__ __launch_bounds__(256) void event_draws_kernel(DrawParams dp, uint64_t chain0, uint32_t n, uint32_t nsteps,
                                                          const int2* __restrict__ events,
                                                          const uint32_t* __restrict__ n_events, double* evd)
{
    const uint32_t c = blockIdx.y * blockDim.x + threadIdx.x;
    const uint32_t e = blockIdx.x;
    if (c >= n || e >= min(*n_events, ev_cap_dev(nsteps))) return;
    const uint64_t chain = chain0 + c, step = (uint64_t)events[e].x;
    const int fl = events[e].y;
    double* o = evd + (size_t)e * 4 * n + c;
    if (fl & FL_DAY) {
        const U4 u = keyed_block(dp.seed, chain, step, TAG_BOUNDARY, 0);
        o[2 * (size_t)n] = normal(u52(u.x, u.y), 0.99, 0.08);
        o[(size_t)n] = 2.14 * gammaincinv(2.69, u52(u.z, u.w));
    }
    if (fl & FL_HOUR) {
        const U4 u = keyed_block(dp.seed, chain, step, TAG_BOUNDARY, 1);
        o[0] = cc_faithful(dp, u52(u.x, u.y));
        o[3 * (size_t)n] = normal(u52(u.z, u.w), 0.99, 0.08);
    }
}

// _next_min draws of every (minute boundary, chain): clearskyindexmodel.py:86-95,109-111
__global__ __launch_bounds__(256) void minute_draws_kernel(DrawParams dp, StateView st, uint64_t chain0, uint32_t n,
                                                           int64_t W0, uint32_t nsteps, int64_t utc0,
                                                           const double* __restrict__ tab64,
                                                           const int2* __restrict__ events,
                                                           const uint32_t* __restrict__ n_events,
                                                           const double* __restrict__ evd, double* mind)
{
    const uint32_t c = blockIdx.y * blockDim.x + threadIdx.x;
    const uint32_t q = blockIdx.x;
    const int64_t j = first_minute(utc0, W0) + 60 * (int64_t)q;
    if (c >= n || j >= (int64_t)nsteps) return;
    const int64_t step = W0 + j;
    const int ne = (int)min(*n_events, ev_cap_dev(nsteps));
    int a = 0, z = ne;   // last event <= step
    while (a < z) {
        const int mid = (a + z) / 2;
        if (events[mid].x <= step) a = mid + 1;
        else z = mid;
    }
    int h0 = -1, h1 = -1;
    for (int i = a - 1; i >= 0 && h1 < 0; --i)
        if (events[i].y & FL_HOUR) {
            if (h0 < 0) h0 = i;
            else h1 = i;
        }
    double pb, pa;   // cloud cover pair after the hour push of this second
    if (h0 < 0) {
        pb = st.sb[S_CC][c];
        pa = st.sa[S_CC][c];
    } else if (h1 < 0) {
        pb = st.sa[S_CC][c];
        pa = evd[(size_t)h0 * 4 * n + c];
    } else {
        pb = evd[(size_t)h1 * 4 * n + c];
        pa = evd[(size_t)h0 * 4 * n + c];
    }
    const double cc = interp(pb, pa, tab64[(size_t)j * ROW + G_HOURF]);
    const U4 u = keyed_block(dp.seed, chain0 + c, (uint64_t)step, TAG_BOUNDARY, 2);
    mind[(size_t)q * 2 * n + c] = normal(u52(u.x, u.y), 1.0, dp.sqrt09 * (0.01 + 0.003 * 8 * cc));
    mind[((size_t)q * 2 + 1) * n + c] = normal(u52(u.z, u.w), 1.0, dp.sqrt09 * (0.001 + 0.0015 * 8 * cc));
}

// cc / clear_day / noise pairs described by `d`, from the draw tables (start = window start)
__device__ __forceinline__ void samplers_at(const BlockDesc& d, const SegView& sg, uint32_t n, uint32_t c, Samp& s)
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
    if (d.q0 >= 0) {
        for (int k = 0; k < 2; ++k) {
            const int si = k == 0 ? S_CLOUDY_NOISE : S_CLEAR_NOISE;
            const double na = sg.mind[((size_t)d.q0 * 2 + k) * n + c];
            s.b[si] = d.q1 >= 0 ? sg.mind[((size_t)d.q1 * 2 + k) * n + c] : s.a[si];
            s.a[si] = na;
        }
    }
}

// ------------------------------------------------------------ sequential kernel
// Advance chains [0, n) over steps [step0, step0 + nsteps), one lane per chain.
template <typename R, int RNG>
__global__ __launch_bounds__(256) void chain_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                    int64_t step0, uint32_t nsteps,
                                                    const double* __restrict__ tab64,
                                                    const float* __restrict__ tab32, InjView inj, TraceView tr,
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
        dr.chain = chain0 + c;
    } else {
        dr.u = inj.u + (size_t)c * inj.stride;
        dr.len = inj.len;
    }
    const uint64_t chain = chain0 + c;
    double* sc = live ? sig_c(st, c) : nullptr;
    double* sl = live ? sig_l(st, c) : nullptr;
    FSamp<R> fs;
    to_real(fs, ch.s);
    Acc acc{0.0, 0.0, 0.0, -INFINITY};
    for (uint32_t j = 0; j < nsteps; ++j) {
        const uint64_t step = (uint64_t)(step0 + j);
        const float* r32 = tab32 + (size_t)j * ROW;
        const double* r64 = tab64 + (size_t)j * ROW;
        const uint32_t fl = __float_as_uint(r32[G_FLAGS]);
        R row[ROW];
#pragma unroll
        for (int i = 0; i < ROW; ++i) row[i] = sizeof(R) == 8 ? (R)r64[i] : (R)r32[i];
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
                    push(ch.s, S_CC, draw_cc(kp, ch, u0));
                    push(ch.s, S_CLEAR_DAY, normal(u1, 0.99, 0.08));
                }
                if (fl & FL_MIN) {                     // _next_min
                    dr.two(ch, step, TAG_BOUNDARY, 2, u0, u1);
                    const double cc = interp(ch.s.b[S_CC], ch.s.a[S_CC], hf);
                    push(ch.s, S_CLOUDY_NOISE, scaled_noise(kp, u0, 0.01, 0.003, cc));
                    push(ch.s, S_CLEAR_NOISE, scaled_noise(kp, u1, 0.001, 0.0015, cc));
                }
                to_real(fs, ch.s);
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
                // keyed: one Philox block per step pair, 32-bit words;
                // the meter is its own process in the reference: always keyed
                const U4 pb = keyed_block(kp.seed, chain, (uint64_t)step >> 1, TAG_STEP2, 0);
                const bool odd = step & 1;
                double ue = u32d(odd ? pb.z : pb.x);
                const double um = u32d(odd ? pb.w : pb.y);
                if constexpr (RNG == TMH_RNG_INJECTED) ue = dr.one(ch, step, TAG_STEP, 0, 0);
                if (ch.status == 0) {
                    const bool covered = ch.sec < ch.t1;
                    cov = covered ? 1 : 0;
                    second_body<R>(kp, row, fl, fs, covered, ue, um, csi, pv, meter, res);
                    ok = true;
                }
            }
        }
        if (live) emit<R>(tr, sv, lds_hist, (uint64_t)j * tr.ld + c, cov, csi, pv, meter, res, acc, ok);
    }
    if (live) {
        store_chain(st, c, ch);
        if (sv.acc) {
            sv.acc[c] += acc.pv;
            sv.acc[(size_t)n + c] += acc.m;
            sv.acc[2 * (size_t)n + c] += acc.r;
            sv.acc[3 * (size_t)n + c] = fmax(sv.acc[3 * (size_t)n + c], acc.mx);
        }
    }
    if (sv.hist) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x)
            if (lds_hist[i]) atomicAdd((unsigned long long*)&sv.hist[i], (unsigned long long)lds_hist[i]);
    }
}

// ------------------------------------------------------------ P1: segments
// One wavefront per chain (keyed, faithful): jump from segment end to segment
// end.  The chain's sigma arrays stay in VGPRs (64 lanes x NCH chunks) for the
// whole window; hour/day fractions come from clock arithmetic (scalar).
// hour / day fractions of step s (clearskyindexmodel.py:114-116) from the window's
// local second-of-day at W0: 32-bit, wave-uniform arithmetic
struct WinClock {
    int32_t sod0;            // local second of day at W0
    int32_t n;               // shifts inside the window
    int32_t step[8], delta[8];   // window-relative shift steps and sizes
};

__device__ __forceinline__ WinClock win_clock(const tmh_clock& ck, int64_t W0)
{
    WinClock w;
    const int64_t l0 = local_at(ck, W0);
    w.sod0 = (int32_t)(l0 - floordiv(l0, 86400) * 86400);
    w.n = 0;
    for (int i = 0; i < ck.n_shifts && i < 8; ++i)
        if (ck.shift_step[i] > W0) {
            w.step[w.n] = (int32_t)(ck.shift_step[i] - W0);
            w.delta[w.n] = ck.shift_delta[i];
            ++w.n;
        }
    return w;
}

__device__ __forceinline__ void fractions_at(const WinClock& w, int32_t j, double& hour_f, double& day_f)
{
    int32_t sod = w.sod0 + j;
    for (int i = 0; i < w.n; ++i)
        if (j >= w.step[i]) sod += w.delta[i];
    sod %= 86400;
    if (sod < 0) sod += 86400;
    const int hour = sod / 3600, minute = (sod / 60) % 60, second = sod % 60;
    double min_f;
    clock_fractions(hour, minute, second, min_f, hour_f, day_f);
}

__global__ __launch_bounds__(256) void segments_kernel(DrawParams dp, StateView st, uint64_t chain0, uint32_t n,
                                                       int64_t W0, uint32_t nsteps, tmh_clock ck,
                                                       const int2* __restrict__ events,
                                                       const uint32_t* __restrict__ n_events, SegView sg)
{
    const int lane = threadIdx.x & 63;
    const uint32_t c = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (c >= n) return;   // whole wave
    const uint64_t chain = chain0 + c;
    const int64_t W1 = W0 + nsteps;
    uint32_t status = st.status[c];
    double ccb = st.sb[S_CC][c], cca = st.sa[S_CC][c], wsb = st.sb[S_WS][c], wsa = st.sa[S_WS][c];
    int32_t fault = INT_MAX;
    uint32_t nrec = 0;
    if (status == 0) {
        double cl = st.cl[c], clr = st.clr[c];
        int L = st.L[c];
        const int32_t sec = st.sec[c];
        double vc[NCH], vl[NCH];
        double* gsc = sig_c(st, c);
        double* gsl = sig_l(st, c);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const int k = ch * 64 + lane;
            vc[ch] = k < L ? gsc[k] : 0.0;
            vl[ch] = k < L ? gsl[k] : 0.0;
        }
        int64_t s_start = W0 - sec;   // step at which sec was 1
        int32_t t1 = ceil_thr(cl), t2 = ceil_thr(cl + clr);
        int64_t e = s_start + t2 - 1;
        int2* rec = sg.rec + (size_t)c * sg.cap;
        if (lane == 0) rec[0] = make_int2((int)(s_start + t1 - 1), (int)e);
        nrec = 1;
        const uint32_t nev = min(*n_events, ev_cap_dev(nsteps));
        uint32_t ev = 0;
        // the next boundary event and its draws, loaded one event ahead of use
        int64_t next_ev = INT64_MAX;
        int ev_fl = 0;
        double ev_cc = 0.0, ev_ws = 0.0;
        auto fetch_event = [&]() {
            if (ev < nev) {
                const int2 r = events[ev];
                next_ev = r.x;
                ev_fl = r.y;
                ev_cc = sg.evd[(size_t)ev * 4 * n + c];
                ev_ws = sg.evd[((size_t)ev * 4 + 1) * n + c];
            } else {
                next_ev = INT64_MAX;
            }
        };
        fetch_event();
        auto apply_events = [&](int64_t upto) {   // _next_day / _next_hour at steps <= upto
            while (next_ev <= upto) {
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
        };
        // try-0 candidates of the next 64 calls (keyed by call number, so they
        // can be drawn before the calls' steps are known)
        uint32_t ncall = st.ncalls[c], kb = ncall;
        double cand_x, cand_u;
        cloud_candidates(dp, chain, kb, lane, cand_x, cand_u);
        const WinClock wck = win_clock(ck, W0);
        while (e < W1) {
            apply_events(e);
            double hf, df;
            fractions_at(wck, (int32_t)(e - W0), hf, df);
            const double hh = interp(ccb, cca, hf);
            const double h = 0.95 < hh ? 0.95 : hh;   // update_parameters
            const double ws = interp(wsb, wsa, df);
            if (ncall - kb >= 64u) {
                kb = ncall;
                cloud_candidates(dp, chain, kb, lane, cand_x, cand_u);
            }
            const int slot = (int)(ncall - kb);
            const double x0 = readlane_f64(cand_x, slot);
            double ncl = x0 / ws, nclr = 0.0;
            uint32_t f = 0;
            if (!next_cloud_fast(vc, vl, L, ncl, 1.0 / h - 1.0, lane, nclr))
                f = next_cloud_regs(dp, vc, vl, gsc, gsl, L, h, ws, chain, ncall, x0, readlane_f64(cand_u, slot), lane,
                                    ncl, nclr);
            ++ncall;
            if (f) {
                status = f;
                fault = (int32_t)(e - W0);
                break;
            }
            cl = ncl;
            clr = nclr;
            t1 = ceil_thr(cl);
            t2 = ceil_thr(cl + clr);
            s_start = e;
            e = s_start + t2 - 1;
            if (nrec >= sg.cap) {
                status = TMH_CHAIN_SEGMENT_OVERFLOW;
                fault = (int32_t)(s_start - W0);
                break;
            }
            if (lane == 0) rec[nrec] = make_int2((int)(s_start + t1 - 1), (int)e);
            ++nrec;
        }
        if (status == 0) apply_events(W1 - 1);   // remaining boundaries of the window
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {   // register chunks back to the state row
            const int k = ch * 64 + lane;
            if (k < L) {
                gsc[k] = vc[ch];
                gsl[k] = vl[ch];
            }
        }
        if (lane == 0) {
            st.sec[c] = (int32_t)(W1 - s_start);   // sec after step W1 - 1
            st.cl[c] = cl;
            st.clr[c] = clr;
            st.L[c] = L;
            st.ncalls[c] = ncall;
        }
    }
    if (lane == 0) {
        sg.count[c] = nrec;
        sg.fault[c] = fault;
        sg.status[c] = status;
        sg.end_p1[c] = ccb;
        sg.end_p1[(size_t)n + c] = cca;
        sg.end_p1[2 * (size_t)n + c] = wsb;
        sg.end_p1[3 * (size_t)n + c] = wsa;
    }
}

// ------------------------------------------------------------ P2: expand
// One work-item per (chain, block of 256 seconds).  The boundary draws come
// from the draw tables, so the per-second loop holds only the R copies of the
// sampler pairs and does no fp64 work in fp32 mode.
template <typename R, int OUT>
__global__ __launch_bounds__(256) void expand_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                     int64_t W0, uint32_t nsteps, int64_t utc0,
                                                     const double* __restrict__ tab64,
                                                     const float* __restrict__ tab32,
                                                     const BlockDesc* __restrict__ desc, SegView sg, TraceView tr,
                                                     StatsView sv)
{
    extern __shared__ uint32_t lds_hist[];
    const uint32_t c = blockIdx.y * blockDim.x + threadIdx.x;   // grid: x = time block, y = chain block
    const uint32_t b = blockIdx.x;
    const bool live = c < n;
    if (sv.hist) {
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x) lds_hist[i] = 0;
        __syncthreads();
    }
    const uint32_t j0 = b * BLOCK_STEPS, j1 = min(j0 + (uint32_t)BLOCK_STEPS, nsteps);
    const uint64_t chain = chain0 + c;
    const int64_t fm = first_minute(utc0, W0);
    Acc acc{0.0, 0.0, 0.0, -INFINITY};
    bool alive = false;
    int32_t fault = INT_MAX;
    int2 seg = make_int2(0, 0);
    const int2* rec = sg.rec + (size_t)(live ? c : 0) * sg.cap;
    uint32_t jr = 0, evi = 0;
    FSamp<R> fs;
    if (live) {
        alive = st.status[c] == 0;
        fault = sg.fault[c];
        Samp s;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            s.b[k] = st.sb[k][c];
            s.a[k] = st.sa[k][c];
        }
        const BlockDesc d = desc[b];
        evi = (uint32_t)d.evi;
        if (alive && b > 0) samplers_at(d, sg, n, c, s);
        to_real(fs, s);
    }
    if (alive) {   // segment containing the block start: first record with next-call step > start
        const int64_t s0 = W0 + j0;
        int lo = 0, hi = (int)sg.count[c] - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((int64_t)rec[mid].y > s0) hi = mid;
            else lo = mid + 1;
        }
        jr = (uint32_t)lo;
        seg = rec[jr];
    }
    const double* evd = sg.evd + c;
    const double* mind = sg.mind + c;
    U4 pair{0, 0, 0, 0};
    bool have_pair = false;
    for (uint32_t j = j0; j < j1; ++j) {
        const int64_t step = W0 + j;
        const float* r32 = tab32 + (size_t)j * ROW;
        const uint32_t fl = __float_as_uint(r32[G_FLAGS]);
        R row[ROW];
#pragma unroll
        for (int i = 0; i < ROW; ++i) row[i] = sizeof(R) == 8 ? (R)tab64[(size_t)j * ROW + i] : (R)r32[i];
        R csi = R(NAN), pv = R(NAN), meter = R(NAN), res = R(NAN);
        uint8_t cov = 255;
        const bool ok = alive && (int32_t)j < fault;
        if (ok) {
            if (fl & (FL_DAY | FL_HOUR)) {            // _next_day, _next_hour
                const size_t eo = (size_t)evi * 4 * n;
                if (fl & FL_DAY) {
                    fs.b[S_CLEAR_DAY] = fs.a[S_CLEAR_DAY];
                    fs.a[S_CLEAR_DAY] = (R)evd[eo + 2 * (size_t)n];
                }
                if (fl & FL_HOUR) {
                    fs.b[S_CC] = fs.a[S_CC];
                    fs.a[S_CC] = (R)evd[eo];
                    fs.b[S_CLEAR_DAY] = fs.a[S_CLEAR_DAY];
                    fs.a[S_CLEAR_DAY] = (R)evd[eo + 3 * (size_t)n];
                }
            }
            if (fl & FL_MIN) {                         // _next_min
                const size_t q = (size_t)((j - fm) / 60);
                fs.b[S_CLOUDY_NOISE] = fs.a[S_CLOUDY_NOISE];
                fs.a[S_CLOUDY_NOISE] = (R)mind[q * 2 * n];
                fs.b[S_CLEAR_NOISE] = fs.a[S_CLEAR_NOISE];
                fs.a[S_CLEAR_NOISE] = (R)mind[(q * 2 + 1) * n];
            }
            while (step >= (int64_t)seg.y) seg = rec[++jr];   // next_cloud happened at seg.y
            const bool covered = step < (int64_t)seg.x;
            cov = covered ? 1 : 0;
            if (!(step & 1) || !have_pair) {   // one Philox block per step pair (uniform branch)
#ifdef TMH_DIAG_NO_RNG   // diagnostic builds only (scripts/diag_variants.sh): cost breakdown
                const uint32_t hsh = (uint32_t)chain * 0x9E3779B9u ^ (uint32_t)step * 0x85EBCA6Bu;
                pair = U4{hsh, hsh >> 3, hsh ^ 0x5555u, hsh >> 5};
#else
                pair = keyed_block(kp.seed, chain, (uint64_t)step >> 1, TAG_STEP2, 0);
#endif
                have_pair = true;
            }
            const bool odd = step & 1;
            second_body<R>(kp, row, fl, fs, covered, u32d(odd ? pair.z : pair.x), u32d(odd ? pair.w : pair.y), csi, pv,
                           meter, res);
        }
        if (fl & (FL_DAY | FL_HOUR)) ++evi;
#ifdef TMH_DIAG_NO_STORE
        if (live && csi == R(-12345))
            emit<R, OUT>(tr, sv, lds_hist, (uint64_t)j * tr.ld + c, cov, csi, pv, meter, res, acc, ok);
#else
        if (live) emit<R, OUT>(tr, sv, lds_hist, (uint64_t)j * tr.ld + c, cov, csi, pv, meter, res, acc, ok);
#endif
    }
    if (live && sv.acc) {
        const size_t o = (size_t)b * n + c, stride = (size_t)sg.nblk * n;
        sg.part[o] = acc.pv;
        sg.part[stride + o] = acc.m;
        sg.part[2 * stride + o] = acc.r;
        sg.part[3 * stride + o] = acc.mx;
    }
    if (sv.hist) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x)
            if (lds_hist[i]) atomicAdd((unsigned long long*)&sv.hist[i], (unsigned long long)lds_hist[i]);
    }
}

// Stats partials -> per-chain accumulators (fixed order: deterministic), then
// the window-end state of P1/P2 -> chain state.
__global__ __launch_bounds__(256) void commit_kernel(StateView st, uint32_t n, SegView sg, StatsView sv,
                                                     const BlockDesc* __restrict__ desc_end)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    if (sv.acc) {
        const size_t stride = (size_t)sg.nblk * n;
        double p = 0.0, m = 0.0, r = 0.0, mx = -INFINITY;
        for (uint32_t b = 0; b < sg.nblk; ++b) {
            const size_t o = (size_t)b * n + c;
            p += sg.part[o];
            m += sg.part[stride + o];
            r += sg.part[2 * stride + o];
            mx = fmax(mx, sg.part[3 * stride + o]);
        }
        sv.acc[c] += p;
        sv.acc[(size_t)n + c] += m;
        sv.acc[2 * (size_t)n + c] += r;
        sv.acc[3 * (size_t)n + c] = fmax(sv.acc[3 * (size_t)n + c], mx);
    }
    if (st.status[c] != 0) return;
    st.status[c] = sg.status[c];
    if (sg.status[c] != 0) return;
    Samp sp;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        sp.b[k] = st.sb[k][c];
        sp.a[k] = st.sa[k][c];
    }
    samplers_at(*desc_end, sg, n, c, sp);
#pragma unroll
    for (int k = 0; k < 5; ++k) {   // cc, clear_day, cloudy_hour (unchanged), noises
        st.sb[k][c] = sp.b[k];
        st.sa[k][c] = sp.a[k];
    }
    st.sb[S_WS][c] = sg.end_p1[2 * (size_t)n + c];
    st.sa[S_WS][c] = sg.end_p1[3 * (size_t)n + c];
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
        case 5: {   // wavefront argmin (first index on ties) of x[wave lanes]; needs full waves
            double dm;
            int km;
            argmin_first(x[i], (int)(i & 63), dm, km);
            v = (double)km;
            break;
        }
        case 6: v = dpp_f64<0x138>(a, x[i]); break;            // wave_shr:1, lane 0 <- a
        case 7: v = readlane_f64(x[i], 63); break;
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

// state field order: sb[6], sa[6], cl, clr, mstate, sec, L, pos, status, ncalls, sigma_cloud, sigma_clear, -, -
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
    v.n = n;
    return v;
}

// plan: tab64 | tab32 | events | n_events | block descriptors
uint32_t ev_cap(uint32_t n_steps) { return n_steps / 1800 + 64; }
uint32_t nblk_of(uint32_t n_steps) { return (n_steps + BLOCK_STEPS - 1) / BLOCK_STEPS; }

struct PlanView {
    double* tab64;
    float* tab32;
    int2* events;
    uint32_t* n_events;
    BlockDesc* desc;
};

size_t plan_layout(uint32_t n_steps, void* base, PlanView* v)
{
    size_t o = 0;
    char* b = (char*)base;
    if (v) v->tab64 = (double*)(b + o);
    o += align_up((size_t)n_steps * ROW * 8);
    if (v) v->tab32 = (float*)(b + o);
    o += align_up((size_t)n_steps * ROW * 4);
    if (v) v->events = (int2*)(b + o);
    o += align_up((size_t)ev_cap(n_steps) * 8);
    if (v) v->n_events = (uint32_t*)(b + o);
    o += ALIGN;
    if (v) v->desc = (BlockDesc*)(b + o);
    o += align_up((size_t)(nblk_of(n_steps) + 1) * sizeof(BlockDesc));
    return o;
}

uint32_t seg_cap(uint32_t n_steps) { return n_steps / 8 + 64; }

size_t scratch_layout(uint32_t n, uint32_t n_steps, void* base, SegView* v)
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
    if (v) v->count = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->fault = (int32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->status = (uint32_t*)(b + o);
    o += align_up((size_t)n * 4);
    if (v) v->end_p1 = (double*)(b + o);
    o += align_up((size_t)n * 4 * 8);
    if (v) v->end_p2 = (double*)(b + o);
    o += align_up((size_t)n * 6 * 8);
    if (v) v->part = (double*)(b + o);
    o += align_up((size_t)n * nblk * 4 * 8);
    const uint32_t evc = ev_cap(n_steps), nmin = n_steps / 60 + 2;
    if (v) {
        v->evcap = evc;
        v->nmin = nmin;
        v->evd = (double*)(b + o);
    }
    o += align_up((size_t)n * evc * 4 * 8);
    if (v) v->mind = (double*)(b + o);
    o += align_up((size_t)n * nmin * 2 * 8);
    return o;
}

}  // namespace

struct tmh_engine {
    KParams kp;
    DrawParams dp;
    GParams gp;
    int device;
    int path;   // resolved kernel path: 1 sequential, 2 time-parallel
    // side stream: the minute draws run beside the segment walk (both need only
    // the event draws); created on first use, never holds device memory
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
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
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
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
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (aux) (void)hipStreamDestroy(aux);
    }
};

extern "C" {

int tmh_abi_version(void) { return TMH_ABI_VERSION; }

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
    return scratch_layout(n_chains, n_steps, nullptr, nullptr);
}

size_t tmh_workspace_bytes(uint32_t n_chains, uint32_t n_steps)
{
    return tmh_plan_bytes(n_steps) + tmh_scratch_bytes(n_chains, n_steps);
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
    bool minutes = ((clock->local0 - clock->utc0) % 60) == 0;
    for (int i = 0; i < clock->n_shifts; ++i) minutes = minutes && (clock->shift_delta[i] % 60) == 0;
    const bool tp_ok = p->rng_mode == TMH_RNG_KEYED && p->cc_mode == TMH_CC_FAITHFUL && minutes;
    int path = p->kernel_path == TMH_PATH_AUTO ? (tp_ok ? TMH_PATH_TIME_PARALLEL : TMH_PATH_SEQUENTIAL)
                                               : p->kernel_path;
    if (path == TMH_PATH_TIME_PARALLEL && !tp_ok)
        return fail(TMH_E_INVAL, "kernel_path time-parallel needs keyed rng, faithful cc mode, whole-minute offsets");
    int ndev = 0;
    if (int rc = hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return rc;
    if (device < 0 || device >= ndev) return fail(TMH_E_INVAL, "device %d out of range (%d devices)", device, ndev);
    tmh_engine* e = new (std::nothrow) tmh_engine;
    if (!e) return fail(TMH_E_NOMEM, "out of host memory");
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
    int fb = 0;   // bin of a fresh generator: searchsorted(edges, 1.0)
    while (fb < 5 && p->edges[fb] < 1.0) ++fb;
    d.fb_is_t = p->shape_is_t[fb];
    d.fb_k = d.fb_is_t ? p->shapes[fb][3] : p->shapes[fb][2];
    d.fb_scale = p->shapes[fb][1];
    d.fb_loc = p->shapes[fb][0];
    e->device = device;
    e->path = path;
    *out = e;
    return TMH_OK;
}

int tmh_engine_destroy(struct tmh_engine* eng)
{
    delete eng;
    return TMH_OK;
}

int tmh_engine_path(const struct tmh_engine* eng) { return eng ? eng->path : TMH_E_INVAL; }

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
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    const tmh_clock& ck = eng->gp.clock;
    int64_t sod = ck.local0 % 86400;
    if (sod < 0) sod += 86400;
    const double hf = ((int)((sod / 60) % 60) + (int)(sod % 60) / 60.0) / 60.0;
    StateView v = make_view(state, n_chains);
    InjView iv{inj ? inj->u : nullptr, inj ? inj->stride : 0, inj ? inj->len : 0};
    dim3 grid((n_chains + 255) / 256), block(256);
    hipStream_t s = (hipStream_t)stream;
    if (eng->kp.rng_mode == TMH_RNG_KEYED)
        hipLaunchKernelGGL(init_kernel<TMH_RNG_KEYED>, grid, block, 0, s, eng->kp, v, chain0, n_chains, hf, iv);
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
                       pv.tab32);
    hipLaunchKernelGGL(events_kernel, dim3(1), dim3(1024), 0, s, pv.tab32, step0, n_steps, eng->gp.clock.utc0,
                       pv.events, ev_cap(n_steps), pv.n_events);
    const uint32_t nb = nblk_of(n_steps);
    hipLaunchKernelGGL(desc_kernel, dim3((nb + 1 + 255) / 256), dim3(256), 0, s, step0, n_steps, eng->gp.clock.utc0,
                       pv.events, pv.n_events, pv.desc, nb);
    return hip_check(hipGetLastError(), "plan kernels launch");
}

int tmh_step(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
             uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
             const void* plan, void* scratch, size_t scratch_bytes, void* stream)
{
    if (!eng || !state || !plan) return fail(TMH_E_INVAL, "NULL engine/state/plan");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    if (step0 < 0 || step0 + (int64_t)n_steps > (int64_t)INT_MAX - (1 << 20))
        return fail(TMH_E_INVAL, "step window [%lld, +%u) outside [0, 2^31 - 2^20)", (long long)step0, n_steps);
    if ((n_chains + 255) / 256 > 65535) return fail(TMH_E_INVAL, "n_chains %u > 16,776,960 per call", n_chains);
    if (eng->kp.rng_mode == TMH_RNG_INJECTED && (!inj || !inj->u || inj->stride < inj->len))
        return fail(TMH_E_INVAL, "injected mode needs a stream with stride >= len");
    if (trace && (trace->csi || trace->pv || trace->meter || trace->residual || trace->covered) &&
        trace->ld < n_chains)
        return fail(TMH_E_INVAL, "trace ld %llu < n_chains %u", (unsigned long long)trace->ld, n_chains);
    if (stats && stats->hist && (stats->n_bins == 0 || stats->n_bins > 16384 || !(stats->hi > stats->lo)))
        return fail(TMH_E_INVAL, "bad histogram spec (n_bins %u in [1,16384], hi > lo)", stats->n_bins);
    const bool tp = eng->path == TMH_PATH_TIME_PARALLEL;
    if (tp && (!scratch || scratch_bytes < tmh_scratch_bytes(n_chains, n_steps)))
        return fail(TMH_E_INVAL, "scratch too small: %zu < %zu", scratch_bytes, tmh_scratch_bytes(n_chains, n_steps));
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
        sv.acc = stats->chain_acc;
        lds = stats->hist ? (size_t)stats->n_bins * 4 : 0;
    }
    hipStream_t s = (hipStream_t)stream;
    const bool f64 = eng->kp.precision == TMH_FP64, keyed = eng->kp.rng_mode == TMH_RNG_KEYED;
    if (!tp) {
        dim3 grid((n_chains + 255) / 256), block(256);
#define LAUNCH(R, M)                                                                                                 \
    hipLaunchKernelGGL((chain_kernel<R, M>), grid, block, lds, s, eng->kp, v, chain0, n_chains, step0, n_steps,      \
                       pv.tab64, pv.tab32, iv, tv, sv)
        if (f64 && keyed) LAUNCH(double, TMH_RNG_KEYED);
        else if (f64) LAUNCH(double, TMH_RNG_INJECTED);
        else if (keyed) LAUNCH(float, TMH_RNG_KEYED);
        else LAUNCH(float, TMH_RNG_INJECTED);
#undef LAUNCH
        return hip_check(hipGetLastError(), "chain_kernel launch");
    }
    SegView sg;
    scratch_layout(n_chains, n_steps, scratch, &sg);
    const uint32_t cb = (n_chains + 255) / 256;
    const int64_t utc0 = eng->gp.clock.utc0;
    if (!eng->aux) {
        if (int rc = hip_check(hipStreamCreateWithFlags(&eng->aux, hipStreamNonBlocking), "hipStreamCreate")) return rc;
        if (int rc = hip_check(hipEventCreateWithFlags(&eng->ev_fork, hipEventDisableTiming), "hipEventCreate"))
            return rc;
        if (int rc = hip_check(hipEventCreateWithFlags(&eng->ev_join, hipEventDisableTiming), "hipEventCreate"))
            return rc;
    }
    hipEvent_t t_step = eng->mark(s);
    hipLaunchKernelGGL(event_draws_kernel, dim3(sg.evcap, cb), dim3(256), 0, s, eng->dp, chain0, n_chains, n_steps,
                       pv.events, pv.n_events, sg.evd);
    // fork: minute draws on the side stream, segment walk on `s`; join before P2
    if (int rc = hip_check(hipEventRecord(eng->ev_fork, s), "hipEventRecord")) return rc;
    if (int rc = hip_check(hipStreamWaitEvent(eng->aux, eng->ev_fork, 0), "hipStreamWaitEvent")) return rc;
    hipEvent_t t_min = eng->mark(eng->aux);
    hipLaunchKernelGGL(minute_draws_kernel, dim3(sg.nmin, cb), dim3(256), 0, eng->aux, eng->dp, v, chain0, n_chains,
                       step0, n_steps, utc0, pv.tab64, pv.events, pv.n_events, sg.evd, sg.mind);
    eng->close(TMH_K_MINUTE_DRAWS, t_min, eng->aux);
    if (int rc = hip_check(hipEventRecord(eng->ev_join, eng->aux), "hipEventRecord")) return rc;
    hipEvent_t t_seg = eng->mark(s);
    hipLaunchKernelGGL(segments_kernel, dim3((n_chains + 3) / 4), dim3(256), 0, s, eng->dp, v, chain0, n_chains,
                       step0, n_steps, eng->gp.clock, pv.events, pv.n_events, sg);
    eng->close(TMH_K_SEGMENTS, t_seg, s);
    if (int rc = hip_check(hipStreamWaitEvent(s, eng->ev_join, 0), "hipStreamWaitEvent")) return rc;
    if (int rc = hip_check(hipGetLastError(), "draws/segments kernels launch")) return rc;
    hipEvent_t t_exp = eng->mark(s);
    dim3 grid2(nblk_of(n_steps), cb);
    const bool no_stats = !sv.hist && !sv.acc;
    const int out = (no_stats && tv.pv && tv.meter && tv.residual && !tv.csi && !tv.covered) ? OUT_TRACE3
                    : (!tv.pv && !tv.meter && !tv.residual && !tv.csi && !tv.covered) ? OUT_STATS
                                                                                      : OUT_ANY;
#define LAUNCH(R, O)                                                                                                 \
    hipLaunchKernelGGL((expand_kernel<R, O>), grid2, dim3(256), lds, s, eng->kp, v, chain0, n_chains, step0, n_steps, \
                       utc0, pv.tab64, pv.tab32, pv.desc, sg, tv, sv)
    if (f64) {
        if (out == OUT_TRACE3) LAUNCH(double, OUT_TRACE3);
        else if (out == OUT_STATS) LAUNCH(double, OUT_STATS);
        else LAUNCH(double, OUT_ANY);
    } else {
        if (out == OUT_TRACE3) LAUNCH(float, OUT_TRACE3);
        else if (out == OUT_STATS) LAUNCH(float, OUT_STATS);
        else LAUNCH(float, OUT_ANY);
    }
#undef LAUNCH
    eng->close(TMH_K_EXPAND, t_exp, s);
    if (int rc = hip_check(hipGetLastError(), "expand_kernel launch")) return rc;
    hipLaunchKernelGGL(commit_kernel, dim3(cb), dim3(256), 0, s, v, n_chains, sg, sv, pv.desc + nblk_of(n_steps));
    eng->close(TMH_K_STEP, t_step, s);
    return hip_check(hipGetLastError(), "commit_kernel launch");
}

int tmh_run(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
            uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
            void* workspace, size_t workspace_bytes, void* stream)
{
    if (!eng || !state) return fail(TMH_E_INVAL, "NULL engine/state");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    const size_t pb = tmh_plan_bytes(n_steps);
    const size_t need = eng->path == TMH_PATH_TIME_PARALLEL ? pb + tmh_scratch_bytes(n_chains, n_steps) : pb;
    if (!workspace || workspace_bytes < need)
        return fail(TMH_E_INVAL, "workspace too small: %zu < %zu", workspace_bytes, need);
    if (int rc = tmh_plan(eng, step0, n_steps, workspace, stream)) return rc;
    return tmh_step(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, workspace,
                    (char*)workspace + pb, workspace_bytes - pb, stream);
}

int tmh_probe(int fn, double a, const double* x, double* out, uint32_t n, void* stream)
{
    if (!x || !out) return fail(TMH_E_INVAL, "NULL probe buffers");
    if (n == 0) return TMH_OK;
    hipLaunchKernelGGL(probe_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, a, x, out, n);
    return hip_check(hipGetLastError(), "probe_kernel launch");
}

}  // extern "C"
