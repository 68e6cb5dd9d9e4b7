// Model pieces shared by every tmhpvsim kernel (gfx950).  Reference lines
// restated are cited at each function (paths relative to tmhpvsim/).
#pragma once
#include <hip/hip_runtime.h>

#include <climits>

#include "tmh_math.h"
#include "tmhpvsim.h"

namespace tmh {

#define CAP TMH_SIGMA_CAP
#define ROW TMH_GEOM_FIELDS

// ------------------------------------------------------------ parameters
// fp32 constants of the PV chain (pvmodel.py:53-80), rounded once on the host
// in the forms pv_power_f evaluates (each an affine map in one variable, so one FMA):
//   tcell = poa (tmod_k + dT / 1000) + temp_air          tk, temp_air
//   Bvmpo = bvmpo + mbvmp (1 - Ee)                        nmbvmp = -mbvmp, bvmpo1 = bvmpo + mbvmp
//   delta log2(Ee) = n k / q (tcell + 273.15) ln(Ee)     nkq = n k / q ln 2, nkq273 = 273.15 nkq
//   A - B, B, C of the SNL inverter, affine in vmp:       (ab1, ab0), (b1, b0), (c1, c0)
// sqrt(0.1 * 60) (0.001 + 0.0015 * 8 cc) of clearskyindexmodel.py:146-147 in fp32: model constants,
// so literals in the kernels (the host checks they equal its PVF::eps0 / eps1)
constexpr double SQRT6 = 2.449489742783178;
constexpr float EPS0F = (float)(SQRT6 * 0.001), EPS1F = (float)(SQRT6 * (0.0015 * 8));
struct PVF {
    // the addends of pv_power_f's affine maps first: the first PVF_VGPR fields can be pinned in
    // VGPRs (a VOP3 FMA reads one SGPR, so a map with two SGPR constants costs a v_mov per use)
    float temp_air, nkq273, impo_c0, bvmpo1, vmpo, ab0, b0, c0;
    float tk, fd, nmbvmp, nkq, impo_c1, aimp, c2ns, c3ns;
    float paco, pso, ab1, b1, c1;
    float pacoc;        // max(Paco, 0): the upper bound of the final clamp
    float eps0, eps1;   // sqrt(6) 0.001, sqrt(6) 0.0015 * 8: the noise scale is eps0 + eps1 cc
};

// fp64 constants of the PV chain, folded on the host like PVF (pv_power_d): the
// products and sums differ from pvmodel.py's order of operations by an ulp or two,
// 1e-16 relative against the fp64 bar of 1e-12.
//   tcell = poa tk + temp_air; Bvmpo = bvmpo1 + nmbvmp Ee; delta = nkq (tcell + 273.15)
//   imp = Ee (impo_c0 + impo_c1 Ee) (aimp0 + aimp tcell); A - B, B, C affine in vmp
struct PV64 {
    double tk, temp_air, fd, nmbvmp, bvmpo1, nkq, impo_c0, impo_c1, aimp0, aimp, vmpo, c2ns, c3ns;
    double paco, pso, ab1, ab0, b1, b0, c1, c0, pnt;   // pnt = -|Pnt| (night tare)
};
constexpr int PV64_N = sizeof(PV64) / 8;

struct KParams {
    int32_t cc_mode, rng_mode, with_pv, precision;
    uint64_t seed;
    double shapes[6][4];
    int32_t is_t[6];
    double edges[6];
    double module[TMH_MOD_COUNT];
    double inverter[TMH_INV_COUNT];
    double alpha, delta, expo, sqrt09, sqrt6;   // cloud_cover_binary.py:35-40, scales
    double temp_air, wind;                      // sapm_celltemp inputs (pvmodel.py:69-70)
    double tmod_k;                              // exp(a + b * wind): constant for the run (wind fixed at 0)
    PVF pvf;                                    // fp32 copies for the fp32 chain
    PV64 pv64;                                  // the fp64 chain's folded constants
    const double* tab;                          // per-chain shape tables [n][6][4] (NULL: shapes)
    const int32_t* tab_t;                       // per-chain Student-t flags [n][6] (NULL: is_t)
    const double* sites;                        // per-chain PV sites [n][8] (NULL: the plan's site)
    const double* site_linke;                   // per-chain monthly Linke turbidity [n][12] (NULL: params)
    const uint32_t* ids;                        // slot -> chain (tmh_set_chain_ids; NULL: slot c is chain c)
    uint32_t ids_n, pad_;                       // chains of the full batch (row count of tables, sites, acc)
};

// The chain in launch slot c (a compacted batch runs only its live chains; its
// keyed draws, tables, sites and statistics stay those of the original chain).
__device__ __forceinline__ uint32_t gid(const uint32_t* ids, uint32_t c) { return ids ? ids[c] : c; }

struct GParams {
    double site[8];
    double linke[12];
    double module[TMH_MOD_COUNT];
    tmh_clock clock;
};

// FL_DISCOK: DISC's zenith test passes (pvlib irradiance.disc max_zenith, the row's
// G_DISCOK as a flag bit, so the fp32 chain tests a scalar instead of a float per lane)
// FL_G_NIGHT / FL_G_DAY (fp32 rows, on the first row of a four-step group of a window whose
// start is on the four-step grid; group_kind_kernel): the group's four seconds are all night,
// or all daylight with DISC valid, and its seconds 1-3 carry no boundary event, so the fp32
// single-site expansion runs the group as straight-line code (expand_tile, FASTG)
enum : uint32_t { FL_DAY = 1, FL_HOUR = 2, FL_MIN = 4, FL_NIGHT = 8, FL_DISCOK = 16, FL_G_NIGHT = 32, FL_G_DAY = 64 };
// clock/geometry table row (TMH_GEOM_FIELDS = 20)
enum {
    G_MINF = 0, G_HOURF = 1, G_DAYF = 2, G_FLAGS = 3, G_COSZ = 4, G_CSIMAX = 5, G_GHICS = 6,
    G_I0H = 7, G_I0 = 8, G_KNC = 9, G_AM = 10, G_F2 = 11, G_RB = 12, G_DNIEXTRA = 13,
    G_TERM2 = 14, G_GFAC = 15, G_COSAOI = 16, G_F1 = 17, G_DISCOK = 18,
    G_LAST = 18,  // DISC's zenith test last: the fp32 single-site kernels read it as FL_DISCOK, so their
                  // scalar loads of a row stop one field early (3 s_loads a second, not 6 around a hole)
    // fp64 rows only (pv_power_d multiplies where pvmodel.py divides): kt = csi GHI_cs / I0h
    // and AI = dni / dni_extra as products, within an ulp or two of the quotients
    G_KTC = 19,     // GHI_cs / I0h
    G_RDNIX = 20    // 1 / dni_extra (field 21 unused: rows of 22 doubles, 16-byte aligned)
};
// fp32 row (ROW32 = 22 floats, the kernels' scalar loads): each clock fraction
// beside its complement 1 - f (rounded in fp32 exactly as the kernels would),
// 8-byte aligned pairs, so an interpolation f a + (1 - f) b is one packed
// multiply on an SGPR pair plus an add; then flags and G_COSZ..G_LAST, i.e. the
// fp64 row's field G_X (X >= FLAGS) sits at G_X + G32.  Kept compact: every
// field is held in SGPRs through the step.
enum { G32_MINF_C = 0, G32_MINF = 1, G32_HOURF_C = 2, G32_HOURF = 3, G32_DAYF_C = 4, G32_DAYF = 5, G32 = 3 };
#define ROW32 22
template <typename R>
constexpr int row_w() { return sizeof(R) == 8 ? ROW : ROW32; }
template <typename R>   // the row as the fp64 field layout (G_FLAGS..G_LAST) sees it
constexpr int row_off() { return sizeof(R) == 8 ? 0 : G32; }

enum { S_CC = 0, S_CLEAR_DAY = 1, S_CLOUDY_HOUR = 2, S_CLOUDY_NOISE = 3, S_CLEAR_NOISE = 4, S_WS = 5 };

// chain state, structure of arrays; sigma arrays chain-major [n][CAP] so the
// wave-cooperative next_cloud scans one chain's arrays with coalesced loads
struct StateView {
    double* sb[6];
    double* sa[6];
    double *cl, *clr, *mstate;
    int32_t *sec, *L;
    uint32_t *pos, *status, *ncalls;
    double *sc, *sl;
    float2* fn[2];   // fp32 mode: the (before, after) cloudy / clear noise pairs the fp32 kernels sample (minute_noise_fast)
    uint32_t n;
};

struct InjView {
    const double* u;
    uint64_t stride, len;
};

struct TraceView {
    void *csi, *pv, *meter, *residual;
    uint8_t* covered;
    uint64_t ld;
};

struct StatsView {
    uint64_t* hist;
    uint32_t n_bins;
    double lo, scale;
    double* acc;
    float scale_f, off_f;   // fp32 kernels' bin position: res scale + off, off = -lo scale
    uint32_t bin64;         // fp32 kernels bin in fp64 (a histogram spec whose fp32 binning error is too large)
};

// the histogram bin of a residual: fp64 kernels (res - lo) scale in fp64; fp32 kernels one
// fp32 FMA and a clamp, no fp64 conversions per second.  That bin position's error is
// below 2^-24 (scale (2 max(|res|, |lo|) + |lo|) + n_bins) bins (the roundings of scale,
// of -lo scale and of the FMA): ~3e-4 of a bin for the default [-300, 9000) W in 4,096
// bins.  The host (step_phases) sets bin64 when that bound exceeds 1e-3 bins (a narrow
// range far from 0, very many bins): such a spec is binned in fp64 like the fp64 kernels
// (a scalar branch per second, taken the same way by every wave).
// B64: bin in fp64 (the fp64 kernels; fp32 kernels built for a bin64 spec, OUT_B64); the
// per-second loops take the choice at compile time, hist_bin_rt (the fixup, the sequential
// kernel) at run time
template <typename R, bool B64 = (sizeof(R) == 8)>
__device__ __forceinline__ int hist_bin(const StatsView& sv, R res)
{
    if constexpr (sizeof(R) == 8 || B64) {
        const double x = ((double)res - sv.lo) * sv.scale;
        return x < 0.0 ? 0 : (x >= (double)(sv.n_bins - 1) ? (int)sv.n_bins - 1 : (int)x);
    } else {
        return (int)__builtin_amdgcn_fmed3f(fmaf((float)res, sv.scale_f, sv.off_f), 0.0f, (float)(sv.n_bins - 1));
    }
}
template <typename R>
__device__ __forceinline__ int hist_bin_rt(const StatsView& sv, R res)
{
    return sv.bin64 ? hist_bin<R, true>(sv, res) : hist_bin<R>(sv, res);
}

struct Samp {
    double b[6], a[6];
};

struct Chain {
    Samp s;
    double cl, clr, mstate;
    int32_t sec, L, t1, t2;
    uint32_t pos, status, ncalls;
};

// ------------------------------------------------------------ rng sources
template <int RNG>
struct Draw;

template <>
struct Draw<TMH_RNG_KEYED> {
    uint64_t seed, chain;
    __device__ __forceinline__ double one(Chain&, uint64_t step, uint32_t tag, uint32_t sub, int half) const
    {
        const U4 b = keyed_block(seed, chain, step, tag, sub);
        return half ? u52(b.z, b.w) : u52(b.x, b.y);
    }
    __device__ __forceinline__ void two(Chain&, uint64_t step, uint32_t tag, uint32_t sub, double& u0,
                                        double& u1) const
    {
        const U4 b = keyed_block(seed, chain, step, tag, sub);
        u0 = u52(b.x, b.y);
        u1 = u52(b.z, b.w);
    }
};

template <>
struct Draw<TMH_RNG_INJECTED> {
    const double* u;
    uint64_t len;
    __device__ __forceinline__ double one(Chain& ch, uint64_t, uint32_t, uint32_t, int) const
    {
        if (ch.pos >= len) {
            if (!ch.status) ch.status = TMH_CHAIN_U_EXHAUSTED;
            return 0.5;
        }
        return u[ch.pos++];
    }
    __device__ __forceinline__ void two(Chain& ch, uint64_t s, uint32_t t, uint32_t sub, double& u0,
                                        double& u1) const
    {
        u0 = one(ch, s, t, sub, 0);
        u1 = one(ch, s, t, sub, 1);
    }
};

__device__ __forceinline__ double keyed_u(uint64_t seed, uint64_t chain, uint64_t step, uint32_t tag, uint32_t sub,
                                          int half)
{
    const U4 b = keyed_block(seed, chain, step, tag, sub);
    return half ? u52(b.z, b.w) : u52(b.x, b.y);
}

// ------------------------------------------------------------ model pieces
// InterpolatedSampler.interpolate, clearskyindexmodel.py:39-40 (op order kept)
__device__ __forceinline__ double interp(double b, double a, double f) { return f * a + (1.0 - f) * b; }

__device__ __forceinline__ void push(Samp& s, int k, double v)
{   // InterpolatedSampler.__next__, clearskyindexmodel.py:34-37
    s.b[k] = s.a[k];
    s.a[k] = v;
}

__device__ __forceinline__ double normal(double u, double loc, double scale) { return ndtri(u) * scale + loc; }

__device__ __forceinline__ double scaled_noise(const KParams& kp, double u, double s0, double s1, double cc)
{   // norm.rvs(loc=1., scale=np.sqrt(0.9) * (sigma0 + sigma1 * 8 * cc)), clearskyindexmodel.py:86-88
    return normal(u, 1.0, kp.sqrt09 * (s0 + s1 * 8 * cc));
}

// _next_min noise draw (clearskyindexmodel.py:86-88, 109-111): the reference's
// fp64 formula.  Shared by every kernel path so the paths agree bit for bit.
// fp64 mode samples it; fp32 mode keeps it in the state's sampler pairs (the
// rare fp64 recomputation of a second, redo_second, needs these values) and
// samples minute_noise_fast.
template <typename R>
__device__ __forceinline__ double minute_noise(double u, double s0, double s1, double cc, double sqrt09)
{
    return normal(u, 1.0, sqrt09 * (s0 + s1 * 8 * cc));
}

// the fp32 path's copy of the same draw: the quantile and the affine map in fp32
// (the scale formed in fp64 and rounded); the state's fn pairs and the fp32
// minute table hold these
__device__ __forceinline__ float minute_noise_fast(double u, double s0, double s1, double cc, double sqrt09)
{
    const float sc = (float)(sqrt09 * (s0 + s1 * 8 * cc));
    return ndtri_f(u) * sc + 1.0f;
}

// hourly cloud cover: next(get_cloud_cover(distributions)) (cloud_cover_hourly.py:309-316);
// faithful = a fresh generator per draw, i.e. state 1.0 (clearskyindexmodel.py:61-63).
// Chain c (index within the launch) draws from its own table when per-chain
// tables are set (tmh_set_shape_tables: a lat/lon sweep, C5).
__device__ __forceinline__ double draw_cc_from(const KParams& kp, uint32_t c, double state, double u)
{
    int bin = 0;
    while (bin < 5 && kp.edges[bin] < state) ++bin;   // np.searchsorted(bins, state)
    double loc, scale, kappa, df;
    int is_t;
    if (kp.tab) {
        const double* sh = kp.tab + (size_t)c * 24 + 4 * bin;
        loc = sh[0];
        scale = sh[1];
        kappa = sh[2];
        df = sh[3];
        is_t = kp.tab_t ? kp.tab_t[(size_t)c * 6 + bin] : kp.is_t[bin];
    } else {
        loc = kp.shapes[bin][0];
        scale = kp.shapes[bin][1];
        kappa = kp.shapes[bin][2];
        df = kp.shapes[bin][3];
        is_t = kp.is_t[bin];
    }
    double v = is_t ? stdtrit(df, u) : al_ppf(u, kappa);
    v = v * scale + loc;                              // scipy rvs: vals * scale + loc
    const double x = state + v;
    return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);      // np.clip(., 0, 1)
}

__device__ __forceinline__ double draw_cc(const KParams& kp, uint32_t c, Chain& ch, double u)
{
    const double state = kp.cc_mode == TMH_CC_MARKOV ? ch.mstate : 1.0;
    const double x = draw_cc_from(kp, c, state, u);
    if (kp.cc_mode == TMH_CC_MARKOV) ch.mstate = x;
    return x;
}

__device__ __forceinline__ int32_t ceil_thr(double x)
{   // sec < x  <=>  sec < ceil(x) for integer sec (cloud_cover_binary.py:111-113)
    // branch-free (round 6: the walk's latency chain): above 2147483000 or NaN -> INT_MAX,
    // below -2147483000 -> INT_MIN + 1, else ceil(x)
    double y = x <= 2147483000.0 ? x : 2147483647.0;
    y = y < -2147483000.0 ? -2147483647.0 : y;
    return (int32_t)ceil(y);
}

__device__ __forceinline__ double* sig_c(const StateView& st, uint32_t c) { return st.sc + (size_t)c * CAP; }
__device__ __forceinline__ double* sig_l(const StateView& st, uint32_t c) { return st.sl + (size_t)c * CAP; }

__device__ void reset_sigma(double* sc, double* sl, Chain& ch, double h)
{   // cloud_cover_binary.py:76-78: cumsum(300 * ones(int(12 h))) is exact
    int L = (int)(h * 12);
    if (L > CAP) L = CAP;
    const double f = 1.0 / h - 1.0;
    double acc = 0.0;
    for (int k = 0; k < L; ++k) {
        acc += 300.0;
        sc[k] = acc;
        sl[k] = f * acc;
    }
    ch.L = L;
}

// cloud_cover_binary.py:80-107, one lane per chain (sequential kernel / init);
// returns 0 or a fault status.  Keyed draws: counter = the chain's next_cloud
// call number (0 = the constructor's call), sub = try >> 1, half = try & 1, so
// the candidate lengths of a call do not depend on the step it happens at.
template <int RNG>
__device__ uint32_t next_cloud(const KParams& kp, double* sc, double* sl, Chain& ch, const Draw<RNG>& dr, double h,
                               double ws, uint32_t tag)
{
    const double f = 1.0 / h - 1.0;
    int tries = 0;
    const uint64_t ctr = ch.ncalls++;
    for (int rec = 0; rec < 2; ++rec) {
        for (int i = 0; i < 20; ++i, ++tries) {
            const double u = dr.one(ch, ctr, tag, (uint32_t)(tries >> 1), tries & 1);
            const double cl = pow(kp.alpha + kp.delta * u, kp.expo) / ws;
            int last = -1;
            double best = 0.0;
            for (int k = 0; k < ch.L; ++k) {
                const double nsc = cl + sc[k];
                const double nsl = f * nsc;
                const double tot = nsc + nsl;
                if (nsl - sl[k] > 0.0 && tot < 5400.0) {
                    const double d = fabs(tot - 3600.0);
                    if (last < 0 || d < best) {
                        best = d;
                        last = k;
                    }
                }
            }
            if (last >= 0) {
                if (last + 2 > CAP) return TMH_CHAIN_SIGMA_OVERFLOW;
                const double clr = f * (cl + sc[last]) - sl[last];
                for (int k = last; k >= 0; --k) {
                    const double nsc = cl + sc[k];
                    sc[k + 1] = nsc;
                    sl[k + 1] = f * nsc;
                }
                sc[0] = cl;
                sl[0] = clr;
                ch.L = last + 2;
                ch.cl = cl;
                ch.clr = clr;
                ch.t1 = ceil_thr(cl);
                ch.t2 = ceil_thr(cl + clr);
                ch.sec = 0;
                return 0;
            }
        }
        if (rec == 0) reset_sigma(sc, sl, ch, h);
    }
    return TMH_CHAIN_ASSERT_BINARY;
}

// next_cloud on freshly reset sigma arrays: the constructor's call
// (CloudCoverBinary.__init__, cloud_cover_binary.py:63-78, then :80-107).  After
// reset_sigma entry k is exactly 300 (k + 1) and f * 300 (k + 1) (both resets of
// the 40-try loop give the same arrays), so the scan computes the entries instead
// of loading them and only the result is stored; same draws, same bits as
// reset_sigma + next_cloud.
template <int RNG>
__device__ uint32_t next_cloud_fresh(const KParams& kp, double* sc, double* sl, Chain& ch, const Draw<RNG>& dr,
                                     double h, double ws, uint32_t tag)
{
    const double f = 1.0 / h - 1.0;
    int L0 = (int)(h * 12);
    if (L0 > CAP) L0 = CAP;
    const uint64_t ctr = ch.ncalls++;
    for (int tries = 0; tries < 40; ++tries) {
        const double u = dr.one(ch, ctr, tag, (uint32_t)(tries >> 1), tries & 1);
        const double cl = pow(kp.alpha + kp.delta * u, kp.expo) / ws;
        int last = -1;
        double best = 0.0;
        for (int k = 0; k < L0; ++k) {
            const double sck = 300.0 * (k + 1);
            const double nsc = cl + sck;
            const double nsl = f * nsc;
            const double tot = nsc + nsl;
            if (nsl - f * sck > 0.0 && tot < 5400.0) {
                const double d = fabs(tot - 3600.0);
                if (last < 0 || d < best) {
                    best = d;
                    last = k;
                }
            }
        }
        if (last >= 0) {
            if (last + 2 > CAP) return TMH_CHAIN_SIGMA_OVERFLOW;
            const double sc_last = 300.0 * (last + 1);
            const double clr = f * (cl + sc_last) - f * sc_last;   // f * (cl + sc[last]) - sl[last]
            for (int k = last; k >= 0; --k) {
                const double nsc = cl + 300.0 * (k + 1);
                sc[k + 1] = nsc;
                sl[k + 1] = f * nsc;
            }
            sc[0] = cl;
            sl[0] = clr;
            ch.L = last + 2;
            ch.cl = cl;
            ch.clr = clr;
            ch.t1 = ceil_thr(cl);
            ch.t2 = ceil_thr(cl + clr);
            ch.sec = 0;
            return 0;
        }
    }
    reset_sigma(sc, sl, ch, h);   // the state an AssertionError leaves (:91)
    return TMH_CHAIN_ASSERT_BINARY;
}

// Small by-value parameter block for the out-of-line / time-parallel paths
// (avoids taking the address of the large kernel-argument struct).
struct DrawParams {
    uint64_t seed;
    double alpha, delta, expo, sqrt09;
    double x_lo, x_hi;               // range of pow(alpha + delta u, expo) over u in [0, 1] (100 m, 1e6 m)
    double fb_k, fb_scale, fb_loc;   // the bin a fresh generator (state 1.0) draws from
    int32_t fb_is_t, fb_bin;
    const double* tab;               // per-chain shape tables (KParams::tab)
    const int32_t* tab_t;
    const uint32_t* ids;             // KParams::ids
    int32_t markov, pad;             // cc_mode markov: hourly draws come from markov_cc_kernel
};

// faithful hourly cloud cover: a fresh get_cloud_cover generator (state 1.0) per draw
__device__ __forceinline__ double cc_faithful(const DrawParams& dp, uint32_t c, double u)
{
    double k = dp.fb_k, scale = dp.fb_scale, loc = dp.fb_loc;
    int is_t = dp.fb_is_t;
    if (dp.tab) {
        const double* sh = dp.tab + (size_t)c * 24 + 4 * dp.fb_bin;
        if (dp.tab_t) is_t = dp.tab_t[(size_t)c * 6 + dp.fb_bin];
        k = is_t ? sh[3] : sh[2];
        scale = sh[1];
        loc = sh[0];
    }
    double v = is_t ? stdtrit(k, u) : al_ppf(u, k);
    v = v * scale + loc;
    const double x = 1.0 + v;
    return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);
}

// CloudCoverBinary.next_cloud (cloud_cover_binary.py:80-107) with the 64 lanes
// of a wavefront cooperating on ONE chain: entry k = chunk * 64 + lane.  The
// first NCH chunks (128 entries: all but ~1e-6 of calls) live in
// VGPRs for the whole window; chunks NCH.. stay in the chain's global sigma row
// and are touched only while L > 128.  The element arithmetic is the
// reference's (identical bits); np.argmin's first-index tie rule is a butterfly
// reduction; the r_[cl, nsc[:last+1]] shift is a lane shuffle by one.
constexpr int NCH = 2;
constexpr int NCH_ALL = CAP / 64;


// ---- wavefront primitives (DPP, readlane): no LDS round trips
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double old, double v)
{
    const uint32_t lo = dpp_u32<CTRL>((uint32_t)__double2loint(old), (uint32_t)__double2loint(v));
    const uint32_t hi = dpp_u32<CTRL>((uint32_t)__double2hiint(old), (uint32_t)__double2hiint(v));
    return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int lane)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// (d, k) lexicographic min; d >= 0 or +inf, so its bit pattern orders like the value
__device__ __forceinline__ bool key_less(uint64_t ad, int ak, uint64_t bd, int bk)
{
    return ad < bd || (ad == bd && ak < bk);
}

template <int CTRL>
__device__ __forceinline__ void argmin_step(uint64_t& d, int& k)
{
    const uint32_t ol = dpp_u32<CTRL>((uint32_t)d, (uint32_t)d);
    const uint32_t oh = dpp_u32<CTRL>((uint32_t)(d >> 32), (uint32_t)(d >> 32));
    const int ok = (int)dpp_u32<CTRL>((uint32_t)k, (uint32_t)k);
    const uint64_t od = ((uint64_t)oh << 32) | ol;
    if (key_less(od, ok, d, k)) {
        d = od;
        k = ok;
    }
}

// np.argmin semantics over the wave: minimal d, first (lowest) k on ties; result uniform
__device__ __forceinline__ void argmin_first(double dval, int kval, double& dmin, int& kmin)
{
    uint64_t d = (uint64_t)__double_as_longlong(dval);
    int k = kval;
    argmin_step<0xB1>(d, k);    // quad_perm [1,0,3,2]
    argmin_step<0x4E>(d, k);    // quad_perm [2,3,0,1]
    argmin_step<0x141>(d, k);   // row_half_mirror
    argmin_step<0x140>(d, k);   // row_mirror: every row of 16 now holds its minimum
    uint64_t bd = 0;
    int bk = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)d, 16 * r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(d >> 32), 16 * r);
        const int rk = __builtin_amdgcn_readlane(k, 16 * r);
        const uint64_t rd = ((uint64_t)hi << 32) | lo;
        if (r == 0 || key_less(rd, rk, bd, bk)) {
            bd = rd;
            bk = rk;
        }
    }
    dmin = __longlong_as_double((long long)bd);
    kmin = bk;
}

// Unscaled candidate lengths pow(alpha + delta u, expo) (cloud_cover_binary.py:35-40)
// of try 0 for the 64 calls [kb, kb + 64): lane i holds call kb + i, plus the
// uniform of try 1 (the other half of the same Philox block).  One pass of
// 64 independent Philox + pow replaces 64 sequential, wave-redundant ones.
__device__ __forceinline__ void cloud_candidates(const DrawParams& dp, uint64_t chain, uint32_t kb, int lane,
                                                 double& x0, double& u1)
{
    const U4 b = keyed_block(dp.seed, chain, (uint64_t)(kb + (uint32_t)lane), TAG_CLOUD, 0);
    u1 = u52(b.z, b.w);
    x0 = pow_d(dp.alpha + dp.delta * u52(b.x, b.y), dp.expo);
}

__device__ __forceinline__ uint32_t next_cloud_regs(const DrawParams& dp, double (&vc)[NCH], double (&vl)[NCH],
                                                    double* gsc, double* gsl, int& L, double h, double ws,
                                                    uint64_t chain, uint32_t ctr, double x0, double u1, int lane,
                                                    double& cl_out, double& clr_out)
{
    const double f = 1.0 / h - 1.0;
    int tries = 0;
    for (int rec = 0; rec < 2; ++rec) {
        for (int i = 0; i < 20; ++i, ++tries) {
            // try 0 comes precomputed; later tries (about 3 % of calls) are drawn here.
            // pow stays out of line: inlining ocml pow and capping the kernel at
            // 128 VGPR (launch_bounds(256, 4)) once broke bit-parity on gfx950
            double x;
            if (tries == 0) x = x0;
            else if (tries == 1) x = pow_d(dp.alpha + dp.delta * u1, dp.expo);
            else x = pow_d(dp.alpha + dp.delta * keyed_u(dp.seed, chain, ctr, TAG_CLOUD, (uint32_t)(tries >> 1), tries & 1),
                           dp.expo);
            const double cl = x / ws;
            double bd = INFINITY;
            int bk = INT_MAX;
            auto scan = [&](int k, double sc, double sl) {   // :83-88
                if (k < L) {
                    const double nsc = cl + sc;
                    const double nsl = f * nsc;
                    const double tot = nsc + nsl;
                    if (nsl - sl > 0.0 && tot < 5400.0) {
                        const double d = fabs(tot - 3600.0);
                        if (d < bd) {   // chunks ascend in k: ties keep the lower k
                            bd = d;
                            bk = k;
                        }
                    }
                }
            };
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
                if (ch * 64 < L) scan(ch * 64 + lane, vc[ch], vl[ch]);
            for (int ch = NCH; ch * 64 < L; ++ch) {
                const int k = ch * 64 + lane;
                if (k < L) scan(k, gsc[k], gsl[k]);
            }
            double dmin;
            int kmin;
            argmin_first(bd, bk, dmin, kmin);
            if (kmin != INT_MAX) {
                const int last = kmin;
                if (last + 2 > CAP) return TMH_CHAIN_SIGMA_OVERFLOW;
                double sc_last = 0.0, sl_last = 0.0;
                if (last < NCH * 64) {
#pragma unroll
                    for (int ch = 0; ch < NCH; ++ch)
                        if (ch == (last >> 6)) {
                            sc_last = readlane_f64(vc[ch], last & 63);
                            sl_last = readlane_f64(vl[ch], last & 63);
                        }
                } else {
                    sc_last = gsc[last];
                    sl_last = gsl[last];
                }
                const double clr = f * (cl + sc_last) - sl_last;
                double carry = 0.0;   // old entry 64 ch - 1 (lane 63 of the previous chunk)
#pragma unroll
                for (int ch = 0; ch < NCH; ++ch) {
                    if (ch * 64 <= last + 1) {
                        const double top = readlane_f64(vc[ch], 63);
                        const double prev = dpp_f64<0x138>(carry, vc[ch]);   // wave_shr:1, lane 0 <- carry
                        const int p = ch * 64 + lane;
                        const double nsc = cl + prev;
                        vc[ch] = p == 0 ? cl : nsc;
                        vl[ch] = p == 0 ? clr : f * nsc;
                        carry = top;
                    }
                }
                for (int ch = NCH; ch * 64 <= last + 1; ++ch) {   // rare: entries 128.. in memory
                    const int k = ch * 64 + lane;
                    const double old = gsc[k];
                    const double top = readlane_f64(old, 63);
                    const double prev = dpp_f64<0x138>(carry, old);
                    const double nsc = cl + prev;
                    gsc[k] = nsc;
                    gsl[k] = f * nsc;
                    carry = top;
                }
                L = last + 2;
                cl_out = cl;
                clr_out = clr;
                return 0;
            }
        }
        if (rec == 0) {   // reset_sigma (cloud_cover_binary.py:76-78); 300 (k+1) is exact
            int nl = (int)(h * 12);
            if (nl > CAP) nl = CAP;
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                const int k = ch * 64 + lane;
                if (k < nl) {
                    vc[ch] = 300.0 * (k + 1);
                    vl[ch] = f * vc[ch];
                }
            }
            for (int ch = NCH; ch * 64 < nl; ++ch) {
                const int k = ch * 64 + lane;
                if (k < nl) {
                    gsc[k] = 300.0 * (k + 1);
                    gsl[k] = f * gsc[k];
                }
            }
            L = nl;
        }
    }
    return TMH_CHAIN_ASSERT_BINARY;
}

// ---- wave min of a double (every lane's value >= 0 or +inf), result uniform
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_f64_rows(double v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), CTRL, ROWS, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), CTRL, ROWS, 0xF, false);
    return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ double wave_min_f64(double v)
{
    v = fmin(v, dpp_f64_rows<0xB1>(v));        // quad_perm [1,0,3,2]
    v = fmin(v, dpp_f64_rows<0x4E>(v));        // quad_perm [2,3,0,1]
    v = fmin(v, dpp_f64_rows<0x141>(v));       // row_half_mirror
    v = fmin(v, dpp_f64_rows<0x140>(v));       // row_mirror: each row of 16 holds its min
    v = fmin(v, dpp_f64_rows<0x142, 0xA>(v));  // row_bcast:15 -> rows 1, 3
    v = fmin(v, dpp_f64_rows<0x143, 0xC>(v));  // row_bcast:31 -> rows 2, 3: lane 63 = wave min
    return readlane_f64(v, 63);
}

// next_cloud fast path (cloud_cover_binary.py:80-107) for the common case: the
// sigma arrays fit the two register chunks (L <= 128) and try 0 finds a
// possible index (97 % of calls).  np.argmin's first-index rule = min over
// the wave, then the lowest set lane of ballot(d == min).  Returns false (no
// state touched) when the general path must run.
__device__ __forceinline__ bool next_cloud_fast(double (&vc)[NCH], double (&vl)[NCH], int& L, double cl, double f,
                                                int lane, double& clr_out)
{
    static_assert(NCH == 2, "fast path written for two register chunks");
    if (L > 128) return false;
    bool ok0, ok1;
    double d0, d1;
    {
        const double nsc = cl + vc[0];
        const double nsl = f * nsc;
        const double tot = nsc + nsl;
        ok0 = lane < L && nsl - vl[0] > 0.0 && tot < 5400.0;
        d0 = ok0 ? fabs(tot - 3600.0) : INFINITY;
    }
    {
        const double nsc = cl + vc[1];
        const double nsl = f * nsc;
        const double tot = nsc + nsl;
        ok1 = 64 + lane < L && nsl - vl[1] > 0.0 && tot < 5400.0;
        d1 = ok1 ? fabs(tot - 3600.0) : INFINITY;
    }
    const double dmin = wave_min_f64(fmin(d0, d1));
    if (!(dmin < INFINITY)) return false;
    const uint64_t m0 = __builtin_amdgcn_ballot_w64(ok0 && d0 == dmin);
    const uint64_t m1 = __builtin_amdgcn_ballot_w64(ok1 && d1 == dmin);
    int last;
    double sc_last, sl_last;
    if (m0) {
        last = __builtin_ctzll(m0);
        sc_last = readlane_f64(vc[0], last);
        sl_last = readlane_f64(vl[0], last);
    } else {
        last = 64 + __builtin_ctzll(m1);
        sc_last = readlane_f64(vc[1], last - 64);
        sl_last = readlane_f64(vl[1], last - 64);
    }
    const double clr = f * (cl + sc_last) - sl_last;
    // sigma_cloud = r_[cl, nsc[:last+1]], sigma_clear = r_[clr, nsl[:last+1]]
    const double top0 = readlane_f64(vc[0], 63);
    {
        const double prev = dpp_f64<0x138>(0.0, vc[0]);   // wave_shr:1
        const double nsc = cl + prev;
        vc[0] = lane == 0 ? cl : nsc;
        vl[0] = lane == 0 ? clr : f * nsc;
    }
    if (last + 1 >= 64) {
        const double prev = dpp_f64<0x138>(top0, vc[1]);   // lane 0 <- old entry 63
        const double nsc = cl + prev;
        vc[1] = nsc;
        vl[1] = f * nsc;
    }
    L = last + 2;
    clr_out = clr;
    return true;
}

// ------------------------------------------------------------ clock + geometry
// min_f = s / 60, hour_f = (m + min_f) / 60, day_f = (h + hour_f) / 24
// (clearskyindexmodel.py:114-116) without fp64 divisions: q = x * (1/d) plus
// one FMA residual correction.  Equal to the IEEE quotient for every one of
// the 86,400 wall-clock seconds (checked exhaustively: oracle orc_check_fractions).
__device__ __forceinline__ double div_exact(double x, double d, double rd)
{
    const double q = x * rd;
    return fma(fma(-q, d, x), rd, q);
}

__device__ __forceinline__ void clock_fractions(int hour, int minute, int second, double& min_f, double& hour_f,
                                                double& day_f)
{
    min_f = div_exact((double)second, 60.0, 1.0 / 60.0);
    hour_f = div_exact(minute + min_f, 60.0, 1.0 / 60.0);
    day_f = div_exact(hour + hour_f, 24.0, 1.0 / 24.0);
}

__device__ __forceinline__ double rad(double d) { return d * (3.14159265358979323846 / 180.0); }
__device__ __forceinline__ double deg(double r) { return r * (180.0 / 3.14159265358979323846); }
__device__ __forceinline__ double cosd(double d) { return cos(rad(d)); }
__device__ __forceinline__ double sind(double d) { return sin(rad(d)); }

__device__ __forceinline__ int64_t local_at(const tmh_clock& ck, int64_t s)
{
    int64_t l = ck.local0 + s;
    for (int i = 0; i < ck.n_shifts && i < 8; ++i)
        if (s >= ck.shift_step[i]) l += ck.shift_delta[i];
    return l;
}

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b)
{
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

// days since 1970-01-01 -> (year, day of year 1..366, leap)
__device__ void civil_doy(int64_t z, int& doy, int& leap)
{
    z += 719468;
    const int64_t era = floordiv(z, 146097);
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doyy = doe - (365 * yoe + yoe / 4 - yoe / 100);   // from March 1
    const int64_t mp = (5 * doyy + 2) / 153;
    const int64_t d = doyy - (153 * mp + 2) / 5 + 1;
    const int64_t m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) ++y;
    leap = ((y % 4 == 0) && (y % 100 != 0)) || (y % 400 == 0);
    static const int cum[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
    doy = cum[m - 1] + (int)d + ((leap && m > 2) ? 1 : 0);
}

__device__ __forceinline__ double extra_rad(int doy, double s0)
{
    const double B = (2.0 * 3.14159265358979323846 / 365.0) * (doy - 1);
    return s0 * (1.00011 + 0.034221 * cos(B) + 0.00128 * sin(B) + 0.000719 * cos(2.0 * B) + 7.7e-05 * sin(2.0 * B));
}

__device__ double linke_at(const double* lts, int doy, int leap)
{
    const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    double x0 = -31.0 / 2.0, y0 = lts[11], cum = 0.0;
    for (int m = 0; m < 13; ++m) {
        double x1, y1;
        if (m < 12) {
            const double d = md[m] + (leap && m == 1 ? 1 : 0);
            cum += d;
            x1 = cum - d / 2.0;
            y1 = lts[m];
        } else {
            x1 = (leap ? 366 : 365) + 28 / 2.0;
            y1 = lts[0];
        }
        if ((double)doy <= x1) return y0 + ((double)doy - x0) * (y1 - y0) / (x1 - x0);
        x0 = x1;
        y0 = y1;
    }
    return lts[0];
}

// ---- solar geometry, split by what it depends on (pvmodel.py:50-76, pvlib 0.6.3
// model choices; NOAA / Meeus low-precision sun + SPA refraction, the oracle's
// restatement).  The sun's place depends on the instant only: one plan row per
// step (sun_at).  The site part runs once per site and step in geom_kernel, or
// per chain-second when every chain has its own site (tmh_set_sites, C5).
// SUN_SDH / SUN_CDH: sine and cosine of the hour angle's advance since the start of the
// step's 128-s expansion block (lane-independent: the site's longitude cancels), so a
// per-chain site rotates its block-start hour angle instead of a sincos per second (lane_row)
enum { SUN_SIND = 0, SUN_COSD, SUN_TAND, SUN_EOT, SUN_MIN, SUN_DNIX, SUN_I0, SUN_TL, SUN_DOY, SUN_LEAP, SUN_RDNIX,
       SUN_SDH, SUN_CDH, SUN_W = 14 };

__device__ void sun_at(int64_t utc, int doy, int leap, const double* linke, double* o)
{
    const double jd = (double)utc / 86400.0 + 2440587.5;
    const double T = (jd - 2451545.0) / 36525.0;
    const double L0 = fmod(280.46646 + T * (36000.76983 + T * 0.0003032), 360.0);
    const double M = 357.52911 + T * (35999.05029 - 0.0001537 * T);
    const double e = 0.016708634 - T * (0.000042037 + 0.0000001267 * T);
    const double Mr = rad(M);
    const double C = sin(Mr) * (1.914602 - T * (0.004817 + 0.000014 * T)) +
                     sin(2.0 * Mr) * (0.019993 - 0.000101 * T) + sin(3.0 * Mr) * 0.000289;
    const double omega = 125.04 - 1934.136 * T;
    const double lam = L0 + C - 0.00569 - 0.00478 * sin(rad(omega));
    const double eps0 = 23.0 + (26.0 + (21.448 - T * (46.815 + T * (0.00059 - T * 0.001813))) / 60.0) / 60.0;
    const double eps = eps0 + 0.00256 * cos(rad(omega));
    const double decl = asin(sin(rad(eps)) * sin(rad(lam)));
    double y = tan(rad(eps) / 2.0);
    y *= y;
    const double L0r = rad(L0);
    const double eot = 4.0 * deg(y * sin(2.0 * L0r) - 2.0 * e * sin(Mr) + 4.0 * e * y * sin(Mr) * cos(2.0 * L0r) -
                                 0.5 * y * y * sin(4.0 * L0r) - 1.25 * e * e * sin(2.0 * Mr));
    int64_t sod = utc % 86400;
    if (sod < 0) sod += 86400;
    o[SUN_SIND] = sin(decl);
    o[SUN_COSD] = cos(decl);
    o[SUN_TAND] = tan(decl);
    o[SUN_EOT] = eot;
    o[SUN_MIN] = (double)sod / 60.0;
    o[SUN_DNIX] = extra_rad(doy, 1366.1);   // ineichen dni_extra
    o[SUN_I0] = extra_rad(doy, 1370.0);     // disc I0
    o[SUN_TL] = linke ? linke_at(linke, doy, leap) : 0.0;
    o[SUN_DOY] = doy;
    o[SUN_LEAP] = leap;
    o[SUN_RDNIX] = 1.0 / o[SUN_DNIX];       // the fp32 row's reciprocal, once per step
}

// sine and cosine of x in [-pi, pi] (the hour angle): quadrant by rint(x 2/pi), the
// Cody-Waite reduction and kernel polynomials of fdlibm's k_sin.c / k_cos.c / e_rem_pio2.c
// (within 2.2e-16 relative on [-pi/4, pi/4], checked against numpy); straight-line,
// about half of ocml's general-argument sincos
__device__ __forceinline__ void sincos_pi(double x, double* sp, double* cp)
{
    const double k = rint(x * 0.63661977236758134308);
    const double r = fma(-k, 6.07710050650619224932e-11, fma(-k, 1.57079632673412561417e+00, x));
    const double z = r * r;
    double ps = 1.58969099521155010221e-10;
    ps = fma(ps, z, -2.50507602534068634195e-08);
    ps = fma(ps, z, 2.75573137070700676789e-06);
    ps = fma(ps, z, -1.98412698298579493134e-04);
    ps = fma(ps, z, 8.33333333332248946124e-03);
    ps = fma(ps, z, -1.66666666666666324348e-01);
    const double sr = fma(r * z, ps, r);
    double pc = -1.13596475577881948265e-11;
    pc = fma(pc, z, 2.08757232129817482790e-09);
    pc = fma(pc, z, -2.75573143513906633035e-07);
    pc = fma(pc, z, 2.48015872894767294178e-05);
    pc = fma(pc, z, -1.38888888888741095749e-03);
    pc = fma(pc, z, 4.16666666666666019037e-02);
    const double cr = fma(z * z, pc, fma(-0.5, z, 1.0));
    const int q = (int)k & 3;
    const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
    *sp = (q & 2) ? -s0 : s0;
    *cp = ((q + 1) & 2) ? -c0 : c0;
}

// x^y for x > 0 as exp2(y log2 x): within a few ulps of pow (|y log2 x| < 16 here),
// about half of ocml's pow (its extra-precise log and special cases)
// x^y for x > 0 from the PV table's log and exp (a few 1e-16 relative for the airmass powers)
template <typename TP>
__device__ __forceinline__ double pow_pos(double x, double y, TP t) { return exp_tab(y * log_tab(x, t), t); }

// per-site constants of the geometry (site row: lat, lon, altitude, tilt, azimuth, albedo)
struct SiteK {
    double lon, slat, clat, pres, refr, alt, fh1, fh2, cg1, cg2, ctilt, stilt, saz, term2, gfac, csaz, ssaz;
};

__device__ __forceinline__ SiteK site_k(const double* site)
{
    SiteK k;
    const double lat = site[0], alt = site[2], tilt = site[3], albedo = site[5];
    k.lon = site[1];
    k.saz = site[4];
    k.alt = alt;
    const double latr = rad(lat);
    k.slat = sin(latr);
    k.clat = cos(latr);
    k.pres = 100.0 * pow((44331.514 - alt) / 11880.516, 1.0 / 0.1902632);   // alt2pres
    k.refr = (k.pres / 100.0 / 1010.0) * (283.0 / (273.0 + 12.0)) * 1.02;    // SPA refraction at 12 C
    k.fh1 = exp(-alt / 8000.0);
    k.fh2 = exp(-alt / 1250.0);
    k.cg1 = 5.09e-05 * alt + 0.868;
    k.cg2 = 3.92e-05 * alt + 0.0387;
    k.ctilt = cosd(tilt);
    k.stilt = sind(tilt);
    k.term2 = 0.5 * (1.0 + cosd(tilt));
    k.gfac = albedo * (1.0 - cos(rad(tilt))) * 0.5;
    sincos(rad(k.saz), &k.ssaz, &k.csaz);
    return k;
}

// geometry row fields G_COSZ..G_LAST of one site and step (fp64); returns true
// when the clear-sky GHI is 0 (pv = 0 whatever the csi).  FULL = false stops
// there at night (the per-chain-second path); FULL fills every field.  t: the PV table
// (g_pv_tab, or an LDS copy of it) for the airmass powers.
// the hour angle (rad) of site k at a sun row: true solar time, fmod(x, 1440) for x in
// (-1440, 2880) as one exact subtraction (Sterbenz) or none
__device__ __forceinline__ double hour_angle(const SiteK& k, const double* sun)
{
    double tst = sun[SUN_MIN] + sun[SUN_EOT] + 4.0 * k.lon;
    if (tst >= 1440.0) tst -= 1440.0;
    if (tst < 0) tst += 1440.0;
    return rad(tst / 4.0 - 180.0);
}

// site_geom from the hour angle's sine and cosine (sha, cha) at this sun row
template <bool FULL, bool F32 = false, typename TP = const double*>
__device__ __forceinline__ bool site_geom_hc(const SiteK& k, const double* sun, double tl, const double* m, double* g,
                                             TP t, double sha, double cha)
{
    double czr = k.slat * sun[SUN_SIND] + k.clat * sun[SUN_COSD] * cha;
    czr = czr > 1.0 ? 1.0 : (czr < -1.0 ? -1.0 : czr);
    // the sun below -0.83 deg elevation (cos z < cos(90.84 deg) = -0.0147): outside the
    // refraction band (de = 0), apparent zenith = zenith > 90 deg, night -- skip the rest
    if (!FULL && czr < -0.015) return true;
    const double zen = deg(acos(czr));
    const double e0 = 90.0 - zen;
    double de = 0.0;
    // F32 rows: the refraction correction (< 0.6 deg) in fp32, relative error ~5e-7 of
    // de, i.e. ~3e-9 deg on the apparent zenith
    if (e0 >= -1.0 * (0.26667 + 0.5667)) {
        if constexpr (F32) {   // all fp32 (fast quotients, ~2 ulp): de within ~5e-7 of its fp64 value
            const float e0f = (float)e0;
            de = (double)__fdividef((float)k.refr * (1.0f / 60.0f),
                                    tanf((e0f + __fdividef(10.3f, e0f + 5.11f)) * 0.0174532925199432958f));
        }
        else de = k.refr / (60.0 * tan(rad(e0 + 10.3 / (e0 + 5.11))));
    }
    const double azen = 90.0 - (e0 + de);
    // cos / sin of the apparent zenith zen - de from the true zenith's (czr, sqrt(1 - czr^2))
    // and the refraction angle's: |de| < 0.6 deg (0 below the horizon band), so its sine and
    // cosine are short Taylor series (truncation < 1e-18): two fp64 sincos calls fewer
    // than sincos(rad(azen)), the same to a few ulps
    double szs, czs;
    {
        // (F32 rows: fp32 sine of the true zenith; it enters czs only through sin(de) <= 0.01)
        const double sz = F32 ? (double)__builtin_sqrtf((float)fmax(1.0 - czr * czr, 0.0)) : sqrt(fmax(1.0 - czr * czr, 0.0));
        const double d = rad(de), d2 = d * d;
        const double sd = d * (1.0 - d2 * (1.0 / 6.0) * (1.0 - d2 * (1.0 / 20.0) * (1.0 - d2 * (1.0 / 42.0))));
        const double cd = 1.0 - d2 * 0.5 * (1.0 - d2 * (1.0 / 12.0) * (1.0 - d2 * (1.0 / 30.0) * (1.0 - d2 * (1.0 / 56.0))));
        czs = czr * cd + sz * sd;
        szs = sz * cd - czr * sd;
    }
    if (!FULL && !(czs > 0.0)) return true;   // ghi_cs = cg1 * .. * max(cos(apparent zenith), 0) = 0
    // azimuth az = atan2(Y, X) + 180 deg (NOAA, the oracle's solpos): only cos(az - saz) is
    // used (Hay-Davies / AOI projection), = -(X cos saz + Y sin saz) / hypot(X, Y)
    const double azY = sha, azX = cha * k.slat - sun[SUN_TAND] * k.clat;
    double caz;
    if constexpr (F32) {   // fp32 reciprocal square root: ~1e-7 relative on the AOI projection
        const float r2 = (float)(azX * azX + azY * azY);
        caz = r2 > 0.0f ? (double)(-(float)(azX * k.csaz + azY * k.ssaz) * __builtin_amdgcn_rsqf(r2)) : -k.csaz;
    } else {
        const double azr = sqrt(azX * azX + azY * azY);
        caz = azr > 0.0 ? -(azX * k.csaz + azY * k.ssaz) / azr : -k.csaz;   // atan2(0, 0) = 0: az = 180
    }
    const double ct = czr;   // cos(rad(deg(acos(czr)))): the same to ~3e-16 absolute
    g[G_COSZ] = ct;
    // pvmodel.py:52-58; F32 (a per-chain site's fp32 row): in fp32, 1e-7 relative -- the bound
    // only clips csi, and a clipped second's fp32 PV carries that relative error, far inside 1e-5
    if constexpr (F32) {
        const float cf = (float)ct;
        g[G_CSIMAX] = fmaf(27.21f, __expf(-114.0f * cf), fmaf(1.665f, __expf(-4.494f * cf), 1.08f));
    } else
        g[G_CSIMAX] = 27.21 * exp(-114 * ct) + 1.665 * exp(-4.494 * ct) + 1.08;
    const double dni_extra = sun[SUN_DNIX];
    // F32 rows: the relative airmass only feeds Ineichen's exponent and the SAPM spectral
    // polynomial (factors of GHI_cs and of the effective irradiance): fp32 power, ~2e-7
    // relative; DISC's airmass (amd, below, ill-conditioned at low sun) stays fp64
    double am_rel, am_abs;
    if constexpr (F32) {   // fp32 quotient; the pressure ratio as a product
        am_rel = azen <= 90.0 ? (double)__builtin_amdgcn_rcpf(
                                    (float)(czs + 0.50572 * (double)__powf((float)(6.07995 + (90.0 - azen)), -1.6364f)))
                              : NAN;
        am_abs = am_rel * (k.pres * (1.0 / 101325.0));
    } else {
        am_rel = azen <= 90.0 ? 1.0 / (czs + 0.50572 * pow_pos(6.07995 + (90.0 - azen), -1.6364, t)) : NAN;
        am_abs = am_rel * k.pres / 101325.0;
    }
    const double cz = czs > 0.0 ? czs : 0.0;
    const double gx = -k.cg2 * am_abs * (k.fh1 + k.fh2 * (tl - 1.0));
    const double gexp = F32 ? (double)__expf((float)gx) : exp(gx);   // F32: ~1e-7 relative on GHI_cs (kt guard band 4e-6)
    const double gmax = isnan(gexp) ? 0.0 : (gexp > 0.0 ? gexp : 0.0);
    // ineichen (pvmodel.py:60); F32 rows drop its tl / tl (an identity to one ulp)
    g[G_GHICS] = F32 ? k.cg1 * dni_extra * cz * gmax : k.cg1 * dni_extra * cz * tl / tl * gmax;
    const double I0 = sun[SUN_I0];
    g[G_I0] = I0;                                                              // disc (pvmodel.py:63)
    g[G_I0H] = I0 * (ct > 0.065 ? ct : 0.065);
    // DISC's airmass from the fp64 zenith (its conditioning at low sun); F32 rows (which hold
    // am and Kn_c as floats) take the reciprocal and Kn_c's polynomial in fp32 (~1e-7)
    double amd;
    if constexpr (F32) amd = zen <= 90.0 ? (double)__builtin_amdgcn_rcpf((float)(ct + 0.15 * pow_pos(93.885 - zen, -1.253, t)))
                                         : NAN;
    else amd = zen <= 90.0 ? 1.0 / (ct + 0.15 * pow_pos(93.885 - zen, -1.253, t)) : NAN;
    if constexpr (!F32) amd = amd * 101325.0 / 101325.0;   // (pvlib's pressure scaling: an identity to one ulp)
    amd = amd < 12.0 ? amd : (isnan(amd) ? amd : 12.0);
    g[G_AM] = amd;
    if constexpr (F32) {
        const float a = (float)amd;
        g[G_KNC] = fmaf(fmaf(fmaf(fmaf(0.000014f, a, -0.000653f), a, 0.0121f), a, -0.122f), a, 0.866f);
    } else {
        const double amd2 = amd * amd;
        g[G_KNC] = 0.866 - 0.122 * amd + 0.0121 * amd2 - 0.000653 * (amd2 * amd) + 0.000014 * (amd2 * amd2);
    }
    g[G_DISCOK] = zen > 87.0 ? 0.0 : 1.0;
    double proj = k.ctilt * czs + k.stilt * szs * caz;                      // haydavies / aoi (pvmodel.py:66-72)
    proj = proj > 1.0 ? 1.0 : (proj < -1.0 ? -1.0 : proj);
    const double cos_tt = proj > 0.0 ? proj : 0.0;
    if constexpr (F32) g[G_RB] = cos_tt * (double)__builtin_amdgcn_rcpf((float)(czs > 0.01745 ? czs : 0.01745));
    else g[G_RB] = cos_tt / (czs > 0.01745 ? czs : 0.01745);
    g[G_DNIEXTRA] = dni_extra;
    g[G_TERM2] = k.term2;
    g[G_GFAC] = k.gfac;
    // F32 rows: the angle of incidence only enters the SAPM AOI-loss polynomial (a factor
    // of the direct POA): fp32 acos, ~1e-7 relative
    const double aoi = F32 ? (double)(acosf((float)proj) * (float)(180.0 / 3.14159265358979323846)) : deg(acos(proj));
    g[G_COSAOI] = proj;   // cos(rad(aoi)): the same to ~3e-16 absolute
    double f1 = (((m[4] * am_abs + m[3]) * am_abs + m[2]) * am_abs + m[1]) * am_abs + m[0];   // sapm spectral
    f1 = isnan(f1) ? 0.0 : f1;
    g[G_F1] = f1 > 0.0 ? f1 : 0.0;
    double f2 = ((((m[10] * aoi + m[9]) * aoi + m[8]) * aoi + m[7]) * aoi + m[6]) * aoi + m[5];   // sapm aoi loss
    f2 = f2 > 0.0 ? f2 : 0.0;
    if (aoi < 0.0) f2 = 0.0;
    g[G_F2] = f2;
    if constexpr (!F32) {   // the fp64 rows' products (the fp32 rows hold reciprocals in place)
        g[G_KTC] = g[G_GHICS] / g[G_I0H];
        g[G_RDNIX] = sun[SUN_RDNIX];
    }
    return g[G_GHICS] == 0.0;
}

template <bool FULL, bool F32 = false, typename TP = const double*>
__device__ __forceinline__ bool site_geom(const SiteK& k, const double* sun, double tl, const double* m, double* g,
                                          TP t = (const double*)g_pv_tab)
{
    double sha, cha;
    sincos_pi(hour_angle(k, sun), &sha, &cha);
    return site_geom_hc<FULL, F32>(k, sun, tl, m, g, t, sha, cha);
}

constexpr double LOG2E = 1.44269504088896340736;   // the fp32 row's airmass is am log2 e (pv_power_f)

// the kernels' row of one chain's own site (fp32 rows carry the reciprocals
// of I0h and dni_extra and the airmass times log2 e, like geom_kernel's fp32 table)
template <typename R>
__device__ __forceinline__ void site_row(const double* g, const double* sun, R* row_base)
{
    R* row = row_base + row_off<R>();
#pragma unroll
    for (int i = G_COSZ; i <= G_LAST; ++i) row[i] = (R)g[i];
    if constexpr (sizeof(R) == 8) {
        row[G_KTC] = g[G_KTC];
        row[G_RDNIX] = g[G_RDNIX];
    } else {
        row[G_I0H] = __builtin_amdgcn_rcpf((float)g[G_I0H]);
        row[G_DNIEXTRA] = (float)sun[SUN_RDNIX];
        row[G_AM] = (float)(g[G_AM] * LOG2E);
        row[G_F1] = (float)(g[G_F1] * 1e-3);   // pv_power_f: Ee = F1 (...) without the / 1000
        row[G_RB] = (float)(g[G_RB] - g[G_TERM2]);   // pv_power_f: sky = dhi (term2 + AI (Rb - term2))
    }
}

// True when the sun at site k stays below the refraction band (cos z < -0.015, where
// site_geom<false> returns night) for the whole block of BLOCK seconds starting at the
// sun row `sun`: cos z at the block start below -0.015 - 0.012.  Over 128 s the hour
// angle moves by 2 pi 128 / 86400 = 0.0093 rad and cos z by at most that (its
// derivative in the hour angle is cos(lat) cos(decl) sin(h) <= 1); the declination's
// and the equation of time's drift add < 1e-5.  Exact: such a block's seconds are all night.
__device__ __forceinline__ bool site_block_night(const SiteK& k, const double* sun)
{
    double tst = sun[SUN_MIN] + sun[SUN_EOT] + 4.0 * k.lon;
    if (tst >= 1440.0) tst -= 1440.0;
    if (tst < 0) tst += 1440.0;
    const double czr = k.slat * sun[SUN_SIND] + k.clat * sun[SUN_COSD] * cos(rad(tst / 4.0 - 180.0));
    return czr < -0.027;
}

// per-chain site state of a kernel lane: constants + the day's Linke turbidity + the hour
// angle's sine and cosine at the current 128-s block's start (lane_anchor)
struct LaneSite {
    SiteK k;
    const double* linke;   // the chain's 12 monthly values, or NULL (the plan's per-step value)
    int tl_doy;
    double tl;
    double s0, c0;
};

// the lane's hour-angle anchor at a block's first sun row (every kernel that evaluates a
// per-chain site sets it at each 128-s block start of the window, so all of them rotate
// from the same anchors and agree bit for bit)
__device__ __forceinline__ void lane_anchor(LaneSite& ls, const double* sun0)
{
    sincos_pi(hour_angle(ls.k, sun0), &ls.s0, &ls.c0);
}

// the geometry of lane site `ls` at the plan's sun row; true = night.  The hour angle's
// sine and cosine: the block-start anchor rotated by the row's advance (SUN_SDH, SUN_CDH;
// four fp64 operations instead of a sincos per chain-second, a few 1e-16 off the direct
// evaluation)
template <typename R, typename TP = const double*>
__device__ __forceinline__ bool lane_row(LaneSite& ls, const double* sun, const double* module, R* row,
                                         TP t = (const double*)g_pv_tab)
{
    double tl = sun[SUN_TL];
    if (ls.linke) {
        const int doy = (int)sun[SUN_DOY];
        if (doy != ls.tl_doy) {
            ls.tl_doy = doy;
            ls.tl = linke_at(ls.linke, doy, (int)sun[SUN_LEAP]);
        }
        tl = ls.tl;
    }
    double g[ROW];
#ifndef TMH_HA_ROTATE
#define TMH_HA_ROTATE 1   // 0: a sincos per chain-second (A/B builds)
#endif
#if TMH_HA_ROTATE
    const double sdh = sun[SUN_SDH], cdh = sun[SUN_CDH];
    const double sha = fma(ls.s0, cdh, ls.c0 * sdh), cha = fma(ls.c0, cdh, -(ls.s0 * sdh));
#else
    double sha, cha;
    sincos_pi(hour_angle(ls.k, sun), &sha, &cha);
#endif
    if (site_geom_hc<false, sizeof(R) == 4>(ls.k, sun, tl, module, g, t, sha, cha)) return true;
    site_row<R>(g, sun, row);
    return g[G_GHICS] == 0.0;
}

// the flags of a per-chain-site second: the table's day / hour / minute bits, then
// night and DISC's zenith test from the lane's own row (lane_row's result and row)
template <typename R>
__device__ __forceinline__ uint32_t lane_flags(uint32_t fl, bool night, const R* row)
{
    fl &= ~(uint32_t)(FL_NIGHT | FL_DISCOK);
    if (night) return fl | FL_NIGHT;
    return row[row_off<R>() + G_DISCOK] != R(0) ? (fl | FL_DISCOK) : fl;
}


// ------------------------------------------------------------ PV (per chain-second)
// pvmodel.py:53-80 on the precomputed geometry row, fp64.  `p` points at the folded
// constants (PV64: in the kernel arguments, or an LDS copy the expansion re-reads each
// second instead of holding 22 doubles in SGPRs across its loop); `lt` is an LDS copy of
// the table of log_tab / exp_tab, or nullptr for the table itself (g_pv_tab).  kt and AI
// multiply by the row's GHI_cs / I0h and 1 / dni_extra; the SAPM and SNL constants are
// PV64's affine forms.
// an LDS pointer re-laundered (its loads cannot move above this point, so the
// constants are read shortly before their use instead of all at the second's start)
template <typename PP>
__device__ __forceinline__ PP lds_fence(PP p)
{
    if constexpr (__is_same(PP, const PV64*)) return p;
    else {
        uint32_t a = (uint32_t)(uintptr_t)p;
        asm volatile("" : "+v"(a));
        return (PP)(uintptr_t)a;
    }
}

// The a * b + c of the chain after DISC's polynomials are one fma each, in pvmodel.py's order
// of operations (the summations keep their order, each product enters exactly): an fp64
// rounding fewer per pair, within 1e-16 relative of the separate multiply and add (the
// kernels build with -ffp-contract=off); fp64 C2 trace loop -5 % VALU.  DISC's polynomials
// keep the multiply-add form: fused as well, the trace kernel took 122 VGPRs instead of 110,
// i.e. two waves per SIMD beside a 146-VGPR walk wave instead of three (measured: alone
// 2.74 against 2.89 ms, in the pipeline 3.05 against 2.94 ms).
#ifndef TMH_DISC64_HORNER
#define TMH_DISC64_HORNER 0   // A/B builds: 9 fmas, but 33 VGPRs spilled in the fp64 trace loop (2.99-3.07 against 2.55-2.70 ms alone, round 6)
#endif
template <typename PP, typename LT>
__device__ __forceinline__ double pv_power_d(PP p, const double* g, double csi, LT lt)
{
    const double c = csi > g[G_CSIMAX] ? g[G_CSIMAX] : csi;
    const double ghi = c * g[G_GHICS];
    double kt = c * g[G_KTC];
    kt = kt > 0.0 ? kt : 0.0;
    kt = kt < 1.0 ? kt : 1.0;
    const double am = g[G_AM];
    double a, b, cc;
#if TMH_DISC64_HORNER
    // Horner with fmas (round 6): within ~1e-16 relative of pvmodel.py's power form (the fp64
    // bar is 1e-12), 9 fmas instead of 14 multiplies and adds
    if (kt <= 0.6) {
        a = fma(fma(fma(-2.222, kt, 2.286), kt, -1.56), kt, 0.512);
        b = fma(0.962, kt, 0.37);
        cc = fma(fma(-2.048, kt, 0.932), kt, -0.28);
    } else {
        a = fma(fma(fma(11.56, kt, -27.49), kt, 21.77), kt, -5.743);
        b = fma(fma(fma(31.9, kt, 66.05), kt, -118.5), kt, 41.4);
        cc = fma(fma(fma(73.81, kt, -222.0), kt, 184.2), kt, -47.01);
    }
#else
    const double kt2 = kt * kt, kt3 = kt2 * kt;
    if (kt <= 0.6) {
        a = 0.512 - 1.56 * kt + 2.286 * kt2 - 2.222 * kt3;
        b = 0.37 + 0.962 * kt;
        cc = -0.28 + 0.932 * kt - 2.048 * kt2;
    } else {
        a = -5.743 + 21.77 * kt - 27.49 * kt2 + 11.56 * kt3;
        b = 41.4 - 118.5 * kt + 66.05 * kt2 + 31.9 * kt3;
        cc = -47.01 + 184.2 * kt - 222.0 * kt2 + 73.81 * kt3;
    }
#endif
    double ex;
    if constexpr (__is_same(LT, decltype(nullptr))) ex = exp_tab(cc * am, (const double*)g_pv_tab);
    else ex = exp_tab(cc * am, lt);
    const double dkn = fma(b, ex, a);
    double dni = (g[G_KNC] - dkn) * g[G_I0];
    if (g[G_DISCOK] == 0.0 || ghi < 0.0 || dni < 0.0) dni = 0.0;
    const double dhi = fma(-dni, g[G_COSZ], ghi);
    const double AI = dni * g[G_RDNIX];
    double sky = dhi * fma(AI, g[G_RB], (1.0 - AI) * g[G_TERM2]);
    sky = sky > 0.0 ? sky : 0.0;
    double poa_direct = dni * g[G_COSAOI];
    poa_direct = poa_direct > 0.0 ? poa_direct : 0.0;
    const double poa_diffuse = fma(ghi, g[G_GFAC], sky);   // sky + ground
    const double poa_global = poa_direct + poa_diffuse;
    // sapm_celltemp, sapm_effective_irradiance, sapm (pvmodel.py:69-77)
    p = lds_fence(p);
    const double tcell = fma(poa_global, p->tk, p->temp_air);
    const double Ee = g[G_F1] * fma(poa_direct, g[G_F2], p->fd * poa_diffuse) * 1e-3;
    const double Bvmpo = fma(p->nmbvmp, Ee, p->bvmpo1);
    const double delta = p->nkq * (tcell + 273.15);
    double logEe;
    if constexpr (__is_same(LT, decltype(nullptr))) logEe = log_tab(Ee, (const double*)g_pv_tab);
    else logEe = log_tab(Ee, lt);
    const double imp = Ee * fma(p->impo_c1, Ee, p->impo_c0) * fma(p->aimp, tcell, p->aimp0);
    const double dl = delta * logEe;
    double vmp = fma(Bvmpo, tcell - 25.0, fma(p->c3ns, dl * dl, fma(p->c2ns, dl, p->vmpo)));
    if (!isnan(vmp)) vmp = vmp > 0.0 ? vmp : 0.0;
    const double pdc = imp * vmp;
    // snlinverter (pvmodel.py:78): A - B, B, C affine in vmp
    p = lds_fence(p);
    const double AB = fma(p->ab1, vmp, p->ab0), B = fma(p->b1, vmp, p->b0), C = fma(p->c1, vmp, p->c0);
    const double pmB = pdc - B;
    double ac = fma(fma(-C, AB, p->paco / AB), pmB, C * (pmB * pmB));
    if (!isnan(ac)) ac = p->paco < ac ? p->paco : ac;
    if (pdc < p->pso) ac = p->pnt;
    if (isnan(ac)) return 0.0;                       // .fillna(0.)
    return ac > 0.0 ? ac : 0.0;                      // .clip(lower=0.)
}


// DISC's Kn polynomials (pvlib irradiance.disc, pvmodel.py:63) re-expanded
// about kt = 0.6f: p(kt) = sum_k d_k t^k with t = kt - 0.6f (exact in fp32 for
// kt in [0.3, 1.2], Sterbenz).  In the literal form the high set's terms reach
// ~30 around kt = 0.6 where a(kt) is ~0.08: fp32 Horner then loses ~9 bits and
// the PV error reaches 4e-5 at airmass 3-4; the shifted coefficients stay of
// the size of the result there (same FMA count).  d_k = sum_{i>=k} C(i,k) c_i x0^(i-k),
// evaluated in fp64 at compile time and rounded once.
struct Cubic {
    double c0, c1, c2, c3;
};
constexpr double DISC_X0 = (double)0.6f;
constexpr float disc_shift(const Cubic& p, int k)
{
    const double x = DISC_X0;
    return (float)(k == 0   ? ((p.c3 * x + p.c2) * x + p.c1) * x + p.c0
                   : k == 1 ? (3.0 * p.c3 * x + 2.0 * p.c2) * x + p.c1
                   : k == 2 ? 3.0 * p.c3 * x + p.c2
                            : p.c3);
}
constexpr Cubic DISC_A_LO{0.512, -1.56, 2.286, -2.222}, DISC_A_HI{-5.743, 21.77, -27.49, 11.56};
constexpr Cubic DISC_B_LO{0.37, 0.962, 0.0, 0.0}, DISC_B_HI{41.4, -118.5, 66.05, 31.9};
constexpr Cubic DISC_C_LO{-0.28, 0.932, -2.048, 0.0}, DISC_C_HI{-47.01, 184.2, -222.0, 73.81};

template <int DEG>   // Horner over the shifted coefficients d_DEG .. d_0
__device__ __forceinline__ float disc_poly(const Cubic& p, float t)
{
    float v = disc_shift(p, DEG);
#pragma unroll
    for (int k = DEG - 1; k >= 0; --k) v = fmaf(v, t, disc_shift(p, k));
    return v;
}

// The same coefficients as a table (round 6): the single-site expansion keeps it in LDS after
// the noise quantile's and reads the lane's set, so DISC's kt split costs an address select
// instead of divergent branches.  Rows {d3, d2, d1, d0} of a, b, c for kt <= 0.6, then for
// kt > 0.6; the low set's missing leading terms are 0, and Horner through a zero leading term
// gives disc_poly's value bit for bit (0 t + 0 = +-0, then +-0 t + d = d exactly, d != 0).
constexpr int DISC_TAB = 6;
__device__ __forceinline__ float4 disc_row(int i)
{
    const Cubic& p = i % 3 == 0 ? (i < 3 ? DISC_A_LO : DISC_A_HI)
                                : (i % 3 == 1 ? (i < 3 ? DISC_B_LO : DISC_B_HI) : (i < 3 ? DISC_C_LO : DISC_C_HI));
    const int deg = i == 1 ? 1 : (i == 2 ? 2 : 3);
    const float d3 = deg >= 3 ? disc_shift(p, 3) : 0.0f, d2 = deg >= 2 ? disc_shift(p, 2) : 0.0f;
    return make_float4(d3, d2, disc_shift(p, 1), disc_shift(p, 0));
}
__device__ __forceinline__ float disc_horner(const float4& d, float t)
{
    return fmaf(fmaf(fmaf(d.x, t, d.y), t, d.z), t, d.w);
}

// Guard band of the fp32 chain's two discontinuities (DISC's kt = 0.6 split and
// the inverter's p_dc < Pso cut-in): a second whose fp32 kt or p_dc lies this
// close to its threshold may have fallen on the other side than the fp64
// reference, and is recomputed in fp64 (pv_fp64_*).  The fp32 kt differs from
// the fp64 one by < 4e-7 (csi <= 4.5e-7 relative, measured over 4e7 points, plus
// three roundings), p_dc by < 1e-5 relative.
constexpr float KT_GUARD = 4e-6f, PDC_GUARD = 1e-4f;

// fp32 PV chain: the model of pv_power<double>, with fused multiply-adds,
// fp32 constants rounded once on the host (KParams::pvf) and the hardware
// exp / log; within 1e-5 of the fp64 oracle.  `risky`: the second
// lies in a guard band and must be recomputed in fp64.
// UROW: the row is wave-uniform (the single-site kernels' scalar loads), so the clamp's bound
// is an SGPR operand of a plain v_min_f32
template <bool UROW = false>
__device__ __forceinline__ float pv_power_f(const PVF& k, const float* g, float csi, bool discok, bool& risky,
                                            const float4* dtab = nullptr)
{
    // min(csi, csimax) as a median with -inf: no canonicalising max of the row's value first.
    // On a NaN csi it returns csimax, as fminf did (tmh_probe fn 10, test_probe_math); a NaN
    // csi occurs only on lanes whose outputs are masked anyway (faulted chains, lanes past the
    // last chain).
    float c;
    if constexpr (UROW)   // v_min_f32 directly (the compiler's minnum first canonicalises the row value: one op more)
        asm("v_min_f32 %0, %1, %2" : "=v"(c) : "s"(g[G_CSIMAX]), "v"(csi));
    else c = __builtin_amdgcn_fmed3f(csi, -INFINITY, g[G_CSIMAX]);
    const float ghi = c * g[G_GHICS];
    const float kt = fminf(fmaxf(ghi * g[G_I0H], 0.0f), 1.0f);
    // DISC Kn: coefficient sets split at kt = 0.6 (compile-time constants, no
    // SGPRs).  Both sets are evaluated and the results selected: cheaper than
    // selecting twelve coefficient pairs per lane.
    // UROW with dtab (the single-site expansion): the lane's set from the LDS table (disc_row)
    const bool lo = kt <= 0.6f;
    const float t = kt - 0.6f;
    float a, b, cc;
    if (UROW && dtab) {
        const float4* d = dtab + (lo ? 0 : 3);
        a = disc_horner(d[0], t);
        b = disc_horner(d[1], t);
        cc = disc_horner(d[2], t);
    } else {
        a = lo ? disc_poly<3>(DISC_A_LO, t) : disc_poly<3>(DISC_A_HI, t);
        b = lo ? disc_poly<1>(DISC_B_LO, t) : disc_poly<3>(DISC_B_HI, t);
        cc = lo ? disc_poly<2>(DISC_C_LO, t) : disc_poly<3>(DISC_C_HI, t);
    }
    // exp(cc am) = exp2(cc * (am log2 e)): the fp32 row holds am log2 e (one rounding)
    const float dkn = fmaf(b, __builtin_amdgcn_exp2f(cc * g[G_AM]), a);
    float dni = (g[G_KNC] - dkn) * g[G_I0];
    dni = (discok && ghi >= 0.0f && dni >= 0.0f) ? dni : 0.0f;
    const float dhi = fmaf(-dni, g[G_COSZ], ghi);
    const float AI = dni * g[G_DNIEXTRA];
    // AI Rb + (1 - AI) term2 = term2 + AI (Rb - term2): the fp32 row's G_RB holds Rb - term2
    const float sky = fmaxf(dhi * fmaf(AI, g[G_RB], g[G_TERM2]), 0.0f);
    const float poa_direct = fmaxf(dni * g[G_COSAOI], 0.0f);
    const float poa_diffuse = fmaf(ghi, g[G_GFAC], sky);
    const float poa_global = poa_direct + poa_diffuse;
    const float tcell = fmaf(poa_global, k.tk, k.temp_air);
    const float Ee = g[G_F1] * fmaf(poa_direct, g[G_F2], k.fd * poa_diffuse);   // the row's F1 holds F1 / 1000
    const float Bvmpo = fmaf(k.nmbvmp, Ee, k.bvmpo1);
    const float delta = fmaf(k.nkq, tcell, k.nkq273);   // delta log2(Ee) = delta_ref ln(Ee)
    // the hardware log2 already gives -inf at +-0 and NaN below 0 or at NaN
    const float logEe = __builtin_amdgcn_logf(Ee);
    const float dt25 = tcell - 25.0f;
    const float imp = fmaf(k.impo_c1, Ee, k.impo_c0) * Ee * fmaf(k.aimp, dt25, 1.0f);
    const float dl = delta * logEe;
    // max(vmp, 0) unless NaN in the reference; a NaN vmp there gives p_dc NaN and pv 0
    // (.fillna), here vmp 0 gives p_dc 0 < Pso and pv 0: the same pv, one op less
    const float vmp = fmaxf(fmaf(Bvmpo, dt25, fmaf(k.c3ns, dl * dl, fmaf(k.c2ns, dl, k.vmpo))), 0.0f);
    const float pdc = imp * vmp;
    const float AmB = fmaf(k.ab1, vmp, k.ab0), B = fmaf(k.b1, vmp, k.b0), C = fmaf(k.c1, vmp, k.c0);
    const float pmB = pdc - B;
    const float ac = fmaf(C, pmB * pmB, fmaf(-C, AmB, k.paco * __builtin_amdgcn_rcpf(AmB)) * pmB);
    risky = fabsf(t) < KT_GUARD || fabsf(pdc - k.pso) < PDC_GUARD * k.pso;
    // min(ac, Paco) unless NaN, -|Pnt| below the cut-in, .fillna(0), .clip(lower=0):
    // -|Pnt| <= 0 clips to 0 and a NaN fills to 0; the rest is one med3 into [0, Paco].
    // v_med3_f32 with a NaN operand returns min3 of its operands, so a NaN ac gives
    // min(0, max(Paco, 0)) = 0 with no separate NaN test (tmh_probe fn 9, test_probe_math)
    return pdc < k.pso ? 0.0f : __builtin_amdgcn_fmed3f(ac, 0.0f, k.pacoc);
}

// ------------------------------------------------------------ fused per-second body
// The kernels' sampler pairs (InterpolatedSampler, clearskyindexmodel.py:12-40) in the
// compute precision.  R = double: (before b, after a), interpolated exactly as the
// reference (f a + (1 - f) b).  R = float (round 6): the after value a and the
// difference d = a - b (held in b[k]), so the interpolation is one FMA, a - (1 - f) d,
// with the row's fp32 1 - f; a push (b <- a, a <- v) is d = v - a, a = v.  Every fp32
// kernel forms d from the same fp32 values (to_real, set_fast_noise, fpush), so the
// sequential and time-parallel fp32 paths agree bit for bit.
template <typename R>
struct FSamp {
    R b[6], a[6];   // R = float: b[k] holds a[k] - before
};

template <typename R>
__device__ __forceinline__ void to_real(FSamp<R>& f, const Samp& s)
{
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        f.a[k] = (R)s.a[k];
        if constexpr (sizeof(R) == 8) f.b[k] = s.b[k];
        else f.b[k] = (float)s.a[k] - (float)s.b[k];
    }
}

// push a new after value (InterpolatedSampler.next, clearskyindexmodel.py:34-37)
template <typename R>
__device__ __forceinline__ void fpush(FSamp<R>& f, int k, R v)
{
    if constexpr (sizeof(R) == 8) f.b[k] = f.a[k];
    else f.b[k] = v - f.a[k];
    f.a[k] = v;
}

// fp32: the noise samplers hold the fast draws (minute_noise_fast), not the state's fp64 ones
template <typename R>
__device__ __forceinline__ void set_fast_noise(FSamp<R>& f, float2 cloudy, float2 clear)
{
    f.a[S_CLOUDY_NOISE] = cloudy.y;
    f.b[S_CLOUDY_NOISE] = cloudy.y - cloudy.x;
    f.a[S_CLEAR_NOISE] = clear.y;
    f.b[S_CLEAR_NOISE] = clear.y - clear.x;
}

template <typename R>
__device__ __forceinline__ R rinterp(const FSamp<R>& f, int k, R frac)
{
    static_assert(sizeof(R) == 8, "the fp32 samplers interpolate from the row's (1 - f) (rinterp_row)");
    return frac * f.a[k] + (R(1) - frac) * f.b[k];
}

// the same from a row's fraction field fi: the fp32 row holds (1 - f, f) as a pair
template <typename R>
__device__ __forceinline__ R rinterp_row(const FSamp<R>& f, int k, const R* row, int fi)
{
    if constexpr (sizeof(R) == 8) return rinterp(f, k, row[fi]);
    else {
        const int pc = fi == G_MINF ? G32_MINF_C : (fi == G_HOURF ? G32_HOURF_C : G32_DAYF_C);
        return fmaf(-row[pc], f.b[k], f.a[k]);   // a - (1 - f) (a - b): one FMA
    }
}

// clearskyindexmodel.py:146-160 + pvmodel.py:53-80 + metersim.py:51 + pvsim.py:83
// per-second draws from the step's two Philox words (keyed mode): the noise's
// standard normal and the meter (metersim.py:51, 9000 u in [0, 9000))
template <typename R>
__device__ __forceinline__ R noise_z(uint32_t w)
{
    // fp64: ndtri64 (<= ~1e-15 relative, far inside the fp64 bar); fp32: the table quantile
    // (ndtri_t, <= 4.6e-7 absolute) read from global memory -- the expansion reads the same
    // values from its LDS copy, so every fp32 kernel draws the same z
    if constexpr (sizeof(R) == 8) return ndtri64(w, (const double*)g_pv_tab);
    else return ndtri_t(w, (const float4*)g_nd32_tab);
}

// the same quantile from the expansion's LDS copy of the fp32 table (the fp64 kernels' is ndtri64's)
template <typename R>
__device__ __forceinline__ R noise_lds(uint32_t w, const float4* nd_lds)
{
    if constexpr (sizeof(R) == 8) return noise_z<R>(w);
    else return ndtri_t(w, nd_lds);
}

template <typename R>
__device__ __forceinline__ R meter_w(uint32_t w)
{
    if constexpr (sizeof(R) == 8) return 9000 * u32d(w);
    // 9000 u = 9000 (w + 1/2) 2^-32 with the scale shrunk by 2^-23 relative: w = 2^32 - 1
    // converts to 2^32 and then lands on 8999.999 (the largest float < 9000), so no clamp
    // is needed to keep [0, 9000); 1.2e-7 relative, far inside the fp32 bar
    else return fmaf((float)w, 9000.0f * 0x1p-32f * (1.0f - 0x1p-23f), 9000.0f * 0x1p-33f);
}

// risky (fp32 only): pv lies in pv_power_f's guard band; the caller recomputes
// the second in fp64 (pv_fp64_*) and replaces pv and res
// (fp64: p64 / lt as pv_power_d's; the defaults read the kernel arguments and ocml's log)
template <typename R, bool UROW = false, typename P64 = decltype(nullptr), typename LT = decltype(nullptr)>
__device__ __forceinline__ void second_body(const KParams& kp, const PVF& pk, const R* row, uint32_t fl,
                                            const FSamp<R>& fs, bool covered, R z, R meter_in, R& csi, R& pv, R& meter,
                                            R& res, bool& risky, P64 p64 = nullptr, LT lt = nullptr,
                                            const float4* dtab = nullptr)
{
    risky = false;
    const R cloudcover = rinterp_row(fs, S_CC, row, G_HOURF);   // == interp() bit for bit when R = double
    R eps;
    if constexpr (sizeof(R) == 8) eps = z * (R(kp.sqrt6) * (R(0.001) + R(0.0015 * 8) * cloudcover)) + R(0);
    else eps = z * fmaf(cloudcover, EPS1F, EPS0F);   // fp32: the scale as one FMA on literals (z is never 0)
    // both branches' factors, then a select on values (a select on the sampler
    // index would make the compiler index the sampler arrays dynamically: scratch)
    const R a_clear = rinterp_row(fs, S_CLEAR_DAY, row, G_DAYF), a_cloudy = rinterp_row(fs, S_CLOUDY_HOUR, row, G_HOURF);
    const R n_clear = rinterp_row(fs, S_CLEAR_NOISE, row, G_MINF), n_cloudy = rinterp_row(fs, S_CLOUDY_NOISE, row, G_MINF);
    csi = (covered ? a_clear : a_cloudy) * ((covered ? n_clear : n_cloudy) + eps);
    if constexpr (sizeof(R) == 8) {
        if constexpr (__is_same(P64, decltype(nullptr)))
            pv = (kp.with_pv && !(fl & FL_NIGHT)) ? pv_power_d(&kp.pv64, row, csi, lt) : R(0);
        else
            pv = (kp.with_pv && !(fl & FL_NIGHT)) ? pv_power_d(p64, row, csi, lt) : R(0);
    }
    else pv = (kp.with_pv && !(fl & FL_NIGHT)) ? pv_power_f<UROW>(pk, row + G32, csi, (fl & FL_DISCOK) != 0, risky, dtab) : 0.0f;
    meter = meter_in;
    res = meter - pv;
}

// streaming trace stores: non-temporal, so the write-once trace does not
// evict the tables and draw buffers the block re-reads
template <typename R>
__device__ __forceinline__ void trace_store(void* p, uint64_t i, R v)
{
    if (p) __builtin_nontemporal_store(v, reinterpret_cast<R*>(p) + i);
}

struct Acc {
    double pv, m, r, mx;
    // fp32 kernels: the residual maximum kept in fp32 (one v_max_f32 per second instead of an
    // fp64 max and its operand canonicalisation); widening is exact and monotonic, so
    // max(mx, mxf) equals the fp64 maximum of the widened residuals bit for bit
    float mxf = -INFINITY;
    __device__ double max() const { return fmax(mx, (double)mxf); }
};

// output specialisations of the time-parallel expansion (chosen on the host)
enum : int {
    OUT_ANY = 0,      // any combination of trace fields and statistics
    OUT_TRACE3 = 1,   // exactly pv, meter, residual traces (the trace-mode hot path)
    OUT_STATS = 2,    // statistics only, no trace
    // flags on OUT_ANY / OUT_STATS (fp32 kernels): OUT_B64 bins in fp64 (a histogram spec whose
    // fp32 bin position is not accurate enough, StatsView::bin64); OUT_BRT decides at run time
    OUT_B64 = 8, OUT_BRT = 16
};
constexpr int out_base(int out) { return out & 7; }

// held: a guard-band second whose pv / residual fixup_kernel replaces; it enters
// the sums here (fixup_kernel adds the exact difference) but not the maximum or
// the histogram (fixup_kernel adds its final value)
// PACK: the workgroup's LDS histogram holds two 16-bit bins per word (a 128-second
// block of 256 chains adds at most 32,768 to a bin), half the LDS of one word each
template <typename R, int OUT = OUT_ANY, bool PACK = false>
__device__ __forceinline__ void emit(const TraceView& tr, const StatsView& sv, uint32_t* lds_hist, uint64_t o,
                                     uint8_t cov, R csi, R pv, R meter, R res, Acc& acc, bool ok, bool held = false)
{
    if constexpr (out_base(OUT) == OUT_TRACE3) {
        __builtin_nontemporal_store(pv, reinterpret_cast<R*>(tr.pv) + o);
        __builtin_nontemporal_store(meter, reinterpret_cast<R*>(tr.meter) + o);
        __builtin_nontemporal_store(res, reinterpret_cast<R*>(tr.residual) + o);
        return;
    }
    if constexpr (out_base(OUT) == OUT_ANY) {
        trace_store<R>(tr.csi, o, csi);
        trace_store<R>(tr.pv, o, pv);
        trace_store<R>(tr.meter, o, meter);
        trace_store<R>(tr.residual, o, res);
        if (tr.covered) tr.covered[o] = cov;
    }
    if (ok) {
        if (sv.acc) {
            // a night second's literal pv = 0 adds nothing (acc.pv starts at +0 and sums values >= 0,
            // so it is never -0 and acc.pv + 0 == acc.pv): no fp64 add for it
            if (!(__builtin_constant_p(pv) && pv == R(0))) acc.pv += (double)pv;
            acc.m += (double)meter;
            acc.r += (double)res;
            if constexpr (sizeof(R) == 4) {   // v_max_f32 directly (fmaxf canonicalises both operands
                float m;                         // first; res is never NaN here: ok lanes only), a select
                asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(acc.mxf), "v"(res));   // for held (no branch)
                acc.mxf = held ? acc.mxf : m;
            } else if (!held) {
                acc.mx = fmax(acc.mx, (double)res);
            }
        }
        if (sv.hist && !held) {
            const int bin = (OUT & OUT_BRT) ? hist_bin_rt<R>(sv, res) : hist_bin<R, sizeof(R) == 8 || (OUT & OUT_B64) != 0>(sv, res);
            if constexpr (PACK) atomicAdd(&lds_hist[bin >> 1], 1u << ((bin & 1) << 4));
            else atomicAdd(&lds_hist[bin], 1u);
        }
    }
}

}  // namespace tmh
