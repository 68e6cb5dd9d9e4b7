// libtmhpvsim — MI355X (gfx950) batched simulator of tmhpvsim's clear-sky-index
// chain + PV model behind the C-ABI of include/tmhpvsim.h.
//
// One work-item per chain (site x scenario).  Chain state lives in registers
// across the in-kernel time loop and in structure-of-arrays HBM buffers
// between calls (every per-lane access is coalesced: element = field[chain]).
// Everything that is the same for all chains at a given second (wall-clock
// fractions, boundary flags, solar geometry, clear-sky irradiance, SAPM
// spectral/AOI factors) is computed once per second by geom_kernel into a
// table that the chain kernel reads with wave-uniform (scalar) loads.
//
// Reference lines restated (tmhpvsim/...):
//   clearskyindexmodel.py:12-40   InterpolatedSampler (interp op order kept)
//   clearskyindexmodel.py:57-99   constructor draw sequence      -> init_kernel
//   clearskyindexmodel.py:101-126 day/hour/minute resampling     -> chain_kernel
//   clearskyindexmodel.py:128-160 per-second CSI                 -> chain_kernel
//   cloud_cover_binary.py:25-117  cloud lengths, CloudCoverBinary-> next_cloud
//   cloud_cover_hourly.py:100-104,290-316 hourly cover draw      -> draw_cc
//   pvmodel.py:50-80              PV chain (pvlib 0.6.3 models)  -> geom_kernel + pv_power
//   metersim.py:49-51, pvsim.py:83 meter + residual              -> chain_kernel
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "tmh_math.h"
#include "tmhpvsim.h"

using namespace tmh;

#define CAP TMH_SIGMA_CAP
#define ROW TMH_GEOM_FIELDS

namespace {

// ------------------------------------------------------------ parameters
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
};

struct GParams {
    double site[8];
    double linke[12];
    double module[TMH_MOD_COUNT];
    tmh_clock clock;
};

enum : uint32_t { FL_DAY = 1, FL_HOUR = 2, FL_MIN = 4, FL_NIGHT = 8 };
// geometry table row (TMH_GEOM_FIELDS = 20)
enum {
    G_MINF = 0, G_HOURF = 1, G_DAYF = 2, G_FLAGS = 3, G_COSZ = 4, G_CSIMAX = 5, G_GHICS = 6,
    G_I0H = 7, G_I0 = 8, G_KNC = 9, G_AM = 10, G_DISCOK = 11, G_RB = 12, G_DNIEXTRA = 13,
    G_TERM2 = 14, G_GFAC = 15, G_COSAOI = 16, G_F1 = 17, G_F2 = 18
};

struct StateView {
    double* sb[6];
    double* sa[6];
    double *cl, *clr, *mstate;
    int32_t *sec, *L;
    uint32_t *pos, *status, *ncalls;
    double *sc, *sl;   // [CAP][n]
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
};

enum { S_CC = 0, S_CLEAR_DAY = 1, S_CLOUDY_HOUR = 2, S_CLOUDY_NOISE = 3, S_CLEAR_NOISE = 4, S_WS = 5 };

struct Chain {
    double sb[6], sa[6];
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

// ------------------------------------------------------------ model pieces
__device__ __forceinline__ double interp(double b, double a, double f) { return f * a + (1.0 - f) * b; }

__device__ __forceinline__ void push(Chain& ch, int k, double v)
{
    ch.sb[k] = ch.sa[k];
    ch.sa[k] = v;
}

__device__ __forceinline__ double normal(double u, double loc, double scale) { return ndtri(u) * scale + loc; }

__device__ __forceinline__ double scaled_noise(const KParams& kp, double u, double s0, double s1, double cc)
{   // norm.rvs(loc=1., scale=np.sqrt(0.9) * (sigma0 + sigma1 * 8 * cc)), clearskyindexmodel.py:86-88
    return normal(u, 1.0, kp.sqrt09 * (s0 + s1 * 8 * cc));
}

// hourly cloud cover: next(get_cloud_cover(distributions)); faithful = fresh generator (state 1.0)
__device__ double draw_cc(const KParams& kp, Chain& ch, double u)
{
    const double state = kp.cc_mode == TMH_CC_MARKOV ? ch.mstate : 1.0;
    int bin = 0;
    while (bin < 5 && kp.edges[bin] < state) ++bin;   // np.searchsorted(bins, state)
    double v = kp.is_t[bin] ? stdtrit(kp.shapes[bin][3], u) : al_ppf(u, kp.shapes[bin][2]);
    v = v * kp.shapes[bin][1] + kp.shapes[bin][0];
    double x = state + v;
    x = x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);
    if (kp.cc_mode == TMH_CC_MARKOV) ch.mstate = x;
    return x;
}

__device__ __forceinline__ int32_t ceil_thr(double x)
{   // sec < x  <=>  sec < ceil(x) for integer sec
    if (!(x <= 2147483000.0)) return INT_MAX;
    if (x < -2147483000.0) return INT_MIN + 1;
    return (int32_t)ceil(x);
}

__device__ void reset_sigma(const StateView& st, uint32_t c, Chain& ch, double h)
{   // cloud_cover_binary.py:76-78
    int L = (int)(h * 12);
    if (L > CAP) L = CAP;
    const double f = 1.0 / h - 1.0;
    double acc = 0.0;
    for (int k = 0; k < L; ++k) {
        acc += 300.0;
        st.sc[(size_t)k * st.n + c] = acc;
        st.sl[(size_t)k * st.n + c] = f * acc;
    }
    ch.L = L;
}

// cloud_cover_binary.py:80-107; returns 0 or a fault status
template <int RNG>
__device__ uint32_t next_cloud(const KParams& kp, const StateView& st, uint32_t c, Chain& ch,
                               const Draw<RNG>& dr, double h, double ws, uint64_t step, uint32_t tag,
                               uint32_t call)
{
    const double f = 1.0 / h - 1.0;
    int tries = 0;
    ch.ncalls++;
    for (int rec = 0; rec < 2; ++rec) {
        for (int i = 0; i < 20; ++i, ++tries) {
            const double u = dr.one(ch, step, tag, (call << 8) | (uint32_t)(tries >> 1), tries & 1);
            const double cl = pow(kp.alpha + kp.delta * u, kp.expo) / ws;
            int last = -1;
            double best = 0.0;
            for (int k = 0; k < ch.L; ++k) {
                const double nsc = cl + st.sc[(size_t)k * st.n + c];
                const double nsl = f * nsc;
                const double tot = nsc + nsl;
                if (nsl - st.sl[(size_t)k * st.n + c] > 0.0 && tot < 5400.0) {
                    const double d = fabs(tot - 3600.0);
                    if (last < 0 || d < best) {
                        best = d;
                        last = k;
                    }
                }
            }
            if (last >= 0) {
                if (last + 2 > CAP) return TMH_CHAIN_SIGMA_OVERFLOW;
                const double clr = f * (cl + st.sc[(size_t)last * st.n + c]) - st.sl[(size_t)last * st.n + c];
                for (int k = last; k >= 0; --k) {
                    const double nsc = cl + st.sc[(size_t)k * st.n + c];
                    st.sc[(size_t)(k + 1) * st.n + c] = nsc;
                    st.sl[(size_t)(k + 1) * st.n + c] = f * nsc;
                }
                st.sc[c] = cl;
                st.sl[c] = clr;
                ch.L = last + 2;
                ch.cl = cl;
                ch.clr = clr;
                ch.t1 = ceil_thr(cl);
                ch.t2 = ceil_thr(cl + clr);
                ch.sec = 0;
                return 0;
            }
        }
        if (rec == 0) reset_sigma(st, c, ch, h);
    }
    return TMH_CHAIN_ASSERT_BINARY;
}

__device__ __forceinline__ void load_chain(const StateView& st, uint32_t c, Chain& ch)
{
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        ch.sb[k] = st.sb[k][c];
        ch.sa[k] = st.sa[k][c];
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
        st.sb[k][c] = ch.sb[k];
        st.sa[k][c] = ch.sa[k];
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
template <int RNG>
__global__ __launch_bounds__(256) void init_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                   double hf, InjView inj)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    Chain ch;
    for (int k = 0; k < 6; ++k) ch.sb[k] = ch.sa[k] = NAN;
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
    // NB: injected mode consumes in exactly this order (clearskyindexmodel.py:61-97)
    ch.sb[S_CC] = draw_cc(kp, ch, u[0]);
    ch.sa[S_CC] = draw_cc(kp, ch, u[1]);
    ch.sb[S_CLEAR_DAY] = normal(u[2], 0.99, 0.08);
    ch.sa[S_CLEAR_DAY] = normal(u[3], 0.99, 0.08);
    bool name_error = false;
    for (int j = 0; j < 2; ++j) {   // :68-82
        const double cc = interp(ch.sb[S_CC], ch.sa[S_CC], hf);
        double v;
        if (cc < 6.0 / 8) v = normal(u[4 + j], 0.6784, 0.2046);
        else if (cc < 7.0 / 8) {
            name_error = true;
            break;
        } else v = gammaincinv(3.5624, u[4 + j]) * 0.0867 + 0.0;
        if (j == 0) ch.sb[S_CLOUDY_HOUR] = v;
        else ch.sa[S_CLOUDY_HOUR] = v;
    }
    if (name_error) {
        // the reference raises after consuming the 4 draws before the cloudy sampler
        if constexpr (RNG == TMH_RNG_INJECTED) ch.pos = ch.pos < 4 ? ch.pos : 4;
        ch.status = TMH_CHAIN_NAMEERROR_INIT;
        store_chain(st, c, ch);
        return;
    }
    const double cch = interp(ch.sb[S_CC], ch.sa[S_CC], hf);
    ch.sb[S_CLOUDY_NOISE] = scaled_noise(kp, u[6], 0.01, 0.003, cch);
    ch.sa[S_CLOUDY_NOISE] = scaled_noise(kp, u[7], 0.01, 0.003, cch);
    ch.sb[S_CLEAR_NOISE] = scaled_noise(kp, u[8], 0.001, 0.0015, cch);
    ch.sa[S_CLEAR_NOISE] = scaled_noise(kp, u[9], 0.001, 0.0015, cch);
    ch.sb[S_WS] = 2.14 * gammaincinv(2.69, u[10]);
    ch.sa[S_WS] = 2.14 * gammaincinv(2.69, u[11]);
    // CloudCoverBinary(cc.interpolate(0), ws.interpolate(0)) (:98-99)
    const double h0 = interp(ch.sb[S_CC], ch.sa[S_CC], 0.0);
    const double h = 0.95 < h0 ? 0.95 : h0;
    const double ws = interp(ch.sb[S_WS], ch.sa[S_WS], 0.0);
    reset_sigma(st, c, ch, h);
    uint32_t f = next_cloud<RNG>(kp, st, c, ch, dr, h, ws, 0, TAG_INIT_CLOUD, 0);
    if (!f) {
        const double us = dr.one(ch, 0, TAG_INIT_SEC, 0, 0);
        ch.sec = (int32_t)((ch.cl + ch.clr) * us);
    }
    if (f && !ch.status) ch.status = f;
    store_chain(st, c, ch);
}

// ------------------------------------------------------------ clock + geometry
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

__device__ void solpos(int64_t utc, double lat, double lon, double pressure_pa, double temp_c, double& zen,
                       double& azen, double& az)
{   // NOAA / Meeus low-precision sun + SPA refraction (same restatement as the oracle)
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
    double tst = fmod((double)sod / 60.0 + eot + 4.0 * lon, 1440.0);
    if (tst < 0) tst += 1440.0;
    const double ha = rad(tst / 4.0 - 180.0);
    const double latr = rad(lat);
    double cz = sin(latr) * sin(decl) + cos(latr) * cos(decl) * cos(ha);
    cz = cz > 1.0 ? 1.0 : (cz < -1.0 ? -1.0 : cz);
    zen = deg(acos(cz));
    az = deg(atan2(sin(ha), cos(ha) * sin(latr) - tan(decl) * cos(latr))) + 180.0;
    const double e0 = 90.0 - zen;
    double de = 0.0;
    if (e0 >= -1.0 * (0.26667 + 0.5667))
        de = (pressure_pa / 100.0 / 1010.0) * (283.0 / (273.0 + temp_c)) * 1.02 /
             (60.0 * tan(rad(e0 + 10.3 / (e0 + 5.11))));
    azen = 90.0 - (e0 + de);
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
    g[G_MINF] = second / 60.0;                       // clearskyindexmodel.py:114-116
    g[G_HOURF] = (minute + g[G_MINF]) / 60.0;
    g[G_DAYF] = (hour + g[G_HOURF]) / 24.0;
    uint32_t fl = 0;
    if (dn != dp) fl |= FL_DAY;                      // :121 prev.day != day
    if (hour != hourp) fl |= FL_HOUR;                // :123
    if (minute != minutep) fl |= FL_MIN;             // :125
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
    const double am_rel = azen <= 90.0 ? 1.0 / (cos(rad(azen)) + 0.50572 * pow(6.07995 + (90.0 - azen), -1.6364))
                                       : NAN;
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
    if (g[G_GHICS] == 0.0) fl |= FL_NIGHT;           // ghi_cs = 0 -> pv = 0 whatever the csi
    g[G_FLAGS] = (double)fl;
    double* o64 = tab64 + (size_t)j * ROW;
    float* o32 = tab32 + (size_t)j * ROW;
    for (int i = 0; i < ROW; ++i) {
        o64[i] = g[i];
        o32[i] = (float)g[i];
    }
    o32[G_FLAGS] = __uint_as_float(fl);
    o32[G_I0H] = (float)(1.0 / g[G_I0H]);              // fp32 path multiplies by reciprocals
    o32[G_DNIEXTRA] = (float)(1.0 / g[G_DNIEXTRA]);
}

// ------------------------------------------------------------ PV (per chain-second)
// pvmodel.py:53-80 on the precomputed geometry row; R = float | double.
template <typename R>
__device__ __forceinline__ R pv_power(const KParams& kp, const R* g, R csi)
{
    const double* m = kp.module;
    const double* iv = kp.inverter;
    R c = csi > g[G_CSIMAX] ? g[G_CSIMAX] : csi;
    const R ghi = c * g[G_GHICS];
    R kt;
    if constexpr (sizeof(R) == 8) kt = ghi / g[G_I0H];
    else kt = ghi * g[G_I0H];
    kt = kt > R(0) ? kt : R(0);
    kt = kt < R(1) ? kt : R(1);
    const R am = g[G_AM], kt2 = kt * kt, kt3 = kt2 * kt;
    R a, b, cc;
    if (kt <= R(0.6)) {
        a = R(0.512) - R(1.56) * kt + R(2.286) * kt2 - R(2.222) * kt3;
        b = R(0.37) + R(0.962) * kt;
        cc = R(-0.28) + R(0.932) * kt - R(2.048) * kt2;
    } else {
        a = R(-5.743) + R(21.77) * kt - R(27.49) * kt2 + R(11.56) * kt3;
        b = R(41.4) - R(118.5) * kt + R(66.05) * kt2 + R(31.9) * kt3;
        cc = R(-47.01) + R(184.2) * kt - R(222.0) * kt2 + R(73.81) * kt3;
    }
    const R dkn = a + b * exp(cc * am);
    R dni = (g[G_KNC] - dkn) * g[G_I0];
    if (g[G_DISCOK] == R(0) || ghi < R(0) || dni < R(0)) dni = R(0);
    const R dhi = ghi - dni * g[G_COSZ];
    R AI;
    if constexpr (sizeof(R) == 8) AI = dni / g[G_DNIEXTRA];
    else AI = dni * g[G_DNIEXTRA];
    R sky = dhi * (AI * g[G_RB] + (R(1) - AI) * g[G_TERM2]);
    sky = sky > R(0) ? sky : R(0);
    const R ground = ghi * g[G_GFAC];
    R poa_direct = dni * g[G_COSAOI];
    poa_direct = poa_direct > R(0) ? poa_direct : R(0);
    const R poa_diffuse = sky + ground;
    const R poa_global = poa_direct + poa_diffuse;
    // sapm_celltemp (pvmodel.py:69-70), open_rack_cell_glassback
    const R tmod = poa_global * exp(R(m[TMH_MOD_TEMP_A]) + R(m[TMH_MOD_TEMP_B]) * R(kp.wind)) + R(kp.temp_air);
    const R tcell = tmod + (poa_global / R(1000)) * R(m[TMH_MOD_TEMP_DT]);
    // sapm_effective_irradiance, suns (pvmodel.py:74-76)
    const R Ee = g[G_F1] * (poa_direct * g[G_F2] + R(m[TMH_MOD_FD]) * poa_diffuse) / R(1000);
    // sapm (pvmodel.py:77)
    const R q = R(1.60218e-19), kb = R(1.38066e-23);
    const R Bvmpo = R(m[TMH_MOD_BVMPO]) + R(m[TMH_MOD_MBVMP]) * (R(1) - Ee);
    R delta;
    if constexpr (sizeof(R) == 8) delta = R(m[TMH_MOD_N]) * kb * (tcell + R(273.15)) / q;
    else delta = R(m[TMH_MOD_N] * (1.38066e-23 / 1.60218e-19)) * (tcell + R(273.15));   // fp32: no 1e-23 subnormals
    const R logEe = Ee > R(0) ? log(Ee) : (Ee == R(0) ? -R(INFINITY) : R(NAN));
    const R imp = R(m[TMH_MOD_IMPO]) * (R(m[TMH_MOD_C0]) * Ee + R(m[TMH_MOD_C1]) * (Ee * Ee)) *
                  (R(1) + R(m[TMH_MOD_AIMP]) * (tcell - R(25)));
    const R dl = delta * logEe;
    R vmp = R(m[TMH_MOD_VMPO]) + R(m[TMH_MOD_C2]) * R(m[TMH_MOD_NS]) * delta * logEe +
            R(m[TMH_MOD_C3]) * R(m[TMH_MOD_NS]) * (dl * dl) + Bvmpo * (tcell - R(25));
    if (!isnan(vmp)) vmp = vmp > R(0) ? vmp : R(0);
    const R pdc = imp * vmp;
    // snlinverter (pvmodel.py:78)
    const R dv = vmp - R(iv[2]);
    const R A = R(iv[1]) * (R(1) + R(iv[5]) * dv);
    const R B = R(iv[3]) * (R(1) + R(iv[6]) * dv);
    const R C = R(iv[4]) * (R(1) + R(iv[7]) * dv);
    R ac = (R(iv[0]) / (A - B) - C * (A - B)) * (pdc - B) + C * ((pdc - B) * (pdc - B));
    if (!isnan(ac)) ac = R(iv[0]) < ac ? R(iv[0]) : ac;
    if (pdc < R(iv[3])) ac = R(-1) * fabs(R(iv[8]));
    if (isnan(ac)) return R(0);                       // .fillna(0.)
    return ac > R(0) ? ac : R(0);                      // .clip(lower=0.)
}

// ------------------------------------------------------------ chain kernel
template <typename R>
__device__ __forceinline__ void trace_store(void* p, uint64_t i, R v)
{
    if (p) reinterpret_cast<R*>(p)[i] = v;
}

// Advance chains [0, n) of this call over steps [step0, step0 + nsteps).
template <typename R, int RNG>
__global__ __launch_bounds__(256) void chain_kernel(KParams kp, StateView st, uint64_t chain0, uint32_t n,
                                                    int64_t step0, uint32_t nsteps,
                                                    const double* __restrict__ tab64,
                                                    const float* __restrict__ tab32, InjView inj,
                                                    TraceView tr, StatsView sv)
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
    // fp32 copies of the sampler pairs (refreshed at boundaries)
    R fb[6], fa[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        fb[k] = (R)ch.sb[k];
        fa[k] = (R)ch.sa[k];
    }
    double acc_pv = 0.0, acc_m = 0.0, acc_r = 0.0, mx = -INFINITY;
    const R sqrt6 = (R)kp.sqrt6, k15 = (R)(0.0015 * 8);
    for (uint32_t j = 0; j < nsteps; ++j) {
        const uint64_t step = (uint64_t)(step0 + j);
        const float* r32 = tab32 + (size_t)j * ROW;
        const uint32_t fl = __float_as_uint(r32[G_FLAGS]);
        R row[ROW];
        if constexpr (sizeof(R) == 8) {
#pragma unroll
            for (int i = 0; i < ROW; ++i) row[i] = tab64[(size_t)j * ROW + i];
        } else {
#pragma unroll
            for (int i = 0; i < ROW; ++i) row[i] = r32[i];
        }
        R csi = R(NAN), pv = R(NAN), meter = R(NAN), res = R(NAN);
        uint8_t cov = 255;
        if (ch.status == 0) {
            const double* r64 = tab64 + (size_t)j * ROW;
            if (fl & (FL_DAY | FL_HOUR | FL_MIN)) {           // _set_time boundaries (:120-126)
                const double hf = r64[G_HOURF];
                double u0, u1;
                if (fl & FL_DAY) {                              // _next_day
                    dr.two(ch, step, TAG_BOUNDARY, 0, u0, u1);
                    push(ch, S_CLEAR_DAY, normal(u0, 0.99, 0.08));
                    push(ch, S_WS, 2.14 * gammaincinv(2.69, u1));
                }
                if (fl & FL_HOUR) {                             // _next_hour (advances clear_day)
                    dr.two(ch, step, TAG_BOUNDARY, 1, u0, u1);
                    push(ch, S_CC, draw_cc(kp, ch, u0));
                    push(ch, S_CLEAR_DAY, normal(u1, 0.99, 0.08));
                }
                if (fl & FL_MIN) {                              // _next_min
                    dr.two(ch, step, TAG_BOUNDARY, 2, u0, u1);
                    const double cc = interp(ch.sb[S_CC], ch.sa[S_CC], hf);
                    push(ch, S_CLOUDY_NOISE, scaled_noise(kp, u0, 0.01, 0.003, cc));
                    push(ch, S_CLEAR_NOISE, scaled_noise(kp, u1, 0.001, 0.0015, cc));
                }
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    fb[k] = (R)ch.sb[k];
                    fa[k] = (R)ch.sa[k];
                }
            }
            ch.sec += 1;                                          // CloudCoverBinary.__next__
            uint32_t call = 0;
            while (ch.sec >= ch.t2 && ch.status == 0) {           // segment over: next_cloud(); next(self)
                const double hh = interp(ch.sb[S_CC], ch.sa[S_CC], r64[G_HOURF]);
                const double h = 0.95 < hh ? 0.95 : hh;           // update_parameters
                const double ws = interp(ch.sb[S_WS], ch.sa[S_WS], r64[G_DAYF]);
                const uint32_t f = next_cloud<RNG>(kp, st, c, ch, dr, h, ws, step, TAG_CLOUD, call++);
                if (f) ch.status = f;
                else ch.sec += 1;
            }
            double ue = 0.5, um = 0.5;
            if (ch.status == 0) {
                if constexpr (RNG == TMH_RNG_KEYED) {
                    dr.two(ch, step, TAG_STEP, 0, ue, um);
                } else {   // the meter is its own process in the reference: always keyed
                    ue = dr.one(ch, step, TAG_STEP, 0, 0);
                    const U4 b = keyed_block(kp.seed, chain, step, TAG_STEP, 0);
                    um = u52(b.z, b.w);
                }
            }
            if (ch.status == 0) {
                const bool covered = ch.sec < ch.t1;
                cov = covered ? 1 : 0;
                R cloudcover, z;
                if constexpr (sizeof(R) == 8) {
                    cloudcover = interp(ch.sb[S_CC], ch.sa[S_CC], row[G_HOURF]);
                    z = ndtri(ue);
                } else {
                    cloudcover = row[G_HOURF] * fa[S_CC] + (R(1) - row[G_HOURF]) * fb[S_CC];
                    z = ndtri_f(ue);
                }
                const R eps = z * (sqrt6 * (R(0.001) + k15 * cloudcover)) + R(0);
                if (covered)
                    csi = (row[G_DAYF] * fa[S_CLEAR_DAY] + (R(1) - row[G_DAYF]) * fb[S_CLEAR_DAY]) *
                          ((row[G_MINF] * fa[S_CLEAR_NOISE] + (R(1) - row[G_MINF]) * fb[S_CLEAR_NOISE]) + eps);
                else
                    csi = (row[G_HOURF] * fa[S_CLOUDY_HOUR] + (R(1) - row[G_HOURF]) * fb[S_CLOUDY_HOUR]) *
                          ((row[G_MINF] * fa[S_CLOUDY_NOISE] + (R(1) - row[G_MINF]) * fb[S_CLOUDY_NOISE]) + eps);
                pv = (kp.with_pv && !(fl & FL_NIGHT)) ? pv_power<R>(kp, row, csi) : R(0);
                if constexpr (sizeof(R) == 8) meter = 9000 * um;
                else meter = (R)(9000 * um);
                res = meter - pv;
                if (sv.acc) {
                    acc_pv += (double)pv;
                    acc_m += (double)meter;
                    acc_r += (double)res;
                    mx = fmax(mx, (double)res);
                }
                if (sv.hist) {
                    double x = ((double)res - sv.lo) * sv.scale;
                    int bin = x < 0.0 ? 0 : (x >= (double)(sv.n_bins - 1) ? (int)sv.n_bins - 1 : (int)x);
                    atomicAdd(&lds_hist[bin], 1u);
                }
            }
        }
        if (live) {
            const uint64_t o = (uint64_t)j * tr.ld + c;
            trace_store<R>(tr.csi, o, csi);
            trace_store<R>(tr.pv, o, pv);
            trace_store<R>(tr.meter, o, meter);
            trace_store<R>(tr.residual, o, res);
            if (tr.covered) tr.covered[o] = cov;
        }
    }
    if (live) {
        store_chain(st, c, ch);
        if (sv.acc) {
            sv.acc[c] += acc_pv;
            sv.acc[(size_t)n + c] += acc_m;
            sv.acc[2 * (size_t)n + c] += acc_r;
            sv.acc[3 * (size_t)n + c] = fmax(sv.acc[3 * (size_t)n + c], mx);
        }
    }
    if (sv.hist) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < sv.n_bins; i += blockDim.x)
            if (lds_hist[i]) atomicAdd((unsigned long long*)&sv.hist[i], (unsigned long long)lds_hist[i]);
    }
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

// field order: sb[6], sa[6], cl, clr, mstate, sec, L, pos, status, ncalls, sigma_cloud, sigma_clear, -, -
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

}  // namespace

struct tmh_engine {
    KParams kp;
    GParams gp;
    int device;
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

size_t tmh_workspace_bytes(uint32_t n_steps) { return align_up((size_t)n_steps * ROW * 8) + align_up((size_t)n_steps * ROW * 4); }

int tmh_engine_create(const tmh_params* p, const tmh_clock* clock, int device, struct tmh_engine** out)
{
    if (!p || !clock || !out) return fail(TMH_E_INVAL, "NULL argument to tmh_engine_create");
    if (p->cc_mode != TMH_CC_FAITHFUL && p->cc_mode != TMH_CC_MARKOV) return fail(TMH_E_INVAL, "bad cc_mode %d", p->cc_mode);
    if (p->rng_mode != TMH_RNG_KEYED && p->rng_mode != TMH_RNG_INJECTED) return fail(TMH_E_INVAL, "bad rng_mode %d", p->rng_mode);
    if (p->precision != TMH_FP32 && p->precision != TMH_FP64) return fail(TMH_E_INVAL, "bad precision %d", p->precision);
    if (clock->n_shifts < 0 || clock->n_shifts > 8) return fail(TMH_E_INVAL, "bad n_shifts %d", clock->n_shifts);
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
    memcpy(e->gp.site, p->site, sizeof e->gp.site);
    memcpy(e->gp.linke, p->linke, sizeof e->gp.linke);
    memcpy(e->gp.module, p->module, sizeof e->gp.module);
    e->gp.clock = *clock;
    e->device = device;
    *out = e;
    return TMH_OK;
}

int tmh_engine_destroy(struct tmh_engine* eng)
{
    delete eng;
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

int tmh_geometry(struct tmh_engine* eng, int64_t step0, uint32_t n_steps, double* table, void* stream)
{
    if (!eng || !table) return fail(TMH_E_INVAL, "NULL engine/table");
    if (n_steps == 0) return TMH_OK;
    if (step0 < 0) return fail(TMH_E_INVAL, "negative step0");
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    float* t32 = (float*)((char*)table + align_up((size_t)n_steps * ROW * 8));
    hipLaunchKernelGGL(geom_kernel, dim3((n_steps + 255) / 256), dim3(256), 0, (hipStream_t)stream, eng->gp, step0,
                       n_steps, table, t32);
    return hip_check(hipGetLastError(), "geom_kernel launch");
}

int tmh_step(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
             uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
             const void* table, void* stream)
{
    if (!eng || !state || !table) return fail(TMH_E_INVAL, "NULL engine/state/table");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    if (step0 < 0) return fail(TMH_E_INVAL, "negative step0");
    if (eng->kp.rng_mode == TMH_RNG_INJECTED && (!inj || !inj->u || inj->stride < inj->len))
        return fail(TMH_E_INVAL, "injected mode needs a stream with stride >= len");
    if (trace && (trace->csi || trace->pv || trace->meter || trace->residual || trace->covered) && trace->ld < n_chains)
        return fail(TMH_E_INVAL, "trace ld %llu < n_chains %u", (unsigned long long)trace->ld, n_chains);
    if (stats && stats->hist && (stats->n_bins == 0 || stats->n_bins > 16384 || !(stats->hi > stats->lo)))
        return fail(TMH_E_INVAL, "bad histogram spec (n_bins %u in [1,16384], hi > lo)", stats->n_bins);
    if (int rc = hip_check(hipSetDevice(eng->device), "hipSetDevice")) return rc;
    const double* t64 = (const double*)table;
    const float* t32 = (const float*)((const char*)table + align_up((size_t)n_steps * ROW * 8));
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
    dim3 grid((n_chains + 255) / 256), block(256);
    hipStream_t s = (hipStream_t)stream;
    const bool f64 = eng->kp.precision == TMH_FP64, keyed = eng->kp.rng_mode == TMH_RNG_KEYED;
#define LAUNCH(R, M)                                                                                                 \
    hipLaunchKernelGGL((chain_kernel<R, M>), grid, block, lds, s, eng->kp, v, chain0, n_chains, step0, n_steps, t64, \
                       t32, iv, tv, sv)
    if (f64 && keyed) LAUNCH(double, TMH_RNG_KEYED);
    else if (f64) LAUNCH(double, TMH_RNG_INJECTED);
    else if (keyed) LAUNCH(float, TMH_RNG_KEYED);
    else LAUNCH(float, TMH_RNG_INJECTED);
#undef LAUNCH
    return hip_check(hipGetLastError(), "chain_kernel launch");
}

int tmh_run(struct tmh_engine* eng, void* state, uint64_t chain0, uint32_t n_chains, int64_t step0,
            uint32_t n_steps, const tmh_ustream* inj, const tmh_trace* trace, const tmh_stats* stats,
            void* workspace, size_t workspace_bytes, void* stream)
{
    if (!eng || !state) return fail(TMH_E_INVAL, "NULL engine/state");
    if (n_chains == 0 || n_steps == 0) return TMH_OK;
    if (!workspace || workspace_bytes < tmh_workspace_bytes(n_steps))
        return fail(TMH_E_INVAL, "workspace too small: %zu < %zu", workspace_bytes, tmh_workspace_bytes(n_steps));
    if (int rc = tmh_geometry(eng, step0, n_steps, (double*)workspace, stream)) return rc;
    return tmh_step(eng, state, chain0, n_chains, step0, n_steps, inj, trace, stats, workspace, stream);
}

int tmh_probe(int fn, double a, const double* x, double* out, uint32_t n, void* stream)
{
    if (!x || !out) return fail(TMH_E_INVAL, "NULL probe buffers");
    if (n == 0) return TMH_OK;
    hipLaunchKernelGGL(probe_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fn, a, x, out, n);
    return hip_check(hipGetLastError(), "probe_kernel launch");
}

}  // extern "C"
