// Device math for the tmhpvsim kernels (gfx950).
//
// Random numbers: Philox4x32-10 (Random123 algorithm; counter layout in
// DESIGN.md "Random numbers"), 52-bit midpoint uniforms u = (2k+1) 2^-53.
// Variates: ONE uniform -> ONE variate by inverse CDF, the mapping the parity
// harness applies to the reference:
//   normal      ndtri(u)                      (scipy.stats.norm._rvs)
//   gamma(a)    P^-1(a, u)                    (scipy.stats.gamma._rvs, np.random.gamma)
//   t(df)       F_t^-1(df, u)                 (scipy.stats.t._rvs)
//   AL(kappa)   cloud_cover_hourly.py:100-104 (generic rv_continuous._rvs)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmh {

// ---------------------------------------------------------------- Philox
struct U4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Random123).  The key (the seed) is wave-uniform: round key r =
// key + r (W0, W1) is one s_add with a literal each, from a base the compiler must
// treat as fresh per call (the empty asm), so it neither hoists twenty
// loop-invariant round keys of a kernel's main loop into SGPRs (held across the
// loop they spill into VGPR lanes and every round pays a v_readlane) nor copies a
// bumped register it still needs.
__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1)
{
    k0 = __builtin_amdgcn_readfirstlane(k0);
    k1 = __builtin_amdgcn_readfirstlane(k1);
    asm volatile("" : "+s"(k0), "+s"(k1));
    const uint32_t kb0 = k0, kb1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        k0 = kb0 + (uint32_t)r * 0x9E3779B9u;
        k1 = kb1 + (uint32_t)r * 0xBB67AE85u;
        // one v_mad_u64_u32 per product (both halves) instead of mul_lo + mul_hi:
        // about 25 % less issue time per block on gfx950 (scripts/micro/philox_bench.hip)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        // rounds 0-1: the counter words are mostly wave-uniform (step, tag, chain
        // high word) and plain xors fold into SALU; from round 2 on both words are
        // per lane and the three-way xor is one gfx950 v_bitop3_b32 (0x96 = a^b^c)
        uint32_t n0, n2;
        if (r < 2) {
            n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
            n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        } else {
            n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
            n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        }
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ double u52(uint32_t lo, uint32_t hi)
{
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    return (double)((v >> 11) | 1ull) * 0x1p-53;
}

// 32-bit midpoint uniform (w + 1/2) 2^-32, exact in fp64 (per-second draws)
__device__ __forceinline__ double u32d(uint32_t w) { return ((double)w + 0.5) * 0x1p-32; }

// draw-family tags (ctr1 = tag << 28 | sub); must match oracle/philox.py
enum : uint32_t {
    TAG_STEP = 1,
    TAG_BOUNDARY = 2,
    TAG_CLOUD = 3,
    TAG_INIT = 4,
    TAG_INIT_CLOUD = 5,
    TAG_INIT_SEC = 6,
    // per-second draws, two streams of one block per four steps g = step >> 2, word step & 3
    // (x, y, z, w): the meter's and the noise's.  A night second needs only its meter word,
    // so four night seconds cost one block (round 2's one block per step pair held both).
    TAG_METER4 = 8,
    TAG_NOISE4 = 9
};

__device__ __forceinline__ uint32_t word_of(const struct U4& b, uint32_t q)   // b.x, .y, .z, .w for q = 0..3
{
    return q == 0 ? b.x : (q == 1 ? b.y : (q == 2 ? b.z : b.w));
}

__device__ __forceinline__ U4 keyed_block(uint64_t seed, uint64_t chain, uint64_t step, uint32_t tag,
                                          uint32_t sub)
{
    return philox4x32_10((uint32_t)step, (tag << 28) | (sub & 0x0FFFFFFFu), (uint32_t)chain,
                         (uint32_t)(chain >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
}

// ------------------------------------------------------------- variates
// standard normal quantile (fp64).  ocml's ncdfinv, polished by one Halley
// step on the erfc/erf residual so the result is within ~1 ulp of the exact
// quantile (the oracle's and scipy's ndtri agree to ~1e-16).
__device__ __noinline__ double ndtri(double p)
{
    double x = normcdfinv(p);
    if (!(p > 0.0) || !(p < 1.0)) return x;
    const double q = p - 0.5;
    double e;
    if (fabs(q) < 0.25) e = 0.5 * erf(x * 0.70710678118654752440) - q;
    else if (q < 0.0) e = 0.5 * erfc(-x * 0.70710678118654752440) - p;
    else e = (1.0 - p) - 0.5 * erfc(x * 0.70710678118654752440);   // upper tail, 1-p exact
    const double u = e * 2.50662827463100050242 * exp(0.5 * x * x);
    return x - u / (1.0 + 0.5 * x * u);
}

// the quantile without the polish (ocml's ncdfinv: within 7e-16 relative of the
// exact quantile on 2e5 32-bit midpoint uniforms); out of line like ndtri, so the
// kernels that call it per second keep their register budget
__device__ __noinline__ double ndtri_fast(double p) { return normcdfinv(p); }

// Giles' single-precision erfinv ("Approximating the erfinv function", GPU
// Computing Gems, 2011) as p(w), w = -log((1 - x)(1 + x)), erfinv(x) = p x:
// central polynomial in w - 2.5 for w < 5 (99.66 % of draws) ...
__device__ __forceinline__ float erfinv_central(float w0)
{
    const float v = w0 - 2.5f;
    float p = 2.81022636e-08f;
    p = fmaf(p, v, 3.43273939e-07f);
    p = fmaf(p, v, -3.5233877e-06f);
    p = fmaf(p, v, -4.39150654e-06f);
    p = fmaf(p, v, 0.00021858087f);
    p = fmaf(p, v, -0.00125372503f);
    p = fmaf(p, v, -0.00417768164f);
    p = fmaf(p, v, 0.246640727f);
    return fmaf(p, v, 1.50140941f);
}

// ... his tail polynomial in sqrt(w) - 3 for 5 <= w < 16, and for 16 <= w <= 21.5
// (t down to 2^-33, the smallest 32-bit midpoint uniform) a quintic in sqrt(w) - 4.3
// fitted here (scripts/fit_ndtri_tail.py: 1.7e-7 relative; Giles' tail is 4e-4 off
// there).  Straight-line code: no nested branch (the library quantile's nest of
// exec-mask branches cost the per-second loop ~20 scalar instructions a step).
__device__ __forceinline__ float erfinv_tail(float w0)
{
    const float s = __builtin_amdgcn_sqrtf(w0);
    const float v = s - 3.0f;
    float p = -0.000200214257f;
    p = fmaf(p, v, 0.000100950558f);
    p = fmaf(p, v, 0.00134934322f);
    p = fmaf(p, v, -0.00367342844f);
    p = fmaf(p, v, 0.00573950773f);
    p = fmaf(p, v, -0.0076224613f);
    p = fmaf(p, v, 0.00943887047f);
    p = fmaf(p, v, 1.00167406f);
    p = fmaf(p, v, 2.83297682f);
    const float e = s - 4.3f;
    float q = -5.854465416632593e-05f;
    q = fmaf(q, e, 0.00019957200856879354f);
    q = fmaf(q, e, -0.000567059323657304f);
    q = fmaf(q, e, 0.000624575128313154f);
    q = fmaf(q, e, 1.010045051574707f);
    q = fmaf(q, e, 4.14272403717041f);
    return w0 < 16.0f ? p : q;
}

// standard normal quantile from a fp64 uniform in fp32 arithmetic:
// ndtri(u) = sqrt(2) erfinv(2u - 1), the log argument (1 - x)(1 + x) = 4u(1 - u)
// formed in fp64 so the tails keep full relative precision.  53-bit uniforms reach
// past w = 21.5 (p < 5e-10 per draw): the fp32 library quantile there.
__device__ __forceinline__ float ndtri_f(double u)
{
    const float x = (float)(2.0 * u - 1.0);
    const float w0 = -__logf((float)(4.0 * u * (1.0 - u)));
    float p = erfinv_central(w0);
    if (w0 >= 5.0f) {
        if (w0 > 21.5f) {
            const double t = u < 0.5 ? u : 1.0 - u;
            const float z = normcdfinvf((float)t);
            return u < 0.5 ? z : -z;
        }
        p = erfinv_tail(w0);
    }
    return 1.41421356237309505f * (p * x);
}

// the same quantile straight from a 32-bit Philox word w, u = (w + 1/2) 2^-32,
// all in fp32: t = min(u, 1 - u) = (min(w, ~w) + 1/2) 2^-32 keeps the tails'
// relative precision, x = 2u - 1 comes from the signed word (per-second noise
// of the fp32 path; the fp64 path uses ndtri(u32d(w)))
__device__ __forceinline__ float ndtri_w(uint32_t w)
{
    const uint32_t m = w < 0x80000000u ? w : ~w;
    const float t = fmaf((float)m, 0x1p-32f, 0x1p-33f);
    const float x = fmaf((float)(int32_t)(w ^ 0x80000000u), 0x1p-31f, 0x1p-32f);
    // -log((1 - x)(1 + x)) = -log(4 t (1 - t)); the argument is >= 2^-31: no denormal path needed
    const float w0 = -0.693147180559945309f * __builtin_amdgcn_logf(fmaf(-4.0f * t, t, 4.0f * t));
    float p = erfinv_central(w0);
    if (w0 >= 5.0f) p = erfinv_tail(w0);   // 0.34 % of draws; w0 <= 21.5 for 32-bit words
    return 1.41421356237309505f * (p * x);
}

// ---- fp32 normal quantile of a 32-bit word from a table (the per-second noise, round 6) ----
// u = (w + 1/2) 2^-32, t = min(w, ~w) (u -> min(u, 1 - u)), uf = the fp32 value of (t + 1/2) 2^-32
// (as ndtri_w forms it).  uf's exponent e and its top ND32_S mantissa bits pick a segment of
// 1/32 octave; ndtri(uf) there is a cubic in the segment's low 18 mantissa bits r, its
// coefficients in g_nd32_tab (written by the host at engine creation: Chebyshev-node
// interpolation of the fp64 quantile, then rounded to fp32; tmh_engine.hip nd32_tab_upload).
// The index is (bits >> 18) & 511: e in [112, 127] (u in [2^-15, 2)), so 16 octaves of which
// e = 112..125 are used and e = 126 (uf rounded up to 0.5) holds zeros; u < 2^-15 (6e-5 of
// the draws) takes ndtri_w.  Measured against scipy's ndtri on every segment (numpy
// emulation of the fp32 Horner): <= 4.6e-7 absolute, the fp32 rounding of |z| ~ 4.
// 13 VALU (3 FMA for the cubic) instead of ndtri_w's ~25 with a log and a tail branch
// taken by a fifth of the waves.
constexpr int ND32_S = 5, ND32_SHIFT = 23 - ND32_S, ND32_N = 512, ND32_EMIN = 112;
__device__ float4 g_nd32_tab[ND32_N];

template <typename TP>   // TP: const float4* (g_nd32_tab or an LDS copy)
__device__ __forceinline__ float ndtri_t(uint32_t w, TP tab)
{
    const uint32_t m = w ^ (uint32_t)((int32_t)w >> 31);   // min(w, ~w)
    const uint32_t bits = __float_as_uint(fmaf((float)m, 0x1p-32f, 0x1p-33f));
    const float4 c = tab[(bits >> ND32_SHIFT) & (uint32_t)(ND32_N - 1)];
    const float r = (float)(bits & ((1u << ND32_SHIFT) - 1u));
    float q = fmaf(fmaf(fmaf(c.w, r, c.z), r, c.y), r, c.x);   // ndtri(min(u, 1 - u)) <= 0
    q = __uint_as_float(__float_as_uint(q) ^ (w & 0x80000000u));   // the upper half by symmetry
    if (__builtin_expect(bits < ((uint32_t)ND32_EMIN << 23), 0)) q = ndtri_w(w);   // the far tails
    return q;
}

__device__ __noinline__ void gamma_pq(double a, double x, double lga, double& P, double& Q)
{
    if (x <= 0.0) {
        P = 0.0;
        Q = 1.0;
        return;
    }
    const double lpre = -x + a * log(x) - lga;
    if (x < a + 1.0) {
        double ap = a, sum = 1.0 / a, del = sum;
        for (int n = 0; n < 1000; ++n) {
            ap += 1.0;
            del *= x / ap;
            sum += del;
            if (fabs(del) < fabs(sum) * 1e-17) break;
        }
        P = sum * exp(lpre);
        Q = 1.0 - P;
    } else {
        double b = x + 1.0 - a, c = 1.0 / 1e-300, d = 1.0 / b, h = d;
        for (int i = 1; i < 1000; ++i) {
            const double an = -i * (i - a);
            b += 2.0;
            d = an * d + b;
            if (fabs(d) < 1e-300) d = 1e-300;
            c = b + an / c;
            if (fabs(c) < 1e-300) c = 1e-300;
            d = 1.0 / d;
            const double del = d * c;
            h *= del;
            if (fabs(del - 1.0) < 1e-17) break;
        }
        Q = exp(lpre) * h;
        P = 1.0 - Q;
    }
}

// inverse regularized lower incomplete gamma (scipy.special.gammaincinv)
__device__ __noinline__ double gammaincinv(double a, double p)
{
    if (!(p > 0.0)) return 0.0;
    if (!(p < 1.0)) return INFINITY;
    const bool upper = p >= 0.5;
    const double target = upper ? 1.0 - p : p;
    const double z = ndtri(p), s = 1.0 / (9.0 * a);
    const double w = 1.0 - s + z * sqrt(s);
    double x = a * w * w * w;
    const double lg = lgamma(a);
    if (!(x > 1e-3 * a)) x = exp((log(p) + lgamma(a + 1.0)) / a);
    for (int it = 0; it < 8; ++it) {   // Halley from Wilson-Hilferty: 2-3 steps reach ~1 ulp
        double P, Q;
        gamma_pq(a, x, lg, P, Q);
        const double f = upper ? Q - target : P - target;
        const double dens = exp(-x + (a - 1.0) * log(x) - lg);
        if (dens == 0.0) break;
        double t = f / dens;
        if (upper) t = -t;
        const double hstep = t / (1.0 - 0.5 * t * ((a - 1.0) / x - 1.0));
        double xn = x - hstep;
        if (xn <= 0.0) xn = 0.5 * x;
        if (fabs(xn - x) <= 1e-15 * xn) {
            x = xn;
            break;
        }
        x = xn;
    }
    return x;
}

__device__ __noinline__ double betacf(double a, double b, double x)
{
    const double qab = a + b, qap = a + 1.0, qam = a - 1.0;
    double c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < 1e-300) d = 1e-300;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m < 10000; ++m) {
        const int m2 = 2 * m;
        double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < 1e-300) d = 1e-300;
        c = 1.0 + aa / c;
        if (fabs(c) < 1e-300) c = 1e-300;
        d = 1.0 / d;
        h *= d * c;
        aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
        d = 1.0 + aa * d;
        if (fabs(d) < 1e-300) d = 1e-300;
        c = 1.0 + aa / c;
        if (fabs(c) < 1e-300) c = 1e-300;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < 1e-16) break;
    }
    return h;
}

__device__ __noinline__ double ibeta(double a, double b, double x)
{
    if (x <= 0.0) return 0.0;
    if (x >= 1.0) return 1.0;
    const double lbt = lgamma(a + b) - lgamma(a) - lgamma(b) + a * log(x) + b * log1p(-x);
    if (x < (a + 1.0) / (a + b + 2.0)) return exp(lbt) * betacf(a, b, x) / a;
    return 1.0 - exp(lbt) * betacf(b, a, 1.0 - x) / b;
}

__device__ __noinline__ double t_resid(double df, double t, double p)
{
    const double t2 = t * t;
    if (t2 < df) return (0.5 - p) - 0.5 * ibeta(0.5, 0.5 * df, t2 / (df + t2));
    return 0.5 * ibeta(0.5 * df, 0.5, df / (df + t2)) - p;
}

// inverse Student-t CDF (scipy.special.stdtrit), lower half; upper by symmetry
__device__ __noinline__ double stdtrit(double df, double p)
{
    if (!(p > 0.0)) return -INFINITY;
    if (!(p < 1.0)) return INFINITY;
    if (p == 0.5) return 0.0;
    double sign = -1.0;
    if (p > 0.5) {
        p = 1.0 - p;
        sign = 1.0;
    }
    const double lc = lgamma(0.5 * (df + 1.0)) - lgamma(0.5 * df) - 0.5 * log(df * 3.14159265358979323846);
    double t;
    if (p < 1e-5) {
        t = -exp((lc + 0.5 * (df + 1.0) * log(df) - log(df) - log(p)) / df);
    } else {
        const double z = ndtri(p), z2 = z * z;
        t = z + (z2 * z + z) / (4.0 * df) + (5.0 * z2 * z2 * z + 16.0 * z2 * z + 3.0 * z) / (96.0 * df * df);
    }
    if (t > -1e-300) t = -1e-300;
    for (int it = 0; it < 200; ++it) {
        const double f = t_resid(df, t, p);
        const double ldens = lc - 0.5 * (df + 1.0) * log1p(t * t / df);
        double tn;
        if (t < -1e3) {
            const double F = f + p;
            const double slope = exp(ldens + log(-t) - log(F));
            tn = -exp(log(-t) + log1p(f / p) / slope);
        } else {
            tn = t - f / exp(ldens);
        }
        if (tn >= 0.0) tn = 0.5 * t;
        if (fabs(tn - t) <= 1e-15 * fabs(tn)) {
            t = tn;
            break;
        }
        t = tn;
    }
    return sign < 0.0 ? t : -t;
}

// asymmetric Laplace ppf, cloud_cover_hourly.py:100-104 (op order kept)
__device__ __noinline__ double al_ppf(double y, double kappa)
{
    const double k2 = kappa * kappa;
    if (y < k2 / (1.0 + k2)) return kappa * log((1.0 + k2) / k2 * y);
    return -1.0 / kappa * log((1.0 + k2) * (1.0 - y));
}

// fp64 pow out of line (cloud lengths, cloud_cover_binary.py:40): keeps callers' registers low
__device__ __noinline__ double pow_d(double x, double y) { return pow(x, y); }

// ---- fp64 natural log from a table (the PV chain's log(Ee), pv_power_d) ----
// x = 2^e m, m in [1, 2); c_i = 1 + (i + 1/2) / 128 for the top 7 bits i of m's
// mantissa, u = m / c_i - 1 (|u| <= 2^-8, as fma(m, 1 / c_i, -1)), and
// log x = e ln 2 + log c_i + log1p(u) with log1p to u^7 / 7 (truncation < 2^-67).
// Absolute error a few 1e-16 (the rounding of e ln 2, 1 / c_i and log c_i; numpy
// emulation over 45,000 x in [1e-8, 2]: at most one ulp of the result): the PV chain
// needs 1e-12 relative.  13 VALU instead of ocml log's ~90.  Zero, negative, NaN,
// infinite and subnormal x take ocml's log (and its -inf / NaN).
// g_pv_tab: t[2 i] = 1 / c_i, t[2 i + 1] = log c_i, then exp_tab's 2^(i / 64) at
// t[EXP_OFF + i], then ndtri64's three pieces at t[NDTRI_OFF + NDTRI_STRIDE q] (the piece's
// center, then its coefficients, degree 0 first); written
// once per engine from the host (tmh_engine_create); every fp64
// PV evaluation reads these same values (the expansion from an LDS copy), so the kernels
// agree bit for bit.
constexpr int LOG_TAB = 128, EXP_TAB = 64, EXP_OFF = 2 * LOG_TAB, NDTRI_OFF = EXP_OFF + EXP_TAB, NDTRI_DEG = 13,
              NDTRI_PIECES = 3, NDTRI_STRIDE = NDTRI_DEG + 2, PV_TAB = NDTRI_OFF + NDTRI_PIECES * NDTRI_STRIDE;
__device__ double g_pv_tab[PV_TAB];
typedef __attribute__((address_space(3))) const double LdsD;

// (out of line: inlined, its constants would be hoisted into registers across the caller's loop)
__device__ __noinline__ double log_edge(double x) { return x > 0.0 ? log(x) : (x == 0.0 ? -INFINITY : NAN); }

template <typename TP>   // TP: LdsD* (an LDS copy) or const double* (g_pv_tab)
__device__ __forceinline__ double log_tab(double x, TP t)
{
    if (__builtin_expect(!(x >= 0x1p-1022) || x == INFINITY, 0)) return log_edge(x);
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    const uint32_t hi = (uint32_t)(bits >> 32);
    const int e = (int)(hi >> 20) - 1023;
    const uint32_t i = (hi >> 13) & (uint32_t)(LOG_TAB - 1);
    const double m = __longlong_as_double((long long)(((uint64_t)((hi & 0x000FFFFFu) | 0x3FF00000u) << 32) |
                                                      (bits & 0xFFFFFFFFull)));
    const double u = fma(m, t[2 * i], -1.0);
    double h = fma(u, 1.0 / 7.0, -1.0 / 6.0);
    h = fma(h, u, 1.0 / 5.0);
    h = fma(h, u, -1.0 / 4.0);
    h = fma(h, u, 1.0 / 3.0);
    h = fma(h, u, -1.0 / 2.0);
    return fma((double)e, 0.693147180559945309417, t[2 * i + 1]) + fma(u * u, h, u);
}

// ---- fp64 normal quantile of a 32-bit word (the per-second noise, noise_z<double>) ----
// p = (w + 1/2) 2^-32, x = 2p - 1 (exact), ndtri(p) = sqrt(2) erfinv(x) = sqrt(2) x f(w')
// with w' = -log(1 - x^2) = -log(4 p (1 - p)) and, for w' < 6.25 (p in ~[5e-4, 1 - 5e-4],
// 99.9 % of the draws), f a degree-13 polynomial in w' - c_q on the lane's piece q of
// [0, 2), [2, 4), [4, 6.25) (Giles' form, "Approximating the erfinv function", refitted in
// pieces: scripts/fit_ndtri_f64.py, <= 3.1e-16 relative in an fp64 Horner evaluation; round 4
// used one piece of degree 22, 9 fmas more per daylight second at 4.2e-16); the rest take
// ocml's quantile out of line (ndtri_fast).  The piece is chosen per lane by table offset,
// not by branch.  The coefficients come from the table (an LDS copy in the expansion, read
// through `tab_fence` in chunks so they are loaded shortly before use).
constexpr double NDTRI_CENTER[NDTRI_PIECES] = {1.0, 3.0, 5.125};
constexpr double NDTRI_COEF[NDTRI_PIECES][NDTRI_DEG + 1] = {   // degree 0 first (the host copies them into g_pv_tab)
    {1.1273743936892275, 0.24783287028621095, 0.004250709244840092, -0.002376369955580531, 0.00010012177598503247,
     3.820187251368197e-05, -4.275584236922046e-06, -5.652253874123589e-07, 1.2231291266949573e-07,
     6.040592330213068e-09, -3.017929272010491e-09, 1.5906520115066905e-11, 6.298924235630103e-11,
     -3.2253159972831256e-12},
    {1.6235420064648298, 0.24163040416615827, -0.0057381352210059446, -0.0008361817769086462, 0.0001950613244170301,
     -1.2716422648914508e-05, -1.7480021231028974e-06, 4.499854856199944e-07, -2.3688647408781946e-08,
     -5.467350086581866e-09, 1.110687588033803e-09, -3.117460148479959e-11, -1.7262109450729976e-11,
     2.5158500392913756e-12},
    {2.1064123296343875, 0.21189284366397468, -0.007210971340179456, 0.00015540013139557572, 4.64226024498019e-05,
     -9.737631064560686e-06, 9.675017285744816e-07, -1.947519718448861e-08, -1.048456228150318e-08,
     1.8905557238598573e-09, -1.415734465250556e-10, -5.179746543640047e-12, 2.839759278393376e-12,
     -3.365321693201019e-13}};

template <typename TP>
__device__ __forceinline__ TP tab_fence(TP t)
{
    if constexpr (__is_same(TP, const double*)) return t;
    else {
        uint32_t a = (uint32_t)(uintptr_t)t;
        asm volatile("" : "+v"(a));
        return (TP)(uintptr_t)a;
    }
}

template <typename TP>
__device__ __forceinline__ double ndtri64(uint32_t w, TP t)
{
    const double p = ((double)w + 0.5) * 0x1p-32;
    const double x = 2.0 * p - 1.0;
    const double ww = -log_tab(4.0 * p * (1.0 - p), t);
    if (__builtin_expect(!(ww < 6.25), 0)) return ndtri_fast(p);
    const int q = NDTRI_OFF + NDTRI_STRIDE * ((ww >= 2.0 ? 1 : 0) + (ww >= 4.0 ? 1 : 0));   // the lane's piece
    t = tab_fence(t);
    const double u = ww - t[q];
    double f = t[q + 1 + NDTRI_DEG];
#pragma unroll
    for (int k = NDTRI_DEG - 1; k >= 0; --k) {
        if (k % 6 == 5) t = tab_fence(t);
        f = fma(f, u, t[q + 1 + k]);
    }
    return (1.4142135623730950488 * x) * f;
}

// ---- fp64 exp from the same table (DISC's exp(c am), pv_power_d) ----
// x = (k / 64) ln 2 + r, k = rint(64 x / ln 2), |r| <= ln 2 / 128 (r from a two-part
// ln 2 / 64 whose high part times k is exact for |k| < 2^16); exp x = 2^(k >> 6)
// 2^((k & 63) / 64) p(r), p to r^6 / 720.  Numpy emulation over 100,000 x in [-40, 3]:
// at most 1.5 ulp.  14 VALU instead of ocml exp's ~31; |x| >= 700 and NaN take ocml's.
__device__ __noinline__ double exp_edge(double x) { return exp(x); }

template <typename TP>
__device__ __forceinline__ double exp_tab(double x, TP t)
{
    if (__builtin_expect(!(fabs(x) < 700.0), 0)) return exp_edge(x);
    const double kf = rint(x * 92.332482616893656768);   // 64 / ln 2
    double r = fma(-kf, 0x1.62e42fefa0000p-7, x);
    r = fma(-kf, 2.572804640231345e-14, r);
    double p = fma(r, 1.0 / 720.0, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int k = (int)kf;
    return ldexp(t[EXP_OFF + (k & (EXP_TAB - 1))] * p, k >> 6);
}

}  // namespace tmh
