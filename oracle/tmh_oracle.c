/* TEST INFRASTRUCTURE ONLY — plain-C restatement of the tmhpvsim hot path.
 *
 * The checker for the HIP kernels (tests/, __graft_entry__.smoke()) and the
 * CPU baseline of bench.py ("kind": "port").  Never linked by the product.
 *
 * Restates, line by line:
 *   InterpolatedSampler            tmhpvsim/clearskyindexmodel.py:12-40
 *   ClearskyindexModel init        tmhpvsim/clearskyindexmodel.py:57-99
 *   _next_day/_next_hour/_next_min tmhpvsim/clearskyindexmodel.py:101-111
 *   _set_time                      tmhpvsim/clearskyindexmodel.py:113-126
 *   next (per-second CSI)          tmhpvsim/clearskyindexmodel.py:128-160
 *   random_windspeed               tmhpvsim/cloud_cover_binary.py:5-23
 *   random_cloudlength_in_s        tmhpvsim/cloud_cover_binary.py:25-40
 *   CloudCoverBinary               tmhpvsim/cloud_cover_binary.py:42-117
 *   asymmetric Laplace ppf         tmhpvsim/cloud_cover_hourly.py:100-104
 *   get_cloud_cover (hourly draw)  tmhpvsim/cloud_cover_hourly.py:290-316
 *   PVModel.populate_cache PV      tmhpvsim/pvmodel.py:50-80 (pvlib 0.6.3 model
 *                                  choices restated from the published models;
 *                                  pvlib is absent here: PV parity vs pvlib is
 *                                  UNPINNED)
 *   get_meter_value                tmhpvsim/metersim.py:49-51
 *   residual = meter - pv          tmhpvsim/pvsim.py:80-83
 *
 * Random numbers: "one uniform -> one variate by inverse CDF" (SURVEY App. D),
 * uniforms either from an injected per-chain stream consumed in reference
 * order, or keyed Philox4x32-10 (see oracle/philox.py for the contract).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_SIGMA_CAP 4096

/* diagnostics: histogram of len(sigma_cloud) after each successful next_cloud */
static uint64_t g_Lhist[ORC_SIGMA_CAP + 1];
void orc_L_hist(uint64_t* out, int reset)
{
    memcpy(out, g_Lhist, sizeof g_Lhist);
    if (reset) memset(g_Lhist, 0, sizeof g_Lhist);
}
/* diagnostics: histogram of tries per successful next_cloud call (index = tries, 0..40) */
static uint64_t g_Thist[41];
void orc_T_hist(uint64_t* out, int reset)
{
    memcpy(out, g_Thist, sizeof g_Thist);
    if (reset) memset(g_Thist, 0, sizeof g_Thist);
}

enum { ST_OK = 0, ST_NAMEERROR_INIT = 1, ST_ASSERT_BINARY = 2, ST_SIGMA_OVERFLOW = 3,
       ST_U_EXHAUSTED = 4 };
enum { TAG_STEP = 1, TAG_BOUNDARY = 2, TAG_CLOUD = 3, TAG_INIT = 4, TAG_INIT_CLOUD = 5, TAG_METER4 = 8, TAG_NOISE4 = 9,
       TAG_INIT_SEC = 6 };
enum { S_CC = 0, S_CLEAR_DAY = 1, S_CLOUDY_HOUR = 2, S_CLOUDY_NOISE = 3, S_CLEAR_NOISE = 4,
       S_WS = 5 };

typedef struct {
    int32_t cc_mode;      /* 0 faithful (reference behaviour), 1 markov (persistent chain) */
    int32_t rng_mode;     /* 0 keyed Philox, 1 injected stream */
    uint64_t seed;        /* keyed seed; the meter always draws keyed (own stream) */
    int32_t with_pv;
    int32_t n_threads;
    double shapes[6][4];  /* loc, scale, kappa, df */
    int32_t shape_is_t[6];
    double edges[6];      /* right edges of the cloud-cover bins */
    double site[8];       /* lat, lon, altitude, tilt, surface azimuth, albedo, temp_air, wind */
    double linke[12];     /* monthly Linke turbidity (LinkeTurbidities.h5 absent offline) */
    double module[26];    /* SAPM: A0..A4 B0..B5 FD Impo Vmpo Aimp C0 C1 C2 C3 Bvmpo Mbvmp N Ns a b dT */
    double inverter[9];   /* Sandia: Paco Pdco Vdco Pso C0 C1 C2 C3 Pnt */
} orc_params;

/* ------------------------------------------------------------------ Philox */
static void philox4x32_10(const uint32_t c[4], const uint32_t k[2], uint32_t o[4])
{
    uint32_t x0 = c[0], x1 = c[1], x2 = c[2], x3 = c[3], k0 = k[0], k1 = k[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        x0 = hi1 ^ x1 ^ k0; x1 = lo1; x2 = hi0 ^ x3 ^ k1; x3 = lo0;
    }
    o[0] = x0; o[1] = x1; o[2] = x2; o[3] = x3;
}

static double u52(uint32_t lo, uint32_t hi)
{
    uint64_t v = ((uint64_t)hi << 32) | lo;
    return (double)((v >> 11) | 1ull) * 0x1p-53;
}

/* injected uniform streams (oracle/philox.py injected_stream, key = (seed, chain),
 * counter = block number, two 53-bit uniforms per block): out[c * len + k] */
void orc_injected_streams(uint64_t seed, uint64_t chain0, uint32_t n_chains, uint32_t len, double* out, int n_threads)
{
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (uint32_t c = 0; c < n_chains; ++c) {
        const uint32_t k[2] = {(uint32_t)seed, (uint32_t)(chain0 + c)};
        double* o = out + (size_t)c * len;
        for (uint32_t b = 0; 2 * b < len; ++b) {
            const uint32_t ctr[4] = {b, 0u, 0u, 0u};
            uint32_t r[4];
            philox4x32_10(ctr, k, r);
            o[2 * b] = u52(r[0], r[1]);
            if (2 * b + 1 < len) o[2 * b + 1] = u52(r[2], r[3]);
        }
    }
}

void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out)
{
    philox4x32_10(ctr, key, out);
}

static double keyed_u(uint64_t seed, uint64_t chain, uint64_t step, uint32_t tag, uint32_t sub,
                      int half)
{
    uint32_t c[4] = {(uint32_t)step, (tag << 28) | (sub & 0x0FFFFFFFu), (uint32_t)chain,
                     (uint32_t)(chain >> 32)};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, o[4];
    philox4x32_10(c, k, o);
    return half ? u52(o[2], o[3]) : u52(o[0], o[1]);
}

/* per-second draws: two streams, the noise's (TAG_NOISE4) and the meter's (TAG_METER4),
 * one block per four steps g = step >> 2, word step & 3; 32-bit midpoint uniforms
 * (w + 1/2) 2^-32 (the device's keyed_block + word_of, tmh_math.h) */
static uint32_t step_word(uint64_t seed, uint64_t chain, uint64_t step, uint32_t tag)
{
    uint32_t c[4] = {(uint32_t)(step >> 2), tag << 28, (uint32_t)chain, (uint32_t)(chain >> 32)};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, o[4];
    philox4x32_10(c, k, o);
    return o[step & 3];
}

static void step_u(uint64_t seed, uint64_t chain, uint64_t step, double* ue, double* um)
{
    *ue = ((double)step_word(seed, chain, step, TAG_NOISE4) + 0.5) * 0x1p-32;
    *um = ((double)step_word(seed, chain, step, TAG_METER4) + 0.5) * 0x1p-32;
}

/* --------------------------------------------------------------- variates */
/* Standard normal quantile: rational first guess + Halley refinement on
 * Phi(x) = erfc(-x/sqrt2)/2 (glibc erfc).  Matches scipy.special.ndtri to
 * ~1 ulp (pinned against tests/golden/functions.npz). */
double orc_ndtri(double p)
{
    if (!(p > 0.0)) return p == 0.0 ? -INFINITY : NAN;
    if (!(p < 1.0)) return p == 1.0 ? INFINITY : NAN;
    if (p > 0.5) return -orc_ndtri(1.0 - p);        /* 1 - p exact for p >= 0.5 */
    static const double a[6] = {-3.969683028665376e+01, 2.209460984245205e+02,
                                -2.759285104469687e+02, 1.383577518672690e+02,
                                -3.066479806614716e+01, 2.506628277459239e+00};
    static const double b[5] = {-5.447609879822406e+01, 1.615858368580409e+02,
                                -1.556989798598866e+02, 6.680131188771972e+01,
                                -1.328068155288572e+01};
    static const double c[6] = {-7.784894002430293e-03, -3.223964580411365e-01,
                                -2.400758277161838e+00, -2.549732539343734e+00,
                                4.374664141464968e+00, 2.938163982698783e+00};
    static const double d[4] = {7.784695709041462e-03, 3.224671290700398e-01,
                                2.445134137142996e+00, 3.754408661907416e+00};
    double x;
    if (p < 0.02425) {
        double q = sqrt(-2.0 * log(p));
        x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
            ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0);
    } else {
        double q = p - 0.5, r = q * q;
        x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
            (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0);
    }
    double q0 = p - 0.5;                              /* exact for p in [0.25, 0.5] */
    for (int it = 0; it < 4; ++it) {
        /* residual Phi(x) - p: erf form near the centre avoids cancellation */
        double e = p > 0.25 ? 0.5 * erf(x / M_SQRT2) - q0 : 0.5 * erfc(-x / M_SQRT2) - p;
        double u = e * sqrt(2.0 * M_PI) * exp(0.5 * x * x);
        double dx = u / (1.0 + 0.5 * x * u);
        x -= dx;
        if (fabs(dx) <= 1e-17 * fabs(x)) break;
    }
    return x;
}

/* regularized lower / upper incomplete gamma (series / Lentz continued fraction) */
static void gamma_pq(double a, double x, double* P, double* Q)
{
    if (x <= 0.0) { *P = 0.0; *Q = 1.0; return; }
    double lpre = -x + a * log(x) - lgamma(a);
    if (x < a + 1.0) {
        double ap = a, sum = 1.0 / a, del = sum;
        for (int n = 0; n < 1000; ++n) {
            ap += 1.0; del *= x / ap; sum += del;
            if (fabs(del) < fabs(sum) * 1e-17) break;
        }
        *P = sum * exp(lpre); *Q = 1.0 - *P;
    } else {
        double b = x + 1.0 - a, c = 1.0 / 1e-300, d = 1.0 / b, h = d;
        for (int i = 1; i < 1000; ++i) {
            double an = -i * (i - a);
            b += 2.0;
            d = an * d + b; if (fabs(d) < 1e-300) d = 1e-300;
            c = b + an / c; if (fabs(c) < 1e-300) c = 1e-300;
            d = 1.0 / d;
            double del = d * c; h *= del;
            if (fabs(del - 1.0) < 1e-17) break;
        }
        *Q = exp(lpre) * h; *P = 1.0 - *Q;
    }
}

/* inverse of the regularized lower incomplete gamma: Wilson-Hilferty start,
 * Halley steps on P (p < 1/2) or Q (p >= 1/2) for relative accuracy. */
double orc_gammaincinv(double a, double p)
{
    if (!(p > 0.0)) return 0.0;
    if (!(p < 1.0)) return INFINITY;
    int upper = p >= 0.5;
    double target = upper ? 1.0 - p : p;
    double z = orc_ndtri(p), s = 1.0 / (9.0 * a);
    double x = a * pow(1.0 - s + z * sqrt(s), 3.0);
    if (!(x > 1e-3 * a)) x = exp((log(p) + lgamma(a + 1.0)) / a);
    double lg = lgamma(a);
    for (int it = 0; it < 8; ++it) {   /* Halley from Wilson-Hilferty: 2-3 steps reach ~1 ulp */
        double P, Q;
        gamma_pq(a, x, &P, &Q);
        double f = upper ? Q - target : P - target;
        double dens = exp(-x + (a - 1.0) * log(x) - lg);
        if (dens == 0.0) break;
        double t = f / dens;                       /* Newton step for P (sign flips for Q) */
        if (upper) t = -t;
        double h = t / (1.0 - 0.5 * t * ((a - 1.0) / x - 1.0));   /* Halley */
        double xn = x - h;
        if (xn <= 0.0) xn = 0.5 * x;
        if (fabs(xn - x) <= 1e-15 * xn) { x = xn; break; }
        x = xn;
    }
    return x;
}

/* regularized incomplete beta I_x(a, b) by continued fraction (Lentz) */
static double betacf(double a, double b, double x)
{
    double qab = a + b, qap = a + 1.0, qam = a - 1.0, c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < 1e-300) d = 1e-300;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m < 10000; ++m) {
        int m2 = 2 * m;
        double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
        d = 1.0 + aa * d; if (fabs(d) < 1e-300) d = 1e-300;
        c = 1.0 + aa / c; if (fabs(c) < 1e-300) c = 1e-300;
        d = 1.0 / d; h *= d * c;
        aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
        d = 1.0 + aa * d; if (fabs(d) < 1e-300) d = 1e-300;
        c = 1.0 + aa / c; if (fabs(c) < 1e-300) c = 1e-300;
        d = 1.0 / d;
        double del = d * c; h *= del;
        if (fabs(del - 1.0) < 1e-16) break;
    }
    return h;
}

static double ibeta(double a, double b, double x)
{
    if (x <= 0.0) return 0.0;
    if (x >= 1.0) return 1.0;
    double lbt = lgamma(a + b) - lgamma(a) - lgamma(b) + a * log(x) + b * log1p(-x);
    if (x < (a + 1.0) / (a + b + 2.0)) return exp(lbt) * betacf(a, b, x) / a;
    return 1.0 - exp(lbt) * betacf(b, a, 1.0 - x) / b;
}

/* Student-t CDF residual F(t) - p for t <= 0, p < 1/2: tail form
 * 0.5 * I_{df/(df+t^2)}(df/2, 1/2) far out, centre form
 * 0.5 - 0.5 * I_{t^2/(df+t^2)}(1/2, df/2) near 0 (no cancellation). */
static double t_resid(double df, double t, double p)
{
    double t2 = t * t;
    if (t2 < df) return (0.5 - p) - 0.5 * ibeta(0.5, 0.5 * df, t2 / (df + t2));
    return 0.5 * ibeta(0.5 * df, 0.5, df / (df + t2)) - p;
}

/* inverse Student-t CDF (scipy.special.stdtrit): Cornish-Fisher start + Newton */
double orc_stdtrit(double df, double p)
{
    if (!(p > 0.0)) return -INFINITY;
    if (!(p < 1.0)) return INFINITY;
    if (p == 0.5) return 0.0;
    if (p > 0.5) return -orc_stdtrit(df, 1.0 - p);
    double lc = lgamma(0.5 * (df + 1.0)) - lgamma(0.5 * df) - 0.5 * log(df * M_PI);
    double t;
    if (p < 1e-5) {   /* tail asymptote F(-|t|) ~ c df^((df+1)/2) |t|^-df / df */
        t = -exp((lc + 0.5 * (df + 1.0) * log(df) - log(df) - log(p)) / df);
    } else {          /* Cornish-Fisher */
        double z = orc_ndtri(p), z2 = z * z;
        t = z + (z2 * z + z) / (4.0 * df) + (5.0 * z2 * z2 * z + 16.0 * z2 * z + 3.0 * z) / (96.0 * df * df);
    }
    if (t > -1e-300) t = -1e-300;
    for (int it = 0; it < 200; ++it) {
        double f = t_resid(df, t, p);
        double ldens = lc - 0.5 * (df + 1.0) * log1p(t * t / df);
        double tn;
        if (t < -1e3) {   /* Newton of log F against log|t| in the far tail */
            double F = f + p;
            double slope = exp(ldens + log(-t) - log(F));   /* -d log F / d log|t| */
            tn = -exp(log(-t) + log1p(f / p) / slope);
        } else {
            tn = t - f / exp(ldens);
        }
        if (tn >= 0.0) tn = 0.5 * t;
        if (fabs(tn - t) <= 1e-15 * fabs(tn)) { t = tn; break; }
        t = tn;
    }
    return t;
}

/* cloud_cover_hourly.py:100-104 — note the op order (1+k2)/k2*y */
double orc_al_ppf(double y, double kappa)
{
    double k2 = kappa * kappa;
    if (y < k2 / (1.0 + k2)) return kappa * log((1.0 + k2) / k2 * y);
    return -1.0 / kappa * log((1.0 + k2) * (1.0 - y));
}

/* ------------------------------------------------------------------- chain */
typedef struct {
    double s[6][2];               /* sampler (before, after) */
    double h, ws;                 /* CloudCoverBinary.hourly_cloudcover / windspeed */
    int64_t sec;
    double cl, clr;
    int L;
    double sc[ORC_SIGMA_CAP], sl[ORC_SIGMA_CAP];
    double mstate;                /* markov-mode persistent hourly state */
    uint64_t ncalls;              /* next_cloud calls so far (keyed counter of CLOUD draws) */
    const double* tab;            /* per-chain shape table [6][4] (NULL: orc_params.shapes) */
    const int32_t* tab_t;
    int status;
    /* rng */
    uint64_t chain;
    const double* inj;
    uint64_t inj_len, pos;
} chain_t;

typedef struct {
    const orc_params* P;
    double omb, alpha, delta, expo;      /* cloud_cover_binary.py:35-40 */
    double sqrt09, sqrt6;
} ctx_t;

static double draw_u(const ctx_t* X, chain_t* ch, uint64_t step, uint32_t tag, uint32_t sub, int half)
{
    if (X->P->rng_mode == 1) {
        if (ch->pos >= ch->inj_len) { if (!ch->status) ch->status = ST_U_EXHAUSTED; return 0.5; }
        return ch->inj[ch->pos++];
    }
    return keyed_u(X->P->seed, ch->chain, step, tag, sub, half);
}

static double interp(const double s[2], double f) { return f * s[1] + (1.0 - f) * s[0]; }

static void push(double s[2], double v) { s[0] = s[1]; s[1] = v; }

/* hourly cloud cover draw: get_cloud_cover(distributions) (cloud_cover_hourly.py:309-316).
 * faithful: a fresh generator per call -> state 1.0 (clearskyindexmodel.py:61-63). */
/* optional per-chain shape tables (a lat/lon sweep, C5): chain c (index within
 * the orc_run call) draws from g_tab[c] when set, else from orc_params.shapes */
static const double* g_tab;
static const int32_t* g_tab_t;
static uint32_t g_tab_n;
void orc_set_tables(const double* shapes /* [n][6][4] */, const int32_t* is_t /* [n][6] */, uint32_t n)
{
    g_tab = shapes;
    g_tab_t = is_t;
    g_tab_n = n;
}

static double draw_cc(const ctx_t* X, chain_t* ch, double u)
{
    const orc_params* P = X->P;
    double state = P->cc_mode == 1 ? ch->mstate : 1.0;
    int bin = 0;
    while (bin < 5 && P->edges[bin] < state) ++bin;        /* searchsorted(bins, state), side=left */
    const double* sh = ch->tab ? ch->tab + 4 * bin : P->shapes[bin];
    const int is_t = ch->tab ? ch->tab_t[bin] : P->shape_is_t[bin];
    double v;
    if (is_t) v = orc_stdtrit(sh[3], u);
    else v = orc_al_ppf(u, sh[2]);
    v = v * sh[1] + sh[0];                               /* scipy rvs: vals * scale + loc */
    double x = state + v;
    x = x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);              /* np.clip(., 0, 1) */
    if (P->cc_mode == 1) ch->mstate = x;
    return x;
}

static double normal(double u, double loc, double scale) { return orc_ndtri(u) * scale + loc; }

static double scaled_noise(const ctx_t* X, double u, double s0, double s1, double cc)
{
    /* norm.rvs(loc=1., scale=np.sqrt(0.9) * (sigma0 + sigma1 * 8 * cc)), clearskyindexmodel.py:86-88 */
    return normal(u, 1.0, X->sqrt09 * (s0 + s1 * 8 * cc));
}

static void reset_sigma(chain_t* ch)                        /* cloud_cover_binary.py:76-78 */
{
    int L = (int)(ch->h * 12);
    if (L > ORC_SIGMA_CAP) L = ORC_SIGMA_CAP;
    double f = 1.0 / ch->h - 1.0;
    double acc = 0.0;
    for (int k = 0; k < L; ++k) { acc += 300.0; ch->sc[k] = acc; ch->sl[k] = f * ch->sc[k]; }
    ch->L = L;
}

/* cloud_cover_binary.py:80-107.  Returns 0 or a fault status. */
static int next_cloud(const ctx_t* X, chain_t* ch, uint32_t tag)
{
    double nsc[ORC_SIGMA_CAP], nsl[ORC_SIGMA_CAP];
    int tries = 0;
    /* keyed counter: the chain's next_cloud call number (0 = constructor's call) */
    const uint64_t ctr = ch->ncalls++;
    for (int rec = 0; rec < 2; ++rec) {
        for (int i = 0; i < 20; ++i, ++tries) {
            double u = draw_u(X, ch, ctr, tag, (uint32_t)(tries >> 1), tries & 1);
            double cl = pow(X->alpha + X->delta * u, X->expo) / ch->ws;
            double f = 1.0 / ch->h - 1.0;
            int last = -1;
            double best = 0.0;
            for (int k = 0; k < ch->L; ++k) {
                nsc[k] = cl + ch->sc[k];
                nsl[k] = f * nsc[k];
                double tot = nsc[k] + nsl[k];
                if (nsl[k] - ch->sl[k] > 0.0 && tot < 5400.0) {
                    double dist = fabs(tot - 3600.0);
                    if (last < 0 || dist < best) { best = dist; last = k; }
                }
            }
            if (last >= 0) {
                if (last + 2 > ORC_SIGMA_CAP) return ST_SIGMA_OVERFLOW;
                double clr = nsl[last] - ch->sl[last];
                for (int k = last; k >= 0; --k) { ch->sc[k + 1] = nsc[k]; ch->sl[k + 1] = nsl[k]; }
                ch->sc[0] = cl;
                ch->sl[0] = clr;
                ch->L = last + 2;
#pragma omp atomic
                g_Lhist[ch->L] += 1;
#pragma omp atomic
                g_Thist[tries + 1] += 1;
                ch->cl = cl;
                ch->clr = clr;
                ch->sec = 0;
                return 0;
            }
        }
        if (rec == 0) reset_sigma(ch);                     /* :90-98 */
    }
    return ST_ASSERT_BINARY;                               /* assert not recurse */
}

typedef struct { int32_t day, hour, minute, second; } fields_t;

static void fractions(const fields_t* t, double* min_f, double* hour_f, double* day_f)
{   /* clearskyindexmodel.py:114-116 */
    *min_f = t->second / 60.0;
    *hour_f = (t->minute + *min_f) / 60.0;
    *day_f = (t->hour + *hour_f) / 24.0;
}

static void chain_init(const ctx_t* X, chain_t* ch, const fields_t* t0)
{
    const orc_params* P = X->P;
    double mf, hf, df;
    fractions(t0, &mf, &hf, &df);
    ch->mstate = 1.0;
#define IU(d) draw_u(X, ch, 0, TAG_INIT, (d) >> 1, (d) & 1)
    ch->s[S_CC][0] = draw_cc(X, ch, IU(0));
    ch->s[S_CC][1] = draw_cc(X, ch, IU(1));
    ch->s[S_CLEAR_DAY][0] = normal(IU(2), 0.99, 0.08);
    ch->s[S_CLEAR_DAY][1] = normal(IU(3), 0.99, 0.08);
    for (int j = 0; j < 2; ++j) {                          /* :68-82 */
        double c = interp(ch->s[S_CC], hf);
        if (c < 6.0 / 8) ch->s[S_CLOUDY_HOUR][j] = normal(IU(4 + j), 0.6784, 0.2046);
        else if (c < 7.0 / 8) { ch->status = ST_NAMEERROR_INIT; return; }
        else ch->s[S_CLOUDY_HOUR][j] = orc_gammaincinv(3.5624, IU(4 + j)) * 0.0867 + 0.0;
    }
    for (int j = 0; j < 2; ++j)
        ch->s[S_CLOUDY_NOISE][j] = scaled_noise(X, IU(6 + j), 0.01, 0.003, interp(ch->s[S_CC], hf));
    for (int j = 0; j < 2; ++j)
        ch->s[S_CLEAR_NOISE][j] = scaled_noise(X, IU(8 + j), 0.001, 0.0015, interp(ch->s[S_CC], hf));
    for (int j = 0; j < 2; ++j)
        ch->s[S_WS][j] = 2.14 * orc_gammaincinv(2.69, IU(10 + j));
#undef IU
    (void)P;
    /* CloudCoverBinary(cc.interpolate(0), ws.interpolate(0)), clearskyindexmodel.py:98-99 */
    double h0 = interp(ch->s[S_CC], 0.0), w0 = interp(ch->s[S_WS], 0.0);
    ch->h = 0.95 < h0 ? 0.95 : h0;
    ch->ws = w0;
    reset_sigma(ch);
    int st = next_cloud(X, ch, TAG_INIT_CLOUD);
    if (st) { ch->status = st; return; }
    double u = draw_u(X, ch, 0, TAG_INIT_SEC, 0, 0);
    ch->sec = (int64_t)((ch->cl + ch->clr) * u);           /* :68, int() truncates */
}

/* -------------------------------------------------------------------- PV */
typedef struct {
    double zenith, app_zenith, azimuth;
} solpos_t;

static double rad(double d) { return d * (M_PI / 180.0); }
static double deg(double r) { return r * (180.0 / M_PI); }
static double cosd(double d) { return cos(rad(d)); }
static double sind(double d) { return sin(rad(d)); }

/* NOAA / Meeus low-precision solar position (<~0.01 deg) + the SPA refraction
 * correction (Reda & Andreas 2004, eq. 42).  pvlib 0.6.3 uses the full SPA
 * (nrel_numpy) whose periodic-term tables are not available offline. */
void orc_solpos(int64_t utc, double lat, double lon, double pressure_pa, double temp_c,
                double* zenith, double* app_zenith, double* azimuth)
{
    double jd = (double)utc / 86400.0 + 2440587.5;
    double T = (jd - 2451545.0) / 36525.0;
    double L0 = fmod(280.46646 + T * (36000.76983 + T * 0.0003032), 360.0);
    double M = 357.52911 + T * (35999.05029 - 0.0001537 * T);
    double e = 0.016708634 - T * (0.000042037 + 0.0000001267 * T);
    double Mr = rad(M);
    double C = sin(Mr) * (1.914602 - T * (0.004817 + 0.000014 * T)) +
               sin(2.0 * Mr) * (0.019993 - 0.000101 * T) + sin(3.0 * Mr) * 0.000289;
    double omega = 125.04 - 1934.136 * T;
    double lam = L0 + C - 0.00569 - 0.00478 * sin(rad(omega));
    double eps0 = 23.0 + (26.0 + (21.448 - T * (46.815 + T * (0.00059 - T * 0.001813))) / 60.0) / 60.0;
    double eps = eps0 + 0.00256 * cos(rad(omega));
    double decl = asin(sin(rad(eps)) * sin(rad(lam)));
    double y = tan(rad(eps) / 2.0);
    y *= y;
    double L0r = rad(L0);
    double eot = 4.0 * deg(y * sin(2.0 * L0r) - 2.0 * e * sin(Mr) + 4.0 * e * y * sin(Mr) * cos(2.0 * L0r) -
                           0.5 * y * y * sin(4.0 * L0r) - 1.25 * e * e * sin(2.0 * Mr));
    int64_t sod = utc % 86400;
    if (sod < 0) sod += 86400;
    double tst = fmod((double)sod / 60.0 + eot + 4.0 * lon, 1440.0);
    if (tst < 0) tst += 1440.0;
    double ha = rad(tst / 4.0 - 180.0);
    double latr = rad(lat);
    double cz = sin(latr) * sin(decl) + cos(latr) * cos(decl) * cos(ha);
    cz = cz > 1.0 ? 1.0 : (cz < -1.0 ? -1.0 : cz);
    double zen = deg(acos(cz));
    double az = deg(atan2(sin(ha), cos(ha) * sin(latr) - tan(decl) * cos(latr))) + 180.0;
    double e0 = 90.0 - zen;
    double de = 0.0;
    if (e0 >= -1.0 * (0.26667 + 0.5667))
        de = (pressure_pa / 100.0 / 1010.0) * (283.0 / (273.0 + temp_c)) * 1.02 /
             (60.0 * tan(rad(e0 + 10.3 / (e0 + 5.11))));
    *zenith = zen;
    *app_zenith = 90.0 - (e0 + de);
    *azimuth = az;
}

static double alt2pres(double alt) { return 100.0 * pow((44331.514 - alt) / 11880.516, 1.0 / 0.1902632); }

static double extra_rad(int doy, double s0)        /* pvlib irradiance.get_extra_radiation, spencer */
{
    double B = (2.0 * M_PI / 365.0) * (doy - 1);
    double r = 1.00011 + 0.034221 * cos(B) + 0.00128 * sin(B) + 0.000719 * cos(2.0 * B) + 7.7e-05 * sin(2.0 * B);
    return s0 * r;
}

static double am_kastenyoung(double z)              /* atmosphere.get_relative_airmass */
{
    if (!(z <= 90.0)) return NAN;
    return 1.0 / (cos(rad(z)) + 0.50572 * pow(6.07995 + (90.0 - z), -1.6364));
}

static double am_kasten1966(double z)
{
    if (!(z <= 90.0)) return NAN;
    return 1.0 / (cos(rad(z)) + 0.15 * pow(93.885 - z, -1.253));
}

static double linke_at(const double lts[12], int doy, int leap)   /* clearsky._interpolate_turbidity */
{
    static const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    double x[14], y[14];
    x[0] = -31.0 / 2.0; y[0] = lts[11];
    double cum = 0.0;
    for (int m = 0; m < 12; ++m) {
        double d = md[m] + (leap && m == 1 ? 1 : 0);
        cum += d;
        x[m + 1] = cum - d / 2.0; y[m + 1] = lts[m];
    }
    x[13] = (leap ? 366 : 365) + 28 / 2.0; y[13] = lts[0];
    double t = doy;
    for (int i = 0; i < 13; ++i)
        if (t <= x[i + 1]) return y[i] + (t - x[i]) * (y[i + 1] - y[i]) / (x[i + 1] - x[i]);
    return y[13];
}

typedef struct {   /* per site-second deterministic part */
    double cosz, csi_max, ghi_cs, i0h_disc, i0_disc, knc, am_disc, disc_ok, cos_zen_disc;
    double rb, ai_scale, term2, gfac, cos_aoi, f1, f2;
} geom_t;

static void geometry(const orc_params* P, int64_t utc, int doy, int leap, geom_t* g)
{
    const double lat = P->site[0], lon = P->site[1], alt = P->site[2], tilt = P->site[3],
                 saz = P->site[4], albedo = P->site[5];
    double pres = alt2pres(alt);
    double zen, azen, az;
    orc_solpos(utc, lat, lon, pres, 12.0, &zen, &azen, &az);
    /* pvmodel.py:52-58 csi upper clip on the (non-refracted) zenith */
    double ct = cos(rad(zen));
    g->cosz = ct;
    g->csi_max = 27.21 * exp(-114 * ct) + 1.665 * exp(-4.494 * ct) + 1.08;
    /* ineichen (pvmodel.py:60), apparent zenith + kastenyoung absolute airmass at site pressure */
    double dni_extra = extra_rad(doy, 1366.1);
    double am_rel = am_kastenyoung(azen);
    double am_abs = am_rel * pres / 101325.0;
    double tl = linke_at(P->linke, doy, leap);
    double fh1 = exp(-alt / 8000.0), fh2 = exp(-alt / 1250.0);
    double cg1 = 5.09e-05 * alt + 0.868, cg2 = 3.92e-05 * alt + 0.0387;
    double cz = cosd(azen);
    cz = cz > 0.0 ? cz : 0.0;
    double gexp = exp(-cg2 * am_abs * (fh1 + fh2 * (tl - 1.0)));
    double gmax = isnan(gexp) ? 0.0 : (gexp > 0.0 ? gexp : 0.0);      /* np.fmax(ghi, 0) */
    g->ghi_cs = cg1 * dni_extra * cz * tl / tl * gmax;
    /* disc (pvmodel.py:63): I0 with S = 1370, kasten1966 airmass at 101325 Pa */
    double I0 = extra_rad(doy, 1370.0);
    double czd = cosd(zen);
    g->cos_zen_disc = czd;
    g->i0_disc = I0;
    g->i0h_disc = I0 * (czd > 0.065 ? czd : 0.065);
    double amd = am_kasten1966(zen);
    amd = amd * 101325.0 / 101325.0;
    amd = amd < 12.0 ? amd : (isnan(amd) ? amd : 12.0);
    g->am_disc = amd;
    g->knc = 0.866 - 0.122 * amd + 0.0121 * pow(amd, 2) - 0.000653 * pow(amd, 3) + 0.000014 * pow(amd, 4);
    g->disc_ok = zen > 87.0 ? 0.0 : 1.0;
    /* haydavies + ground diffuse + aoi on the APPARENT zenith (pvmodel.py:66-68) */
    double proj = cosd(tilt) * cosd(azen) + sind(tilt) * sind(azen) * cosd(az - saz);
    proj = proj > 1.0 ? 1.0 : (proj < -1.0 ? -1.0 : proj);
    double cos_tt = proj > 0.0 ? proj : 0.0;
    double czs = cosd(azen);
    g->rb = cos_tt / (czs > 0.01745 ? czs : 0.01745);
    g->ai_scale = dni_extra;
    g->term2 = 0.5 * (1.0 + cosd(tilt));
    g->gfac = albedo * (1.0 - cos(rad(tilt))) * 0.5;
    double aoi = deg(acos(proj));
    g->cos_aoi = cos(rad(aoi));
    /* sapm spectral (airmass_absolute, pvmodel.py:73-76) and aoi losses */
    const double* m = P->module;
    double f1 = (((m[4] * am_abs + m[3]) * am_abs + m[2]) * am_abs + m[1]) * am_abs + m[0];
    f1 = isnan(f1) ? 0.0 : f1;
    g->f1 = f1 > 0.0 ? f1 : 0.0;
    double f2 = ((((m[10] * aoi + m[9]) * aoi + m[8]) * aoi + m[7]) * aoi + m[6]) * aoi + m[5];
    f2 = f2 > 0.0 ? f2 : 0.0;
    if (aoi < 0.0) f2 = 0.0;
    g->f2 = f2;
}

/* per chain-second stochastic part: pvmodel.py:53-80 */
static double pv_power(const orc_params* P, const geom_t* g, double csi)
{
    const double* m = P->module;
    const double* iv = P->inverter;
    double c = csi > g->csi_max ? g->csi_max : csi;        /* np.clip(a_max=...) */
    if (isnan(csi)) c = csi;
    double ghi = c * g->ghi_cs;
    /* disc: clearness index + _disc_kn */
    double kt = ghi / g->i0h_disc;
    kt = kt > 0.0 ? kt : 0.0;
    kt = kt < 1.0 ? kt : 1.0;
    double am = g->am_disc, kt2 = kt * kt, kt3 = kt2 * kt, a, b, cc;
    if (kt <= 0.6) {
        a = 0.512 - 1.56 * kt + 2.286 * kt2 - 2.222 * kt3;
        b = 0.37 + 0.962 * kt;
        cc = -0.28 + 0.932 * kt - 2.048 * kt2;
    } else {
        a = -5.743 + 21.77 * kt - 27.49 * kt2 + 11.56 * kt3;
        b = 41.4 - 118.5 * kt + 66.05 * kt2 + 31.9 * kt3;
        cc = -47.01 + 184.2 * kt - 222.0 * kt2 + 73.81 * kt3;
    }
    double dkn = a + b * exp(cc * am);
    double dni = (g->knc - dkn) * g->i0_disc;
    if (g->disc_ok == 0.0 || ghi < 0.0 || dni < 0.0) dni = 0.0;
    double dhi = ghi - dni * g->cosz;
    /* haydavies sky diffuse + ground diffuse + beam */
    double AI = dni / g->ai_scale;
    double sky = dhi * (AI * g->rb + (1.0 - AI) * g->term2);
    sky = sky > 0.0 ? sky : 0.0;
    double ground = ghi * g->gfac;
    double poa_direct = dni * g->cos_aoi;
    poa_direct = poa_direct > 0.0 ? poa_direct : 0.0;
    double poa_diffuse = sky + ground;
    double poa_global = poa_direct + poa_diffuse;
    /* sapm_celltemp, wind 0, air 20 C */
    double wind = P->site[7], tair = P->site[6];
    double tmod = poa_global * exp(m[23] + m[24] * wind) + tair;
    double tcell = tmod + (poa_global / 1000.0) * m[25];
    /* sapm_effective_irradiance (suns) */
    double Ee = g->f1 * (poa_direct * g->f2 + m[11] * poa_diffuse) / 1000.0;
    /* sapm */
    const double q = 1.60218e-19, kb = 1.38066e-23;
    double Bvmpo = m[19] + m[20] * (1.0 - Ee);
    double delta = m[21] * kb * (tcell + 273.15) / q;
    double logEe = Ee > 0.0 ? log(Ee) : (Ee == 0.0 ? -INFINITY : NAN);
    double imp = m[12] * (m[15] * Ee + m[16] * (Ee * Ee)) * (1.0 + m[14] * (tcell - 25.0));
    double dl = delta * logEe;
    double vmp = m[13] + m[17] * m[22] * delta * logEe + m[18] * m[22] * (dl * dl) + Bvmpo * (tcell - 25.0);
    if (!isnan(vmp)) vmp = vmp > 0.0 ? vmp : 0.0;
    double pdc = imp * vmp;
    /* snlinverter */
    double A = iv[1] * (1.0 + iv[5] * (vmp - iv[2]));
    double B = iv[3] * (1.0 + iv[6] * (vmp - iv[2]));
    double C = iv[4] * (1.0 + iv[7] * (vmp - iv[2]));
    double ac = (iv[0] / (A - B) - C * (A - B)) * (pdc - B) + C * ((pdc - B) * (pdc - B));
    if (!isnan(ac)) ac = iv[0] < ac ? iv[0] : ac;
    if (pdc < iv[3]) ac = -1.0 * fabs(iv[8]);
    /* ac.clip(lower=0.).fillna(0.) */
    if (isnan(ac)) return 0.0;
    return ac > 0.0 ? ac : 0.0;
}

void orc_geometry(const orc_params* P, int64_t utc, int doy, int leap, double* out16)
{
    geom_t g;
    geometry(P, utc, doy, leap, &g);
    memcpy(out16, &g, sizeof(g));
}

double orc_pv(const orc_params* P, int64_t utc, int doy, int leap, double csi)
{
    geom_t g;
    geometry(P, utc, doy, leap, &g);
    return pv_power(P, &g, csi);
}

/* optional per-chain PV sites (C5): chain c (index within the orc_run call)
 * uses site columns 0-5 of g_sites[c] (temp_air and wind stay P's) and, when
 * set, the monthly Linke turbidity g_site_linke[c]; its geometry is then
 * evaluated per chain-step */
static const double* g_sites;
static const double* g_site_linke;
static uint32_t g_sites_n;
void orc_set_sites(const double* sites /* [n][8] */, const double* linke /* [n][12] or NULL */, uint32_t n)
{
    g_sites = sites;
    g_site_linke = linke;
    g_sites_n = n;
}

/* optional global chain ids (tests comparing scattered chains of a large GPU batch
 * in one run): chain c of the orc_run call is global chain g_ids[c] instead of
 * chain0 + c; keyed draws follow the global id exactly as on the GPU */
static const uint64_t* g_ids;
static uint32_t g_ids_n;
void orc_set_chain_ids(const uint64_t* ids, uint32_t n)
{
    g_ids = ids;
    g_ids_n = n;
}

/* optional on-host statistics of orc_run (the GPU's stats mode, tmh_stats): per
 * chain c: acc[c][4] = sum pv, sum meter, sum residual (W s), max residual over
 * its good seconds; hist[c][n_bins] its residual histogram (edge bins absorb
 * out-of-range, bin = floor((r - lo) n_bins / (hi - lo))); amb[c] the seconds
 * whose bin coordinate lies within amb_eps of a bin edge (a tolerance-sized
 * error may move them) */
static double* g_acc;
static uint64_t* g_hist;
static uint64_t* g_amb;
static uint32_t g_nbins;
static double g_lo, g_scale, g_amb_eps;

void orc_set_stats(double* acc, uint64_t* hist, uint64_t* amb, uint32_t n_bins, double lo, double hi, double amb_eps)
{
    g_acc = acc;
    g_hist = hist;
    g_amb = amb;
    g_nbins = n_bins;
    g_lo = lo;
    g_scale = hist ? n_bins / (hi - lo) : 0.0;
    g_amb_eps = amb_eps;
}

static void stats_add(uint32_t c, double pv, double meter, double res)
{
    double* a = g_acc + 4 * (size_t)c;
    a[0] += pv;
    a[1] += meter;
    a[2] += res;
    a[3] = a[3] > res ? a[3] : res;
    if (g_hist) {
        const double x = (res - g_lo) * g_scale;
        const int bin = x < 0.0 ? 0 : (x >= (double)(g_nbins - 1) ? (int)g_nbins - 1 : (int)x);
        g_hist[(size_t)c * g_nbins + bin] += 1;
        const double fr = x - floor(x);
        if (g_amb && x > 0.0 && x < (double)(g_nbins - 1) && (fr < g_amb_eps || fr > 1.0 - g_amb_eps)) g_amb[c] += 1;
    }
}

/* -------------------------------------------------------------------- run */
/* cal: n_steps x 6 int32 = (day of month, hour, minute, second, day of year, leap) local fields.
 * Outputs time-major [step][chain]; any pointer may be NULL.
 * calls (optional): per next_cloud call (chain, step, pos_before, pos_after, cl, clr, L_after) */
int orc_run(const orc_params* P, uint64_t chain0, uint32_t n_chains, uint32_t n_steps,
            const int32_t* cal, const int64_t* utc, const double* inj, uint64_t inj_stride,
            double* csi_out, uint8_t* cov_out, double* pv_out, double* meter_out,
            double* resid_out, uint32_t* pos_out, uint8_t* status_out,
            double* init_out /* [n_chains][16] samplers + sec,cl,clr,pos */)
{
    ctx_t X;
    X.P = P;
    X.omb = 1.0 - 1.66;
    X.alpha = pow(1e6, X.omb);
    X.delta = pow(0.1e3, X.omb) - X.alpha;
    X.expo = 1.0 / X.omb;
    X.sqrt09 = sqrt(0.9);
    X.sqrt6 = sqrt(0.1 * 60);

    geom_t* G = NULL;
    if (P->with_pv) {
        G = (geom_t*)malloc(sizeof(geom_t) * (size_t)n_steps);
        if (!G) return -3;
#pragma omp parallel for schedule(static) num_threads(P->n_threads > 0 ? P->n_threads : 1)
        for (uint32_t s = 0; s < n_steps; ++s)
            geometry(P, utc[s], cal[6 * s + 4], cal[6 * s + 5], &G[s]);
    }
    int nt = P->n_threads > 0 ? P->n_threads : 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
    for (uint32_t c = 0; c < n_chains; ++c) {
        chain_t* ch = (chain_t*)calloc(1, sizeof(chain_t));
        ch->chain = (g_ids && c < g_ids_n) ? g_ids[c] : chain0 + c;
        orc_params Pc;
        const orc_params* Ps = P;   /* the chain's PV site */
        if (g_sites && c < g_sites_n) {
            Pc = *P;
            memcpy(Pc.site, g_sites + 8 * (size_t)c, 6 * sizeof(double));
            if (g_site_linke) memcpy(Pc.linke, g_site_linke + 12 * (size_t)c, 12 * sizeof(double));
            Ps = &Pc;
        }
        if (g_tab && c < g_tab_n) {
            ch->tab = g_tab + 24 * (size_t)c;
            ch->tab_t = g_tab_t + 6 * (size_t)c;
        }
        if (inj) { ch->inj = inj + (uint64_t)c * inj_stride; ch->inj_len = inj_stride; }
        if (g_acc) {
            double* a = g_acc + 4 * (size_t)c;
            a[0] = a[1] = a[2] = 0.0;
            a[3] = -INFINITY;
        }
        fields_t t0 = {cal[0], cal[1], cal[2], cal[3]};
        chain_init(&X, ch, &t0);
        if (init_out) {
            double* o = init_out + 16 * (size_t)c;
            for (int k = 0; k < 6; ++k) { o[2 * k] = ch->s[k][0]; o[2 * k + 1] = ch->s[k][1]; }
            o[12] = (double)ch->sec; o[13] = ch->cl; o[14] = ch->clr; o[15] = (double)ch->pos;
        }
        fields_t prev = t0;
        for (uint32_t s = 0; s < n_steps; ++s) {
            size_t o = (size_t)s * n_chains + c;
            fields_t t = {cal[6 * s], cal[6 * s + 1], cal[6 * s + 2], cal[6 * s + 3]};
            double mf, hf, df;
            fractions(&t, &mf, &hf, &df);
            double csi = NAN;
            int cov = 255;
            if (!ch->status) {
                uint64_t step = s;
                if (prev.day != t.day) {                       /* _next_day */
                    push(ch->s[S_CLEAR_DAY], normal(draw_u(&X, ch, step, TAG_BOUNDARY, 0, 0), 0.99, 0.08));
                    push(ch->s[S_WS], 2.14 * orc_gammaincinv(2.69, draw_u(&X, ch, step, TAG_BOUNDARY, 0, 1)));
                }
                if (prev.hour != t.hour) {                     /* _next_hour (advances clear_day) */
                    push(ch->s[S_CC], draw_cc(&X, ch, draw_u(&X, ch, step, TAG_BOUNDARY, 1, 0)));
                    push(ch->s[S_CLEAR_DAY], normal(draw_u(&X, ch, step, TAG_BOUNDARY, 1, 1), 0.99, 0.08));
                }
                if (prev.minute != t.minute) {                 /* _next_min */
                    double u0 = draw_u(&X, ch, step, TAG_BOUNDARY, 2, 0);
                    push(ch->s[S_CLOUDY_NOISE], scaled_noise(&X, u0, 0.01, 0.003, interp(ch->s[S_CC], hf)));
                    double u1 = draw_u(&X, ch, step, TAG_BOUNDARY, 2, 1);
                    push(ch->s[S_CLEAR_NOISE], scaled_noise(&X, u1, 0.001, 0.0015, interp(ch->s[S_CC], hf)));
                }
                double cloudcover = interp(ch->s[S_CC], hf);
                double hh = interp(ch->s[S_CC], hf);
                ch->h = 0.95 < hh ? 0.95 : hh;                 /* update_parameters */
                ch->ws = interp(ch->s[S_WS], df);
                ch->sec += 1;                                  /* CloudCoverBinary.__next__ */
                for (;;) {
                    if ((double)ch->sec < ch->cl) { cov = 1; break; }
                    if ((double)ch->sec < ch->cl + ch->clr) { cov = 0; break; }
                    int st = next_cloud(&X, ch, TAG_CLOUD);
                    if (st) { ch->status = st; break; }
                    ch->sec += 1;
                }
                if (!ch->status) {
                    double ue, um_unused;
                    step_u(P->seed, ch->chain, step, &ue, &um_unused);
                    if (P->rng_mode == 1) ue = draw_u(&X, ch, step, TAG_STEP, 0, 0);
                    double eps = orc_ndtri(ue) *
                                 (X.sqrt6 * (0.001 + 0.0015 * 8 * cloudcover)) + 0.0;
                    if (cov) csi = interp(ch->s[S_CLEAR_DAY], df) * (interp(ch->s[S_CLEAR_NOISE], mf) + eps);
                    else csi = interp(ch->s[S_CLOUDY_HOUR], hf) * (interp(ch->s[S_CLOUDY_NOISE], mf) + eps);
                }
                if (ch->status) { csi = NAN; cov = 255; }
            }
            prev = t;
            if (csi_out) csi_out[o] = csi;
            if (cov_out) cov_out[o] = (uint8_t)cov;
            if (pos_out) pos_out[o] = (uint32_t)ch->pos;
            double pv = NAN, meter = NAN;
            if (!ch->status) {
                if (P->with_pv && Ps != P) {
                    geom_t gs;
                    geometry(Ps, utc[s], cal[6 * s + 4], cal[6 * s + 5], &gs);
                    pv = pv_power(Ps, &gs, csi);
                } else {
                    pv = P->with_pv ? pv_power(P, &G[s], csi) : 0.0;
                }
                double ue_unused, um;
                step_u(P->seed, ch->chain, s, &ue_unused, &um);
                meter = 9000 * um;
            }
            if (pv_out) pv_out[o] = pv;
            if (meter_out) meter_out[o] = meter;
            if (resid_out) resid_out[o] = meter - pv;
            if (g_acc && !ch->status) stats_add(c, pv, meter, meter - pv);
        }
        if (status_out) status_out[c] = (uint8_t)ch->status;
        free(ch);
    }
    free(G);
    return 0;
}

/* expose constants for tests */
void orc_constants(double* out4)
{
    double omb = 1.0 - 1.66;
    out4[0] = pow(1e6, omb);
    out4[1] = pow(0.1e3, omb) - out4[0];
    out4[2] = 1.0 / omb;
    out4[3] = sqrt(0.1 * 60);
}

/* The device computes the wall-clock fractions (clearskyindexmodel.py:114-116)
 * as q = x * (1/d) plus one FMA residual correction instead of an IEEE division.
 * Returns the number of the 86,400 seconds of a day for which that differs from
 * the divisions the reference performs (expected 0). */
int orc_check_fractions(void)
{
    int bad = 0;
    for (int h = 0; h < 24; ++h)
        for (int m = 0; m < 60; ++m)
            for (int s = 0; s < 60; ++s) {
                double mf = s / 60.0, hf = (m + mf) / 60.0, df = (h + hf) / 24.0;
                double q = s * (1.0 / 60.0);
                double mf2 = fma(fma(-q, 60.0, (double)s), 1.0 / 60.0, q);
                double x = m + mf2;
                q = x * (1.0 / 60.0);
                double hf2 = fma(fma(-q, 60.0, x), 1.0 / 60.0, q);
                x = h + hf2;
                q = x * (1.0 / 24.0);
                double df2 = fma(fma(-q, 24.0, x), 1.0 / 24.0, q);
                bad += (mf2 != mf) + (hf2 != hf) + (df2 != df);
            }
    return bad;
}
