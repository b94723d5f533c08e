/*
 * gsm_oracle_math.h -- deterministic scalar math for the oracle (TEST INFRASTRUCTURE).
 *
 * The reference compiles its Metal kernels with -ffast-math
 * (/root/reference/compile_shaders.sh:50), so its transcendentals are not
 * reproducible off Apple hardware.  DESIGN.md "Numeric contract" fixes one
 * definition for each, and this header restates it for the CPU:
 *   - fp32 atan2/log2/exp2: fixed minimax-style polynomials (tools/fit_polys.py),
 *     evaluated with fmaf (correctly rounded on every IEEE platform);
 *   - sin/cos of the 65536 quantised ellipse angles and e^x of every fp16 x:
 *     double-precision Taylor series with only + - * / (no libm), then rounded
 *     to nearest-even fp32 / fp16.
 * Every other operation is a single IEEE-754 op with no contraction
 * (compile with -ffp-contract=off).
 */
#ifndef GSM_ORACLE_MATH_H
#define GSM_ORACLE_MATH_H
#include <math.h>
#include <stdint.h>
#include <string.h>

#define OGM_PI_F 3.14159265358979323846f

static inline uint32_t ogm_fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float ogm_bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* atan(t)/t = P(t^2), t in [0,1] */
static const float OGM_ATAN_P[12] = {
    0x1.000000p+0f, -0x1.555554p-2f, 0x1.999918p-3f, -0x1.248880p-3f,
    0x1.c65610p-4f, -0x1.6fa1e4p-4f, 0x1.2836b8p-4f, -0x1.ba8a46p-5f,
    0x1.15ba34p-5f, -0x1.043f50p-6f, 0x1.37ac38p-8f, -0x1.5e0120p-11f};
/* log2(m) = u*Q(u^2), u = (m-1)/(m+1), m in [sqrt(1/2), sqrt(2)) */
static const float OGM_LOG2_Q[6] = {
    0x1.715476p+1f, 0x1.ec709ep-1f, 0x1.2776c2p-1f,
    0x1.a61a2cp-2f, 0x1.4795a8p-2f, 0x1.21ac98p-2f};
/* 2^f = R(f), f in [-1/2, 1/2] */
static const float OGM_EXP2_R[8] = {
    0x1.000000p+0f, 0x1.62e430p-1f, 0x1.ebfbe0p-3f, 0x1.c6b08ap-5f,
    0x1.3b29dcp-7f, 0x1.5d8aa0p-10f, 0x1.4469d4p-13f, 0x1.fde104p-17f};

static inline float ogm_atan2f(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y);
    if (isnan(x) || isnan(y)) return x + y;
    float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    float r;
    if (mx == 0.0f) {
        r = 0.0f;
    } else if (isinf(mx)) {
        r = isinf(mn) ? (OGM_PI_F * 0.25f) : 0.0f;
    } else {
        float t = mn / mx;
        float s = t * t;
        float p = OGM_ATAN_P[11];
        for (int i = 10; i >= 0; --i) p = fmaf(p, s, OGM_ATAN_P[i]);
        r = t * p;
    }
    if (ay > ax) r = (OGM_PI_F * 0.5f) - r;
    if (signbit(x)) r = OGM_PI_F - r;
    if (signbit(y)) r = -r;
    return r;
}

static inline float ogm_log2f(float x) {
    if (isnan(x) || x < 0.0f) return NAN;
    if (x == 0.0f) return -INFINITY;
    if (isinf(x)) return INFINITY;
    uint32_t u = ogm_fbits(x);
    int e;
    if ((u & 0x7F800000u) == 0) { /* subnormal: scale by 2^23 (exact) */
        x = x * 8388608.0f;
        u = ogm_fbits(x);
        e = (int)((u >> 23) & 0xFF) - 127 - 23;
    } else {
        e = (int)((u >> 23) & 0xFF) - 127;
    }
    float m = ogm_bitsf((u & 0x007FFFFFu) | 0x3F800000u); /* [1,2) */
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float num = m - 1.0f, den = m + 1.0f;
    float uu = num / den;
    float u2 = uu * uu;
    float q = OGM_LOG2_Q[5];
    for (int i = 4; i >= 0; --i) q = fmaf(q, u2, OGM_LOG2_Q[i]);
    return fmaf(uu, q, (float)e);
}

static inline float ogm_exp2f(float x) {
    if (isnan(x)) return x;
    if (x >= 128.0f) return INFINITY;
    if (x < -150.0f) return 0.0f;
    float n = rintf(x); /* round-half-even */
    float f = x - n;    /* exact */
    float r = OGM_EXP2_R[7];
    for (int i = 6; i >= 0; --i) r = fmaf(r, f, OGM_EXP2_R[i]);
    return ldexpf(r, (int)n);
}

/* powr(x, y) for x > 0: the reference's fast::powr (GaussianShared.h:120). */
static inline float ogm_powrf(float x, float y) { return ogm_exp2f(y * ogm_log2f(x)); }

/* ---- double-precision series (table builders) ---- */
static inline double ogm_sin_series(double x) { /* |x| <= pi/2 */
    double x2 = x * x, term = x, sum = x;
    for (int k = 1; k < 14; ++k) {
        term = term * (-x2) / (double)((2 * k) * (2 * k + 1));
        sum = sum + term;
    }
    return sum;
}
static inline double ogm_cos_series(double x) { /* |x| <= pi/2 */
    double x2 = x * x, term = 1.0, sum = 1.0;
    for (int k = 1; k < 14; ++k) {
        term = term * (-x2) / (double)((2 * k - 1) * (2 * k));
        sum = sum + term;
    }
    return sum;
}
/* sin/cos of x in [0, pi + 1e-3]: reflect about pi/2 so the series argument is small. */
static inline void ogm_sincos_d(double x, double *s, double *c) {
    const double half_pi = 1.5707963267948966192;
    if (x <= half_pi) {
        *s = ogm_sin_series(x);
        *c = ogm_cos_series(x);
    } else {
        double r = x - 2.0 * half_pi; /* x - pi in [-pi/2, 0] */
        *s = -ogm_sin_series(r);
        *c = -ogm_cos_series(r);
    }
}
/* e^x in double for |x| <= 20: e^x = (e^(x/64))^64 with a 24-term series. */
static inline double ogm_exp_d(double x) {
    double y = x / 64.0, term = 1.0, sum = 1.0;
    for (int k = 1; k < 24; ++k) {
        term = term * y / (double)k;
        sum = sum + term;
    }
    for (int k = 0; k < 6; ++k) sum = sum * sum;
    return sum;
}

/* sin/cos of an unquantised fp32 angle th in [0, pi] (conicFromThetaSigmas' fast::sincos,
 * GaussianShared.h:490-494, as the DepthFirst stereo projection calls it with the fp32 theta,
 * DepthFirstShaders.metal:455,471).  Reflected about pi/2 like ogm_sincos_d, then Horner
 * polynomials in double with the Taylor coefficients +-1/n! (compile-time correctly rounded
 * doubles), only * and + (no contraction), one rounding to fp32.  The GPU evaluates the same
 * expression (gsm_detmath.h det_sincos_theta) with IEEE double ops, so the bits agree. */
static inline void ogm_sincos_theta(float th, float *s, float *c) {
    static const double S[11] = {1.0, -1.0 / 6.0, 1.0 / 120.0, -1.0 / 5040.0, 1.0 / 362880.0,
                                 -1.0 / 39916800.0, 1.0 / 6227020800.0, -1.0 / 1307674368000.0,
                                 1.0 / 355687428096000.0, -1.0 / 121645100408832000.0,
                                 1.0 / 51090942171709440000.0};
    static const double K[11] = {1.0, -1.0 / 2.0, 1.0 / 24.0, -1.0 / 720.0, 1.0 / 40320.0,
                                 -1.0 / 3628800.0, 1.0 / 479001600.0, -1.0 / 87178291200.0,
                                 1.0 / 20922789888000.0, -1.0 / 6402373705728000.0,
                                 1.0 / 2432902008176640000.0};
    const double half_pi = 1.5707963267948966192;
    double x = (double)th, sg = 1.0;
    if (!(x <= half_pi)) {
        x = x - 2.0 * half_pi;
        sg = -1.0;
    }
    double x2 = x * x, ps = S[10], pc = K[10];
    for (int i = 9; i >= 0; --i) {
        ps = ps * x2 + S[i];
        pc = pc * x2 + K[i];
    }
    *s = (float)(sg * (x * ps));
    *c = (float)(sg * pc);
}

#endif
