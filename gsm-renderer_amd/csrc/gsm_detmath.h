// gsm_detmath.h -- the deterministic numeric contract for gfx950.
//
// The reference's Metal kernels are built with -ffast-math
// (/root/reference/compile_shaders.sh:50); their transcendentals are not reproducible.
// This build fixes one definition per function, evaluated identically on the GPU
// and on the CPU checker:
//   * atan2 / log2 / exp2 in fp32: fixed polynomials (tools/fit_polys.py) with
//     fmaf (v_fma_f32 on gfx950, correctly rounded);
//   * sin/cos of the 65536 quantised ellipse angles and e^x of every fp16 x:
//     built on the host once per renderer (double-precision series, only + - * /,
//     one final rounding) and read from tables by the kernels.
// Every other op is a single IEEE op; the library is compiled with
// -ffp-contract=off and correctly rounded fp32 division / sqrt.
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace gsm {

#define GSM_HD __host__ __device__ __forceinline__

constexpr float kPiF = 3.14159265358979323846f;

GSM_HD float det_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// atan(t)/t = P(t^2) on [0,1].
GSM_HD float det_atan2f(float y, float x) {
    const float P[12] = {0x1.000000p+0f, -0x1.555554p-2f, 0x1.999918p-3f, -0x1.248880p-3f,
                         0x1.c65610p-4f, -0x1.6fa1e4p-4f, 0x1.2836b8p-4f, -0x1.ba8a46p-5f,
                         0x1.15ba34p-5f, -0x1.043f50p-6f, 0x1.37ac38p-8f, -0x1.5e0120p-11f};
    if (__builtin_isnan(x) || __builtin_isnan(y)) return x + y;
    float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
    float mx = __builtin_fmaxf(ax, ay), mn = __builtin_fminf(ax, ay);
    float r;
    if (mx == 0.0f) {
        r = 0.0f;
    } else if (__builtin_isinf(mx)) {
        r = __builtin_isinf(mn) ? (kPiF * 0.25f) : 0.0f;
    } else {
        float t = mn / mx;
        float s = t * t;
        float p = P[11];
#pragma unroll
        for (int i = 10; i >= 0; --i) p = det_fma(p, s, P[i]);
        r = t * p;
    }
    if (ay > ax) r = (kPiF * 0.5f) - r;
    if (__builtin_signbit(x)) r = kPiF - r;
    if (__builtin_signbit(y)) r = -r;
    return r;
}

GSM_HD uint32_t f32_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
GSM_HD float bits_f32(uint32_t u) { return __builtin_bit_cast(float, u); }

// log2 via u = (m-1)/(m+1), m in [sqrt(1/2), sqrt(2)).
GSM_HD float det_log2f(float x) {
    const float Q[6] = {0x1.715476p+1f, 0x1.ec709ep-1f, 0x1.2776c2p-1f,
                        0x1.a61a2cp-2f, 0x1.4795a8p-2f, 0x1.21ac98p-2f};
    if (__builtin_isnan(x) || x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -__builtin_inff();
    if (__builtin_isinf(x)) return __builtin_inff();
    uint32_t u = f32_bits(x);
    int e;
    if ((u & 0x7F800000u) == 0) {
        x = x * 8388608.0f;
        u = f32_bits(x);
        e = (int)((u >> 23) & 0xFF) - 127 - 23;
    } else {
        e = (int)((u >> 23) & 0xFF) - 127;
    }
    float m = bits_f32((u & 0x007FFFFFu) | 0x3F800000u);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e += 1;
    }
    float uu = (m - 1.0f) / (m + 1.0f);
    float u2 = uu * uu;
    float q = Q[5];
#pragma unroll
    for (int i = 4; i >= 0; --i) q = det_fma(q, u2, Q[i]);
    return det_fma(uu, q, (float)e);
}

GSM_HD float det_exp2f(float x) {
    const float R[8] = {0x1.000000p+0f, 0x1.62e430p-1f, 0x1.ebfbe0p-3f, 0x1.c6b08ap-5f,
                        0x1.3b29dcp-7f, 0x1.5d8aa0p-10f, 0x1.4469d4p-13f, 0x1.fde104p-17f};
    if (__builtin_isnan(x)) return x;
    if (x >= 128.0f) return __builtin_inff();
    if (x < -150.0f) return 0.0f;
    float n = __builtin_rintf(x);
    float f = x - n;
    float r = R[7];
#pragma unroll
    for (int i = 6; i >= 0; --i) r = det_fma(r, f, R[i]);
    return __builtin_ldexpf(r, (int)n);
}

// fast::powr(x, y), x > 0 (GaussianShared.h:120).
GSM_HD float det_powrf(float x, float y) { return det_exp2f(y * det_log2f(x)); }

// gaussianComputePower (GaussianShared.h:595-597).
GSM_HD float det_compute_power(float opacity) {
    const float LN2 = 0.693147180559945f;
    return LN2 * 8.0f + LN2 * det_log2f(__builtin_fmaxf(opacity, 1e-6f));
}

// ---- host-side table builders (double series, no libm) ----
inline double det_sin_series(double x) {
    double x2 = x * x, term = x, sum = x;
    for (int k = 1; k < 14; ++k) {
        term = term * (-x2) / (double)((2 * k) * (2 * k + 1));
        sum = sum + term;
    }
    return sum;
}
inline double det_cos_series(double x) {
    double x2 = x * x, term = 1.0, sum = 1.0;
    for (int k = 1; k < 14; ++k) {
        term = term * (-x2) / (double)((2 * k - 1) * (2 * k));
        sum = sum + term;
    }
    return sum;
}
inline void det_sincos_table_entry(uint32_t q, float* s, float* c) {
    const float kscale = kPiF / 65535.0f;  // unpackThetaPi (GaussianShared.h:442-444)
    float th = (float)q * kscale;
    const double half_pi = 1.5707963267948966192;
    double x = (double)th, sd, cd;
    if (x <= half_pi) {
        sd = det_sin_series(x);
        cd = det_cos_series(x);
    } else {
        double r = x - 2.0 * half_pi;
        sd = -det_sin_series(r);
        cd = -det_cos_series(r);
    }
    *s = (float)sd;
    *c = (float)cd;
}
// sin/cos of an unquantised fp32 angle in [0, pi] (conicFromThetaSigmas' fast::sincos for the
// DepthFirst stereo projection's fp32 theta, DepthFirstShaders.metal:455,471): reflected about
// pi/2, Horner polynomials in double with the Taylor coefficients +-1/n! (compile-time
// correctly rounded), only * and + (no contraction), one rounding to fp32.  Evaluated per
// gaussian on the GPU with IEEE double ops; oracle/gsm_oracle_math.h ogm_sincos_theta is the
// same expression.
GSM_HD void det_sincos_theta(float th, float* s, float* c) {
    constexpr double S[11] = {1.0, -1.0 / 6.0, 1.0 / 120.0, -1.0 / 5040.0, 1.0 / 362880.0,
                              -1.0 / 39916800.0, 1.0 / 6227020800.0, -1.0 / 1307674368000.0,
                              1.0 / 355687428096000.0, -1.0 / 121645100408832000.0,
                              1.0 / 51090942171709440000.0};
    constexpr double K[11] = {1.0, -1.0 / 2.0, 1.0 / 24.0, -1.0 / 720.0, 1.0 / 40320.0,
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
#pragma unroll
    for (int i = 9; i >= 0; --i) {
        ps = ps * x2 + S[i];
        pc = pc * x2 + K[i];
    }
    *s = (float)(sg * (x * ps));
    *c = (float)(sg * pc);
}
inline double det_exp_double(double x) {  // |x| <= 20
    double y = x / 64.0, term = 1.0, sum = 1.0;
    for (int k = 1; k < 24; ++k) {
        term = term * y / (double)k;
        sum = sum + term;
    }
    for (int k = 0; k < 6; ++k) sum = sum * sum;
    return sum;
}

// IEEE binary16 helpers for the host.
inline float half_bits_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0) {
        float f = (float)m * 5.9604644775390625e-08f;
        return (h & 0x8000u) ? -f : f;
    }
    uint32_t bits = (e == 31) ? (sign | 0x7F800000u | (m << 13)) : (sign | ((e + 112u) << 23) | (m << 13));
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}
// double -> fp16, round to nearest even, one rounding.
inline uint16_t double_to_half_bits(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    uint16_t sign = (uint16_t)((u >> 48) & 0x8000u);
    if (std::isnan(d)) return (uint16_t)(sign | 0x7E00u | (uint16_t)((u >> 42) & 0x1FFu));
    double a = std::fabs(d);
    if (a >= 65520.0) return (uint16_t)(sign | 0x7C00u);
    if (a < 6.103515625e-05) return (uint16_t)(sign | (uint16_t)std::nearbyint(a * 16777216.0));
    int e;
    double m = std::frexp(a, &e);
    double r = std::nearbyint(std::ldexp(m, 11));
    if (r == 2048.0) {
        r = 1024.0;
        e += 1;
    }
    int he = e - 1 + 15;
    if (he >= 31) return (uint16_t)(sign | 0x7C00u);
    return (uint16_t)(sign | (uint16_t)(he << 10) | (uint16_t)((int)r - 1024));
}
inline uint16_t float_to_half_bits(float f) { return double_to_half_bits((double)f); }

// The projection's table of the u8 channel values c = 0..255 (k_project, stored behind the 65536 sincos
// entries): x = the tile-test level 2 computePower(c) of an opacity byte (tileCountIndirectKernel,
// GlobalShaders.metal:563-616), y = the bits of fp16(float(c) / 255) (getColor/getOpacity,
// GlobalShaders.metal:9-15) -- the same single IEEE operations the kernels evaluated per gaussian before r06.
inline void det_byte_lut_entry(uint32_t c, float* level, uint32_t* div255) {
    *level = 2.0f * det_compute_power((float)c);
    *div255 = float_to_half_bits((float)c / 255.0f);
}
// e^x for fp16 x: one rounding of the double series.
inline uint16_t det_exp_half_bits(uint16_t xb) {
    float x = half_bits_to_float(xb);
    if (std::isnan(x)) return float_to_half_bits(x);
    if (x < -18.0f) return 0;
    if (x > 12.0f) return 0x7C00u;
    return double_to_half_bits(det_exp_double((double)x));
}
// The blend's per-pixel exp: exp(-0.5h * p) for every fp16 quadratic-form value p
// (GlobalShaders.metal:1124-1131), indexed by the bits of p.
inline uint16_t blend_exp_table_entry(uint16_t pb) {
    float p = half_bits_to_float(pb);
    uint16_t arg = float_to_half_bits(-0.5f * p);  // fp16 multiply: exact product, one rounding
    return det_exp_half_bits(arg);
}
// The DepthFirst stereo blend's alpha factor: p > r2Max = 9 gives alpha 0 without the exp
// (DepthFirstShaders.metal:1898-1905); opacity * 0 = 0 and min(0, 0.99) = 0, so the cutoff
// folds into the table.  NaN p compares false and keeps the exp entry.
inline uint16_t stereo_exp_table_entry(uint16_t pb) {
    const float p = half_bits_to_float(pb);
    if (p > 9.0f) return 0;
    return blend_exp_table_entry(pb);
}

}  // namespace gsm
