/*
 * gsm_oracle.c -- CPU restatement of the reference GlobalRenderer frame.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline); see gsm_oracle.h.
 * Every function cites the reference file:line it restates.  Paths are
 * relative to /root/reference.  Compile with -ffp-contract=off (oracle/Makefile).
 */
#include "gsm_oracle.h"
#include "gsm_oracle_math.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

/* ------------------------------------------------------------------ */
/* fp16                                                                */
/* ------------------------------------------------------------------ */
static float g_h2f[65536];
static uint16_t g_exp_h[65536];
static float g_sin_t[65536], g_cos_t[65536];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

uint16_t og_d2h(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    uint16_t sign = (uint16_t)((u >> 48) & 0x8000u);
    double a = fabs(d);
    if (isnan(d)) return (uint16_t)(sign | 0x7E00u | (uint16_t)((u >> 42) & 0x1FFu));
    if (a >= 65520.0) return (uint16_t)(sign | 0x7C00u);
    if (a < 6.103515625e-05) { /* subnormal: quantum 2^-24 */
        double r = nearbyint(a * 16777216.0);
        return (uint16_t)(sign | (uint16_t)r);
    }
    int e;
    double m = frexp(a, &e); /* a = m * 2^e, m in [0.5, 1) */
    double r = nearbyint(ldexp(m, 11));
    if (r == 2048.0) { r = 1024.0; e += 1; }
    int he = e - 1 + 15;
    if (he >= 31) return (uint16_t)(sign | 0x7C00u);
    return (uint16_t)(sign | (uint16_t)(he << 10) | (uint16_t)((int)r - 1024));
}

static float h2f_slow(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) bits = sign;
        else { /* subnormal: m * 2^-24, exact in fp32 */
            float f = (float)m * 5.9604644775390625e-08f;
            return (h & 0x8000u) ? -f : f;
        }
    } else if (e == 31) {
        bits = sign | 0x7F800000u | (m << 13);
    } else {
        bits = sign | ((e + 112u) << 23) | (m << 13);
    }
    return ogm_bitsf(bits);
}

/* fp32 -> fp16, round to nearest even (the GPU's v_cvt_f16_f32 in default mode). */
uint16_t og_f2h(float f) {
    uint32_t x = ogm_fbits(f);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) {
        if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));
        return (uint16_t)(sign | 0x7C00u);
    }
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u); /* >= 65520 */
    if (ax >= 0x38800000u) {                                   /* normal fp16 */
        uint32_t m = ax - 0x38000000u;
        m = m + 0x0FFFu + ((m >> 13) & 1u);
        return (uint16_t)(sign | (m >> 13));
    }
    float v = ogm_bitsf(ax) * 16777216.0f; /* exact scaling */
    return (uint16_t)(sign | (uint16_t)rintf(v));
}

static void ensure_init(void);
float og_h2f(uint16_t h) { ensure_init(); return g_h2f[h]; }

/* e^x for fp16 x (DESIGN.md numeric contract): double series, one rounding to fp16. */
static uint16_t exp_h_build(uint16_t xb) {
    float x = h2f_slow(xb);
    if (isnan(x)) return og_f2h(x);
    if (x < -18.0f) return 0;
    if (x > 12.0f) return 0x7C00u;
    return og_d2h(ogm_exp_d((double)x));
}

static void init_tables(void) {
    for (uint32_t i = 0; i < 65536; ++i) g_h2f[i] = h2f_slow((uint16_t)i);
    for (uint32_t i = 0; i < 65536; ++i) g_exp_h[i] = exp_h_build((uint16_t)i);
    /* unpackThetaPi (GaussianShared.h:442-444) then sin/cos of the fp32 angle. */
    const float kscale = OGM_PI_F / 65535.0f;
    for (uint32_t i = 0; i < 65536; ++i) {
        float th = (float)i * kscale;
        double s, c;
        ogm_sincos_d((double)th, &s, &c);
        g_sin_t[i] = (float)s;
        g_cos_t[i] = (float)c;
    }
}
static void ensure_init(void) { pthread_once(&g_once, init_tables); }

uint16_t og_exp_h(uint16_t x) { ensure_init(); return g_exp_h[x]; }
float og_atan2f(float y, float x) { return ogm_atan2f(y, x); }
float og_log2f(float x) { return ogm_log2f(x); }
float og_exp2f(float x) { return ogm_exp2f(x); }

/* fp16 arithmetic: one fp32 op then one rounding == the correctly rounded fp16 op
 * for + - * / (24 >= 2*11+2, so double rounding is innocuous). */
static inline float H(uint16_t h) { return g_h2f[h]; }
static inline uint16_t hadd(uint16_t a, uint16_t b) { return og_f2h(H(a) + H(b)); }
static inline uint16_t hsub(uint16_t a, uint16_t b) { return og_f2h(H(a) - H(b)); }
static inline uint16_t hmul(uint16_t a, uint16_t b) { return og_f2h(H(a) * H(b)); }

/* next fp16 bit pattern above / below a finite h (signed zeros step to the smallest subnormals) */
static uint16_t h_next_up(uint16_t h) {
    if (h == 0x8000u) return 0x0001u;
    return (h & 0x8000u) ? (uint16_t)(h - 1u) : (uint16_t)(h + 1u);
}
static uint16_t h_next_down(uint16_t h) {
    if (h == 0x0000u) return 0x8001u;
    return (h & 0x8000u) ? (uint16_t)(h + 1u) : (uint16_t)(h - 1u);
}

/* fp16 fused multiply-add a*b + c with ONE rounding to nearest even (the GPU's v_pk_fma_f16;
 * the blend's `C += c * w` accumulations, GlobalShaders.metal:1137-1145).  The
 * product is exact in double (22 significant bits); s = p + c rounds at most once and TwoSum
 * gives its exact error e.  Rounding s to fp16 is the correct rounding of p + c unless s lies
 * exactly on an fp16 midpoint, where the sign of e decides. */
static uint16_t hfma(uint16_t a, uint16_t b, uint16_t c) {
    const double p = (double)H(a) * (double)H(b), cc = (double)H(c);
    const double s = p + cc;
    const uint16_t h = og_d2h(s);
    if (!isfinite(s) || (h & 0x7C00u) == 0x7C00u) return h;
    const double bb = s - p;
    const double e = (p - (s - bb)) + (cc - bb);
    const double v = (double)H(h);
    if (e == 0.0 || v == s) return h;
    const uint16_t n = s > v ? h_next_up(h) : h_next_down(h);
    if ((n & 0x7C00u) == 0x7C00u) return h;
    const double nv = (double)H(n);
    if (s != 0.5 * (v + nv)) return h;  /* not a midpoint: s and p + c round alike */
    return (e > 0.0) == (nv > v) ? n : h;
}
uint16_t og_hfma(uint16_t a, uint16_t b, uint16_t c) { ensure_init(); return hfma(a, b, c); }
/* IEEE minNum / maxNum (a NaN operand yields the other operand). */
static inline uint16_t hmin(uint16_t a, uint16_t b) {
    float fa = H(a), fb = H(b);
    if (isnan(fa)) return b;
    if (isnan(fb)) return a;
    return fb < fa ? b : a;
}
static inline uint16_t hmax(uint16_t a, uint16_t b) {
    float fa = H(a), fb = H(b);
    if (isnan(fa)) return b;
    if (isnan(fb)) return a;
    return fb > fa ? b : a;
}

/* ------------------------------------------------------------------ */
/* small vector/matrix helpers (column-major like simd / Metal)        */
/* ------------------------------------------------------------------ */
typedef struct { float x, y; } f2;
typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;
typedef struct { f3 c[3]; } m3; /* columns */
typedef struct { f2 c[2]; } m2;

static inline float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
static inline float saturatef(float v) { return clampf(v, 0.0f, 1.0f); }
static inline float m3get(const m3 *m, int col, int row) {
    const float *p = &m->c[col].x;
    return p[row];
}
static inline void m3set(m3 *m, int col, int row, float v) {
    float *p = &m->c[col].x;
    p[row] = v;
}

/* float4x4 * float4 = sum_j col_j * v_j, left to right. */
static inline f4 mat4_mul_vec(const float *m, f4 v) {
    const float vv[4] = {v.x, v.y, v.z, v.w};
    float r[4];
    for (int i = 0; i < 4; ++i) {
        float acc = m[0 * 4 + i] * vv[0];
        acc = acc + m[1 * 4 + i] * vv[1];
        acc = acc + m[2 * 4 + i] * vv[2];
        acc = acc + m[3 * 4 + i] * vv[3];
        r[i] = acc;
    }
    f4 o = {r[0], r[1], r[2], r[3]};
    return o;
}
/* float3x3 * float3x3: (A*B)[c] = sum_k A[k] * B[c][k]. */
static inline m3 mat3_mul(const m3 *A, const m3 *B) {
    m3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) {
            float acc = m3get(A, 0, r) * m3get(B, c, 0);
            acc = acc + m3get(A, 1, r) * m3get(B, c, 1);
            acc = acc + m3get(A, 2, r) * m3get(B, c, 2);
            m3set(&R, c, r, acc);
        }
    return R;
}
static inline m3 mat3_transpose(const m3 *A) {
    m3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) m3set(&R, c, r, m3get(A, r, c));
    return R;
}

/* ------------------------------------------------------------------ */
/* GaussianShared.h restatements                                       */
/* ------------------------------------------------------------------ */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2_0 = 1.0925484305920792f;
static const float SH_C2_1 = -1.0925484305920792f;
static const float SH_C2_2 = 0.31539156525252005f;
static const float SH_C2_3 = -1.0925484305920792f;
static const float SH_C2_4 = 0.5462742152960396f;
static const float SH_C3_0 = -0.5900435899266435f;
static const float SH_C3_1 = 2.890611442640554f;
static const float SH_C3_2 = -0.4570457994644658f;
static const float SH_C3_3 = 0.3731763325901154f;
static const float SH_C3_4 = -0.4570457994644658f;
static const float SH_C3_5 = 1.445305721320277f;
static const float SH_C3_6 = -0.5900435899266435f;

/* GlobalProjectCullEncoder.swift:19-26: function constant SH_DEGREE from shComponents. */
static uint32_t sh_degree(uint32_t k) {
    if (k <= 1) return 0;
    if (k <= 4) return 1;
    if (k <= 9) return 2;
    return 3;
}

/* normalize(v) := v / sqrt(dot(v, v)) (declared choice). */
static inline f3 normalize3(f3 v) {
    float d = v.x * v.x + v.y * v.y;
    d = d + v.z * v.z;
    float n = sqrtf(d);
    f3 o = {v.x / n, v.y / n, v.z / n};
    return o;
}
static inline f2 normalize2(f2 v) {
    float d = v.x * v.x + v.y * v.y;
    float n = sqrtf(d);
    f2 o = {v.x / n, v.y / n};
    return o;
}

/* computeSHColor (GaussianShared.h:38-116). */
static f3 compute_sh_color(const void *harm, int half_harm, uint32_t gid, f3 pos, f3 cam,
                           uint32_t sh_components) {
    uint32_t deg = sh_degree(sh_components);
#define HV(i) (half_harm ? H(((const uint16_t *)harm)[(i)]) : ((const float *)harm)[(i)])
    if (deg == 0 || sh_components == 0) {
        size_t base = (size_t)gid * 3u;
        f3 o = {HV(base) * SH_C0, HV(base + 1) * SH_C0, HV(base + 2) * SH_C0};
        return o;
    }
    f3 d0 = {cam.x - pos.x, cam.y - pos.y, cam.z - pos.z};
    f3 dir = normalize3(d0);
    float xx = dir.x * dir.x, yy = dir.y * dir.y, zz = dir.z * dir.z;
    float xy = dir.x * dir.y, yz = dir.y * dir.z, xz = dir.x * dir.z;
    float b[16];
    b[0] = SH_C0;
    b[1] = (-SH_C1) * dir.y;
    b[2] = SH_C1 * dir.z;
    b[3] = (-SH_C1) * dir.x;
    if (deg >= 2) {
        b[4] = SH_C2_0 * xy;
        b[5] = SH_C2_1 * yz;
        b[6] = SH_C2_2 * ((2.0f * zz - xx) - yy);
        b[7] = SH_C2_3 * xz;
        b[8] = SH_C2_4 * (xx - yy);
    }
    if (deg >= 3) {
        b[9] = (SH_C3_0 * dir.y) * (3.0f * xx - yy);
        b[10] = (SH_C3_1 * xy) * dir.z;
        b[11] = (SH_C3_2 * dir.y) * ((4.0f * zz - xx) - yy);
        b[12] = (SH_C3_3 * dir.z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
        b[13] = (SH_C3_4 * dir.x) * ((4.0f * zz - xx) - yy);
        b[14] = (SH_C3_5 * dir.z) * (xx - yy);
        b[15] = (SH_C3_6 * dir.x) * (xx - 3.0f * yy);
    }
    uint32_t k = deg == 1 ? 4u : (deg == 2 ? 9u : 16u);
    size_t base = (size_t)gid * k * 3u;
    f3 c = {0.0f, 0.0f, 0.0f};
    for (uint32_t i = 0; i < k; ++i) {
        c.x = c.x + HV(base + i) * b[i];
        c.y = c.y + HV(base + k + i) * b[i];
        c.z = c.z + HV(base + 2 * k + i) * b[i];
    }
#undef HV
    return c;
}

/* srgbToLinearChannel (GaussianShared.h:118-121). */
static float srgb_to_linear(float c) {
    c = clampf(c, 0.0f, 1.0f);
    return (c <= 0.04045f) ? (c / 12.92f) : ogm_powrf((c + 0.055f) / 1.055f, 2.4f);
}

/* normalizeQuaternion (GaussianShared.h:289-295). */
static f4 normalize_quat(f4 q) {
    float d = q.x * q.x + q.y * q.y;
    d = d + q.z * q.z;
    d = d + q.w * q.w;
    float n = sqrtf(fmaxf(d, 1e-8f));
    if (n < 1e-8f) { f4 o = {1.0f, 0.0f, 0.0f, 0.0f}; return o; }
    f4 o = {q.x / n, q.y / n, q.z / n, q.w / n};
    return o;
}

/* quaternionToMatrix + matrixFromRows (GaussianShared.h:141-147, 297-305). */
static m3 quat_to_matrix(f4 q) {
    float x = q.x, y = q.y, z = q.z, r = q.w;
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, xz = x * z, yz = y * z;
    f3 row0 = {1.0f - 2.0f * (yy + zz), 2.0f * (xy - r * z), 2.0f * (xz + r * y)};
    f3 row1 = {2.0f * (xy + r * z), 1.0f - 2.0f * (xx + zz), 2.0f * (yz - r * x)};
    f3 row2 = {2.0f * (xz - r * y), 2.0f * (yz + r * x), 1.0f - 2.0f * (xx + yy)};
    m3 M;
    M.c[0].x = row0.x; M.c[0].y = row1.x; M.c[0].z = row2.x;
    M.c[1].x = row0.y; M.c[1].y = row1.y; M.c[1].z = row2.y;
    M.c[2].x = row0.z; M.c[2].y = row1.z; M.c[2].z = row2.z;
    return M;
}

/* buildCovariance3D (GaussianShared.h:307-324). */
static m3 build_cov3d(f3 s, f4 quat) {
    f4 q = normalize_quat(quat);
    m3 R = quat_to_matrix(q);
    f3 a = {R.c[0].x * s.x, R.c[0].y * s.x, R.c[0].z * s.x};
    f3 b = {R.c[1].x * s.y, R.c[1].y * s.y, R.c[1].z * s.y};
    f3 c = {R.c[2].x * s.z, R.c[2].y * s.z, R.c[2].z * s.z};
#define DOT3(p, q) ((a.p * a.q + b.p * b.q) + c.p * c.q)
    m3 C;
    C.c[0].x = DOT3(x, x); C.c[0].y = DOT3(x, y); C.c[0].z = DOT3(x, z);
    C.c[1].x = DOT3(y, x); C.c[1].y = DOT3(y, y); C.c[1].z = DOT3(y, z);
    C.c[2].x = DOT3(z, x); C.c[2].y = DOT3(z, y); C.c[2].z = DOT3(z, z);
#undef DOT3
    return C;
}

/* projectCovariance2D (GaussianShared.h:326-388). */
static m2 project_cov2d(const m3 *cov3d, f3 vp, const float *view, const float *proj,
                        float sw, float sh) {
    m3 W;
    for (int c = 0; c < 3; ++c) {
        W.c[c].x = view[c * 4 + 0];
        W.c[c].y = view[c * 4 + 1];
        W.c[c].z = view[c * 4 + 2];
    }
    float absZ = fabsf(vp.z);
    float signZ = (vp.z >= 0.0f) ? 1.0f : -1.0f;
    float safeAbsZ = fmaxf(absZ, 1e-4f);
    float invAbsZ = 1.0f / safeAbsZ;
    float invAbsZ2 = invAbsZ * invAbsZ;
    float p00 = proj[0], p11 = proj[5];
    float tanHalfFovX = 1.0f / fmaxf(fabsf(p00), 1e-4f);
    float tanHalfFovY = 1.0f / fmaxf(fabsf(p11), 1e-4f);
    float limX = 1.3f * tanHalfFovX;
    float limY = 1.3f * tanHalfFovY;
    float tx = vp.x * invAbsZ;
    float ty = vp.y * invAbsZ;
    float xClamped = clampf(tx, -limX, limX) * safeAbsZ;
    float yClamped = clampf(ty, -limY, limY) * safeAbsZ;
    float focalX = sw * fabsf(p00) * 0.5f;
    float focalY = sh * fabsf(p11) * 0.5f;
    m3 J;
    J.c[0].x = focalX * invAbsZ; J.c[0].y = 0.0f; J.c[0].z = 0.0f;
    J.c[1].x = 0.0f; J.c[1].y = focalY * invAbsZ; J.c[1].z = 0.0f;
    J.c[2].x = -focalX * xClamped * signZ * invAbsZ2;
    J.c[2].y = -focalY * yClamped * signZ * invAbsZ2;
    J.c[2].z = 0.0f;
    m3 T = mat3_mul(&J, &W);
    m3 M1 = mat3_mul(&T, cov3d);
    m3 Tt = mat3_transpose(&T);
    m3 F = mat3_mul(&M1, &Tt);
    m2 c2;
    c2.c[0].x = F.c[0].x; c2.c[0].y = F.c[0].y;
    c2.c[1].x = F.c[1].x; c2.c[1].y = F.c[1].y;
    c2.c[0].x = c2.c[0].x + 0.3f;
    c2.c[1].y = c2.c[1].y + 0.3f;
    return c2;
}

/* stabilizeCovariance2D (GaussianShared.h:655-714). */
static m2 stabilize_cov2d(m2 cov, float sw, float sh) {
    const float kMinVar = 1e-4f, kMinDet = 1e-8f, kMaxRatio = 256.0f, kBounds = 3.0f;
    float maxCond = kMaxRatio * kMaxRatio;
    float maxDim = fmaxf(sw, sh);
    float maxExtentPx = maxDim * 2.0f;
    float maxEig = maxExtentPx / kBounds;
    maxEig = maxEig * maxEig;
    float a = cov.c[0].x;
    float b = 0.5f * (cov.c[0].y + cov.c[1].x);
    float d = cov.c[1].y;
    if (!isfinite(a) || !isfinite(b) || !isfinite(d)) {
        m2 I = {{{1.0f, 0.0f}, {0.0f, 1.0f}}};
        return I;
    }
    a = fmaxf(a, kMinVar);
    d = fmaxf(d, kMinVar);
    float det = a * d - b * b;
    if (!isfinite(det) || det < kMinDet) {
        float bump = (kMinDet - det) + kMinVar;
        a = a + bump;
        d = d + bump;
        det = a * d - b * b;
    }
    float mid = 0.5f * (a + d);
    float disc = fmaxf(mid * mid - det, 0.0f);
    float sqrtDisc = sqrtf(disc);
    float l1 = mid + sqrtDisc;
    float l2 = fmaxf(mid - sqrtDisc, kMinVar);
    f2 v1;
    if (fabsf(b) > 1e-8f) {
        float vx = b, vy = l1 - a;
        float vlen = sqrtf(vx * vx + vy * vy);
        float dn = fmaxf(vlen, 1e-8f);
        v1.x = vx / dn;
        v1.y = vy / dn;
    } else if (a >= d) {
        v1.x = 1.0f; v1.y = 0.0f;
    } else {
        v1.x = 0.0f; v1.y = 1.0f;
    }
    f2 v2 = {v1.y, -v1.x};
    l1 = fminf(l1, maxEig);
    l2 = fmaxf(l2, l1 / maxCond);
    m2 o;
    o.c[0].x = l1 * (v1.x * v1.x) + l2 * (v2.x * v2.x);
    o.c[0].y = l1 * (v1.x * v1.y) + l2 * (v2.x * v2.y);
    o.c[1].x = l1 * (v1.y * v1.x) + l2 * (v2.y * v2.x);
    o.c[1].y = l1 * (v1.y * v1.y) + l2 * (v2.y * v2.y);
    return o;
}

/* fmod(theta, pi) for the atan2 range |theta| <= pi_f (exact, GaussianShared.h:436/481). */
static inline float fmod_pi(float t) { return fmodf(t, OGM_PI_F); }

/* covarianceToThetaSigmas (GaussianShared.h:446-488). */
static int cov_to_theta_sigmas(m2 cov, float *theta, float *s1, float *s2) {
    float a = cov.c[0].x;
    float b = 0.5f * (cov.c[0].y + cov.c[1].x);
    float d = cov.c[1].y;
    if (!isfinite(a) || !isfinite(b) || !isfinite(d)) return 0;
    a = fmaxf(a, 1e-8f);
    d = fmaxf(d, 1e-8f);
    float det = a * d - b * b;
    if (!isfinite(det) || det <= 0.0f) return 0;
    float mid = 0.5f * (a + d);
    float disc = fmaxf(mid * mid - det, 0.0f);
    float sq = sqrtf(disc);
    float l1 = fmaxf(mid + sq, 1e-8f);
    float l2 = fmaxf(mid - sq, 1e-8f);
    f2 v1;
    if (fabsf(b) > 1e-8f) {
        f2 t = {b, l1 - a};
        v1 = normalize2(t);
    } else if (a >= d) {
        v1.x = 1.0f; v1.y = 0.0f;
    } else {
        v1.x = 0.0f; v1.y = 1.0f;
    }
    float th = ogm_atan2f(v1.y, v1.x);
    th = fmod_pi(th);
    if (th < 0.0f) th = th + OGM_PI_F;
    if (th >= OGM_PI_F) th = th - OGM_PI_F;
    *theta = th;
    *s1 = sqrtf(l1);
    *s2 = sqrtf(l2);
    return isfinite(th) && isfinite(*s1) && isfinite(*s2);
}

/* packThetaPi (GaussianShared.h:434-440). */
static uint16_t pack_theta_pi(float th) {
    th = fmod_pi(th);
    if (th < 0.0f) th = th + OGM_PI_F;
    float u = th * (65535.0f / OGM_PI_F);
    return (uint16_t)clampf(u + 0.5f, 0.0f, 65535.0f);
}

/* computeOBBExtents (GaussianShared.h:402-427). */
static f2 obb_extents(m2 cov, float k) {
    float a = cov.c[0].x, b = cov.c[0].y, d = cov.c[1].y;
    float det = a * d - b * b;
    float mid = 0.5f * (a + d);
    float disc = fmaxf(mid * mid - det, 1e-6f);
    float sq = sqrtf(disc);
    float l1 = mid + sq;
    float l2 = fmaxf(mid - sq, 1e-6f);
    float e1 = k * sqrtf(fmaxf(l1, 1e-6f));
    float e2 = k * sqrtf(fmaxf(l2, 1e-6f));
    f2 v1;
    if (fabsf(b) > 1e-6f) {
        float vx = b, vy = l1 - a;
        float vlen = sqrtf(vx * vx + vy * vy);
        float dn = fmaxf(vlen, 1e-6f);
        v1.x = vx / dn;
        v1.y = vy / dn;
    } else if (a >= d) {
        v1.x = 1.0f; v1.y = 0.0f;
    } else {
        v1.x = 0.0f; v1.y = 1.0f;
    }
    f2 o = {fabsf(v1.x) * e1 + fabsf(v1.y) * e2, fabsf(v1.y) * e1 + fabsf(v1.x) * e2};
    return o;
}

/* cullByTotalInkFromCov + computeDepthFactor (GaussianShared.h:275-278, 739-768).
 * pow(s, 2.0f) := s*s; farPlane * 0.02 is a float product (Metal has no double). */
static int cull_total_ink(float opacity, m2 cov, float depth, float nearp, float farp,
                          float thr) {
    float a = cov.c[0].x;
    float b = 0.5f * (cov.c[0].y + cov.c[1].x);
    float d = cov.c[1].y;
    float det = a * d - b * b;
    if (thr <= 0.0f) return 0;
    float ink = opacity * 6.283185f * sqrtf(fmaxf(det, 1e-12f));
    float adjFar = farp * 0.02f;
    float s = saturatef((adjFar - depth) / (adjFar - nearp));
    float depthFactor = 1.0f - s * s;
    float adjThr = depthFactor * thr;
    return ink < adjThr;
}

/* conicFromThetaSigmas (GaussianShared.h:490-510) for a quantised angle. */
typedef struct { float A, B, C; } conic3;
static inline conic3 conic_from_quant(uint16_t theta_q, float sigma1, float sigma2) {
    float s = g_sin_t[theta_q], c = g_cos_t[theta_q];
    float sig1 = fmaxf(sigma1, 1e-4f);
    float sig2 = fmaxf(sigma2, 1e-4f);
    float iv1 = 1.0f / (sig1 * sig1);
    float iv2 = 1.0f / (sig2 * sig2);
    float cc = c * c, ss = s * s, cs = c * s;
    conic3 o;
    o.A = cc * iv1 + ss * iv2;
    o.B = cs * (iv1 - iv2);
    o.C = ss * iv1 + cc * iv2;
    return o;
}

/* FlashGS-style ellipse/rect test (GaussianShared.h:595-653). */
static inline int seg_ellipse(float a, float b, float c, float d, float l, float r) {
    float delta = b * b - 4.0f * a * c;
    float t1 = (l - d) * (2.0f * a) + b;
    float t2 = (r - d) * (2.0f * a) + b;
    return delta >= 0.0f && (t1 <= 0.0f || t1 * t1 <= delta) && (t2 >= 0.0f || t2 * t2 <= delta);
}
static inline int intersects_tile(int pminx, int pminy, int pmaxx, int pmaxy, float cx, float cy,
                                  conic3 k, float power) {
    if (cx >= (float)pminx && cx <= (float)pmaxx && cy >= (float)pminy && cy <= (float)pmaxy)
        return 1;
    float w = 2.0f * power;
    float dx, dy, a, b, c;
    if (cx * 2.0f < (float)(pminx + pmaxx)) dx = cx - (float)pminx;
    else dx = cx - (float)pmaxx;
    a = k.C;
    b = -2.0f * k.B * dx;
    c = k.A * dx * dx - w;
    if (seg_ellipse(a, b, c, cy, (float)pminy, (float)pmaxy)) return 1;
    if (cy * 2.0f < (float)(pminy + pmaxy)) dy = cy - (float)pminy;
    else dy = cy - (float)pmaxy;
    a = k.A;
    b = -2.0f * k.B * dy;
    c = k.C * dy * dy - w;
    if (seg_ellipse(a, b, c, cx, (float)pminx, (float)pmaxx)) return 1;
    return 0;
}
/* gaussianComputePower (GaussianShared.h:595-597). */
static inline float compute_power(float opacity) {
    const float LN2 = 0.693147180559945f;
    return LN2 * 8.0f + LN2 * ogm_log2f(fmaxf(opacity, 1e-6f));
}

/* ------------------------------------------------------------------ */
/* threading                                                           */
/* ------------------------------------------------------------------ */
typedef void (*range_fn)(void *ctx, uint32_t lo, uint32_t hi);
typedef struct { range_fn fn; void *ctx; uint32_t lo, hi; } job_t;
static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    j->fn(j->ctx, j->lo, j->hi);
    return NULL;
}
static void parallel_for(int nthreads, uint32_t n, range_fn fn, void *ctx) {
    if (nthreads <= 1 || n < 1024) { fn(ctx, 0, n); return; }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    uint32_t chunk = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; ++t) {
        uint32_t lo = (uint32_t)t * chunk, hi = lo + chunk;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t].fn = fn; jobs[t].ctx = ctx; jobs[t].lo = lo; jobs[t].hi = hi;
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
        used++;
    }
    for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}
/* interleaved variant for load balance (tiles): thread t takes i = t, t+T, ... */
typedef struct { range_fn fn; void *ctx; uint32_t t, nt, n; } ijob_t;
static void *ijob_run(void *p) {
    ijob_t *j = (ijob_t *)p;
    for (uint32_t i = j->t; i < j->n; i += j->nt) j->fn(j->ctx, i, i + 1);
    return NULL;
}
static void parallel_for_interleaved(int nthreads, uint32_t n, range_fn fn, void *ctx) {
    if (nthreads <= 1) { fn(ctx, 0, n); return; }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    ijob_t jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].fn = fn; jobs[t].ctx = ctx; jobs[t].t = (uint32_t)t;
        jobs[t].nt = (uint32_t)nthreads; jobs[t].n = n;
        pthread_create(&th[t], NULL, ijob_run, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------ */
/* frame                                                               */
/* ------------------------------------------------------------------ */
typedef struct {
    const og_config *cfg;
    const void *gaussians, *harmonics;
    uint32_t count, shk;
    const og_camera *cam;
    float width, height; /* camera.width/height = frame size (KernelTypes.swift:107-123) */
    uint32_t tiles_x, tiles_y;
    og_frame *f;
    uint32_t *offsets;
    conic3 *conic;
    float *power;
} frame_ctx;

static inline void mark_culled(og_frame *f, uint32_t gid) {
    int32_t *b = f->bounds + 4 * (size_t)gid;
    b[0] = 0; b[1] = -1; b[2] = 0; b[3] = -1;
    f->mask[gid] = 0;
}

/* globalProjectCull (GlobalShaders.metal:19-123). */
static void project_range(void *vctx, uint32_t lo, uint32_t hi) {
    frame_ctx *X = (frame_ctx *)vctx;
    og_frame *f = X->f;
    const og_camera *cam = X->cam;
    const int half_in = X->cfg->precision == 1;
    const float W = X->width, Hh = X->height;
    const float alphaThreshold = 0.005f, totalInkThreshold = 2.0f;
    const int tileW = 32, tileH = 16;
    for (uint32_t gid = lo; gid < hi; ++gid) {
        f3 pos, scale;
        float opacity;
        f4 rot;
        if (half_in) {
            const og_world16 *g = (const og_world16 *)X->gaussians + gid;
            pos.x = g->px; pos.y = g->py; pos.z = g->pz;
            scale.x = H(g->sx); scale.y = H(g->sy); scale.z = H(g->sz);
            opacity = H(g->opacity);
            rot.x = H(g->rx); rot.y = H(g->ry); rot.z = H(g->rz); rot.w = H(g->rw);
        } else {
            const og_world32 *g = (const og_world32 *)X->gaussians + gid;
            pos.x = g->px; pos.y = g->py; pos.z = g->pz;
            scale.x = g->sx; scale.y = g->sy; scale.z = g->sz;
            opacity = g->opacity;
            rot.x = g->rot[0]; rot.y = g->rot[1]; rot.z = g->rot[2]; rot.w = g->rot[3];
        }
        /* cullByScale (GaussianShared.h:719-722) */
        if (fmaxf(scale.x, fmaxf(scale.y, scale.z)) < 0.0005f) { mark_culled(f, gid); continue; }
        f4 p4 = {pos.x, pos.y, pos.z, 1.0f};
        f4 vp = mat4_mul_vec(cam->view, p4);
        f4 clip = mat4_mul_vec(cam->proj, vp);
        float depth = clip.w;
        if (!(clip.w > cam->near_plane)) { mark_culled(f, gid); continue; }
        float ndcx = clip.x / clip.w, ndcy = clip.y / clip.w;
        /* ndcToScreenCentered (GaussianShared.h:184-189) */
        float sx = ((ndcx + 1.0f) * W - 1.0f) * 0.5f;
        float sy = ((ndcy + 1.0f) * Hh - 1.0f) * 0.5f;
        if (opacity < alphaThreshold) { mark_culled(f, gid); continue; }
        f4 quat = normalize_quat(rot);
        m3 cov3d = build_cov3d(scale, quat);
        f3 vp3 = {vp.x, vp.y, vp.z};
        m2 cov2d = project_cov2d(&cov3d, vp3, cam->view, cam->proj, W, Hh);
        cov2d = stabilize_cov2d(cov2d, W, Hh);
        float theta, s1, s2;
        if (!cov_to_theta_sigmas(cov2d, &theta, &s1, &s2)) { mark_culled(f, gid); continue; }
        float radius = 3.0f * fmaxf(s1, s2);
        if (radius < 0.5f) { mark_culled(f, gid); continue; }
        if (cull_total_ink(opacity, cov2d, depth, cam->near_plane, cam->far_plane, totalInkThreshold)) {
            mark_culled(f, gid);
            continue;
        }
        f2 obb = obb_extents(cov2d, 3.0f);
        /* cullByScreenBounds (GaussianShared.h:771-781) */
        if (sx + obb.x < 0.0f || sx - obb.x > W || sy + obb.y < 0.0f || sy - obb.y > Hh) {
            mark_culled(f, gid);
            continue;
        }
        f3 camc = {cam->position[0], cam->position[1], cam->position[2]};
        f3 col = compute_sh_color(X->harmonics, half_in, gid, pos, camc, X->shk);
        col.x = fmaxf(col.x + 0.5f, 0.0f);
        col.y = fmaxf(col.y + 0.5f, 0.0f);
        col.z = fmaxf(col.z + 0.5f, 0.0f);
        if (X->cfg->color_space == 1) { /* maybeDecodeSRGBToLinear (GaussianShared.h:131-133) */
            col.x = srgb_to_linear(col.x);
            col.y = srgb_to_linear(col.y);
            col.z = srgb_to_linear(col.z);
        }
        og_render_data rd;
        rd.meanX = og_f2h(sx);
        rd.meanY = og_f2h(sy);
        rd.theta = pack_theta_pi(theta);
        rd.sigma1 = og_f2h(s1);
        rd.sigma2 = og_f2h(s2);
        rd.depth = og_f2h(depth);
        rd.colorR = (uint8_t)clampf(col.x * 255.0f, 0.0f, 255.0f);
        rd.colorG = (uint8_t)clampf(col.y * 255.0f, 0.0f, 255.0f);
        rd.colorB = (uint8_t)clampf(col.z * 255.0f, 0.0f, 255.0f);
        rd.opacity = (uint8_t)clampf(opacity * 255.0f, 0.0f, 255.0f);
        f->render_data[gid] = rd;
        /* computeTileBounds (GaussianShared.h:791-828) */
        float xmin = sx - obb.x, xmax = sx + obb.x, ymin = sy - obb.y, ymax = sy + obb.y;
        float maxW = W - 1.0f, maxH = Hh - 1.0f;
        xmin = clampf(xmin, 0.0f, maxW);
        xmax = clampf(xmax, 0.0f, maxW);
        ymin = clampf(ymin, 0.0f, maxH);
        ymax = clampf(ymax, 0.0f, maxH);
        int minTX = (int)floorf(xmin / (float)tileW);
        int maxTX = (int)ceilf(xmax / (float)tileW) - 1;
        int minTY = (int)floorf(ymin / (float)tileH);
        int maxTY = (int)ceilf(ymax / (float)tileH) - 1;
        if (minTX < 0) minTX = 0;
        if (minTY < 0) minTY = 0;
        if (maxTX > (int)X->tiles_x - 1) maxTX = (int)X->tiles_x - 1;
        if (maxTY > (int)X->tiles_y - 1) maxTY = (int)X->tiles_y - 1;
        int32_t *b = f->bounds + 4 * (size_t)gid;
        b[0] = minTX; b[1] = maxTX; b[2] = minTY; b[3] = maxTY;
        f->mask[gid] = 1;
    }
}

/* tileCountIndirectKernel (GlobalShaders.metal:563-616); the compaction of
 * :169-208 keeps ascending gid order, so counting in gid order is equivalent. */
static void count_range(void *vctx, uint32_t lo, uint32_t hi) {
    frame_ctx *X = (frame_ctx *)vctx;
    og_frame *f = X->f;
    for (uint32_t gid = lo; gid < hi; ++gid) {
        const int32_t *r = f->bounds + 4 * (size_t)gid;
        f->tile_counts[gid] = 0;
        if (r[0] > r[1] || r[2] > r[3]) continue;
        const og_render_data *g = &f->render_data[gid];
        float alpha = (float)g->opacity;
        if (alpha < 1e-4f) continue;
        float cx = H(g->meanX), cy = H(g->meanY);
        conic3 k = conic_from_quant(g->theta, H(g->sigma1), H(g->sigma2));
        float power = compute_power(alpha);
        X->conic[gid] = k;
        X->power[gid] = power;
        uint32_t n = 0;
        for (int ty = r[2]; ty <= r[3]; ++ty)
            for (int tx = r[0]; tx <= r[1]; ++tx) {
                int px0 = tx * 32, py0 = ty * 16;
                if (intersects_tile(px0, py0, px0 + 31, py0 + 15, cx, cy, k, power)) n++;
            }
        f->tile_counts[gid] = n;
    }
}

/* tileScatterIndirectKernel (GlobalShaders.metal:623-678) fused with
 * computeSortKeysKernel (GlobalShaders.metal:266-295). */
static void scatter_range(void *vctx, uint32_t lo, uint32_t hi) {
    frame_ctx *X = (frame_ctx *)vctx;
    og_frame *f = X->f;
    const uint32_t maxA = f->max_assignments;
    for (uint32_t gid = lo; gid < hi; ++gid) {
        if (f->tile_counts[gid] == 0) continue;
        const int32_t *r = f->bounds + 4 * (size_t)gid;
        const og_render_data *g = &f->render_data[gid];
        float cx = H(g->meanX), cy = H(g->meanY);
        conic3 k = X->conic[gid];
        float power = X->power[gid];
        uint32_t wp = X->offsets[gid];
        for (int ty = r[2]; ty <= r[3]; ++ty)
            for (int tx = r[0]; tx <= r[1]; ++tx) {
                int px0 = tx * 32, py0 = ty * 16;
                if (intersects_tile(px0, py0, px0 + 31, py0 + 15, cx, cy, k, power)) {
                    if (wp < maxA) {
                        uint32_t tile = (uint32_t)(ty * (int)X->tiles_x + tx);
                        f->keys[wp] = og_sort_key(tile, g->depth);
                        f->values[wp] = (int32_t)gid;
                        wp++;
                    }
                }
            }
    }
}

uint32_t og_sort_key(uint32_t tile, uint16_t depth_h) {
    uint32_t depthBits = (uint32_t)depth_h ^ 0x8000u;
    return (tile << 16) | (depthBits & 0xFFFFu);
}

/* Stable LSD radix sort, 8-bit digits: the semantics of RadixSortEncoder.encode
 * (RadixSortEncoder.swift:41-101) + radixHistogram/Scan/Apply/Scatter kernels
 * (GlobalShaders.metal:768-1028). */
void og_radix_sort_pairs(uint32_t *keys, int32_t *values, uint32_t n) {
    if (n < 2) return;
    uint32_t *k2 = (uint32_t *)malloc(sizeof(uint32_t) * n);
    int32_t *v2 = (int32_t *)malloc(sizeof(int32_t) * n);
    uint32_t *ks = keys, *kd = k2;
    int32_t *vs = values, *vd = v2;
    for (int pass = 0; pass < 4; ++pass) {
        uint32_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        int sh = pass * 8;
        for (uint32_t i = 0; i < n; ++i) cnt[((ks[i] >> sh) & 0xFFu) + 1]++;
        for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t d = (ks[i] >> sh) & 0xFFu;
            uint32_t p = cnt[d]++;
            kd[p] = ks[i];
            vd[p] = vs[i];
        }
        uint32_t *tk = ks; ks = kd; kd = tk;
        int32_t *tv = vs; vs = vd; vd = tv;
    }
    /* 4 passes: result is back in the caller's arrays */
    free(k2);
    free(v2);
}

/* globalRender (GlobalShaders.metal:1030-1187) for one active tile. */
typedef struct {
    uint16_t mx, my, cxx, cyy, cxy2, op, cr, cg, cb, dep;
} blend_rec;
typedef struct {
    og_frame *f;
    blend_rec *rec; /* per gaussian */
    uint32_t *active;
} blend_ctx;

static void blend_tiles(void *vctx, uint32_t lo, uint32_t hi) {
    blend_ctx *B = (blend_ctx *)vctx;
    og_frame *f = B->f;
    const uint16_t H_ONE = 0x3C00u, H_ZERO = 0;
    const uint16_t thr = og_f2h(1.0f / 255.0f); /* half(1.0h/255.0h) */
    const uint16_t c099 = og_d2h(0.99);         /* 0.99h */
    const uint32_t W = f->width, Hh = f->height;
    for (uint32_t ai = lo; ai < hi; ++ai) {
        uint32_t tile = B->active[ai];
        uint32_t start = f->headers[2 * tile], count = f->headers[2 * tile + 1];
        uint32_t tileX = tile % f->tiles_x, tileY = tile / f->tiles_x;
        for (uint32_t ly = 0; ly < 8; ++ly)
            for (uint32_t lx = 0; lx < 8; ++lx) {
                uint32_t baseX = tileX * 32 + lx * 4, baseY = tileY * 16 + ly * 2;
                uint16_t posx[4], posy[2];
                for (int i = 0; i < 4; ++i) posx[i] = og_f2h((float)(baseX + (uint32_t)i));
                for (int j = 0; j < 2; ++j) posy[j] = og_f2h((float)(baseY + (uint32_t)j));
                uint16_t T[8], C[8][3], D[8];
                for (int q = 0; q < 8; ++q) { T[q] = H_ONE; C[q][0] = C[q][1] = C[q][2] = H_ZERO; D[q] = H_ZERO; }
                uint32_t i = 0;
                for (; i < count; ++i) {
                    uint16_t m0 = hmax(hmax(T[0], T[1]), hmax(T[2], T[3]));
                    uint16_t m1 = hmax(hmax(T[4], T[5]), hmax(T[6], T[7]));
                    if (H(hmax(m0, m1)) < H(thr)) break;
                    int32_t gi = f->sorted_values[start + i];
                    if (gi < 0) continue;
                    const blend_rec *g = &B->rec[gi];
                    uint16_t a[8];
                    int any = 0;
                    for (int j = 0; j < 2; ++j)
                        for (int ii = 0; ii < 4; ++ii) {
                            int q = j * 4 + ii;
                            uint16_t dx = hsub(posx[ii], g->mx), dy = hsub(posy[j], g->my);
                            uint16_t t2 = hmul(hmul(dx, dx), g->cxx);
                            uint16_t t4 = hmul(hmul(dy, dy), g->cyy);
                            uint16_t t7 = hmul(hmul(dx, dy), g->cxy2);
                            uint16_t p = hadd(hadd(t2, t4), t7);
                            uint16_t arg = og_f2h(-0.5f * H(p));
                            uint16_t e = g_exp_h[arg];
                            a[q] = hmin(hmul(g->op, e), c099);
                            if (H(a[q]) != 0.0f) any = 1;
                        }
                    if (!any) continue;
                    for (int q = 0; q < 8; ++q) {
                        uint16_t w = hmul(a[q], T[q]);
                        C[q][0] = hfma(g->cr, w, C[q][0]);  /* color += gColor * w: fused */
                        C[q][1] = hfma(g->cg, w, C[q][1]);
                        C[q][2] = hfma(g->cb, w, C[q][2]);
                        D[q] = hfma(g->dep, w, D[q]);
                        T[q] = hmul(T[q], hsub(H_ONE, a[q]));
                    }
                }
                f->group_iters[(size_t)tile * 64 + ly * 8 + lx] = i;
                for (int j = 0; j < 2; ++j)
                    for (int ii = 0; ii < 4; ++ii) {
                        uint32_t x = baseX + (uint32_t)ii, y = baseY + (uint32_t)j;
                        if (x >= W || y >= Hh) continue;
                        int q = j * 4 + ii;
                        uint16_t *px = f->color + 4 * ((size_t)y * W + x);
                        px[0] = C[q][0]; px[1] = C[q][1]; px[2] = C[q][2];
                        px[3] = hsub(H_ONE, T[q]);
                        f->depth[(size_t)y * W + x] = D[q];
                    }
            }
    }
}

typedef struct { og_frame *f; blend_rec *rec; } rec_ctx;
static void rec_range(void *vctx, uint32_t lo, uint32_t hi) {
    rec_ctx *R = (rec_ctx *)vctx;
    og_frame *f = R->f;
    for (uint32_t gid = lo; gid < hi; ++gid) {
        if (!f->mask[gid]) continue;
        const og_render_data *g = &f->render_data[gid];
        /* per-entry values of globalRender (GlobalShaders.metal:1094-1105, :9-15) */
        conic3 k = conic_from_quant(g->theta, H(g->sigma1), H(g->sigma2));
        blend_rec *r = &R->rec[gid];
        r->mx = g->meanX;
        r->my = g->meanY;
        r->cxx = og_f2h(k.A);
        r->cyy = og_f2h(k.C);
        r->cxy2 = og_f2h(2.0f * k.B);
        r->op = og_f2h(H(og_f2h((float)g->opacity)) / 255.0f);
        r->cr = og_f2h(H(og_f2h((float)g->colorR)) / 255.0f);
        r->cg = og_f2h(H(og_f2h((float)g->colorG)) / 255.0f);
        r->cb = og_f2h(H(og_f2h((float)g->colorB)) / 255.0f);
        r->dep = g->depth;
    }
}

void og_frame_free(og_frame *f) {
    if (!f) return;
    free(f->render_data); free(f->bounds); free(f->mask); free(f->tile_counts);
    free(f->keys); free(f->values); free(f->sorted_keys); free(f->sorted_values);
    free(f->headers); free(f->color); free(f->depth); free(f->group_iters);
    free(f);
}

/* GlobalRenderer.render -> encodeRenderToTargetTexture (GlobalRenderer.swift:201-370). */
int og_render(const og_config *cfg, const void *gaussians, const void *harmonics,
              uint32_t count, uint32_t shk, const og_camera *cam, uint32_t width,
              uint32_t height, int nthreads, og_frame **out) {
    ensure_init();
    *out = NULL;
    if (!cfg || !cam || (count > 0 && (!gaussians || !harmonics))) return OG_ERR_INVALID_ARGUMENT;
    if (cfg->max_gaussians > 30000000u) return OG_ERR_INVALID_GAUSSIAN_COUNT;
    uint32_t maxG = cfg->max_gaussians ? cfg->max_gaussians : 1u;
    if (count > maxG) return OG_ERR_INVALID_GAUSSIAN_COUNT; /* validateLimits :372-376 */
    uint32_t maxW = cfg->max_width ? cfg->max_width : 1u;
    uint32_t maxH = cfg->max_height ? cfg->max_height : 1u;
    if (width == 0 || height == 0 || width > maxW || height > maxH) return OG_ERR_INVALID_DIMENSIONS;
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads < 1) nthreads = 1;

    og_frame *f = (og_frame *)calloc(1, sizeof(og_frame));
    if (!f) return OG_ERR_OUT_OF_MEMORY;
    f->count = count;
    f->width = width;
    f->height = height;
    /* RendererLimits (GlobalRenderer.swift:6-51): tile grid from max dims, 32x16 tiles */
    f->tiles_x = (maxW + 31u) / 32u;
    f->tiles_y = (maxH + 15u) / 16u;
    f->tile_count = f->tiles_x * f->tiles_y;
    f->max_assignments = 4u * maxG; /* GlobalResources.swift:79 */
    size_t n = count ? count : 1;
    f->render_data = (og_render_data *)calloc(n, sizeof(og_render_data));
    f->bounds = (int32_t *)calloc(n * 4, sizeof(int32_t));
    f->mask = (uint8_t *)calloc(n, 1);
    f->tile_counts = (uint32_t *)calloc(n, sizeof(uint32_t));
    f->headers = (uint32_t *)calloc((size_t)f->tile_count * 2, sizeof(uint32_t));
    f->color = (uint16_t *)calloc((size_t)width * height * 4, sizeof(uint16_t));
    f->depth = (uint16_t *)calloc((size_t)width * height, sizeof(uint16_t));
    f->group_iters = (uint32_t *)calloc((size_t)f->tile_count * 64, sizeof(uint32_t));
    uint32_t *offsets = (uint32_t *)calloc(n, sizeof(uint32_t));
    conic3 *conic = (conic3 *)calloc(n, sizeof(conic3));
    float *power = (float *)calloc(n, sizeof(float));
    if (!f->render_data || !f->bounds || !f->mask || !f->tile_counts || !f->headers || !f->color ||
        !f->depth || !f->group_iters || !offsets || !conic || !power) {
        free(offsets); free(conic); free(power);
        og_frame_free(f);
        return OG_ERR_OUT_OF_MEMORY;
    }

    frame_ctx X;
    memset(&X, 0, sizeof(X));
    X.cfg = cfg; X.gaussians = gaussians; X.harmonics = harmonics;
    X.count = count; X.shk = shk; X.cam = cam;
    X.width = (float)width; X.height = (float)height;
    X.tiles_x = f->tiles_x; X.tiles_y = f->tiles_y;
    X.f = f; X.offsets = offsets; X.conic = conic; X.power = power;

    double t0 = now_s();
    parallel_for(nthreads, count, project_range, &X);
    double t1 = now_s();
    parallel_for(nthreads, count, count_range, &X);
    /* exclusive prefix sum of tile counts (TwoPassTileAssignEncoder.swift:288-325) */
    uint64_t total = 0;
    uint32_t visible = 0;
    for (uint32_t i = 0; i < count; ++i) {
        offsets[i] = (uint32_t)(total > 0xFFFFFFFFull ? 0xFFFFFFFFu : total);
        total += f->tile_counts[i];
        visible += f->mask[i];
    }
    f->visible = visible;
    /* prepareAssignmentDispatchKernel clamp (GlobalShaders.metal:694-701) */
    uint32_t tot = (uint32_t)(total > f->max_assignments ? f->max_assignments : total);
    f->overflow = total > f->max_assignments ? 1u : 0u;
    f->total_assignments = tot;
    size_t na = tot ? tot : 1;
    f->keys = (uint32_t *)calloc(na, sizeof(uint32_t));
    f->values = (int32_t *)calloc(na, sizeof(int32_t));
    f->sorted_keys = (uint32_t *)calloc(na, sizeof(uint32_t));
    f->sorted_values = (int32_t *)calloc(na, sizeof(int32_t));
    if (!f->keys || !f->values || !f->sorted_keys || !f->sorted_values) {
        free(offsets); free(conic); free(power);
        og_frame_free(f);
        return OG_ERR_OUT_OF_MEMORY;
    }
    parallel_for(nthreads, count, scatter_range, &X);
    double t2 = now_s();
    memcpy(f->sorted_keys, f->keys, sizeof(uint32_t) * tot);
    memcpy(f->sorted_values, f->values, sizeof(int32_t) * tot);
    og_radix_sort_pairs(f->sorted_keys, f->sorted_values, tot);
    double t3 = now_s();
    /* buildHeadersFromSortedKernel (GlobalShaders.metal:304-363) */
    uint32_t *active = (uint32_t *)calloc(f->tile_count ? f->tile_count : 1, sizeof(uint32_t));
    uint32_t nact = 0;
    for (uint32_t tile = 0; tile < f->tile_count; ++tile) {
        if (tot == 0) { f->headers[2 * tile] = 0; f->headers[2 * tile + 1] = 0; continue; }
        uint32_t l = 0, r = tot;
        while (l < r) {
            uint32_t mid = (l + r) >> 1;
            if ((f->sorted_keys[mid] >> 16) < tile) l = mid + 1; else r = mid;
        }
        uint32_t s = l;
        l = s; r = tot;
        while (l < r) {
            uint32_t mid = (l + r) >> 1;
            if ((f->sorted_keys[mid] >> 16) <= tile) l = mid + 1; else r = mid;
        }
        uint32_t e = l;
        f->headers[2 * tile] = s;
        f->headers[2 * tile + 1] = e > s ? e - s : 0u;
        if (e > s) active[nact++] = tile;
    }
    f->active_tiles = nact;
    double t4 = now_s();
    /* clearRenderTexturesKernel (GlobalShaders.metal:140-154): color (0,0,0,1), depth 0 */
    for (size_t i = 0; i < (size_t)width * height; ++i) {
        f->color[4 * i + 0] = 0; f->color[4 * i + 1] = 0; f->color[4 * i + 2] = 0;
        f->color[4 * i + 3] = 0x3C00u;
        f->depth[i] = 0;
    }
    blend_rec *rec = (blend_rec *)calloc(n, sizeof(blend_rec));
    rec_ctx RC = {f, rec};
    parallel_for(nthreads, count, rec_range, &RC);
    blend_ctx B = {f, rec, active};
    parallel_for_interleaved(nthreads, nact, blend_tiles, &B);
    double t5 = now_s();
    free(rec); free(active); free(offsets); free(conic); free(power);
    f->t_project = t1 - t0;
    f->t_assign = t2 - t1;
    f->t_sort = t3 - t2;
    f->t_headers = t4 - t3;
    f->t_blend = t5 - t4;
    *out = f;
    return OG_OK;
}

/* ------------------------------------------------------------------ */
/* reference test fixtures (TestUtils.swift)                           */
/* ------------------------------------------------------------------ */
void og_srand48(long seed) { srand48(seed); }
double og_drand48(void) { return drand48(); }

void og_gen_visible_gaussians(uint32_t count, long seed, og_world32 *world, float *harm) {
    srand48(seed);
    for (uint32_t i = 0; i < count; ++i) {
        float z = (float)(drand48() * 8.0 + 1.5);
        float spread = z * 0.6f;
        float x = (float)(drand48() * 2.0 - 1.0) * spread;
        float y = (float)(drand48() * 2.0 - 1.0) * spread;
        float s = (float)(drand48() * 0.15 + 0.08);
        float op = (float)(drand48() * 0.5 + 0.5);
        float r = (float)drand48(), g = (float)drand48(), b = (float)drand48();
        og_world32 *w = &world[i];
        memset(w, 0, sizeof(*w));
        w->px = x; w->py = y; w->pz = z;
        w->opacity = op;
        w->sx = s; w->sy = s; w->sz = s;
        w->rot[0] = 0.0f; w->rot[1] = 0.0f; w->rot[2] = 0.0f; w->rot[3] = 1.0f;
        harm[3 * i + 0] = r; harm[3 * i + 1] = g; harm[3 * i + 2] = b;
    }
}

void og_gen_grid_gaussians(uint32_t count, long seed, og_world32 *world, float *harm) {
    srand48(seed);
    uint32_t grid = (uint32_t)sqrt((double)count) + 1u;
    for (uint32_t i = 0; i < count; ++i) {
        float x = (float)(i % grid) / (float)grid * 4.0f - 2.0f;
        float y = (float)(i / grid) / (float)grid * 4.0f - 2.0f;
        float z = (float)(drand48() * 3.0 + 2.0);
        float s = (float)(drand48() * 0.1 + 0.05);
        float op = (float)(drand48() * 0.5 + 0.5);
        float r = (float)(drand48() * 0.5), g = (float)(drand48() * 0.5), b = (float)(drand48() * 0.5);
        og_world32 *w = &world[i];
        memset(w, 0, sizeof(*w));
        w->px = x; w->py = y; w->pz = z;
        w->opacity = op;
        w->sx = s; w->sy = s; w->sz = s;
        w->rot[3] = 1.0f;
        harm[3 * i + 0] = r; harm[3 * i + 1] = g; harm[3 * i + 2] = b;
    }
}

void og_make_camera(uint32_t width, uint32_t height, og_camera *cam) {
    memset(cam, 0, sizeof(*cam));
    const float nearp = 0.1f, farp = 10.0f;
    float aspect = (float)width / (float)height;
    float fov = 60.0f * OGM_PI_F / 180.0f;
    float f = 1.0f / tanf(fov / 2.0f);
    float *P = cam->proj;
    P[0] = f / aspect;
    P[5] = f;
    P[10] = farp / (farp - nearp);
    P[11] = 1.0f;
    P[14] = -(farp * nearp) / (farp - nearp);
    for (int i = 0; i < 4; ++i) cam->view[i * 4 + i] = 1.0f;
    cam->focal_x = (float)width * f / (2.0f * aspect);
    cam->focal_y = (float)height * f / 2.0f;
    cam->near_plane = nearp;
    cam->far_plane = farp;
}

/* Metal's conversion of the half4 a texture write stores (GlobalShaders.metal:1155-1186) into the
 * target's pixel format, as declared in include/gsm_renderer.h: unorm8 = RTNE(clamp * 255) with
 * IEEE maxNum/minNum clamping (NaN -> 0); sRGB formats encode R, G, B first with
 * c <= 0.0031308 ? 12.92 c : 1.055 powr(c, 1 / 2.4) - 0.055 (fp32, contract powr). */
static float og_clamp01(float x) {
    x = (x > 0.0f || x != x) ? (x != x ? 0.0f : x) : 0.0f; /* maxNum(x, 0) */
    return x < 1.0f ? x : 1.0f;                               /* minNum(x, 1) */
}
static uint32_t og_unorm8(float x) { return (uint32_t)nearbyintf(x * 255.0f); }
int og_convert_color(const uint16_t *src, size_t n, int format, void *dst) {
    ensure_init();
    if (format == 0) {
        memcpy(dst, src, n * 8);
        return 8;
    }
    for (size_t i = 0; i < n; ++i) {
        float c[4];
        for (int k = 0; k < 4; ++k) c[k] = g_h2f[src[4 * i + k]];
        if (format == 1) {
            memcpy((uint8_t *)dst + 16 * i, c, 16);
            continue;
        }
        if (format < 2 || format > 5) return 0;
        const int srgb = format == 3 || format == 5;
        uint32_t u[4];
        for (int k = 0; k < 4; ++k) {
            float x = og_clamp01(c[k]);
            if (srgb && k < 3) x = x <= 0.0031308f ? x * 12.92f : 1.055f * ogm_powrf(x, 1.0f / 2.4f) - 0.055f;
            u[k] = og_unorm8(x);
        }
        const int bgra = format >= 4;
        const uint32_t p = (bgra ? u[2] : u[0]) | (u[1] << 8) | ((bgra ? u[0] : u[2]) << 16) | (u[3] << 24);
        memcpy((uint8_t *)dst + 4 * i, &p, 4);
    }
    return format == 1 ? 16 : 4;
}

/* ================================================================== */
/* DepthFirst stereo side-by-side              */
/* Sources/Renderer/DepthFirstRenderer/DepthFirstRenderer.swift:469-831 */
/* and DepthFirstShaders.metal (kernels cited per function).           */
/* ================================================================== */

/* float_to_sortable_uint (DepthFirstShaders.metal:33-37). */
static inline uint32_t df_sortable(float v) {
    uint32_t b = ogm_fbits(v);
    return b ^ ((b & 0x80000000u) ? 0xFFFFFFFFu : 0x80000000u);
}

void og_sincos_theta(float th, float *s, float *c) { ogm_sincos_theta(th, s, c); }
uint32_t og_float_to_sortable(float v) { return df_sortable(v); }

/* conicFromThetaSigmas (GaussianShared.h:490-510) for an fp32 angle (sincos: numeric contract). */
static inline conic3 conic_from_theta(float th, float sigma1, float sigma2) {
    float s, c;
    ogm_sincos_theta(th, &s, &c);
    float sig1 = fmaxf(sigma1, 1e-4f);
    float sig2 = fmaxf(sigma2, 1e-4f);
    float iv1 = 1.0f / (sig1 * sig1);
    float iv2 = 1.0f / (sig2 * sig2);
    float cc = c * c, ss = s * s, cs = c * s;
    conic3 o;
    o.A = cc * iv1 + ss * iv2;
    o.B = cs * (iv1 - iv2);
    o.C = ss * iv1 + cc * iv2;
    return o;
}

/* EyeProjectionResult (DepthFirstShaders.metal:236-247). */
typedef struct {
    int visible;
    float sx, sy, theta, s1, s2, det_cov, depth;
    int32_t tb[4];
} df_eye;

/* projectToEye (DepthFirstShaders.metal:249-339). */
static df_eye df_project_eye(f3 pos, f3 scale, f4 quat, const float *scene, float scene_scale,
                             const float *view, const float *proj, float W, float Hh, float nearp,
                             float farp, int tiles_x, int tiles_y) {
    df_eye e;
    memset(&e, 0, sizeof(e));
    e.tb[0] = 0; e.tb[1] = -1; e.tb[2] = 0; e.tb[3] = -1;
    f4 p4 = {pos.x, pos.y, pos.z, 1.0f};
    f4 wp = mat4_mul_vec(scene, p4);
    f4 vp = mat4_mul_vec(view, wp);
    f4 clip = mat4_mul_vec(proj, vp);
    e.depth = clip.w;
    if (!(clip.w > nearp)) return e;  /* isInFrontOfCameraClipW */
    if (e.depth > farp) return e;     /* cullByFarPlane (GaussianShared.h:732-734) */
    float ndcx = clip.x / clip.w, ndcy = clip.y / clip.w;
    /* ndcToScreen (GaussianShared.h:150-155): no pixel-centre shift */
    e.sx = (ndcx + 1.0f) * 0.5f * W;
    e.sy = (ndcy + 1.0f) * 0.5f * Hh;
    f3 ss = {scale.x * scene_scale, scale.y * scene_scale, scale.z * scene_scale};
    m3 cov3d = build_cov3d(ss, quat);
    f3 vp3 = {vp.x, vp.y, vp.z};
    m2 cov2d = project_cov2d(&cov3d, vp3, view, proj, W, Hh);
    cov2d = stabilize_cov2d(cov2d, W, Hh);
    float th, s1, s2;
    if (!cov_to_theta_sigmas(cov2d, &th, &s1, &s2)) return e;
    e.theta = th; e.s1 = s1; e.s2 = s2;
    float a = cov2d.c[0].x, b = 0.5f * (cov2d.c[0].y + cov2d.c[1].x), d = cov2d.c[1].y;
    e.det_cov = fmaxf(a * d - b * b, 0.0f);
    float radius = 3.0f * fmaxf(s1, s2);
    if (radius < 0.5f) return e; /* cullByRadius */
    f2 obb = obb_extents(cov2d, 3.0f);
    if (e.sx + obb.x < 0.0f || e.sx - obb.x > W || e.sy + obb.y < 0.0f || e.sy - obb.y > Hh) return e;
    /* computeTileBounds (GaussianShared.h:791-828), 16x16 tiles (DepthFirstRenderer.swift:8-9) */
    float xmin = clampf(e.sx - obb.x, 0.0f, W - 1.0f), xmax = clampf(e.sx + obb.x, 0.0f, W - 1.0f);
    float ymin = clampf(e.sy - obb.y, 0.0f, Hh - 1.0f), ymax = clampf(e.sy + obb.y, 0.0f, Hh - 1.0f);
    int minTX = (int)floorf(xmin / 16.0f), maxTX = (int)ceilf(xmax / 16.0f) - 1;
    int minTY = (int)floorf(ymin / 16.0f), maxTY = (int)ceilf(ymax / 16.0f) - 1;
    if (minTX < 0) minTX = 0;
    if (minTY < 0) minTY = 0;
    if (maxTX > tiles_x - 1) maxTX = tiles_x - 1;
    if (maxTY > tiles_y - 1) maxTY = tiles_y - 1;
    e.tb[0] = minTX; e.tb[1] = maxTX; e.tb[2] = minTY; e.tb[3] = maxTY;
    e.visible = 1;
    return e;
}

typedef struct {
    const og_config *cfg;
    const void *gaussians, *harmonics;
    uint32_t shk;
    const og_camera *left, *right;
    const float *scene;
    float scene_scale;
    float W, H;
    int tiles_x, tiles_y;
    og_df_frame *f;
} df_ctx;

static void df_mark_culled(og_df_frame *f, uint32_t gid) {
    int32_t *b = f->bounds + 4 * (size_t)gid;
    b[0] = 0; b[1] = -1; b[2] = 0; b[3] = -1;
    f->touched[gid] = 0;
    f->depth_keys[gid] = 0xFFFFFFFFu;
}

/* depthFirstStereoProjectCullKernel (DepthFirstShaders.metal:341-499). */
static void df_project_range(void *vctx, uint32_t lo, uint32_t hi) {
    df_ctx *X = (df_ctx *)vctx;
    og_df_frame *f = X->f;
    const int half_in = X->cfg->precision == 1;
    const float nearp = X->left->near_plane, farp = X->left->far_plane; /* StereoCameraUniforms: left eye's */
    const float alphaThreshold = 0.005f, totalInkThreshold = 2.0f;
    const uint16_t hneg = og_f2h(-1e10f);
    for (uint32_t gid = lo; gid < hi; ++gid) {
        f3 pos, scale;
        float opacity;
        f4 rot;
        if (half_in) {
            const og_world16 *g = (const og_world16 *)X->gaussians + gid;
            pos.x = g->px; pos.y = g->py; pos.z = g->pz;
            scale.x = H(g->sx); scale.y = H(g->sy); scale.z = H(g->sz);
            opacity = H(g->opacity);
            rot.x = H(g->rx); rot.y = H(g->ry); rot.z = H(g->rz); rot.w = H(g->rw);
        } else {
            const og_world32 *g = (const og_world32 *)X->gaussians + gid;
            pos.x = g->px; pos.y = g->py; pos.z = g->pz;
            scale.x = g->sx; scale.y = g->sy; scale.z = g->sz;
            opacity = g->opacity;
            rot.x = g->rot[0]; rot.y = g->rot[1]; rot.z = g->rot[2]; rot.w = g->rot[3];
        }
        if (fmaxf(scale.x, fmaxf(scale.y, scale.z)) < 0.0005f) { df_mark_culled(f, gid); continue; }
        if (opacity < alphaThreshold) { df_mark_culled(f, gid); continue; }
        f4 quat = normalize_quat(rot);
        df_eye L = df_project_eye(pos, scale, quat, X->scene, X->scene_scale, X->left->view, X->left->proj,
                                  X->W, X->H, nearp, farp, X->tiles_x, X->tiles_y);
        df_eye R = df_project_eye(pos, scale, quat, X->scene, X->scene_scale, X->right->view, X->right->proj,
                                  X->W, X->H, nearp, farp, X->tiles_x, X->tiles_y);
        if (!L.visible && !R.visible) { df_mark_culled(f, gid); continue; }
        float checkDepth = L.visible ? L.depth : R.depth;
        if (L.visible && R.visible) checkDepth = (L.depth + R.depth) * 0.5f;
        float detCov = L.visible ? L.det_cov : R.det_cov;
        if (L.visible && R.visible) detCov = fmaxf(L.det_cov, R.det_cov);
        { /* cullByTotalInk (GaussianShared.h:739-751) + computeDepthFactor (:275-278) */
            float ink = opacity * 6.283185f * sqrtf(fmaxf(detCov, 1e-12f));
            float adjFar = farp * 0.02f;
            float s = saturatef((adjFar - checkDepth) / (adjFar - nearp));
            float depthFactor = 1.0f - s * s;
            if (ink < depthFactor * totalInkThreshold) { df_mark_culled(f, gid); continue; }
        }
        f3 mid = {(X->left->position[0] + X->right->position[0]) * 0.5f,
                  (X->left->position[1] + X->right->position[1]) * 0.5f,
                  (X->left->position[2] + X->right->position[2]) * 0.5f};
        f3 col = compute_sh_color(X->harmonics, half_in, gid, pos, mid, X->shk);
        col.x = fmaxf(col.x + 0.5f, 0.0f);
        col.y = fmaxf(col.y + 0.5f, 0.0f);
        col.z = fmaxf(col.z + 0.5f, 0.0f);
        if (X->cfg->color_space == 1) {
            col.x = srgb_to_linear(col.x);
            col.y = srgb_to_linear(col.y);
            col.z = srgb_to_linear(col.z);
        }
        int32_t ub[4];
        if (L.visible && R.visible) {
            ub[0] = L.tb[0] < R.tb[0] ? L.tb[0] : R.tb[0];
            ub[1] = L.tb[1] > R.tb[1] ? L.tb[1] : R.tb[1];
            ub[2] = L.tb[2] < R.tb[2] ? L.tb[2] : R.tb[2];
            ub[3] = L.tb[3] > R.tb[3] ? L.tb[3] : R.tb[3];
        } else {
            const int32_t *t = L.visible ? L.tb : R.tb;
            ub[0] = t[0]; ub[1] = t[1]; ub[2] = t[2]; ub[3] = t[3];
        }
        int ux = ub[1] - ub[0] + 1, uy = ub[3] - ub[2] + 1;
        if (ux < 0) ux = 0;
        if (uy < 0) uy = 0;
        uint32_t touched = (uint32_t)(ux * uy);
        if (touched == 0) { df_mark_culled(f, gid); continue; }
        og_stereo_render_data rd;
        memset(&rd, 0, sizeof(rd));
        const df_eye *eyes[2] = {&L, &R};
        uint16_t *dst[2] = {&rd.leftMeanX, &rd.rightMeanX};
        for (int e = 0; e < 2; ++e) {
            uint16_t *o = dst[e]; /* meanX, meanY, cxx, cyy, cxy2, depth */
            if (eyes[e]->visible) {
                conic3 k = conic_from_theta(eyes[e]->theta, eyes[e]->s1, eyes[e]->s2);
                o[0] = og_f2h(eyes[e]->sx);
                o[1] = og_f2h(eyes[e]->sy);
                o[2] = og_f2h(k.A);
                o[3] = og_f2h(k.C);
                o[4] = og_f2h(2.0f * k.B);
                o[5] = og_f2h(eyes[e]->depth);
            } else {
                o[0] = hneg; o[1] = hneg; o[2] = 0; o[3] = 0; o[4] = 0; o[5] = 0;
            }
        }
        rd.colorR = (uint8_t)clampf(col.x * 255.0f, 0.0f, 255.0f);
        rd.colorG = (uint8_t)clampf(col.y * 255.0f, 0.0f, 255.0f);
        rd.colorB = (uint8_t)clampf(col.z * 255.0f, 0.0f, 255.0f);
        rd.opacity = (uint8_t)clampf(opacity * 255.0f, 0.0f, 255.0f);
        rd.centerDepth = og_f2h(checkDepth);
        f->render_data[gid] = rd;
        int32_t *b = f->bounds + 4 * (size_t)gid;
        b[0] = ub[0]; b[1] = ub[1]; b[2] = ub[2]; b[3] = ub[3];
        f->touched[gid] = touched;
        f->depth_keys[gid] = df_sortable(checkDepth);
    }
}

/* depthFirstStereoRender (DepthFirstShaders.metal:1825-1982) for one active tile. */
typedef struct { og_df_frame *f; uint32_t *active; } df_blend_ctx;

static void df_blend_tiles(void *vctx, uint32_t lo, uint32_t hi) {
    df_blend_ctx *B = (df_blend_ctx *)vctx;
    og_df_frame *f = B->f;
    const uint16_t ONE = 0x3C00u;
    const uint16_t thr = og_f2h(1.0f / 255.0f); /* half(1.0h/255.0h) */
    const uint16_t c099 = og_d2h(0.99);
    const float r2max = 9.0f;                   /* half(9.0f) */
    const uint32_t W = f->width, Hh = f->height;
    for (uint32_t ai = lo; ai < hi; ++ai) {
        uint32_t tile = B->active[ai];
        uint32_t start = f->headers[2 * tile], count = f->headers[2 * tile + 1];
        uint32_t tileX = tile % f->tiles_x, tileY = tile / f->tiles_x;
        for (uint32_t ly = 0; ly < 8; ++ly)
            for (uint32_t lx = 0; lx < 8; ++lx) {
                uint32_t baseX = tileX * 16 + lx * 2, baseY = tileY * 16 + ly * 2;
                /* pixel q = (q & 1, q >> 1): 00, 10, 01, 11 */
                uint16_t px[4], py[4];
                for (int q = 0; q < 4; ++q) {
                    px[q] = og_f2h((float)(baseX + (uint32_t)(q & 1)));
                    py[q] = og_f2h((float)(baseY + (uint32_t)(q >> 1)));
                }
                uint16_t T[2][4], C[2][4][3];
                for (int e = 0; e < 2; ++e)
                    for (int q = 0; q < 4; ++q) { T[e][q] = ONE; C[e][q][0] = C[e][q][1] = C[e][q][2] = 0; }
                for (uint32_t i = 0; i < count; ++i) {
                    uint16_t mt[2];
                    for (int e = 0; e < 2; ++e) mt[e] = hmax(hmax(T[e][0], T[e][1]), hmax(T[e][2], T[e][3]));
                    if (H(hmax(mt[0], mt[1])) < H(thr)) break;
                    int32_t gi = f->inst_gids[start + i];
                    if (gi < 0) continue;
                    const og_stereo_render_data *g = &f->render_data[gi];
                    uint16_t op = og_f2h(H(og_f2h((float)g->opacity)) / 255.0f);
                    uint16_t gc[3] = {og_f2h(H(og_f2h((float)g->colorR)) / 255.0f),
                                      og_f2h(H(og_f2h((float)g->colorG)) / 255.0f),
                                      og_f2h(H(og_f2h((float)g->colorB)) / 255.0f)};
                    for (int e = 0; e < 2; ++e) {
                        if (!(H(mt[e]) >= H(thr))) continue;
                        const uint16_t *ev = e == 0 ? &g->leftMeanX : &g->rightMeanX;
                        if (!(H(ev[0]) >= -60000.0f)) continue;
                        uint16_t p[4], a[4];
                        int all_out = 1;
                        for (int q = 0; q < 4; ++q) {
                            uint16_t dx = hsub(px[q], ev[0]), dy = hsub(py[q], ev[1]);
                            p[q] = hadd(hadd(hmul(hmul(dx, dx), ev[2]), hmul(hmul(dy, dy), ev[3])),
                                        hmul(hmul(dx, dy), ev[4]));
                            if (!(H(p[q]) > r2max)) all_out = 0;
                        }
                        int any = 0;
                        for (int q = 0; q < 4; ++q) {
                            a[q] = 0;
                            if (!all_out && !(H(p[q]) > r2max))
                                a[q] = hmin(hmul(op, g_exp_h[og_f2h(-0.5f * H(p[q]))]), c099);
                            if (H(a[q]) != 0.0f) any = 1;
                        }
                        if (!any) continue;
                        for (int q = 0; q < 4; ++q) {
                            uint16_t w = hmul(a[q], T[e][q]);
                            for (int ch = 0; ch < 3; ++ch) C[e][q][ch] = hfma(gc[ch], w, C[e][q][ch]);
                            T[e][q] = hmul(T[e][q], hsub(ONE, a[q]));
                        }
                    }
                }
                for (int e = 0; e < 2; ++e)
                    for (int q = 0; q < 4; ++q) {
                        uint32_t x = baseX + (uint32_t)(q & 1), y = baseY + (uint32_t)(q >> 1);
                        if (x >= W || y >= Hh) continue;
                        uint16_t *o = f->eye_color + 4 * ((size_t)e * W * Hh + (size_t)y * W + x);
                        o[0] = C[e][q][0]; o[1] = C[e][q][1]; o[2] = C[e][q][2];
                        o[3] = hsub(ONE, T[e][q]);
                    }
            }
    }
}

void og_df_frame_free(og_df_frame *f) {
    if (!f) return;
    free(f->render_data); free(f->bounds); free(f->touched); free(f->depth_keys);
    free(f->depth_order); free(f->inst_tiles); free(f->inst_gids); free(f->headers);
    free(f->eye_color); free(f->color);
    free(f);
}

/* DepthFirstRenderer.renderStereo(.sideBySide) -> renderStereoSideBySideRaster ->
 * encodeStereoPipeline (DepthFirstRenderer.swift:205-223, 469-512, 595-831). */
int og_df_render_stereo(const og_config *cfg, const void *gaussians, const void *harmonics,
                        uint32_t count, uint32_t shk, const og_camera *left, const og_camera *right,
                        const float *scene_transform, uint32_t width, uint32_t height, int nthreads,
                        og_df_frame **out) {
    ensure_init();
    *out = NULL;
    if (!cfg || !left || !right || (count > 0 && (!gaussians || !harmonics))) return OG_ERR_INVALID_ARGUMENT;
    if (cfg->max_gaussians > 30000000u) return OG_ERR_INVALID_GAUSSIAN_COUNT; /* DepthFirstRenderer.swift:51-56 */
    uint32_t maxG = cfg->max_gaussians ? cfg->max_gaussians : 1u;
    if (count > maxG) return OG_ERR_INVALID_GAUSSIAN_COUNT; /* encodeStereoPipeline guard :607 */
    uint32_t maxW = cfg->max_width ? cfg->max_width : 1u, maxH = cfg->max_height ? cfg->max_height : 1u;
    if (width == 0 || height == 0 || width > maxW || height > maxH) return OG_ERR_INVALID_DIMENSIONS;
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads < 1) nthreads = 1;
    static const float identity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const float *scene = scene_transform ? scene_transform : identity;

    og_df_frame *f = (og_df_frame *)calloc(1, sizeof(og_df_frame));
    if (!f) return OG_ERR_OUT_OF_MEMORY;
    f->count = count;
    f->width = width;
    f->height = height;
    /* buildBinningParams(gaussianCount:width:height:) (GlobalRenderer.swift:54-70), 16x16 tiles */
    f->tiles_x = (width + 15u) / 16u;
    f->tiles_y = (height + 15u) / 16u;
    f->tile_count = f->tiles_x * f->tiles_y;
    f->max_instances = 4u * maxG; /* DepthFirstResources.swift:399 */
    size_t n = count ? count : 1;
    f->render_data = (og_stereo_render_data *)calloc(n, sizeof(og_stereo_render_data));
    f->bounds = (int32_t *)calloc(n * 4, sizeof(int32_t));
    f->touched = (uint32_t *)calloc(n, sizeof(uint32_t));
    f->depth_keys = (uint32_t *)calloc(n, sizeof(uint32_t));
    f->depth_order = (int32_t *)calloc(n, sizeof(int32_t));
    f->headers = (uint32_t *)calloc((size_t)f->tile_count * 2, sizeof(uint32_t));
    f->eye_color = (uint16_t *)calloc((size_t)2 * width * height * 4, sizeof(uint16_t));
    f->color = (uint16_t *)calloc((size_t)2 * width * height * 4, sizeof(uint16_t));
    if (!f->render_data || !f->bounds || !f->touched || !f->depth_keys || !f->depth_order || !f->headers ||
        !f->eye_color || !f->color) {
        og_df_frame_free(f);
        return OG_ERR_OUT_OF_MEMORY;
    }
    df_ctx X;
    memset(&X, 0, sizeof(X));
    X.cfg = cfg; X.gaussians = gaussians; X.harmonics = harmonics; X.shk = shk;
    X.left = left; X.right = right; X.scene = scene;
    /* length(sceneTransform[0].xyz) (DepthFirstShaders.metal:293): sqrt(dot) */
    {
        float d = scene[0] * scene[0] + scene[1] * scene[1];
        d = d + scene[2] * scene[2];
        X.scene_scale = sqrtf(d);
    }
    X.W = (float)width; X.H = (float)height;
    X.tiles_x = (int)f->tiles_x; X.tiles_y = (int)f->tiles_y;
    X.f = f;
    double t0 = now_s();
    parallel_for(nthreads, count, df_project_range, &X);
    double t1 = now_s();
    /* visibilityScatterCompactKernel (DepthFirstShaders.metal:589-621): ascending gid */
    uint32_t V = 0;
    uint32_t *keys = (uint32_t *)malloc(sizeof(uint32_t) * n);
    if (!keys) { og_df_frame_free(f); return OG_ERR_OUT_OF_MEMORY; }
    for (uint32_t g = 0; g < count; ++g)
        if (f->touched[g] > 0) { keys[V] = f->depth_keys[g]; f->depth_order[V] = (int32_t)g; V++; }
    f->visible = V;
    /* DepthRadixSortEncoder .bits32: 4 stable 8-bit LSD passes (DepthRadixSortEncoder.swift:14-22) */
    og_radix_sort_pairs(keys, f->depth_order, V);
    free(keys);
    /* applyDepthOrderingKernel + prefix sum + createInstancesStereoKernel (:623-640, :790-826) */
    uint64_t total = 0;
    for (uint32_t i = 0; i < V; ++i) total += f->touched[f->depth_order[i]];
    f->overflow = total > f->max_instances ? 1u : 0u; /* prepareDepthFirstDispatchKernel (:2191-2194) */
    uint32_t tot = (uint32_t)(total > f->max_instances ? f->max_instances : total);
    f->total_instances = tot;
    size_t na = tot ? tot : 1;
    uint32_t *tiles = (uint32_t *)malloc(sizeof(uint32_t) * na);
    int32_t *gids = (int32_t *)malloc(sizeof(int32_t) * na);
    f->inst_tiles = (uint32_t *)calloc(na, sizeof(uint32_t));
    f->inst_gids = (int32_t *)calloc(na, sizeof(int32_t));
    uint32_t *cnt = (uint32_t *)calloc((size_t)f->tile_count + 1, sizeof(uint32_t));
    if (!tiles || !gids || !f->inst_tiles || !f->inst_gids || !cnt) {
        free(tiles); free(gids); free(cnt);
        og_df_frame_free(f);
        return OG_ERR_OUT_OF_MEMORY;
    }
    uint64_t off = 0;
    for (uint32_t i = 0; i < V; ++i) {
        int32_t g = f->depth_order[i];
        const int32_t *b = f->bounds + 4 * (size_t)g;
        for (int ty = b[2]; ty <= b[3]; ++ty)
            for (int tx = b[0]; tx <= b[1]; ++tx) {
                if (off < f->max_instances) {
                    tiles[off] = (uint32_t)(ty * (int)f->tiles_x + tx) & 0xFFFFu; /* ushort tile id */
                    gids[off] = g;
                }
                off++;
            }
    }
    /* TileSortEncoder: stable sort of the instances by tile id (a 16-bit LSD radix sort) */
    for (uint32_t i = 0; i < tot; ++i) cnt[tiles[i] + 1]++;
    for (uint32_t t = 0; t < f->tile_count; ++t) cnt[t + 1] += cnt[t];
    for (uint32_t i = 0; i < tot; ++i) {
        uint32_t p = cnt[tiles[i]]++;
        f->inst_tiles[p] = tiles[i];
        f->inst_gids[p] = gids[i];
    }
    free(tiles); free(gids); free(cnt);
    double t2 = now_s();
    /* extractTileRangesKernel (DepthFirstShaders.metal:1258-1313) */
    uint32_t *active = (uint32_t *)calloc(f->tile_count ? f->tile_count : 1, sizeof(uint32_t));
    if (!active) { og_df_frame_free(f); return OG_ERR_OUT_OF_MEMORY; }
    uint32_t nact = 0;
    for (uint32_t tile = 0; tile < f->tile_count; ++tile) {
        if (tot == 0) { f->headers[2 * tile] = 0; f->headers[2 * tile + 1] = 0; continue; }
        uint32_t l = 0, r = tot;
        while (l < r) { uint32_t m = (l + r) >> 1; if (f->inst_tiles[m] < tile) l = m + 1; else r = m; }
        uint32_t s = l;
        l = s; r = tot;
        while (l < r) { uint32_t m = (l + r) >> 1; if (f->inst_tiles[m] <= tile) l = m + 1; else r = m; }
        f->headers[2 * tile] = s;
        f->headers[2 * tile + 1] = l > s ? l - s : 0u;
        if (l > s) active[nact++] = tile;
    }
    f->active_tiles = nact;
    /* clearStereoRenderTextureKernel (:1813-1823): both slices (0,0,0,1) */
    for (size_t i = 0; i < (size_t)2 * width * height; ++i) {
        f->eye_color[4 * i] = 0; f->eye_color[4 * i + 1] = 0; f->eye_color[4 * i + 2] = 0;
        f->eye_color[4 * i + 3] = 0x3C00u;
    }
    df_blend_ctx B = {f, active};
    parallel_for_interleaved(nthreads, nact, df_blend_tiles, &B);
    free(active);
    /* DepthFirstStereoCopyEncoder (DepthFirstStereoCopyEncoder.swift:29-99): a full-screen
     * triangle per eye viewport (left at x = 0, right at x = width, StereoConfiguration origin
     * DepthFirstRenderer.swift:480-485) sampling slice `eye` at uv = clamp(uv, 0, 1) with the
     * vertex uv (0,0) at NDC (-1,-1) (DepthFirstShaders.metal:1990-2018).  At pixel centres of a
     * 1:1 viewport the linear filter lands on texel centres (weight 1), and the bottom NDC edge
     * maps to texture row 0: target row y of eye e is slice e's row height-1-y. */
    for (uint32_t e = 0; e < 2; ++e)
        for (uint32_t y = 0; y < height; ++y)
            memcpy(f->color + 4 * ((size_t)y * 2 * width + (size_t)e * width),
                   f->eye_color + 4 * ((size_t)e * width * height + (size_t)(height - 1 - y) * width),
                   (size_t)width * 8);
    double t3 = now_s();
    f->t_project = t1 - t0;
    f->t_sort = t2 - t1;
    f->t_blend = t3 - t2;
    *out = f;
    return OG_OK;
}
