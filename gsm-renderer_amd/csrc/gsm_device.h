// gsm_device.h -- device helpers shared by the gfx950 kernels of the GlobalRenderer
// (gsm_kernels.hip) and the DepthFirst stereo path (gsm_depthfirst.hip): fp16 bit casts,
// column-major matrix products, the GaussianShared.h pieces and block/wave scans.
// Numeric contract: DESIGN.md (built with -ffp-contract=off, IEEE div/sqrt).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gsm_renderer.h"
#include "gsm_detmath.h"
#include "gsm_internal.h"
#include "gsm_types.h"

namespace gsm {

typedef _Float16 h1;
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float hbits_to_f(uint16_t b) { return (float)__builtin_bit_cast(h1, b); }
__device__ __forceinline__ uint16_t f_to_hbits(float f) { return __builtin_bit_cast(uint16_t, (h1)f); }

__device__ __forceinline__ float clampf(float v, float lo, float hi) {
    return __builtin_fminf(__builtin_fmaxf(v, lo), hi);
}

// ---------------------------------------------------------------------------
// Cheaper sequences with the numeric contract's results (r06).  Checked bit for bit
// against the compiler's correctly rounded sequences (-fhip-fp32-correctly-rounded-divide-sqrt) over EVERY
// 32-bit input on gfx950 (tools/exp/crmath_check.hip, profiles/r06_crmath_check.txt):
//  * sqrt_cr: v_sqrt_f32 and the IEEE sequence's two-neighbour residual test, without its tiny-input scaling
//    and its special-class select (9 instead of 15 VALU) -- the same bits as __builtin_sqrtf for every
//    x >= 4.6e-32 (the largest input that differs is 0x0b6e9372 = 4.59e-32), +0, -0, +inf and NaN;
//    callers pass x >= 1e-16 by construction (a max with a positive constant, or a sum of squares of a
//    term beyond 1e-8);
//  * rcp_cr: v_rcp_f32 and one fma Newton step (3 instead of 9 VALU and the denormal-mode switches) -- the
//    same bits as 1.0f / b for every b in [2^-126, 2^126] (b above 2^126: 1/b subnormal, differs).
__device__ __forceinline__ float sqrt_cr(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    const float r = rd <= 0.0f ? sd : s;
    return ru > 0.0f ? su : r;
}
__device__ __forceinline__ float rcp_cr(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
}

// ---------------------------------------------------------------------------
// Correctly rounded a[k] / b for K numerators over one divisor -- bit for bit the IEEE a[k] / b of the
// oracle -- at one division's cost: y = RN(1 / b), then per numerator q = RN(a y), r = RN(a - b q) (exact
// by the fma), q' = RN(q + r y): Markstein's correction, correctly rounded when y is the correctly
// rounded reciprocal, q is normal and r does not underflow (Muller et al., Handbook of Floating-Point
// Arithmetic, division via fma).  r = 0 keeps q (so a = -0 gives -0).  The fast path takes numerators
// that are zero or of magnitude in [2^-96, 2^96] (finite; below 2^-96 r could underflow) over divisors
// in [2^-29, 2^29], so every quotient lies in [2^-125, 2^125]: normal, no overflow (r05, ADVICE r04: the
// earlier [2^-100, 2^100] divisor range let quotients go subnormal or overflow).  A wave holding any
// other operand takes the divisions themselves.  Checked on random, signed-zero, fp16-valued and
// arbitrary-bit-pattern pairs against IEEE division (tools/exp/markstein_div.c, tests/test_markstein_div.py).
// b > 0 (norms).
template <int K>
__device__ __forceinline__ void div_many(float (&a)[K], float b) {
    bool slow = !(b >= 0x1p-29f && b <= 0x1p29f);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t x = __float_as_uint(a[k]) & 0x7FFFFFFFu;
        slow = slow || (x != 0u && x - (31u << 23) > (192u << 23));  // 0 < |a| < 2^-96, |a| > 2^96, inf, NaN
    }
    if (__ballot(slow) != 0ull) {  // (rare; wave-uniform)
#pragma unroll
        for (int k = 0; k < K; ++k) a[k] = a[k] / b;
        return;
    }
    const float y = rcp_cr(b);  // = 1.0f / b: b in [2^-29, 2^29] here
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float q = a[k] * y;
        const float r = __builtin_fmaf(-q, b, a[k]);
        a[k] = r == 0.0f ? q : __builtin_fmaf(r, y, q);
    }
}

// small column-major matrix helpers (simd / Metal layout)
// ---------------------------------------------------------------------------
struct M3 {
    float m[3][3];  // m[col][row]
};

__device__ __forceinline__ M3 m3_mul(const M3& A, const M3& B) {
    M3 R;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            float acc = A.m[0][r] * B.m[c][0];
            acc = acc + A.m[1][r] * B.m[c][1];
            acc = acc + A.m[2][r] * B.m[c][2];
            R.m[c][r] = acc;
        }
    return R;
}

// float4x4 * float4 (column-major): sum_j col_j * v_j left to right.
__device__ __forceinline__ void m4_mul_v(const float* M, const float v[4], float out[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = M[0 * 4 + i] * v[0];
        acc = acc + M[1 * 4 + i] * v[1];
        acc = acc + M[2 * 4 + i] * v[2];
        acc = acc + M[3 * 4 + i] * v[3];
        out[i] = acc;
    }
}

// ---------------------------------------------------------------------------
// GaussianShared.h pieces
// ---------------------------------------------------------------------------
struct Cov2 {
    float a, b, c, d;  // col0 = (a, b), col1 = (c, d)
};

// conicFromThetaSigmas (GaussianShared.h:490-510) for a quantised angle.
struct Conic {
    float A, B, C;
};
__device__ __forceinline__ Conic conic_from_quant(const float2* __restrict__ sincos, uint16_t thq,
                                                  float sigma1, float sigma2) {
    float2 sc = sincos[thq];
    float s = sc.x, c = sc.y;
    float sig1 = __builtin_fmaxf(sigma1, 1e-4f);
    float sig2 = __builtin_fmaxf(sigma2, 1e-4f);
    // sig^2 is in [1e-8, 65504^2] or +inf (an fp16 sigma >= 1e-4: inf when the fp32 sigma passed 65504 --
    // adversarial scales reach it, tests/adversarial.py): rcp_cr's exact range, and IEEE 1 / inf = +0
    const float q1 = sig1 * sig1, q2 = sig2 * sig2;
    float iv1 = q1 < __builtin_inff() ? rcp_cr(q1) : 0.0f;
    float iv2 = q2 < __builtin_inff() ? rcp_cr(q2) : 0.0f;
    float cc = c * c, ss = s * s, cs = c * s;
    Conic k;
    k.A = cc * iv1 + ss * iv2;
    k.B = cs * (iv1 - iv2);
    k.C = ss * iv1 + cc * iv2;
    return k;
}

// gaussianComputePower (GaussianShared.h:595-597; gsm_detmath.h).
__device__ __forceinline__ float compute_power(float opacity) { return det_compute_power(opacity); }

// gaussianSegmentIntersectEllipse .. intersectsTile (GaussianShared.h:599-653).
__device__ __forceinline__ bool seg_ellipse(float a, float b, float c, float d, float l, float r) {
    float delta = b * b - 4.0f * a * c;
    float t1 = (l - d) * (2.0f * a) + b;
    float t2 = (r - d) * (2.0f * a) + b;
    return delta >= 0.0f && (t1 <= 0.0f || t1 * t1 <= delta) && (t2 >= 0.0f || t2 * t2 <= delta);
}
__device__ __forceinline__ bool intersects_tile(int tx, int ty, float cx, float cy, const Conic& k,
                                                float w) {
    const int pminx = tx * (int)kTileWidth, pminy = ty * (int)kTileHeight;
    const int pmaxx = pminx + (int)kTileWidth - 1, pmaxy = pminy + (int)kTileHeight - 1;
    if (cx >= (float)pminx && cx <= (float)pmaxx && cy >= (float)pminy && cy <= (float)pmaxy)
        return true;
    float dx = (cx * 2.0f < (float)(pminx + pmaxx)) ? cx - (float)pminx : cx - (float)pmaxx;
    if (seg_ellipse(k.C, -2.0f * k.B * dx, k.A * dx * dx - w, cy, (float)pminy, (float)pmaxy))
        return true;
    float dy = (cy * 2.0f < (float)(pminy + pmaxy)) ? cy - (float)pminy : cy - (float)pmaxy;
    if (seg_ellipse(k.A, -2.0f * k.B * dy, k.C * dy * dy - w, cx, (float)pminx, (float)pmaxx))
        return true;
    return false;
}

constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f;
constexpr float SH_C2_1 = -1.0925484305920792f;
constexpr float SH_C2_2 = 0.31539156525252005f;
constexpr float SH_C2_3 = -1.0925484305920792f;
constexpr float SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f;
constexpr float SH_C3_1 = 2.890611442640554f;
constexpr float SH_C3_2 = -0.4570457994644658f;
constexpr float SH_C3_3 = 0.3731763325901154f;
constexpr float SH_C3_4 = -0.4570457994644658f;
constexpr float SH_C3_5 = 1.445305721320277f;
constexpr float SH_C3_6 = -0.5900435899266435f;

template <bool HALF>
__device__ __forceinline__ float load_harm(const void* __restrict__ h, size_t i) {
    if constexpr (HALF) {
        return hbits_to_f(((const uint16_t*)h)[i]);
    } else {
        return ((const float*)h)[i];
    }
}

// fp32(h) * b for the fp16 in the low / high half of w: one v_fma_mix_f32 (the fp16 operand widened
// exactly inside the instruction, fma(h, b, -0) = the correctly rounded product) instead of a
// v_cvt_f32_f16 and a v_mul_f32 -- the same bits as the contract's convert-then-multiply
__device__ __forceinline__ float mul_h_lo(uint32_t w, float b) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(b), "v"(-0.0f));
    return r;
}
__device__ __forceinline__ float mul_h_hi(uint32_t w, float b) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(b), "v"(-0.0f));
    return r;
}

// computeSHColor (GaussianShared.h:38-116) specialised by degree like the
// SH_DEGREE function constant (GlobalProjectCullEncoder.swift:19-45).
template <bool HALF, int DEG>
__device__ __forceinline__ void sh_color(const void* __restrict__ harm, uint32_t gid,
                                         const float pos[3], const float cam[3], uint32_t shk,
                                         float col[3]) {
    if (DEG == 0 || shk == 0) {
        const size_t base = (size_t)gid * 3u;
        col[0] = load_harm<HALF>(harm, base) * SH_C0;
        col[1] = load_harm<HALF>(harm, base + 1) * SH_C0;
        col[2] = load_harm<HALF>(harm, base + 2) * SH_C0;
        return;
    }
    constexpr int K = DEG == 1 ? 4 : (DEG == 2 ? 9 : 16);
    float d0 = cam[0] - pos[0], d1 = cam[1] - pos[1], d2 = cam[2] - pos[2];
    float dd = d0 * d0 + d1 * d1;
    dd = dd + d2 * d2;
    float n = __builtin_sqrtf(dd);
    float dn3[3] = {d0, d1, d2};
    div_many(dn3, n);  // d / n, each correctly rounded
    float x = dn3[0], y = dn3[1], z = dn3[2];
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, yz = y * z, xz = x * z;
    float b[16];
    b[0] = SH_C0;
    b[1] = (-SH_C1) * y;
    b[2] = SH_C1 * z;
    b[3] = (-SH_C1) * x;
    if constexpr (DEG >= 2) {
        b[4] = SH_C2_0 * xy;
        b[5] = SH_C2_1 * yz;
        b[6] = SH_C2_2 * ((2.0f * zz - xx) - yy);
        b[7] = SH_C2_3 * xz;
        b[8] = SH_C2_4 * (xx - yy);
    }
    if constexpr (DEG >= 3) {
        b[9] = (SH_C3_0 * y) * (3.0f * xx - yy);
        b[10] = (SH_C3_1 * xy) * z;
        b[11] = (SH_C3_2 * y) * ((4.0f * zz - xx) - yy);
        b[12] = (SH_C3_3 * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
        b[13] = (SH_C3_4 * x) * ((4.0f * zz - xx) - yy);
        b[14] = (SH_C3_5 * z) * (xx - yy);
        b[15] = (SH_C3_6 * x) * (xx - 3.0f * yy);
    }
    const size_t base = (size_t)gid * (size_t)K * 3u;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    if constexpr (HALF && DEG == 3) {
        // 96 B per gaussian, 16-B aligned: six dwordx4 loads.
        const uint4* p = (const uint4*)((const uint16_t*)harm + base);
        uint32_t hw[24];  // coefficient 2k in the low half of hw[k], 2k + 1 in the high half
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            uint4 v = p[q];
            hw[4 * q] = v.x;
            hw[4 * q + 1] = v.y;
            hw[4 * q + 2] = v.z;
            hw[4 * q + 3] = v.w;
        }
        auto mulc = [&](int c, float bb) { return (c & 1) ? mul_h_hi(hw[c >> 1], bb) : mul_h_lo(hw[c >> 1], bb); };
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            cr = cr + mulc(i, b[i]);
            cg = cg + mulc(16 + i, b[i]);
            cb = cb + mulc(32 + i, b[i]);
        }
    } else {  // (v_fma_mix here, on 2-byte loads: DepthFirst SH2 projection 60.3 -> 63.5 us, not kept)
#pragma unroll
        for (int i = 0; i < K; ++i) {
            cr = cr + load_harm<HALF>(harm, base + i) * b[i];
            cg = cg + load_harm<HALF>(harm, base + K + i) * b[i];
            cb = cb + load_harm<HALF>(harm, base + 2 * K + i) * b[i];
        }
    }
    col[0] = cr;
    col[1] = cg;
    col[2] = cb;
}

// srgbToLinearChannel (GaussianShared.h:118-121).
__device__ __forceinline__ float srgb_to_linear(float c) {
    c = clampf(c, 0.0f, 1.0f);
    return (c <= 0.04045f) ? (c / 12.92f) : det_powrf((c + 0.055f) / 1.055f, 2.4f);
}

__device__ __forceinline__ float fmod_pi(float t) {
    // fmod(t, pi_f) for |t| < 2 pi_f (atan2 range): exact by Sterbenz.
    float a = __builtin_fabsf(t);
    if (a >= kPiF) {
        float r = a - kPiF;
        return __builtin_copysignf(r, t);
    }
    return t;
}

// normalizeQuaternion (GaussianShared.h:289-295) applied twice -- by the projection kernels
// (GlobalShaders.metal:64, DepthFirstShaders.metal:393) and again inside buildCovariance3D
// (GaussianShared.h:308) -- then quaternionToMatrix (:297-305) and R S S^T R^T (:307-324).
__device__ __forceinline__ M3 build_cov3d(const float scale[3], const float rot[4]) {
    float q[4] = {rot[0], rot[1], rot[2], rot[3]};
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        float d = q[0] * q[0] + q[1] * q[1];
        d = d + q[2] * q[2];
        d = d + q[3] * q[3];
        float nrm = sqrt_cr(__builtin_fmaxf(d, 1e-8f));
        if (nrm < 1e-8f) {
            q[0] = 1.0f; q[1] = 0.0f; q[2] = 0.0f; q[3] = 0.0f;
        } else {
            div_many(q, nrm);  // q / nrm, each correctly rounded
        }
    }
    float x = q[0], y = q[1], z = q[2], r = q[3];
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
    M3 R;
    R.m[0][0] = 1.0f - 2.0f * (yy + zz); R.m[1][0] = 2.0f * (xy - r * z); R.m[2][0] = 2.0f * (xz + r * y);
    R.m[0][1] = 2.0f * (xy + r * z); R.m[1][1] = 1.0f - 2.0f * (xx + zz); R.m[2][1] = 2.0f * (yz - r * x);
    R.m[0][2] = 2.0f * (xz - r * y); R.m[1][2] = 2.0f * (yz + r * x); R.m[2][2] = 1.0f - 2.0f * (xx + yy);
    float RS[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) RS[c][rr] = R.m[c][rr] * scale[c];
    M3 C3;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr)
            C3.m[c][rr] = (RS[0][c] * RS[0][rr] + RS[1][c] * RS[1][rr]) + RS[2][c] * RS[2][rr];
    return C3;
}

// projectCovariance2D (GaussianShared.h:326-375) with its uniform terms (tan clamp limits and
// focal lengths from the projection matrix and viewport) evaluated once per frame on the host.
__device__ __forceinline__ Cov2 project_cov2d(const M3& C3, const float vp[3], const float* view, float limX,
                                              float limY, float focalX, float focalY) {
    M3 W;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) W.m[c][rr] = view[c * 4 + rr];
    float absZ = __builtin_fabsf(vp[2]);
    float signZ = (vp[2] >= 0.0f) ? 1.0f : -1.0f;
    float safeAbsZ = __builtin_fmaxf(absZ, 1e-4f);
    float invAbsZ = 1.0f / safeAbsZ;
    float invAbsZ2 = invAbsZ * invAbsZ;
    float xCl = clampf(vp[0] * invAbsZ, -limX, limX) * safeAbsZ;
    float yCl = clampf(vp[1] * invAbsZ, -limY, limY) * safeAbsZ;
    M3 J;
    J.m[0][0] = focalX * invAbsZ; J.m[0][1] = 0.0f; J.m[0][2] = 0.0f;
    J.m[1][0] = 0.0f; J.m[1][1] = focalY * invAbsZ; J.m[1][2] = 0.0f;
    J.m[2][0] = -focalX * xCl * signZ * invAbsZ2;
    J.m[2][1] = -focalY * yCl * signZ * invAbsZ2;
    J.m[2][2] = 0.0f;
    M3 T = m3_mul(J, W);
    M3 M1 = m3_mul(T, C3);
    M3 Tt;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) Tt.m[c][rr] = T.m[rr][c];
    M3 F = m3_mul(M1, Tt);
    Cov2 cov;
    cov.a = F.m[0][0] + 0.3f;
    cov.b = F.m[0][1];
    cov.c = F.m[1][0];
    cov.d = F.m[1][1] + 0.3f;
    return cov;
}

// stabilizeCovariance2D (GaussianShared.h:655-714); maxEig = ((max(W, H) * 2) / 3)^2 from the host.
__device__ __forceinline__ Cov2 stabilize_cov2d(Cov2 cov, float maxEig) {
    const float kMinVar = 1e-4f, kMinDet = 1e-8f;
    float a = cov.a, b = 0.5f * (cov.b + cov.c), d = cov.d;
    if (!__builtin_isfinite(a) || !__builtin_isfinite(b) || !__builtin_isfinite(d)) {
        cov.a = 1.0f; cov.b = 0.0f; cov.c = 0.0f; cov.d = 1.0f;
        return cov;
    }
    a = __builtin_fmaxf(a, kMinVar);
    d = __builtin_fmaxf(d, kMinVar);
    float det = a * d - b * b;
    if (!__builtin_isfinite(det) || det < kMinDet) {
        float bump = (kMinDet - det) + kMinVar;
        a = a + bump;
        d = d + bump;
        det = a * d - b * b;
    }
    float mid = 0.5f * (a + d);
    float sq = __builtin_sqrtf(__builtin_fmaxf(mid * mid - det, 0.0f));
    float l1 = mid + sq;
    float l2 = __builtin_fmaxf(mid - sq, kMinVar);
    float v1x, v1y;
    if (__builtin_fabsf(b) > 1e-8f) {
        float vx = b, vy = l1 - a;
        float dn = __builtin_fmaxf(sqrt_cr(vx * vx + vy * vy), 1e-8f);  // (|vx| > 1e-8: the sum >= 1e-16)
        float v2[2] = {vx, vy};
        div_many(v2, dn);
        v1x = v2[0];
        v1y = v2[1];
    } else if (a >= d) {
        v1x = 1.0f; v1y = 0.0f;
    } else {
        v1x = 0.0f; v1y = 1.0f;
    }
    float v2x = v1y, v2y = -v1x;
    l1 = __builtin_fminf(l1, maxEig);
    l2 = __builtin_fmaxf(l2, l1 * (1.0f / 65536.0f));  // l1 / 256^2: exact power of two
    cov.a = l1 * (v1x * v1x) + l2 * (v2x * v2x);
    cov.b = l1 * (v1x * v1y) + l2 * (v2x * v2y);
    cov.c = l1 * (v1y * v1x) + l2 * (v2y * v2x);
    cov.d = l1 * (v1y * v1y) + l2 * (v2y * v2y);
    return cov;
}

// covarianceToThetaSigmas (GaussianShared.h:446-488): theta in [0, pi), sigmas = sqrt(eigenvalues).
__device__ __forceinline__ bool theta_sigmas(const Cov2& cov, float* theta, float* s1, float* s2) {
    float a = cov.a, b = 0.5f * (cov.b + cov.c), d = cov.d;
    if (!(__builtin_isfinite(a) && __builtin_isfinite(b) && __builtin_isfinite(d))) return false;
    a = __builtin_fmaxf(a, 1e-8f);
    d = __builtin_fmaxf(d, 1e-8f);
    float det = a * d - b * b;
    if (!(__builtin_isfinite(det) && det > 0.0f)) return false;
    float mid = 0.5f * (a + d);
    float sq = __builtin_sqrtf(__builtin_fmaxf(mid * mid - det, 0.0f));
    float l1 = __builtin_fmaxf(mid + sq, 1e-8f);
    float l2 = __builtin_fmaxf(mid - sq, 1e-8f);
    float v1x, v1y;
    if (__builtin_fabsf(b) > 1e-8f) {
        float tx = b, ty = l1 - a;
        float nn = sqrt_cr(tx * tx + ty * ty);  // (|tx| > 1e-8: the sum >= 1e-16)
        float v2[2] = {tx, ty};
        div_many(v2, nn);
        v1x = v2[0];
        v1y = v2[1];
    } else if (a >= d) {
        v1x = 1.0f; v1y = 0.0f;
    } else {
        v1x = 0.0f; v1y = 1.0f;
    }
    float th = det_atan2f(v1y, v1x);
    th = fmod_pi(th);
    if (th < 0.0f) th = th + kPiF;
    if (th >= kPiF) th = th - kPiF;
    *theta = th;
    *s1 = sqrt_cr(l1);  // (l1, l2 >= 1e-8)
    *s2 = sqrt_cr(l2);
    return __builtin_isfinite(th) && __builtin_isfinite(*s1) && __builtin_isfinite(*s2);
}

// computeOBBExtents (GaussianShared.h:402-427) at k = 3 sigma.
__device__ __forceinline__ void obb_extents(const Cov2& cov, float* ex, float* ey) {
    float a = cov.a, b = cov.b, d = cov.d;
    float det = a * d - b * b;
    float mid = 0.5f * (a + d);
    float sq = sqrt_cr(__builtin_fmaxf(mid * mid - det, 1e-6f));
    float l1 = mid + sq;
    float l2 = __builtin_fmaxf(mid - sq, 1e-6f);
    float e1 = 3.0f * sqrt_cr(__builtin_fmaxf(l1, 1e-6f));
    float e2 = 3.0f * sqrt_cr(__builtin_fmaxf(l2, 1e-6f));
    float v1x, v1y;
    if (__builtin_fabsf(b) > 1e-6f) {
        float vx = b, vy = l1 - a;
        float dn = __builtin_fmaxf(sqrt_cr(vx * vx + vy * vy), 1e-6f);  // (|vx| > 1e-6: the sum >= 1e-12)
        float v2[2] = {vx, vy};
        div_many(v2, dn);
        v1x = v2[0];
        v1y = v2[1];
    } else if (a >= d) {
        v1x = 1.0f; v1y = 0.0f;
    } else {
        v1x = 0.0f; v1y = 1.0f;
    }
    *ex = __builtin_fabsf(v1x) * e1 + __builtin_fabsf(v1y) * e2;
    *ey = __builtin_fabsf(v1y) * e1 + __builtin_fabsf(v1x) * e2;
}

// Tile-level zero test of the blends' per-pixel fp16 quadratic form (DepthFirst skip flags, Global
// unit lists).  The blends evaluate, per pixel, p = fl(fl(fl(fl(dx*dx)*cxx) + fl(fl(dy*dy)*cyy)) +
// fl(fl(dx*dy)*cxy2)) with dx = fl(px - mx).  With Q the same form in real arithmetic on the same fp16
// inputs, a = cxx dx^2, b = cyy dy^2 and rho = |cxy2| / (2 sqrt(cxx cyy)): every product and sum above
// rounds once with relative error <= u = 2^-11 while nothing overflows, so
// p >= (1 - u) (Q - 9.02 u (a + b)), and |c| <= rho (a + b), Q >= (1 - rho)(a + b) give
// p >= (1 - u) Q (1 - 9.02 u / (1 - rho)).  quad_exceeds() is true only when that bound exceeds the
// threshold for the minimum of Q over the pixel rectangle (continuous, so it bounds every pixel), with
// rho <= 15/16, |dx|, |dy| <= 200 and a + b <= 16000 over the rectangle (no fp16 overflow, no NaN),
// the rectangle widened by the fp16 rounding of its pixel coordinates (fp16_coord_margin: exact below
// 2048) and finite positive cxx, cyy.  Divisions and square roots
// use the hardware approximations (v_rcp_f32, v_rsq_f32, ~1 ulp): they move the edge minimiser t by
// ~1e-7 relative (Q rises by at most cyy * (2e-5)^2 there) and rho by ~1e-6 (the factor by ~1.3e-6),
// inside the 1e-3 absolute and 1e-5 relative slack; fp32 evaluation of the bounded quantities adds
// < 1e-6 relative.
struct QuadBound {
    float mx, my, cxx, cyy, cxy, factor, hx, hy;  // hx = 1 / (2 cxx), hy = 1 / (2 cyy)
    int mode;  // 0: test per rectangle, 1: always true (the caller's mean test fails), 2: never
};
// meanW, ccW: fp16 pairs {mx, my}, {cxx, cyy}; cxyW: fp16 cxy2 in the low half
__device__ __forceinline__ QuadBound quad_bound_setup(uint32_t meanW, uint32_t ccW, uint32_t cxyW,
                                                      bool meanTest) {
    QuadBound e;
    e.mx = hbits_to_f((uint16_t)(meanW & 0xFFFFu));
    e.my = hbits_to_f((uint16_t)(meanW >> 16));
    e.cxx = hbits_to_f((uint16_t)(ccW & 0xFFFFu));
    e.cyy = hbits_to_f((uint16_t)(ccW >> 16));
    e.cxy = hbits_to_f((uint16_t)(cxyW & 0xFFFFu));
    e.factor = 0.0f;
    e.hx = e.hy = 0.0f;
    e.mode = 2;
    if (meanTest && !(e.mx >= -60000.0f)) {  // DepthFirst: the blend's mean test skips the eye anyway
        e.mode = 1;
        return e;
    }
    if (!(e.cxx > 0.0f && e.cyy > 0.0f && e.cxx < 65504.0f && e.cyy < 65504.0f && __builtin_fabsf(e.cxy) < 65504.0f &&
          __builtin_fabsf(e.mx) < 65504.0f && __builtin_fabsf(e.my) < 65504.0f))
        return e;
    const float rho = 0.5f * __builtin_fabsf(e.cxy) * __builtin_amdgcn_rsqf(e.cxx * e.cyy);
    if (!(rho <= 15.0f / 16.0f)) return e;
    const float u = 1.0f / 2048.0f;
    e.factor = (1.0f - u) * (1.0f - 10.0f * u * __builtin_amdgcn_rcpf(1.0f - rho)) * (1.0f - 1e-5f);
    e.hx = __builtin_amdgcn_rcpf(2.0f * e.cxx);
    e.hy = __builtin_amdgcn_rcpf(2.0f * e.cyy);
    e.mode = 0;
    return e;
}
// fp16 pixel coordinates: integers below 2048 are exact; in [2048, 4096) the blends' fp16(x) moves
// a coordinate by at most 1, in [4096, 8192) by at most 2 -- the rectangle grows by that margin
__device__ __forceinline__ int fp16_coord_margin(int maxCoord) {
    return maxCoord < 2048 ? 0 : (maxCoord < 4096 ? 1 : (maxCoord < 8192 ? 2 : -1));
}
// every pixel (x, y) with x0 <= x <= x0 + wm1, y0 <= y <= y0 + hm1 has p > thresh
__device__ __forceinline__ bool quad_exceeds(const QuadBound& e, int x0, int y0, int wm1, int hm1, float thresh) {
    if (e.mode != 0) return e.mode == 1;
    const int mxm = fp16_coord_margin(x0 + wm1), mym = fp16_coord_margin(y0 + hm1);
    if (mxm < 0 || mym < 0) return false;
    x0 -= mxm;
    wm1 += 2 * mxm;
    y0 -= mym;
    hm1 += 2 * mym;
    const float dx0 = (float)x0 - e.mx, dx1 = dx0 + (float)wm1;
    const float dy0 = (float)y0 - e.my, dy1 = dy0 + (float)hm1;
    if (!(__builtin_fabsf(dx0) <= 200.0f && __builtin_fabsf(dx1) <= 200.0f && __builtin_fabsf(dy0) <= 200.0f &&
          __builtin_fabsf(dy1) <= 200.0f))
        return false;
    if (dx0 <= 0.0f && dx1 >= 0.0f && dy0 <= 0.0f && dy1 >= 0.0f) return false;  // the mean is inside: Q min = 0
    const float ax = __builtin_fmaxf(dx0 * dx0, dx1 * dx1), ay = __builtin_fmaxf(dy0 * dy0, dy1 * dy1);
    if (!(e.cxx * ax + e.cyy * ay <= 16000.0f)) return false;
    // min of Q over the rectangle: on its boundary (Q is convex with its minimum at the mean, outside)
    auto q = [&](float dx, float dy) { return e.cxx * dx * dx + e.cyy * dy * dy + e.cxy * dx * dy; };
    auto along_y = [&](float X) {  // edge dx = X: minimise over dy in [dy0, dy1]
        const float t = __builtin_fminf(__builtin_fmaxf(-e.cxy * X * e.hy, dy0), dy1);
        return q(X, t);
    };
    auto along_x = [&](float Y) {
        const float t = __builtin_fminf(__builtin_fmaxf(-e.cxy * Y * e.hx, dx0), dx1);
        return q(t, Y);
    };
    const float qmin = __builtin_fminf(__builtin_fminf(along_y(dx0), along_y(dx1)),
                                       __builtin_fminf(along_x(dy0), along_x(dy1)));
    return qmin * e.factor > thresh + 1e-3f;
}

// Column-band zero test for the Global blend's half-tile lists (k_scatter skip flags).  With the
// notation above, Q(dx, dy) >= dx^2 det / cyy for every dy (det = cxx cyy - (cxy2 / 2)^2, the minimum
// over dy), so every pixel whose real dx satisfies |dx| > ex, ex = sqrt(L' cyy / det), has Q > L' and,
// by the same rounding bound as quad_exceeds, p >= factor Q > factor L' = thresh + 1e-3.  A band of
// pixel columns [x0, x1] has fp16 coordinates in [x0 - m, x1 + m] (fp16_coord_margin), so when that
// interval lies beyond ex on one side of the mean every pixel of the band, in any row, has p > thresh.
// The rounding bound's preconditions are checked over the band and the tile's rows (|dx|, |dy| <= 200,
// cxx dx^2 + cyy dy^2 <= 16000, rho <= 15/16, finite positive cxx, cyy); ex carries a 1e-5 relative and
// 1e-4 absolute margin for the fp32 evaluation (hardware rsq/rcp, ~1 ulp).  k_scatter checks the
// preconditions once over a gaussian's whole tile rect (band_rect_ok) and then needs two compares per
// band (half_skip_flags): cheap enough for every (gaussian, tile) of the frame.
struct BandSkip {
    float mx, my, cxx, cyy, ex;
    bool valid;
};
__device__ __forceinline__ BandSkip band_skip_setup(uint32_t meanW, uint32_t ccW, uint32_t cxyW, float thresh) {
    BandSkip b;
    b.mx = hbits_to_f((uint16_t)(meanW & 0xFFFFu));
    b.my = hbits_to_f((uint16_t)(meanW >> 16));
    b.cxx = hbits_to_f((uint16_t)(ccW & 0xFFFFu));
    b.cyy = hbits_to_f((uint16_t)(ccW >> 16));
    const float cxy = hbits_to_f((uint16_t)(cxyW & 0xFFFFu));
    b.ex = 0.0f;
    b.valid = false;
    if (!(b.cxx > 0.0f && b.cyy > 0.0f && b.cxx < 65504.0f && b.cyy < 65504.0f && __builtin_fabsf(cxy) < 65504.0f &&
          __builtin_fabsf(b.mx) < 65504.0f && __builtin_fabsf(b.my) < 65504.0f))
        return b;
    const float rho = 0.5f * __builtin_fabsf(cxy) * __builtin_amdgcn_rsqf(b.cxx * b.cyy);
    if (!(rho <= 15.0f / 16.0f)) return b;
    const float u = 1.0f / 2048.0f;
    const float factor = (1.0f - u) * (1.0f - 10.0f * u * __builtin_amdgcn_rcpf(1.0f - rho)) * (1.0f - 1e-5f);
    const float L = (thresh + 1e-3f) * __builtin_amdgcn_rcpf(factor) * (1.0f + 1e-5f);
    const float det = b.cxx * b.cyy - 0.25f * cxy * cxy;
    if (!(det > 0.0f)) return b;
    // det >= (1 - rho^2) cxx cyy > 0.12 cxx cyy: no cancellation worth more than the relative margin
    // hardware square root (v_sqrt_f32, ~1 ulp; r06): inside the 1e-5 relative margin like rsq / rcp above
    // (the argument is >= L / cxx > 5e-4: never subnormal); the flags only drop entries, the image is the same
    b.ex = __builtin_amdgcn_sqrtf(L * b.cyy * __builtin_amdgcn_rcpf(det)) * (1.0f + 1e-5f) + 1e-4f;
    b.valid = __builtin_isfinite(b.ex);
    return b;
}
// Colour target store of one rgba16f pixel in config.color_format (include/gsm_renderer.h
// conversion rules; oracle og_convert_color): rgba32f widens, the 8-bit formats clamp to
// [0, 1], sRGB-encode rgb and round to nearest.
__device__ __forceinline__ float srgb_encode_px(float c) {
    return c <= 0.0031308f ? c * 12.92f : 1.055f * det_powrf(c, 1.0f / 2.4f) - 0.055f;
}
__device__ __forceinline__ void store_color_px(int fmt, char* dst, uint32_t rg, uint32_t ba) {
    if (fmt == GSM_COLOR_FORMAT_RGBA16F) {  // 4-byte stores: any 4-byte aligned pitch
        ((uint32_t*)dst)[0] = rg;
        ((uint32_t*)dst)[1] = ba;
        return;
    }
    float c[4] = {hbits_to_f((uint16_t)(rg & 0xFFFFu)), hbits_to_f((uint16_t)(rg >> 16)),
                  hbits_to_f((uint16_t)(ba & 0xFFFFu)), hbits_to_f((uint16_t)(ba >> 16))};
    if (fmt == GSM_COLOR_FORMAT_RGBA32F) {
        float* o = (float*)dst;
        o[0] = c[0]; o[1] = c[1]; o[2] = c[2]; o[3] = c[3];
        return;
    }
    const bool srgb = fmt == GSM_COLOR_FORMAT_RGBA8_UNORM_SRGB || fmt == GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB;
    uint32_t u8[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float x = clampf(c[k], 0.0f, 1.0f);
        if (srgb && k < 3) x = srgb_encode_px(x);
        u8[k] = (uint32_t)__builtin_rintf(x * 255.0f);
    }
    const bool bgra = fmt >= GSM_COLOR_FORMAT_BGRA8_UNORM;
    *(uint32_t*)dst = (bgra ? u8[2] : u8[0]) | (u8[1] << 8) | ((bgra ? u8[0] : u8[2]) << 16) | (u8[3] << 24);
}

template <int BLOCK>
__device__ __forceinline__ uint32_t block_reduce_add(uint32_t v, uint32_t* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_scan_incl(v);  // (DPP; lane 63 holds the wave's sum)
    if (lane == 63) lds[wave] = v;
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) s += lds[w];
    return s;
}

// Inclusive scan inside a wave of 64 lanes.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) { return wave_scan_incl(v); }
// Exclusive scan over a block; returns the block total in *total.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        uint32_t s = lds[w];
        if (w < wave) off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

}  // namespace gsm
