// gsm_blend_exact.h -- the exact re-walk of one blend unit, shared by k_blend_px and k_blend_pw.
//
// The reference skips a list entry for a 4x2 pixel group when the group's eight alphas are all zero
// (GlobalShaders.metal:1133, `if (all(alphaRow0 == 0.0h) && all(alphaRow1 == 0.0h)) continue;`).  The
// fast walks blend such an entry with alpha 0 instead: T * (1 - 0) = T, and c * (0 * T) = 0 leaves
// every colour channel bit for bit (the colours are u8 / 255, finite) -- and the depth channel too,
// unless the record's fp16 depth is inf or NaN (a view depth past 65504 overflows fp16, and the Global
// path has no far-plane cull): inf * 0 = NaN where the reference keeps the depth.  The fast walks test
// every 64-entry batch they stage for such a record (one ballot per batch); a unit that meets one is
// walked again here, after its fast walk, with the group test, and all of its pixels are written again.
// Same fp16 operations in the same order as the fast walks (quadratic form, table word, alpha, group
// break, fused accumulation); entries at a time, records staged per 64-entry batch in the wave's LDS
// stage.  Slow, but only for units that hold such a record.
#pragma once
#include <hip/hip_runtime.h>

#include "gsm_types.h"

namespace gsm {
namespace blend_exact {

typedef _Float16 xh1;
typedef _Float16 xh2 __attribute__((ext_vector_type(2)));
typedef unsigned short xu16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ xh2 x_h2(uint32_t u) { return __builtin_bit_cast(xh2, u); }
__device__ __forceinline__ uint32_t x_u32(xh2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ xh2 x_lo(xh2 v) { return xh2{v.x, v.x}; }
__device__ __forceinline__ xh2 x_hi(xh2 v) { return xh2{v.y, v.y}; }
template <int CTRL>
__device__ __forceinline__ uint32_t x_dpp_or(uint32_t v) {
    return v | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t x_dpp_max(uint32_t v) {
    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
    return v > o ? v : o;
}

// a staged batch (one record word b | depth << 16 per lane) holds a record of inf / NaN fp16 depth
__device__ __forceinline__ bool batch_depth_nonfinite(uint32_t recB) {
    return __ballot(((recB >> 16) & 0x7C00u) == 0x7C00u) != 0ull;
}

// One unit at (ux, uy) walked exactly.  P = 2: a 16x16 half tile, lane = 2x2 pixels (k_blend_px's
// half-tile layout: a 4x2 group on lanes 2g, 2g + 1); P = 1: a 16x8 quadrant, lane = one pixel pair
// (a group on a lane quad).  stA / stB: the wave's 64-entry LDS record stage.  write(px, py, A, R, G,
// B, D) stores the pixel pair (px, py), (px + 1, py).
template <int P, typename Write>
__device__ __forceinline__ void walk_unit_exact(const uint32_t* __restrict__ lst, uint32_t count, const BlendRecord* __restrict__ rec,
                                const uint16_t* tbl, uint4* stA, uint32_t* stB, uint32_t ux, uint32_t uy,
                                uint32_t thrBits, Write&& write) {
    static_assert(P == 1 || P == 2, "quadrant or half-tile units");
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t offX, offY0, offY1;
    if (P == 1) {
        const uint32_t grp = lane >> 2;
        offX = (grp & 3u) * 4u + (lane & 1u) * 2u;
        offY0 = offY1 = (grp >> 2) * 2u + ((lane >> 1) & 1u);
    } else {
        const uint32_t grp = lane >> 1;
        offX = (grp & 3u) * 4u + (lane & 1u) * 2u;
        offY0 = (grp >> 2) * 2u;
        offY1 = offY0 + 1u;
    }
    const xh2 ONE = {(xh1)1.0f, (xh1)1.0f}, ZERO = {(xh1)0.0f, (xh1)0.0f};
    const xh1 c099 = (xh1)0.99;
    const xh2 C099 = {c099, c099};
    const xh2 X = {(xh1)(float)(ux + offX), (xh1)(float)(ux + offX + 1u)};
    const xh2 Yv = {(xh1)(float)(uy + offY0), (xh1)(float)(uy + offY1)};
    xh2 T[P], R[P], G[P], B[P], D[P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
        T[q] = ONE;
        R[q] = G[q] = B[q] = D[q] = ZERO;
    }
    bool alive = true;
    const uint32_t last = count - 1u;
    const uint4 pad = make_uint4(x_u32(xh2{(xh1)(float)ux, (xh1)(float)uy}), 0u, 0u, 0u);
    for (uint32_t b0 = 0; b0 < count; b0 += 64u) {
        const uint32_t gi = lst[min(b0 + lane, last)];
        uint4 a = *(const uint4*)(rec + gi);
        uint32_t b = rec[gi].b;
        if (b0 + lane >= count) {
            a = pad;
            b = 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (earlier reads of the stage are done)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        stA[lane] = a;
        stB[lane] = b;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t n = min(64u, count - b0);
        for (uint32_t j = 0; j < n; ++j) {
            // group break before the entry (GlobalShaders.metal:1086-1088): max T of the 4x2 group
            xu16x2 tm = __builtin_bit_cast(xu16x2, T[0]);
#pragma unroll
            for (int q = 1; q < P; ++q) tm = __builtin_elementwise_max(tm, __builtin_bit_cast(xu16x2, T[q]));
            const uint32_t tb = __builtin_bit_cast(uint32_t, tm);
            uint32_t gm = max(tb & 0xFFFFu, tb >> 16);
            gm = x_dpp_max<0xB1>(gm);
            if (P == 1) gm = x_dpp_max<0x4E>(gm);
            alive = alive && !(gm < thrBits);
            if (__ballot(alive) == 0ull) break;
            const uint4 ra = stA[j];
            const uint32_t bd = stB[j];
            // p = ((dx*dx)*cxx + (dy*dy)*cyy) + (dx*dy)*cxy2 (GlobalShaders.metal:1115-1122)
            const xh2 mean = x_h2(ra.x), cc = x_h2(ra.y), oc = x_h2(ra.z);
            const xh2 dyv = Yv - x_hi(mean);
            const xh2 dyy = (dyv * dyv) * x_hi(cc);
            const xh2 dx = X - x_lo(mean);
            xh2 pq[P];
            if constexpr (P == 2) {
                const xh2 dxx = (dx * dx) * x_lo(cc);
                pq[0] = (dxx + x_lo(dyy)) + (dx * x_lo(dyv)) * x_lo(oc);
                pq[1] = (dxx + x_hi(dyy)) + (dx * x_hi(dyv)) * x_lo(oc);
            } else {
                pq[0] = ((dx * dx) * x_lo(cc) + x_lo(dyy)) + (dx * x_lo(dyv)) * x_lo(oc);
            }
            xh2 ac[P], om[P];
            uint32_t nz = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const uint32_t pb = x_u32(pq[q]);
                const xh2 ek = x_h2((uint32_t)tbl[pb & 0xFFFFu] | ((uint32_t)tbl[pb >> 16] << 16));
                // a = min(opacity * exp(-0.5h * p), 0.99h) (GlobalShaders.metal:1124-1131)
                ac[q] = __builtin_elementwise_min(x_hi(oc) * ek, C099);
                om[q] = ONE - ac[q];
                nz |= x_u32(ac[q]) & 0x7FFF7FFFu;
            }
            nz = x_dpp_or<0xB1>(nz);
            if (P == 1) nz = x_dpp_or<0x4E>(nz);
            if (alive && nz != 0u) {  // the group's alphas are not all zero (GlobalShaders.metal:1133)
                const xh2 rgv = x_h2(ra.w), bdv = x_h2(bd);
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const xh2 w = ac[q] * T[q];  // (GlobalShaders.metal:1137-1149)
                    T[q] = T[q] * om[q];
                    R[q] = __builtin_elementwise_fma(x_lo(rgv), w, R[q]);
                    G[q] = __builtin_elementwise_fma(x_hi(rgv), w, G[q]);
                    B[q] = __builtin_elementwise_fma(x_lo(bdv), w, B[q]);
                    D[q] = __builtin_elementwise_fma(x_hi(bdv), w, D[q]);
                }
            }
        }
        if (__ballot(alive) == 0ull) break;
    }
    write(ux + offX, uy + offY0, ONE - T[0], R[0], G[0], B[0], D[0]);
    if (P == 2) write(ux + offX, uy + offY1, ONE - T[P - 1], R[P - 1], G[P - 1], B[P - 1], D[P - 1]);
}

}  // namespace blend_exact
}  // namespace gsm
