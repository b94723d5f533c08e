// gsm_blend_pw.hip -- the GlobalRenderer's blend with two half-tile units per wave (r05).
//
// Same per-pixel operations and order as k_blend_px (globalRender, GlobalShaders.metal:1030-1187; the
// numeric contract), so bit-identical output; what changes is which lanes hold which
// pixels.  A wave takes a PAIR of half-tile units (16x16 pixels, 32 groups of the reference's 4x2
// pixels each) -- consecutive positions of the longest-first schedule, so of similar walk -- and walks
// both half-tile lists in lockstep (entry e of unit 0 on lanes 0-31, entry e of unit 1 on lanes 32-63),
// in three lane layouts that follow the live groups:
//   W8: one group per lane (8 pixels, 4 packed pairs): 64 groups, ~78 VALU per entry -- 9.75 per pixel
//       against 10.65 for 4 pixels per lane; the group break needs no cross-lane step;
//   W4: a group on 2 lanes (4 pixels per lane, k_blend_px's half-tile layout), entered once at most
//       32 groups of the pair live;
//   W2: a group on 4 lanes (2 pixels per lane, k_blend_px's compacted layout), entered at <= 16.
// The tails of the two units (their last live groups) share one wave instead of holding one wave
// each -- the per-unit alive curves put this at -14 % wave-instructions at config 2 and -18 % at
// config 3 (tools/blend_pair_model.py).  The schedule's longest units (the top-priority
// first unit of waves 0-3 of each workgroup) still run alone, in W4 from their first entry, so the
// longest job is no longer than before.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "../../include/gsm_renderer.h"
#include "gsm_blend_exact.h"
#include "gsm_detmath.h"
#include "gsm_internal.h"
#include "gsm_types.h"

namespace gsm {
namespace {

typedef _Float16 h1;
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 splat_lo(h2 v) { return h2{v.x, v.x}; }
__device__ __forceinline__ h2 splat_hi(h2 v) { return h2{v.y, v.y}; }
// `color += gColor * w`: one fused multiply-add per channel
__device__ __forceinline__ h2 acc_fma(h2 acc, h2 c, h2 w) { return __builtin_elementwise_fma(c, w, acc); }
__device__ __forceinline__ float hbits2f(uint16_t b) { return (float)__builtin_bit_cast(h1, b); }
__device__ __forceinline__ float srgb_enc(float c) {
    return c <= 0.0031308f ? c * 12.92f : 1.055f * det_powrf(c, 1.0f / 2.4f) - 0.055f;
}
__device__ __forceinline__ void pw_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t pw_bperm(uint32_t srcLane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(srcLane * 4u), (int)v);
}
__device__ __forceinline__ h2 pw_bperm(uint32_t srcLane, h2 v) { return as_h2(pw_bperm(srcLane, as_u32(v))); }

// the table index of a packed pair of quadratic forms: its fp16 bits (the far-field clamp / dead-column
// variants: tools/exp/rejected_variants.patch)
__device__ __forceinline__ uint32_t pw_tbl_bits(h2 p) {
    return as_u32(p);
}

struct PwTarget {
    uint8_t* color;
    size_t colorPitch;
    uint8_t* depth;
    size_t depthPitch;
    uint32_t W, H;
    int flags;  // bit 0: 16-B colour / 4-B depth stores allowed; bits 4-7: gsm_color_format
};

// one pixel pair (px, py), (px + 1, py) in the target's format (GlobalShaders.metal:1152-1186;
// conversion rules in include/gsm_renderer.h) -- k_blend_px's write_pair without the multi-GPU paths
__device__ __forceinline__ void pw_write_pair(const PwTarget& t, uint32_t px, uint32_t py, h2 Av, h2 Rq, h2 Gq, h2 Bq,
                                              h2 Dq) {
    if (py >= t.H) return;
    uint8_t* crow = t.color + (size_t)py * t.colorPitch;
    const uint32_t ur = as_u32(Rq), ug = as_u32(Gq), ub = as_u32(Bq), ua = as_u32(Av), ud = as_u32(Dq);
    const int fmt = (t.flags >> 4) & 15;
    if (fmt == GSM_COLOR_FORMAT_RGBA16F) {
        const uint32_t p0a = (ur & 0xFFFFu) | (ug << 16);
        const uint32_t p0b = (ub & 0xFFFFu) | (ua << 16);
        const uint32_t p1a = (ur >> 16) | (ug & 0xFFFF0000u);
        const uint32_t p1b = (ub >> 16) | (ua & 0xFFFF0000u);
        if ((t.flags & 1) && px + 1 < t.W) {
            *(uint4*)(crow + (size_t)px * 8) = make_uint4(p0a, p0b, p1a, p1b);
        } else {
            if (px < t.W) {
                *(uint32_t*)(crow + (size_t)px * 8) = p0a;
                *(uint32_t*)(crow + (size_t)px * 8 + 4) = p0b;
            }
            if (px + 1 < t.W) {
                *(uint32_t*)(crow + (size_t)(px + 1) * 8) = p1a;
                *(uint32_t*)(crow + (size_t)(px + 1) * 8 + 4) = p1b;
            }
        }
    } else {
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            if (px + i >= t.W) break;
            const uint32_t sh = 16u * i;
            float c[4] = {hbits2f((uint16_t)(ur >> sh)), hbits2f((uint16_t)(ug >> sh)), hbits2f((uint16_t)(ub >> sh)),
                          hbits2f((uint16_t)(ua >> sh))};
            if (fmt == GSM_COLOR_FORMAT_RGBA32F) {
                uint8_t* o = crow + (size_t)(px + i) * 16;
                if (t.flags & 1) {
                    *(uint4*)o = make_uint4(__float_as_uint(c[0]), __float_as_uint(c[1]), __float_as_uint(c[2]),
                                            __float_as_uint(c[3]));
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) ((uint32_t*)o)[k] = __float_as_uint(c[k]);
                }
                continue;
            }
            const bool srgb = fmt == GSM_COLOR_FORMAT_RGBA8_UNORM_SRGB || fmt == GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB;
            uint32_t u8[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float x = __builtin_fminf(__builtin_fmaxf(c[k], 0.0f), 1.0f);
                if (srgb && k < 3) x = srgb_enc(x);
                u8[k] = (uint32_t)__builtin_rintf(x * 255.0f);
            }
            const bool bgra = fmt >= GSM_COLOR_FORMAT_BGRA8_UNORM;
            *(uint32_t*)(crow + (size_t)(px + i) * 4) =
                (bgra ? u8[2] : u8[0]) | (u8[1] << 8) | ((bgra ? u8[0] : u8[2]) << 16) | (u8[3] << 24);
        }
    }
    if (t.depth) {
        uint8_t* drow = t.depth + (size_t)py * t.depthPitch;
        if ((t.flags & 1) && px + 1 < t.W) {
            *(uint32_t*)(drow + (size_t)px * 2) = ud;
        } else {
            if (px < t.W) *(uint16_t*)(drow + (size_t)px * 2) = (uint16_t)(ud & 0xFFFFu);
            if (px + 1 < t.W) *(uint16_t*)(drow + (size_t)(px + 1) * 2) = (uint16_t)(ud >> 16);
        }
    }
}

}  // namespace

template <int NT>
__global__ __launch_bounds__(NT) void k_blend_pw(
    const uint32_t* __restrict__ tileStart, const BlendRecord* __restrict__ rec,
    const uint16_t* __restrict__ expTable, uint32_t* __restrict__ queue, uint32_t numTiles, uint32_t tilesX,
    PwTarget tg, const uint32_t* __restrict__ order, uint16_t* __restrict__ unitCost,
    unsigned long long* __restrict__ trace, const uint32_t* __restrict__ half0, const uint32_t* __restrict__ half1,
    const uint32_t* __restrict__ halfCount, uint32_t tileCount, uint32_t* __restrict__ costMax, uint32_t rowBegin,
    uint32_t rowStride, int flags) {
    constexpr uint32_t NW = NT / 64;
    constexpr uint32_t NTOP = 4;  // one top-priority single unit per SIMD (the schedule's longest)
    static_assert(NW > NTOP, "pairs need waves beyond the top-priority ones");
    __shared__ __attribute__((aligned(16))) uint16_t tbl[65536];
    __shared__ uint32_t cscr[NW][32];                                // layout changes: the live groups
    __shared__ __attribute__((aligned(16))) uint4 lrecA[NW][64];   // staged records: unit k at 32 k (pairs)
    __shared__ uint32_t lrecB[NW][64];
    GSM_EXP_TABLE_TO_LDS(NT, expTable, tbl);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const bool agePrio = (flags & 2) != 0, split = (flags & 4) != 0;
    const h2 ONE = {(h1)1.0f, (h1)1.0f};
    const h2 ZERO = {(h1)0.0f, (h1)0.0f};
    const uint32_t thrBits = (uint32_t)__builtin_bit_cast(uint16_t, (h1)(1.0f / 255.0f));
    const h1 c099 = (h1)0.99;
    const h2 C099 = {c099, c099};
    const uint32_t numUnits = numTiles * 2u;
    uint32_t* const cs = cscr[wv];
    uint4* const LA = lrecA[wv];
    uint32_t* const LB = lrecB[wv];

    // Jobs (order = the longest-first permutation of the units): job J < NS is the unit at
    // position J alone, job J >= NS the pair at positions NS + 2 (J - NS) and + 1, where NS (written by
    // the schedule, unit_order_block) counts the units whose last walk is too long to share a wave.  The
    // first job of every wave is static -- with the schedule on, waves 0-3 of each workgroup (one per SIMD)
    // take jobs 0 .. 4 gridDim.x - 1 at top priority -- then jobs come from the striped queue (claimed
    // after a job ends).
    const uint32_t gridWaves = gridDim.x * NW;
    uint32_t NS = order ? min(__builtin_amdgcn_readfirstlane(costMax[kCostMaxSlots]), numUnits) : 0u;
    const uint32_t PE = numUnits;
    const uint32_t NPJ = (PE - NS + 1u) / 2u;
    uint32_t job = !split ? blockIdx.x * NW + wv
                          : (wv < NTOP ? blockIdx.x * NTOP + wv : gridDim.x * NTOP + blockIdx.x * (NW - NTOP) + (wv - NTOP));
    bool topPrio = split && wv < NTOP;
    auto jobPos = [&](uint32_t J, bool& single) {
        if (J < NS) {
            single = true;
            return J;
        }
        if (J < NS + NPJ) {
            const uint32_t p = NS + 2u * (J - NS);
            single = p + 1u >= PE;  // (an odd pair range ends with one unit)
            return p;
        }
        single = true;
        return PE + (J - NS - NPJ);
    };
    bool single;
    uint32_t pos = jobPos(job, single);
    const uint32_t stripes = (gridDim.x % kQueueStripes) == 0 ? kQueueStripes : 1u;
    const uint32_t stripe = blockIdx.x % stripes;
    uint32_t* const myQueue = queue + stripe * kQueueStride;
    uint32_t waveMax = 0;

    while (pos < numUnits) {
        const bool pair = !single && pos + 1u < PE;
        // the two units (scalars, not arrays: a lane-dependent pick from an array would go to scratch)
        uint32_t Uu0 = 0, Uu1 = 0, UX0 = 0, UX1 = 0, UY0 = 0, UY1 = 0, CNT0 = 0, CNT1 = 0, FULL0 = 0, FULL1 = 0;
        const uint32_t *LST0 = half0, *LST1 = half0;
        auto unitOf = [&](uint32_t k, uint32_t& uo, uint32_t& uxo, uint32_t& uyo, uint32_t& cnto, uint32_t& fullo,
                          const uint32_t*& lsto) {
            uint32_t u = order ? __builtin_amdgcn_readfirstlane(order[pos + k]) : pos + k;
            if (u >= numUnits) u = pos + k;  // a schedule is a permutation of [0, numUnits); never trust it further
            const uint32_t tile = u >> 1, part = u & 1u;
            const uint32_t tileX = tile % tilesX, tileY = rowBegin + (tile / tilesX) * rowStride;
            uo = u;
            uxo = tileX * kTileWidth + part * 16u;
            uyo = tileY * kTileHeight;
            const uint32_t start = __builtin_amdgcn_readfirstlane(tileStart[tile]);
            fullo = __builtin_amdgcn_readfirstlane(tileStart[tile + 1]) - start;
            cnto = __builtin_amdgcn_readfirstlane(halfCount[part * tileCount + tile]);
            lsto = (part ? half1 : half0) + start;
        };
        unitOf(0u, Uu0, UX0, UY0, CNT0, FULL0, LST0);
        if (pair) unitOf(1u, Uu1, UX1, UY1, CNT1, FULL1, LST1);
        unsigned long long tStart = 0;
        if (trace) tStart = __builtin_amdgcn_s_memrealtime();
        const uint32_t maxCnt = max(CNT0, CNT1);
        uint32_t walk0 = 0u, walk1 = 0u;
        bool done0 = CNT0 == 0u, done1 = !pair || CNT1 == 0u;

        // ---- lane state: up to 4 pixel pairs; coordinates of the lane's first pair (px, py)
        h2 T[4], R[4], G[4], B[4], D[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            T[q] = ONE;
            R[q] = G[q] = B[q] = D[q] = ZERO;
        }
        uint32_t ku, px, py;
        bool valid = true;
        int layout;
        if (pair) {  // W8: lane = 32 ku + group, group g = (gx, gy) of the unit's 4 x 8 groups
            ku = lane >> 5;
            const uint32_t g = lane & 31u;
            px = (ku ? UX1 : UX0) + (g & 3u) * 4u;
            py = (ku ? UY1 : UY0) + (g >> 2) * 2u;
            layout = 8;
        } else {  // W4: group lane >> 1, columns 2 (lane & 1) .. + 1 (k_blend_px's half-tile layout)
            ku = 0;
            const uint32_t g = lane >> 1;
            px = UX0 + (g & 3u) * 4u + (lane & 1u) * 2u;
            py = UY0 + (g >> 2) * 2u;
            layout = 4;
        }
        bool alive = (ku ? CNT1 : CNT0) > 0u;
        // the job met a record of inf / NaN fp16 depth: its units are walked again exactly at its end
        // (gsm_blend_exact.h; one ballot per staged batch)
        bool exactD = false;

        if (maxCnt > 0u) {
            // ---- record batches: BS entries per unit and batch (32 for pairs: lanes 0-31 unit 0, 32-63
            // unit 1; 64 for a single unit), staged in LDS and read back per lane; the next batch's records
            // in registers and the index of the one after (unpredicated clamped loads issued a batch ahead
            // of use -- a batch is >= 32 entries of ~40-80 VALU each, far longer than a miss)
            const uint32_t BS = pair ? 32u : 64u;
            const uint32_t lu = pair ? (lane >> 5) : 0u, lo = pair ? (lane & 31u) : lane;
            const uint32_t cntL = lu ? CNT1 : CNT0;
            // an empty list reads half0[0] (always allocated; its value is masked) -- never a word past a list
            const uint32_t* const lstL = cntL ? (lu ? LST1 : LST0) : half0;
            const uint32_t lastL = cntL ? cntL - 1u : 0u;
            const uint4 padL = make_uint4(as_u32(h2{(h1)(float)(lu ? UX1 : UX0), (h1)(float)(lu ? UY1 : UY0)}), 0u,
                                          0u, 0u);
            auto gidx = [&](uint32_t i) {  // (unpredicated: a predicated load would wait in the loop)
                const uint32_t v = lstL[min(i, lastL)];
                return cntL ? v : 0u;
            };
            uint32_t b0 = 0;  // first entry of the batch staged in LDS
            uint4 A1;
            uint32_t B1, I2;
            {
                const uint32_t g0 = gidx(lo), g1 = gidx(BS + lo);
                uint4 A0 = *(const uint4*)(rec + g0);
                uint32_t B0 = rec[g0].b;
                A1 = *(const uint4*)(rec + g1);
                B1 = rec[g1].b;
                I2 = gidx(2u * BS + lo);
                if (lo >= cntL) {
                    A0.x = padL.x;
                    A0.y = A0.z = A0.w = 0u;
                    B0 = 0u;
                }
                LA[lane] = A0;
                LB[lane] = B0;
                pw_wave_sync();
                exactD = blend_exact::batch_depth_nonfinite(B0) || blend_exact::batch_depth_nonfinite(B1);
            }
            // the batch at b0 + BS goes into LDS (neutral records past the lane's list); the registers
            // move one batch on
            auto restage = [&]() {
                const bool in = b0 + BS + lo < cntL;
                LA[lane] = make_uint4(in ? A1.x : padL.x, in ? A1.y : 0u, in ? A1.z : 0u, in ? A1.w : 0u);
                LB[lane] = in ? B1 : 0u;
                pw_wave_sync();
                exactD = exactD || blend_exact::batch_depth_nonfinite(in ? B1 : 0u);
                A1 = *(const uint4*)(rec + I2);
                B1 = rec[I2].b;
                I2 = gidx(b0 + 3u * BS + lo);
                b0 += BS;
            };
            uint32_t e = 0;  // next entry of both lists (lockstep)
            // slot of entry b0 + i of the lane's unit: 32 ku + i (pairs) or i (single)
            auto laneSlot = [&]() { return pair ? ku * 32u : 0u; };

            // ---- one walk in layout NP pixel pairs per lane (4: W8, 2: W4, 1: W2), from entry e (a
            // multiple of 16) to the checkpoint that ends it; returns 0 = done, 1 = change layout
            auto walk = [&](auto npTag) -> int {
                constexpr int NP = decltype(npTag)::value;
                constexpr uint32_t U = 4u / NP;  // entries per pipeline group
                constexpr uint32_t NG = 16u / U; // groups per 16-entry stretch (one checkpoint)
                h2 X0, X1, Yv;
                if (NP == 4) {
                    X0 = h2{(h1)(float)px, (h1)(float)(px + 1u)};
                    X1 = h2{(h1)(float)(px + 2u), (h1)(float)(px + 3u)};
                    Yv = h2{(h1)(float)py, (h1)(float)(py + 1u)};
                } else if (NP == 2) {
                    X0 = X1 = h2{(h1)(float)px, (h1)(float)(px + 1u)};
                    Yv = h2{(h1)(float)py, (h1)(float)(py + 1u)};
                } else {
                    X0 = X1 = h2{(h1)(float)px, (h1)(float)(px + 1u)};
                    Yv = h2{(h1)(float)py, (h1)(float)py};
                }
                // p = ((dx*dx)*cxx + (dy*dy)*cyy) + (dx*dy)*cxy2 (GlobalShaders.metal:1115-1122), the dx
                // terms once per column pair, the dy terms once per row pair; pair q = 2 row + column
                auto quadform = [&](uint32_t r0, uint32_t r1, uint32_t r2, h2 (&pq)[NP]) {
                    const h2 mean = as_h2(r0), cc = as_h2(r1), oc = as_h2(r2);
                    const h2 dyv = Yv - splat_hi(mean);
                    const h2 dyy = (dyv * dyv) * splat_hi(cc);
                    const h2 dx0 = X0 - splat_lo(mean);
                    const h2 dxx0 = (dx0 * dx0) * splat_lo(cc);
                    if constexpr (NP == 4) {
                        const h2 dx1 = X1 - splat_lo(mean);
                        const h2 dxx1 = (dx1 * dx1) * splat_lo(cc);
                        pq[0] = (dxx0 + splat_lo(dyy)) + (dx0 * splat_lo(dyv)) * splat_lo(oc);
                        pq[1] = (dxx1 + splat_lo(dyy)) + (dx1 * splat_lo(dyv)) * splat_lo(oc);
                        pq[2] = (dxx0 + splat_hi(dyy)) + (dx0 * splat_hi(dyv)) * splat_lo(oc);
                        pq[3] = (dxx1 + splat_hi(dyy)) + (dx1 * splat_hi(dyv)) * splat_lo(oc);
                    } else if constexpr (NP == 2) {
                        pq[0] = (dxx0 + splat_lo(dyy)) + (dx0 * splat_lo(dyv)) * splat_lo(oc);
                        pq[1] = (dxx0 + splat_hi(dyy)) + (dx0 * splat_hi(dyv)) * splat_lo(oc);
                    } else {
                        pq[0] = (dxx0 + splat_lo(dyy)) + (dx0 * splat_lo(dyv)) * splat_lo(oc);
                    }
                };
                h2 ac[U][NP], om[U][NP];
                uint32_t rgc[U], bdc[U], rgn[U], bdn[U], opn[U];
                u16x2 en[U][NP];
                // prime the group at e (the batch in LDS holds it: e - b0 < BS)
                if (e - b0 == BS) restage();
                uint32_t hb = laneSlot() + (e - b0);  // slot of entry e
#pragma unroll
                for (uint32_t k = 0; k < U; ++k) {
                    const uint4 ra = LA[hb + k];
                    h2 pq[NP];
                    quadform(ra.x, ra.y, ra.z, pq);
                    rgc[k] = ra.w;
                    bdc[k] = LB[hb + k];
#pragma unroll
                    for (int q = 0; q < NP; ++q) {
                        const uint32_t pb = pw_tbl_bits(pq[q]);
                        const h2 ek = as_h2((uint32_t)tbl[pb & 0xFFFFu] | ((uint32_t)tbl[pb >> 16] << 16));
                        // a = min(opacity * exp(-0.5h * p), 0.99h) (GlobalShaders.metal:1124-1131)
                        ac[k][q] = __builtin_elementwise_min(splat_hi(as_h2(ra.z)) * ek, C099);
                        om[k][q] = ONE - ac[k][q];
                    }
                }
                for (;;) {
                    // one checkpoint interval: entries e .. e + 15 (hb = slot of e)
#pragma unroll
                    for (uint32_t gi = 0; gi < NG; ++gi) {
                        // stage 1: the next group's records and table words go in flight
                        {
                            uint32_t nb = hb + (gi + 1u) * U;
                            if (gi + 1u == NG) {  // the next group opens the next stretch
                                if (e + 16u - b0 == BS) {  // ... and the next batch
                                    restage();
                                    nb = laneSlot();
                                }
                            }
#pragma unroll
                            for (uint32_t k = 0; k < U; ++k) {
                                const uint4 ra = LA[nb + k];
                                h2 pq[NP];
                                opn[k] = ra.z;
                                quadform(ra.x, ra.y, ra.z, pq);
                                rgn[k] = ra.w;
                                bdn[k] = LB[nb + k];
#pragma unroll
                                for (int q = 0; q < NP; ++q) {
                                    const uint32_t pb = pw_tbl_bits(pq[q]);
                                    en[k][q].x = tbl[pb & 0xFFFFu];
                                    en[k][q].y = tbl[pb >> 16];
                                }
                            }
                        }
                        // stage 2: blend the current group
#pragma unroll
                        for (uint32_t k = 0; k < U; ++k) {
                            // group break (GlobalShaders.metal:1086-1088): max T of the 4x2 group (T >= 0: the
                            // u16 bit patterns order like the values)
                            u16x2 tm = __builtin_bit_cast(u16x2, T[0]);
#pragma unroll
                            for (int q = 1; q < NP; ++q) tm = __builtin_elementwise_max(tm, __builtin_bit_cast(u16x2, T[q]));
                            const uint32_t tb = __builtin_bit_cast(uint32_t, tm);
                            uint32_t gm = max(tb & 0xFFFFu, tb >> 16);
                            if constexpr (NP == 2) {
                                const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)gm, 0xB1, 0xF, 0xF, false);
                                gm = max(gm, o);
                            } else if constexpr (NP == 1) {
                                const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)gm, 0xB1, 0xF, 0xF, false);
                                gm = max(gm, a);
                                const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)gm, 0x4E, 0xF, 0xF, false);
                                gm = max(gm, b);
                            }
                            alive = alive && !(gm < thrBits);
                            const h2 rgv = as_h2(rgc[k]), bdv = as_h2(bdc[k]);
                            if (alive) {  // dead lanes keep T and C (under an EXEC mask)
#pragma unroll
                                for (int q = 0; q < NP; ++q) {
                                    const h2 w = ac[k][q] * T[q];  // (GlobalShaders.metal:1137-1149)
                                    T[q] = T[q] * om[k][q];
                                    R[q] = acc_fma(R[q], splat_lo(rgv), w);
                                    G[q] = acc_fma(G[q], splat_hi(rgv), w);
                                    B[q] = acc_fma(B[q], splat_lo(bdv), w);
                                    D[q] = acc_fma(D[q], splat_hi(bdv), w);
                                }
                            }
                        }
                        if (gi + 1u == NG) {
                            // checkpoint after entry e + 15: a unit whose list ended is final (later entries of
                            // its lanes would be neutral records); per unit, its walk ends here when none of its
                            // groups lives (the next frame's schedule key, as k_blend_px's nproc)
                            e += 16u;
                            alive = alive && e < (ku ? CNT1 : CNT0);
                            if (!done0 && __ballot(alive && ku == 0u) == 0ull) {
                                done0 = true;
                                walk0 = e;
                            }
                            if (!done1 && __ballot(alive && ku == 1u) == 0ull) {
                                done1 = true;
                                walk1 = e;
                            }
                            const uint64_t am = __ballot(alive);
                            if (am == 0ull) return 0;
                            if constexpr (NP == 4) {
                                if (__popcll(am) <= 32) return 1;
                            } else if constexpr (NP == 2) {
                                if (__popcll(am & 0x5555555555555555ull) <= 16) return 1;
                            }
                            // priority rises with the walk's age (k_blend_px)
                            if (topPrio) {
                                if (e == 16u) __builtin_amdgcn_s_setprio(3);
                            } else if (agePrio) {
                                if (e == 16u) __builtin_amdgcn_s_setprio(1);
                                else if (e == 128u) __builtin_amdgcn_s_setprio(2);
                                else if (e == 320u && !split) __builtin_amdgcn_s_setprio(3);
                            }
                            hb = (e - b0 == 0u) ? laneSlot() : hb + 16u;
                        }
                        // stage 3: the next group's alphas
#pragma unroll
                        for (uint32_t k = 0; k < U; ++k) {
#pragma unroll
                            for (int q = 0; q < NP; ++q) {
                                const h2 ek = __builtin_bit_cast(h2, en[k][q]);
                                ac[k][q] = __builtin_elementwise_min(splat_hi(as_h2(opn[k])) * ek, C099);
                                om[k][q] = ONE - ac[k][q];
                            }
                            rgc[k] = rgn[k];
                            bdc[k] = bdn[k];
                        }
                    }
                }
            };

            for (;;) {
                int r;
                if (layout == 8) r = walk(std::integral_constant<int, 4>{});
                else if (layout == 4) r = walk(std::integral_constant<int, 2>{});
                else r = walk(std::integral_constant<int, 1>{});
                if (r == 0) break;
                const uint64_t amAll = __ballot(alive);
                if (layout == 8) {
                    // W8 -> W4: the dead groups are final (written now); the <= 32 live ones move to two lanes
                    // each: slot s = L >> 1 holds live group s (in lane order), lane L its columns 2 (L & 1)..+1
                    if (!alive) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const h2 A = (ku ? FULL1 : FULL0) > 0u ? ONE - T[q] : ONE;
                            pw_write_pair(tg, px + 2u * (uint32_t)(q & 1), py + (uint32_t)(q >> 1), A, R[q], G[q], B[q], D[q]);
                        }
                    }
                    const uint32_t ng = (uint32_t)__popcll(amAll);
                    if (alive) cs[__popcll(amAll & ((1ull << lane) - 1ull))] = lane;
                    pw_wave_sync();
                    const uint32_t s = lane >> 1, c = lane & 1u;
                    valid = s < ng;
                    const uint32_t src = cs[valid ? s : 0u];
                    auto mv2 = [&](h2 (&V)[4]) {
                        const h2 a0 = pw_bperm(src, V[0]), a1 = pw_bperm(src, V[1]);
                        const h2 a2 = pw_bperm(src, V[2]), a3 = pw_bperm(src, V[3]);
                        V[0] = c ? a1 : a0;
                        V[1] = c ? a3 : a2;
                    };
                    mv2(T);
                    mv2(R);
                    mv2(G);
                    mv2(B);
                    mv2(D);
                    ku = src >> 5;
                    const uint32_t g = src & 31u;
                    px = (ku ? UX1 : UX0) + (g & 3u) * 4u + 2u * c;
                    py = (ku ? UY1 : UY0) + (g >> 2) * 2u;
                    alive = valid;
                    layout = 4;
                    if ((uint32_t)__popcll(__ballot(alive) & 0x5555555555555555ull) > 16u) continue;
                }
                {
                    // W4 -> W2 (k_blend_px's compaction): the dead groups are final; the <= 16 live ones move
                    // to four lanes each: group g'' = L >> 2, lane L its columns 2 (L & 1)..+1 of row (L >> 1) & 1
                    if (valid && !alive) {
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            const h2 A = (ku ? FULL1 : FULL0) > 0u ? ONE - T[q] : ONE;
                            pw_write_pair(tg, px, py + (uint32_t)q, A, R[q], G[q], B[q], D[q]);
                        }
                    }
                    const uint64_t am = __ballot(alive) & 0x5555555555555555ull;
                    const uint32_t ng = (uint32_t)__popcll(am);
                    if (alive && (lane & 1u) == 0u) cs[__popcll(am & ((1ull << lane) - 1ull))] = lane >> 1;
                    pw_wave_sync();
                    const uint32_t g2 = lane >> 2, kk = lane & 1u, rr = (lane >> 1) & 1u;
                    valid = g2 < ng;
                    const uint32_t src = 2u * cs[valid ? g2 : 0u] + kk;
                    auto mv1 = [&](h2 (&V)[4]) {
                        const h2 a0 = pw_bperm(src, V[0]), a1 = pw_bperm(src, V[1]);
                        V[0] = rr ? a1 : a0;
                    };
                    mv1(T);
                    mv1(R);
                    mv1(G);
                    mv1(B);
                    mv1(D);
                    px = pw_bperm(src, px);
                    py = pw_bperm(src, py) + rr;
                    ku = pw_bperm(src, ku);
                    alive = valid;
                    layout = 2;
                }
            }
        }
        // write (GlobalShaders.metal:1152-1186); empty tiles keep the clear colour (0,0,0,1)
        if (valid) {
            const bool fullL = (ku ? FULL1 : FULL0) > 0u;
            if (layout == 8) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    pw_write_pair(tg, px + 2u * (uint32_t)(q & 1), py + (uint32_t)(q >> 1), fullL ? ONE - T[q] : ONE, R[q],
                                  G[q], B[q], D[q]);
            } else if (layout == 4) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    pw_write_pair(tg, px, py + (uint32_t)q, fullL ? ONE - T[q] : ONE, R[q], G[q], B[q], D[q]);
            } else {
                pw_write_pair(tg, px, py, fullL ? ONE - T[0] : ONE, R[0], G[0], B[0], D[0]);
            }
        }
        if (exactD) {  // (rare) every pixel of the job's units written again
            auto wr = [&](uint32_t x, uint32_t y, h2 A, h2 r, h2 g, h2 b, h2 d) { pw_write_pair(tg, x, y, A, r, g, b, d); };
            if (CNT0) blend_exact::walk_unit_exact<2>(LST0, CNT0, rec, tbl, LA, LB, UX0, UY0, thrBits, wr);
            if (pair && CNT1) blend_exact::walk_unit_exact<2>(LST1, CNT1, rec, tbl, LA, LB, UX1, UY1, thrBits, wr);
        }
        auto finishUnit = [&](uint32_t uu, uint32_t cnt, bool done, uint32_t walk) {
            const uint32_t wk = min(cnt ? (done ? walk : (cnt + 15u) / 16u * 16u) : 0u, 65535u);
            if (unitCost && lane == 0) unitCost[uu] = (uint16_t)wk;
            waveMax = max(waveMax, wk);
            if (trace && lane == 0) {
                unsigned long long* t = trace + (size_t)uu * 4;
                t[0] = tStart;
                t[1] = __builtin_amdgcn_s_memrealtime();
                t[2] = ((unsigned long long)cnt << 32) | wk;
                const unsigned long long xcc = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (3 << 11));  // XCC_ID
                t[3] = (xcc << 48) | ((unsigned long long)(pair ? 1u : 0u) << 40) |
                       (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));
            }
        };
        finishUnit(Uu0, CNT0, done0, walk0);
        if (pair) finishUnit(Uu1, CNT1, done1, walk1);
        if (agePrio || topPrio) __builtin_amdgcn_s_setprio(0);
        topPrio = false;
        uint32_t nextQ = 0;
        if (lane == 0) nextQ = atomicAdd(myQueue, 1u);  // claimed after the job
        job = gridWaves + stripe + stripes * __builtin_amdgcn_readfirstlane(nextQ);
        pos = jobPos(job, single);
    }
    if (unitCost && lane == 0 && waveMax) atomicMax(&costMax[(blockIdx.x * NW + wv) % kCostMaxSlots], waveMax);
}

// the pair walk for a frame of half-tile units on one GPU (no multi-GPU gather); `waves` per workgroup
void launch_blend_pw(const FrameGeometry& g, const DeviceArena& A, void* color, size_t colorPitch, void* depth,
                     size_t depthPitch, int numCUs, bool costOrder, int colorFormat, hipStream_t s, int waves) {
    const uint32_t numTiles = g.rowCount * g.tilesX;
    if (numTiles == 0) return;
    const int vec = ((((uintptr_t)color) & 15u) == 0 && (colorPitch & 15u) == 0 &&
                     (depth == nullptr || ((((uintptr_t)depth) & 3u) == 0 && (depthPitch & 3u) == 0)))
                        ? 1
                        : 0;
    const PwTarget tg{(uint8_t*)color, colorPitch, (uint8_t*)depth, depthPitch, g.width, g.height,
                      vec | ((colorFormat & 15) << 4)};
    const int flags = 2 | (costOrder ? 4 : 0);
    const uint32_t units = numTiles * 2u;
    // (at most two units per wave in the first round)
    uint32_t grid = (units + (uint32_t)(2 * waves) - 1u) / (uint32_t)(2 * waves);
    if (grid > (uint32_t)numCUs) grid = (uint32_t)numCUs;
    if (grid == 0) grid = 1;
    const uint32_t* order = costOrder ? A.unitOrder : nullptr;
#define GSM_LAUNCH_PW(NTH)                                                                                          \
    hipLaunchKernelGGL((k_blend_pw<NTH>), dim3(grid), dim3(NTH), 0, s, A.tileStart, A.rec, A.expTable, A.tileQueue, \
                       numTiles, g.tilesX, tg, order, A.unitCost, A.blendTrace, A.halfVals[0], A.halfVals[1],      \
                       A.halfCount, g.tileCount, A.costMax, g.rowBegin, g.rowStride, flags)
    if (waves >= 16) GSM_LAUNCH_PW(1024);
    else if (waves >= 12) GSM_LAUNCH_PW(768);
    else GSM_LAUNCH_PW(512);
#undef GSM_LAUNCH_PW
}

}  // namespace gsm
