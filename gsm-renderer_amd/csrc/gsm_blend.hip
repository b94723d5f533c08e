// gsm_blend.hip -- the GlobalRenderer's blend stage on gfx950: clear + front-to-back
// alpha blending of every tile's depth-sorted list (globalRender, GlobalShaders.metal:1030-1187;
// clear: :140-154), plus the load-balancing schedule of its work units.
//
// Persistent workgroups: one workgroup per CU holds the 128 KiB fp16 exp table in LDS and its
// waves pull work units (parts of tiles) from a device counter.  Bit-exact with the oracle: the
// per-thread saturation break of the reference (one 4x2 pixel group) is evaluated per group on
// every list entry.  Numeric contract: DESIGN.md.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/gsm_debug.h"
#include "../../include/gsm_renderer.h"
#include "gsm_blend_exact.h"
#include "gsm_detmath.h"
#include "gsm_internal.h"
#include "gsm_types.h"

namespace gsm {

// entries between the walks' exit / compaction checkpoints (a multiple of 4: the compacted walk's groups;
// 4 and 8 measured no faster)
constexpr uint32_t kBlendExit = 16;
// waves per workgroup that take the schedule's longest units first, at the top priority (waves map
// to SIMDs round-robin: 4 = one per SIMD; 0 and 8 measured slower)
constexpr uint32_t kBlendTopWaves = 4;
// quadrant units (P = 1) up to this many tiles per CU, half tiles beyond
constexpr uint32_t kBlendP1TilesPerCu = 8;

typedef _Float16 h1;
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
// `color += gColor * w` (GlobalShaders.metal:1137-1145, DepthFirstShaders.metal:1783-1786): one
// fused multiply-add, a single rounding per channel (the numeric contract; the oracle's hfma)
__device__ __forceinline__ h2 blend_acc(h2 acc, h2 c, h2 w) { return __builtin_elementwise_fma(c, w, acc); }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ float h_bits_to_f(uint16_t b) { return (float)__builtin_bit_cast(h1, b); }
// linear -> sRGB encode of a [0, 1] value (include/gsm_renderer.h), powr of the numeric contract
__device__ __forceinline__ float srgb_encode(float c) {
    return c <= 0.0031308f ? c * 12.92f : 1.055f * det_powrf(c, 1.0f / 2.4f) - 0.055f;
}
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 splat_lo(h2 v) { return h2{v.x, v.x}; }
__device__ __forceinline__ h2 splat_hi(h2 v) { return h2{v.y, v.y}; }

// The table index of a packed pair of quadratic forms: its fp16 bits.  (The far-field clamp and the
// dead-lane columns that cut the gathers' bank conflicts, and the duplicate-read attribution build, are
// kept as tools/exp/rejected_variants.patch: bit-exact, no faster)
__device__ __forceinline__ uint32_t tbl_bits(h2 p) {
    return as_u32(p);
}

// exp table lookup for a packed pair of quadratic forms: the table is indexed by the fp16 bits
// of p and holds fp16(exp(fp16(-0.5 * p))), correctly rounded (gsm_detmath.h)
__device__ __forceinline__ h2 lookup2(const uint16_t* tbl, h2 p) {
    const uint32_t pb = tbl_bits(p);
    const uint32_t lo = tbl[pb & 0xFFFFu];
    const uint32_t hi = tbl[pb >> 16];
    return as_h2(lo | (hi << 16));
}

// max over the 4 lanes of a quad: DPP quad_perm [1,0,3,2] then [2,3,0,1]
__device__ __forceinline__ uint32_t quad_max_u32(uint32_t v) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v = v > a ? v : a;
    const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    return v > b ? v : b;
}

// ---------------------------------------------------------------------------
// k_blend_px: one wave per blend unit, P pixel pairs per lane.
//   P = 1: 16x8 quadrant of a tile (4 units per tile), a 4x2 group spans 4 lanes
//   P = 2: 16x16 half tile (2 units per tile), a group spans 2 lanes (rows)
// More pairs per lane give every list entry's uniform work (5 readlanes, the dy terms of
// the quadratic form) to more pixels and P independent T chains per lane; fewer give
// shorter walks (a unit walks until its slowest group breaks).  The list is walked in
// groups of U = 4/P entries through a three-stage software pipeline (stage 1: next group's
// p and table reads; stage 2: blend this group; stage 3: next group's alphas).
// ---------------------------------------------------------------------------
// Lanes of one wave hand LDS words to each other: the compiler must not forward a lane's own
// store past them (no instruction; the hardware keeps a wave's LDS operations in order).
__device__ __forceinline__ void blend_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The records of the walk's current 64-entry batch are staged in LDS and read back with uniform
// addresses (one ds_read_b128 + one ds_read_b32 broadcast per entry) instead of 5 v_readlane;
// 2-entry pipeline groups at P = 2 (4-entry groups measured no gain).
template <int NT, int P, bool COMPACT = false>
__global__ __launch_bounds__(NT) void k_blend_px(
    const uint32_t* __restrict__ tileStart, const BlendRecord* __restrict__ rec,
    const uint16_t* __restrict__ expTable, uint32_t* __restrict__ queue, uint32_t tileBegin,
    uint32_t numTiles, uint32_t tilesX, uint32_t W, uint32_t H, uint8_t* __restrict__ color,
    size_t colorPitch, uint8_t* __restrict__ depth, size_t depthPitch, int flags,
    const uint32_t* __restrict__ order, uint16_t* __restrict__ unitCost,
    unsigned long long* __restrict__ trace, const uint32_t* __restrict__ half0,
    const uint32_t* __restrict__ half1, const uint32_t* __restrict__ halfCount, uint32_t tileCount,
    uint32_t* __restrict__ costMax, uint32_t rowBegin, uint32_t rowStride, MgArrive arrive) {
    static_assert(P == 1 || P == 2, "pairs per lane: quadrant or half-tile units (half-tile lists)");
    static_assert(!COMPACT || P == 2, "compaction: half tiles");
    constexpr uint32_t U = 4 / P;  // entries per pipeline group
    constexpr uint32_t NG = 64 / U;      // groups per 64-entry batch
    constexpr uint32_t EXITG = kBlendExit / U;  // exit test every kBlendExit entries
    constexpr uint32_t UPT = 4 / P;      // units per tile
    constexpr uint32_t NW = NT / 64;
    constexpr uint32_t UNROLL = NG;
    const bool agePrio = (flags & 2) != 0;
    __shared__ __attribute__((aligned(16))) uint16_t tbl[65536];
    __shared__ uint32_t cscr[NW][16];  // compaction: the alive groups of each wave, in order
    __shared__ __attribute__((aligned(16))) uint4 lrecA[NW][64];  // current batch records
    __shared__ uint32_t lrecB[NW][64];
    __shared__ uint32_t exitCount;  // a gathered multi-GPU frame: waves of this workgroup past their last unit
    if (threadIdx.x == 0) exitCount = 0;
    GSM_EXP_TABLE_TO_LDS(NT, expTable, tbl);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    // write (GlobalShaders.metal:1152-1186): one pixel pair (px, py), (px + 1, py) in the target's
    // format (flags bits 4-7, gsm_color_format; conversion rules in include/gsm_renderer.h)
    const int colorFmt = (flags >> 4) & 15;
    // plain stores, also into rank 0's gathered frame of a multi-GPU frame (flags bit 12: released by the
    // workgroup's L2 write-back at its exit; write-through pixel stores measured slower)
    auto st128 = [&](uint8_t* p, uint4 v) { *(uint4*)p = v; };
    auto st32 = [&](uint8_t* p, uint32_t v) { *(uint32_t*)p = v; };
    auto std32 = [&](uint8_t* p, uint32_t v) { *(uint32_t*)p = v; };
    auto std16 = [&](uint8_t* p, uint16_t v) { *(uint16_t*)p = v; };
    auto write_pair = [&](uint32_t px, uint32_t py, h2 Av, h2 Rq, h2 Gq, h2 Bq, h2 Dq) {
        if (py >= H) return;
        uint8_t* crow = color + (size_t)py * colorPitch;
        // integer packing (extracting .y of a half2 via __builtin_bit_cast miscompiled)
        const uint32_t ur = as_u32(Rq), ug = as_u32(Gq), ub = as_u32(Bq), ua = as_u32(Av);
        const uint32_t ud = as_u32(Dq);
        if (colorFmt == GSM_COLOR_FORMAT_RGBA16F) {
            const uint32_t p0a = (ur & 0xFFFFu) | (ug << 16);
            const uint32_t p0b = (ub & 0xFFFFu) | (ua << 16);
            const uint32_t p1a = (ur >> 16) | (ug & 0xFFFF0000u);
            const uint32_t p1b = (ub >> 16) | (ua & 0xFFFF0000u);
            if ((flags & 1) && px + 1 < W) {
                st128(crow + (size_t)px * 8, make_uint4(p0a, p0b, p1a, p1b));
            } else {
                if (px < W) {  // 4-byte stores: any 4-byte aligned pitch
                    st32(crow + (size_t)px * 8, p0a);
                    st32(crow + (size_t)px * 8 + 4, p0b);
                }
                if (px + 1 < W) {
                    st32(crow + (size_t)(px + 1) * 8, p1a);
                    st32(crow + (size_t)(px + 1) * 8 + 4, p1b);
                }
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 2; ++i) {
                if (px + i >= W) break;
                const uint32_t sh = 16u * i;
                float c[4] = {h_bits_to_f((uint16_t)(ur >> sh)), h_bits_to_f((uint16_t)(ug >> sh)),
                              h_bits_to_f((uint16_t)(ub >> sh)), h_bits_to_f((uint16_t)(ua >> sh))};
                if (colorFmt == GSM_COLOR_FORMAT_RGBA32F) {
                    uint8_t* o = crow + (size_t)(px + i) * 16;
                    if (flags & 1) {
                        st128(o, make_uint4(__float_as_uint(c[0]), __float_as_uint(c[1]), __float_as_uint(c[2]),
                                            __float_as_uint(c[3])));
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) st32(o + 4 * k, __float_as_uint(c[k]));
                    }
                    continue;
                }
                const bool srgb = colorFmt == GSM_COLOR_FORMAT_RGBA8_UNORM_SRGB ||
                                  colorFmt == GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB;
                uint32_t u8[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float x = __builtin_fminf(__builtin_fmaxf(c[k], 0.0f), 1.0f);
                    if (srgb && k < 3) x = srgb_encode(x);
                    u8[k] = (uint32_t)__builtin_rintf(x * 255.0f);
                }
                const bool bgra = colorFmt >= GSM_COLOR_FORMAT_BGRA8_UNORM;
                const uint32_t px32 = (bgra ? u8[2] : u8[0]) | (u8[1] << 8) | ((bgra ? u8[0] : u8[2]) << 16) | (u8[3] << 24);
                st32(crow + (size_t)(px + i) * 4, px32);
            }
        }
        if (depth) {
            if ((flags & 1) && px + 1 < W) {
                std32(depth + (size_t)py * depthPitch + (size_t)px * 2, ud);
            } else {
                if (px < W) std16(depth + (size_t)py * depthPitch + (size_t)px * 2, (uint16_t)(ud & 0xFFFFu));
                if (px + 1 < W) std16(depth + (size_t)py * depthPitch + (size_t)(px + 1) * 2, (uint16_t)(ud >> 16));
            }
        }
    };
    // pixel pair k of this lane sits at (px[k], py[k]) and (px[k] + 1, py[k]) inside the unit
    uint32_t offX[P], offY[P];
    if (P == 1) {
        const uint32_t grp = lane >> 2;
        offX[0] = (grp & 3u) * 4u + (lane & 1u) * 2u;
        offY[0] = (grp >> 2) * 2u + ((lane >> 1) & 1u);
    } else {
        // a 4x2 group on lanes 2g (columns 0-1) and 2g + 1 (columns 2-3), each lane 2x2 pixels:
        // pair 0 = row 0, pair 1 = row 1 of the same two columns, so the dx terms of the quadratic
        // form are shared by the lane's pairs and the dy terms come as one pair of rows
        const uint32_t grp = lane >> 1;
        offX[0] = offX[P - 1] = (grp & 3u) * 4u + (lane & 1u) * 2u;
        offY[0] = (grp >> 2) * 2u;
        offY[P - 1] = offY[0] + 1u;
    }
    const h2 ONE = {(h1)1.0f, (h1)1.0f};
    const h2 ZERO = {(h1)0.0f, (h1)0.0f};
    const uint32_t thrBits = (uint32_t)__builtin_bit_cast(uint16_t, (h1)(1.0f / 255.0f));
    const h1 c099 = (h1)0.99;
    const h2 C099 = {c099, c099};
    const uint32_t numUnits = numTiles * UPT;
    const uint32_t gridWaves = gridDim.x * NW;

    // First unit static, then the queue.  With the schedule on (flags bit 2), the first half of
    // every workgroup's waves (one per SIMD) take the gridDim.x * NW/2 longest units and run
    // them at the top priority, so each SIMD pairs one long walk with one shorter one and the
    // long walk issues nearly as fast as a wave alone (the makespan is the longest walk's).
    const uint32_t wv = threadIdx.x >> 6;
    const bool split = (flags & 4) != 0;
    constexpr uint32_t NTOP = kBlendTopWaves;
    uint32_t qi = !split ? blockIdx.x * NW + wv
                         : (wv < NTOP ? blockIdx.x * NTOP + wv
                                      : gridDim.x * NTOP + blockIdx.x * (NW - NTOP) + (wv - NTOP));
    bool topPrio = split && wv < NTOP;
    // When a wave claims its next unit from the queue (flags bits 8-9): 1 (default) after the current
    // unit, 0 at its start, 2 one 64-entry batch before the walk it made last frame ends (unitCost).
    // A claim made at the start hides the atomic's latency but hands the next position of the
    // longest-first order to a wave that stays busy for the rest of its unit, so mid-length units
    // started late and ran past the end of the work (r03, config 2: blend 140.4 -> 116.8 us late).
    const uint32_t claimMode = ((uint32_t)flags >> 8) & 3u;
    uint32_t waveMax = 0;  // this wave's longest walk, for the next frame's schedule (costMax)
    // dynamic units: positions gridWaves + stripe + stripes * k from this workgroup's counter
    const uint32_t stripes = (gridDim.x % kQueueStripes) == 0 ? kQueueStripes : 1u;
    const uint32_t stripe = blockIdx.x % stripes;
    uint32_t* const myQueue = queue + stripe * kQueueStride;
    while (qi < numUnits) {
        uint32_t u = order ? __builtin_amdgcn_readfirstlane(order[qi]) : qi;
        if (u >= numUnits) u = qi;  // a schedule is a permutation of [0, numUnits); never trust it further
        const uint32_t tile = tileBegin + u / UPT, part = u % UPT;
        const uint32_t tileX = tile % tilesX, tileY = rowBegin + (tile / tilesX) * rowStride;
        const uint32_t ux = tileX * kTileWidth + (part & 1u) * 16u;
        const uint32_t uy = tileY * kTileHeight + (P == 1 ? (part >> 1) * 8u : 0u);
        // the unit walks its half's list: the tile's sorted entries without those whose skip flag for
        // this half is set (k_scatter, k_half_lists) -- they would leave every pixel of it unchanged
        const uint32_t start = __builtin_amdgcn_readfirstlane(tileStart[tile]);
        const uint32_t full = __builtin_amdgcn_readfirstlane(tileStart[tile + 1]) - start;
        const uint32_t hsel = part & 1u;
        const uint32_t count = __builtin_amdgcn_readfirstlane(halfCount[hsel * tileCount + tile]);
        unsigned long long tStart = 0;
        if (trace) tStart = __builtin_amdgcn_s_memrealtime();
        uint32_t nproc = 0;
        uint32_t ncomp = 0;  // entry at which the unit moved to one pair per lane (trace only)
        uint32_t nextQ = 0;
        bool claimed = false;
        // claimMode 2: the walk this unit made last frame (before this frame's walk overwrites it)
        const uint32_t expWalk = (claimMode == 2 && unitCost) ? __builtin_amdgcn_readfirstlane((uint32_t)unitCost[u]) : 0u;
        auto claim = [&]() {
            if (!claimed) {
                if (lane == 0) nextQ = atomicAdd(myQueue, 1u);
                claimed = true;
            }
        };

        h2 T[P], R[P], G[P], B[P], D[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            T[k] = ONE;
            R[k] = G[k] = B[k] = D[k] = ZERO;
        }
        // the unit met a record of inf / NaN fp16 depth: walked again exactly at its end (gsm_blend_exact.h)
        bool exactD = false;
        if (count > 0) {
            h2 X[P], Yv;  // Yv: the lane's (up to) two rows
#pragma unroll
            for (int k = 0; k < P; ++k) X[k] = h2{(h1)(float)(ux + offX[k]), (h1)(float)(ux + offX[k] + 1u)};
            Yv = h2{(h1)(float)(uy + offY[0]), (h1)(float)(uy + offY[P - 1])};
            const uint32_t* lst = (hsel ? half1 : half0) + start;
            // Batch registers: lane l of bA/bB holds list entry b0 + l, nA/nB entry b0 + 64 + l,
            // mA/mB entry b0 + 128 + l, nI the index of entry b0 + 192 + l.  Loads are
            // unpredicated (clamped index) and issued one batch ahead of their first use, so
            // the group loop never waits on memory (a predicated load would merge with the old
            // register value and force a copy -- and a vmcnt wait -- into the loop).  Lanes past
            // the list end hold a neutral record: mean = unit origin, conic = 0, opacity = 0
            // gives p = 0, alpha = 0 exactly, which leaves T, C and the break state unchanged.
            const uint32_t last = count - 1u;
            const uint4 pad = make_uint4(as_u32(h2{(h1)(float)ux, (h1)(float)uy}), 0u, 0u, 0u);
            const uint32_t gi0 = lst[min(lane, last)];
            const uint32_t gi1 = lst[min(64u + lane, last)];
            const uint32_t gi2 = lst[min(128u + lane, last)];
            uint4 bA = *(const uint4*)(rec + gi0);
            uint32_t bB = rec[gi0].b;
            uint4 nA = *(const uint4*)(rec + gi1);
            uint32_t nB = rec[gi1].b;
            uint4 mA = *(const uint4*)(rec + gi2);
            uint32_t mB = rec[gi2].b;
            uint32_t nI = lst[min(192u + lane, last)];
            if (claimMode == 0 || (claimMode == 2 && expWalk <= 64u)) claim();
            if (lane >= count) {
                bA = pad;
                bB = 0u;
            }
            if (64u + lane >= count) {
                nA = pad;
                nB = 0u;
            }
            exactD = blend_exact::batch_depth_nonfinite(bB) || blend_exact::batch_depth_nonfinite(nB);

            h2 ac[U][P], om[U][P];
            uint32_t rgc[U], bdc[U], rgn[U], bdn[U], opn[U];
            u16x2 en[U][P];  // next group's exp table words (d16 loads into both halves)
            bool alive = true;
            uint32_t eC = 0, b0C = 0;  // compaction: next entry, its batch base
            // p = ((dx*dx)*cxx + (dy*dy)*cyy) + (dx*dy)*cxy2 (GlobalShaders.metal:1115-1122);
            // the dy terms are computed once for the lane's rows, at P = 2 the dx terms once for its
            // two columns (the same operations per pixel, fewer of them per lane)
            auto quadform = [&](uint32_t r0, uint32_t r1, uint32_t r2, h2 (&pq)[P]) {
                const h2 mean = as_h2(r0), cc = as_h2(r1), oc = as_h2(r2);
                const h2 dyv = Yv - splat_hi(mean);
                const h2 dyy = (dyv * dyv) * splat_hi(cc);
                if constexpr (P == 2) {
                    const h2 dx = X[0] - splat_lo(mean);
                    const h2 dxx = (dx * dx) * splat_lo(cc);
                    pq[0] = (dxx + splat_lo(dyy)) + (dx * splat_lo(dyv)) * splat_lo(oc);
                    pq[P - 1] = (dxx + splat_hi(dyy)) + (dx * splat_hi(dyv)) * splat_lo(oc);
                    return;
                }
                // P = 1: one pair per lane
                const h2 dx = X[0] - splat_lo(mean);
                pq[0] = ((dx * dx) * splat_lo(cc) + splat_lo(dyy)) + (dx * splat_lo(dyv)) * splat_lo(oc);
            };
            lrecA[wv][lane] = bA;
            lrecB[wv][lane] = bB;
            blend_wave_sync();
            // prime group 0
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) {
                const uint32_t r2 = __builtin_amdgcn_readlane(bA.z, k);
                h2 pq[P];
                quadform(__builtin_amdgcn_readlane(bA.x, k), __builtin_amdgcn_readlane(bA.y, k), r2, pq);
                rgc[k] = __builtin_amdgcn_readlane(bA.w, k);
                bdc[k] = __builtin_amdgcn_readlane(bB, k);
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    // a = min(opacity * exp(-0.5h * p), 0.99h) (GlobalShaders.metal:1124-1131)
                    ac[k][q] = __builtin_elementwise_min(splat_hi(as_h2(r2)) * lookup2(tbl, pq[q]), C099);
                    om[k][q] = ONE - ac[k][q];
                }
            }
            for (uint32_t b0 = 0;; b0 += 64u) {
                if (claimMode == 2 && b0 + 64u >= expWalk) claim();
#pragma unroll UNROLL
                for (uint32_t gi = 0; gi < NG; ++gi) {
                    // stage 1: the next group's table words go in flight (independent of T)
                    {
                        const bool nb = gi + 1 == NG;
                        if (nb) {  // every entry of this batch was read: stage the next one
                            lrecA[wv][lane] = nA;
                            lrecB[wv][lane] = nB;
                            blend_wave_sync();
                            exactD = exactD || blend_exact::batch_depth_nonfinite(nB);
                        }
#pragma unroll
                        for (uint32_t k = 0; k < U; ++k) {
                            const uint32_t j = ((gi + 1) * U + k) & 63u;
                            h2 pq[P];
                            const uint4 ra = lrecA[wv][j];
                            opn[k] = ra.z;
                            quadform(ra.x, ra.y, ra.z, pq);
                            rgn[k] = ra.w;
                            bdn[k] = lrecB[wv][j];
#pragma unroll
                            for (int q = 0; q < P; ++q) {
                                // raw table words: first used in stage 3, after the current
                                // group's blend, so the LDS latency hides behind it
                                const uint32_t pb = tbl_bits(pq[q]);
                                en[k][q].x = tbl[pb & 0xFFFFu];
                                en[k][q].y = tbl[pb >> 16];
                            }
                        }
                    }
                    // stage 2: blend the current group
#pragma unroll
                    for (uint32_t k = 0; k < U; ++k) {
                        // group break (GlobalShaders.metal:1086-1088): max T of the 4x2 group
                        // T >= 0, so the u16 bit patterns order like the values (v_pk_max_u16,
                        // no canonicalising of the fp16 inputs)
                        u16x2 tm = __builtin_bit_cast(u16x2, T[0]);
#pragma unroll
                        for (int q = 1; q < P; ++q) tm = __builtin_elementwise_max(tm, __builtin_bit_cast(u16x2, T[q]));
                        const uint32_t tb = __builtin_bit_cast(uint32_t, tm);
                        uint32_t gm = max(tb & 0xFFFFu, tb >> 16);
                        if (P == 1) gm = quad_max_u32(gm);
                        if (P == 2) {
                            const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)gm, 0xB1, 0xF, 0xF, false);
                            gm = max(gm, o);
                        }
                        alive = alive && !(gm < thrBits);  // T >= 0: fp16 order == bit order
                        const h2 rgv = as_h2(rgc[k]), bdv = as_h2(bdc[k]);
                        // a dead lane keeps T and C (alpha 0 would give the same bits: C + c*0 == C,
                        // T*1 == T): the updates run under an EXEC mask of the live lanes
                        if (alive) {
#pragma unroll
                            for (int q = 0; q < P; ++q) {
                                const h2 w = ac[k][q] * T[q];  // (GlobalShaders.metal:1137-1149)
                                T[q] = T[q] * om[k][q];
                                R[q] = blend_acc(R[q], splat_lo(rgv), w);
                                G[q] = blend_acc(G[q], splat_hi(rgv), w);
                                B[q] = blend_acc(B[q], splat_lo(bdv), w);
                                D[q] = blend_acc(D[q], splat_hi(bdv), w);
                            }
                        }
                    }
                    const uint32_t g1 = b0 + (gi + 1) * U;
                    // late exits are harmless: neutral records past the end, dead lanes blend nothing
                    if ((gi + 1) % EXITG == 0) {
                        const uint64_t am = __ballot(alive);
                        if (g1 >= count || am == 0) {
                            nproc = g1;
                            goto unit_done;
                        }
                        // at most 16 of the 32 groups alive: continue them one pixel pair per lane
                        // (two 32-bit counts: a 64-bit popcount's compare goes to the VALU)
                        if (COMPACT && (uint32_t)__builtin_popcount((uint32_t)am & 0x55555555u) +
                                               (uint32_t)__builtin_popcount((uint32_t)(am >> 32) & 0x55555555u) <= 16u) {
                            eC = g1;
                            b0C = b0;
                            goto compact_phase;
                        }
                    }
                    // stage 3: the next group's alphas
#pragma unroll
                    for (uint32_t k = 0; k < U; ++k) {
#pragma unroll
                        for (int q = 0; q < P; ++q) {
                            const h2 ek = __builtin_bit_cast(h2, en[k][q]);
                            ac[k][q] = __builtin_elementwise_min(splat_hi(as_h2(opn[k])) * ek, C099);
                            om[k][q] = ONE - ac[k][q];
                        }
                        rgc[k] = rgn[k];
                        bdc[k] = bdn[k];
                    }
                }
                if (topPrio) {
                    if (b0 == 0) __builtin_amdgcn_s_setprio(3);
                } else if (agePrio) {
                    if (b0 == 0) __builtin_amdgcn_s_setprio(1);
                    else if (b0 == 128u) __builtin_amdgcn_s_setprio(2);
                    else if (b0 == 320u && !split) __builtin_amdgcn_s_setprio(3);
                }
                bA = nA;
                bB = nB;
                const bool mv = b0 + 128u + lane < count;
                nA = mv ? mA : pad;
                nB = mv ? mB : 0u;
                mA = *(const uint4*)(rec + nI);
                mB = rec[nI].b;
                nI = lst[min(b0 + 256u + lane, last)];
            }
        compact_phase:
            if constexpr (COMPACT) {
                // Groups that broke keep their pixels: written now, in the half-tile layout.
                if (!alive) {
#pragma unroll
                    for (int q = 0; q < P; ++q)
                        write_pair(ux + offX[q], uy + offY[q], ONE - T[q], R[q], G[q], B[q], D[q]);
                }
                // The alive groups (<= 16) move to one pixel pair per lane: group g' of the new
                // layout owns lanes 4g'..4g'+3 (pair k of row r at lane 4g' + 2r + k), so its
                // break is again a quad max.  State comes over by ds_bpermute from lane 2g + r.
                const uint64_t am = __ballot(alive) & 0x5555555555555555ull;
                const uint32_t ng = (uint32_t)__popcll(am);
                if (alive && (lane & 1u) == 0) cscr[wv][__popcll(am & ((1ull << lane) - 1ull))] = lane >> 1;
                blend_wave_sync();
                const uint32_t gp = lane >> 2, kk = lane & 1u, rr = (lane >> 1) & 1u;
                const bool valid1 = gp < ng;
                const uint32_t sg = cscr[wv][valid1 ? gp : 0u];
                // half-tile layout: columns 2kk..2kk+1 of group sg sit on lane 2sg + kk, row rr in pair rr
                const int srcAddr = (int)((2u * sg + kk) * 4u);
                auto pick = [&](h2 v0, h2 v1) {
                    const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(srcAddr, (int)as_u32(v0));
                    const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(srcAddr, (int)as_u32(v1));
                    return as_h2(rr ? a1 : a0);
                };
                h2 T1 = pick(T[0], T[1]), R1 = pick(R[0], R[1]), G1 = pick(G[0], G[1]);
                h2 B1 = pick(B[0], B[1]), D1 = pick(D[0], D[1]);
                const uint32_t px1 = ux + (sg & 3u) * 4u + 2u * kk, py1 = uy + (sg >> 2) * 2u + rr;
                h2 X1 = h2{(h1)(float)px1, (h1)(float)(px1 + 1u)};
                const h2 Y1 = h2{(h1)(float)py1, (h1)(float)py1};
                bool alive1 = valid1;
                // the same per-pixel operations as the half-tile walk (quadform above)
                auto quad1 = [&](uint32_t r0, uint32_t r1, uint32_t r2) {
                    const h2 mean = as_h2(r0), cc = as_h2(r1), oc = as_h2(r2);
                    const h2 dyv = Y1 - splat_hi(mean);
                    const h2 dyy = (dyv * dyv) * splat_hi(cc);
                    const h2 dx = X1 - splat_lo(mean);
                    return ((dx * dx) * splat_lo(cc) + splat_lo(dyy)) + (dx * splat_lo(dyv)) * splat_lo(oc);
                };
                auto rotate = [&](uint32_t base) {  // batches move one 64-entry step (as above)
                    bA = nA;
                    bB = nB;
                    const bool mv = base + 128u + lane < count;
                    nA = mv ? mA : pad;
                    nB = mv ? mB : 0u;
                    mA = *(const uint4*)(rec + nI);
                    mB = rec[nI].b;
                    nI = lst[min(base + 256u + lane, last)];
                    exactD = exactD || blend_exact::batch_depth_nonfinite(nB);
                };
                uint32_t e = eC, bb = b0C;
                ncomp = eC;
                if (e - bb == 64u) {
                    rotate(bb);
                    bb += 64u;
                }
                constexpr uint32_t U1 = 4;  // entries per pipeline group
                h2 ac1[U1], om1[U1];
                uint32_t rgc1[U1], bdc1[U1], rgn1[U1], bdn1[U1], opn1[U1];
                u16x2 en1[U1];
                // The records come from the LDS stage of the current batch (uniform-address reads, as
                // in the half-tile walk) -- it holds batch bb here: the walk staged it,
                // or staged the next one and the rotation above made that batch bb -- instead of five
                // v_readlane per entry from the batch registers.
#pragma unroll
                for (uint32_t k = 0; k < U1; ++k) {  // prime the group at e
                    const uint32_t j = e - bb + k;
                    const uint4 ra = lrecA[wv][j];
                    const uint32_t r2 = ra.z;
                    const h2 pq = quad1(ra.x, ra.y, r2);
                    rgc1[k] = ra.w;
                    bdc1[k] = lrecB[wv][j];
                    ac1[k] = __builtin_elementwise_min(splat_hi(as_h2(r2)) * lookup2(tbl, pq), C099);
                    om1[k] = ONE - ac1[k];
                }
                for (;;) {
                    if (claimMode == 2 && e + 64u >= expWalk) claim();
                    // stage 1: the next group's records and table words
                    {
                        const uint32_t jn = e + U1 - bb;  // 4..64
                        const bool nb = jn >= 64u;
                        if (nb) {  // the next group opens the next batch: stage it (this batch is all read)
                            lrecA[wv][lane] = nA;
                            lrecB[wv][lane] = nB;
                            blend_wave_sync();
                            exactD = exactD || blend_exact::batch_depth_nonfinite(nB);
                        }
#pragma unroll
                        for (uint32_t k = 0; k < U1; ++k) {
                            const uint32_t j = (jn + k) & 63u;
                            const uint4 ra = lrecA[wv][j];
                            opn1[k] = ra.z;
                            const h2 pq = quad1(ra.x, ra.y, opn1[k]);
                            rgn1[k] = ra.w;
                            bdn1[k] = lrecB[wv][j];
                            const uint32_t pb = tbl_bits(pq);
                            en1[k].x = tbl[pb & 0xFFFFu];
                            en1[k].y = tbl[pb >> 16];
                        }
                    }
                    // stage 2: blend the current group
#pragma unroll
                    for (uint32_t k = 0; k < U1; ++k) {
                        const uint32_t tb = as_u32(T1);
                        const uint32_t gm = quad_max_u32(max(tb & 0xFFFFu, tb >> 16));
                        alive1 = alive1 && !(gm < thrBits);
                        if (alive1) {
                            const h2 rgv = as_h2(rgc1[k]), bdv = as_h2(bdc1[k]);
                            const h2 w = ac1[k] * T1;  // (GlobalShaders.metal:1137-1149)
                            T1 = T1 * om1[k];
                            R1 = blend_acc(R1, splat_lo(rgv), w);
                            G1 = blend_acc(G1, splat_hi(rgv), w);
                            B1 = blend_acc(B1, splat_lo(bdv), w);
                            D1 = blend_acc(D1, splat_hi(bdv), w);
                        }
                    }
                    e += U1;
                    if ((e & (kBlendExit - 1u)) == 0) {
                        if (e >= count || __ballot(alive1) == 0) break;
                    }
                    // stage 3: the next group's alphas
#pragma unroll
                    for (uint32_t k = 0; k < U1; ++k) {
                        const h2 ek = __builtin_bit_cast(h2, en1[k]);
                        ac1[k] = __builtin_elementwise_min(splat_hi(as_h2(opn1[k])) * ek, C099);
                        om1[k] = ONE - ac1[k];
                        rgc1[k] = rgn1[k];
                        bdc1[k] = bdn1[k];
                    }
                    if (e - bb == 64u) {
                        rotate(bb);
                        bb += 64u;
                    }
                }
                nproc = e;
                if (valid1) write_pair(px1, py1, ONE - T1, R1, G1, B1, D1);
                goto unit_end;
            }
        unit_done:;
        } else {
            if (claimMode != 1) claim();
        }
        // write (GlobalShaders.metal:1152-1186); empty tiles keep the clear colour (0,0,0,1)
#pragma unroll
        for (int q = 0; q < P; ++q)
            write_pair(ux + offX[q], uy + offY[q], (full > 0) ? (ONE - T[q]) : ONE, R[q], G[q], B[q], D[q]);
    unit_end:
        if (exactD)  // (rare: a record of inf / NaN fp16 depth; every pixel of the unit is written again)
            blend_exact::walk_unit_exact<P>((hsel ? half1 : half0) + start, count, rec, tbl, lrecA[wv], lrecB[wv], ux,
                                            uy, thrBits, write_pair);
        if (unitCost && lane == 0) unitCost[u] = (uint16_t)min(nproc, 65535u);
        waveMax = max(waveMax, min(nproc, 65535u));
        if (trace && lane == 0) {
            unsigned long long* t = trace + (size_t)u * 4;
            t[0] = tStart;
            t[1] = __builtin_amdgcn_s_memrealtime();
            t[2] = ((unsigned long long)count << 32) | nproc;
            const unsigned long long xcc = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (3 << 11));  // XCC_ID
            t[3] = (xcc << 48) | ((unsigned long long)(ncomp & 0xFFFFu) << 32) |
                   (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        }
        if (agePrio || topPrio) __builtin_amdgcn_s_setprio(0);
        topPrio = false;
        claim();  // (no-op when claimed during the walk)
        qi = gridWaves + stripe + stripes * __builtin_amdgcn_readfirstlane(nextQ);
    }
    if (unitCost && lane == 0 && waveMax) atomicMax(&costMax[(blockIdx.x * NW + wv) % kCostMaxSlots], waveMax);
    // multi-GPU frame gathered on rank 0 (gsm_multigpu.hip): the pixels were plain stores; the
    // workgroup's last exiting wave writes the XCD's L2 back at system scope (covering every wave of the
    // workgroup: each drained its stores before its count) and arrives at barrier 2 for the workgroup
    if (arrive.done) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(&exitCount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(old) == NW - 1u) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            mg_arrive_unit(arrive, blockIdx.x);
        }
    }
}



int blend_pairs_per_lane(uint32_t numTiles, int numCUs) {
    // Half tiles (2 pairs per lane) while the tiles outnumber the 8-wave slots; a smaller frame
    // or a slab of a multi-GPU frame has fewer units than slots, its blend time is its longest
    // unit's walk, and quadrant units (1 pair per lane, ~38 instead of ~61 VALU per entry)
    // shorten that (measured on 1/2, 1/4, 1/8 of the 1080p rows: 149/130/118 -> 138/105/96 us)
    return numTiles <= (uint32_t)numCUs * kBlendP1TilesPerCu ? 1 : 2;
}

uint32_t blend_units_per_tile(uint32_t numTiles, int numCUs) {
    return 4u / (uint32_t)blend_pairs_per_lane(numTiles, numCUs);
}

static int blend_waves_per_wg(uint32_t numTiles, int numCUs) {
    // 16 waves per CU hide more latency once every wave slot gets >= 6 units (4K: 16200 tiles);
    // with fewer units per slot the tail weighs more: 12 waves from 2 units per slot (1080p: 8160
    // units, 3213 -> 3268 frames/s; two 1440x1600 views 1046 -> 1086, r02 fused-accumulate blend),
    // 8 below (r03, late queue claim: DESIGN.md 10)
    const uint64_t units = (uint64_t)numTiles * blend_units_per_tile(numTiles, numCUs);
    if (units >= 6ull * (uint64_t)numCUs * 16u) return 16;
    return units >= 2ull * (uint64_t)numCUs * 12u ? 12 : 8;
}



// Measured schedule choices: units longest-first by last frame's walk (costOrder;
// 1080p 8 waves 293 -> 248 us, 4K 16 waves 703 -> 660), the longest on one top-priority wave per
// SIMD (flags bit 2), later units' priority rising with the age of their walk (flags bit 1).
int launch_blend(const FrameGeometry& g, const DeviceArena& A, void* color,
                  size_t colorPitch, void* depth, size_t depthPitch, int numCUs, bool costOrder, int colorFormat,
                  hipStream_t s, int wavesOverride, int claim, const MgArrive* arrive, bool pairs) {
    // local tile ids: tile t = k * tilesX + tx of the renderer's row k (pixel row rowBegin + k * rowStride)
    const uint32_t numTiles = g.rowCount * g.tilesX;
    if (numTiles == 0) return 0;
    const uint32_t t0 = 0;
    const int vec = ((((uintptr_t)color) & 15u) == 0 && (colorPitch & 15u) == 0 &&
                     (depth == nullptr || ((((uintptr_t)depth) & 7u) == 0 && (depthPitch & 7u) == 0)))
                        ? 1
                        : 0;
    const int flags = vec | 2 | (costOrder ? 4 : 0) | ((colorFormat & 15) << 4) | ((claim & 3) << 8) |
                      (arrive ? 4096 : 0) |  // (a gathered multi-GPU frame: the L2 write-back at exit)
                      ((depth && (((uintptr_t)depth) & 15u) == 0 && (depthPitch & 15u) == 0) ? 2048 : 0);
    // A.tileQueue was zeroed by k_scan_blocks earlier in the frame
    const int P = blend_pairs_per_lane(numTiles, numCUs);
    const int waves = wavesOverride ? wavesOverride : blend_waves_per_wg(numTiles, numCUs);
    // One GPU's half-tile frame with >= 6 units per wave slot (16 waves per CU: the 4K frame): two units
    // per wave (r05, k_blend_pw).  The pairs cut the VALU work (-10 %) but halve the waves walking: a gain
    // where the walk is VALU-bound (config 3: blend 370 -> 327 us), a loss where it is bound by its
    // longest units and latency (config 2: 121 -> 129-147 us at every split tried).
    if (pairs && P == 2 && !arrive && waves == 16) {
        launch_blend_pw(g, A, color, colorPitch, depth, depthPitch, numCUs, costOrder, colorFormat, s, waves);
        return GSM_BLEND_KERNEL_PAIR_WALK;
    }
    const uint32_t units = numTiles * (4u / (uint32_t)P);
    uint32_t grid = (units + (uint32_t)waves - 1) / (uint32_t)waves;
    if (grid > (uint32_t)numCUs) grid = (uint32_t)numCUs;
    const uint32_t* order = costOrder ? A.unitOrder : nullptr;
    MgArrive ar{};
    if (arrive) {
        ar = *arrive;
        ar.total = grid;  // every workgroup arrives once, at its exit
    }
#define GSM_LAUNCH_BLEND(NTH, PP, CMP)                                                                       \
    hipLaunchKernelGGL((k_blend_px<NTH, PP, CMP>), dim3(grid), dim3(NTH), 0, s, A.tileStart, A.rec, \
                       A.expTable, A.tileQueue, t0, numTiles, g.tilesX, g.width, g.height,          \
                       (uint8_t*)color, colorPitch, (uint8_t*)depth, depthPitch, flags, order, A.unitCost,  \
                       A.blendTrace, A.halfVals[0], A.halfVals[1], A.halfCount, g.tileCount, A.costMax, \
                       g.rowBegin, g.rowStride, ar)
    // half tiles compact to one pair per lane once <= 16 of their 32 groups are alive
    if (P == 1) {
        if (waves == 16) GSM_LAUNCH_BLEND(1024, 1, false);
        else if (waves == 12) GSM_LAUNCH_BLEND(768, 1, false);
        else GSM_LAUNCH_BLEND(512, 1, false);
    } else {
        if (waves == 16) GSM_LAUNCH_BLEND(1024, 2, true);
        else if (waves == 12) GSM_LAUNCH_BLEND(768, 2, true);
        else GSM_LAUNCH_BLEND(512, 2, true);
    }
#undef GSM_LAUNCH_BLEND
    return P == 1 ? GSM_BLEND_KERNEL_QUADRANT : GSM_BLEND_KERNEL_HALF_TILE;
}

}  // namespace gsm
