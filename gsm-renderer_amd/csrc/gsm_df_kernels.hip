// gsm_df_kernels.hip -- gfx950 kernels of the DepthFirst stereo side-by-side frame
// (SURVEY.md 8(f) rank 1).  Reference: Sources/Renderer/DepthFirstRenderer/DepthFirstShaders.metal
// and Sources/Renderer/Shared/GaussianShared.h; host order DepthFirstRenderer.swift:595-831.
//
// Frame: project both eyes once per gaussian (k_df_project) -> compact the visible ones with
// their 32-bit depth keys (k_df_compact) -> stable LSD depth sort (gsm_sort.hip) -> per-gaussian
// tile counts in depth order, scan, instance expansion of the union rect (k_df_icount,
// k_df_expand) -> stable LSD sort by tile id, its last pass writing the tile ranges
// (radix_sort_tiles) -> one persistent
// blend kernel that clears, composites each (tile, eye) of 16x16 pixels and writes the two eyes
// side by side with the copy pass's row flip (k_df_blend_eye).
// Numeric contract: DESIGN.md (built with -ffp-contract=off, IEEE div/sqrt); bit-exact with
// oracle/gsm_oracle.c og_df_render_stereo.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/gsm_renderer.h"
#include "gsm_detmath.h"
#include "gsm_device.h"
#include "gsm_df_internal.h"
#include "gsm_internal.h"
#include "gsm_types.h"

// The blend's kept entries' means are valid by construction (the per-entry mean test and the integer
// "every alpha is 0" test it replaced: tools/exp/rejected_variants.patch)

namespace gsm {

// ---------------------------------------------------------------------------
// 1. projection of both eyes (depthFirstStereoProjectCullKernel, DepthFirstShaders.metal:341-499)
// ---------------------------------------------------------------------------
// EyeProjectionResult (DepthFirstShaders.metal:236-247)
struct DfEyeOut {
    bool visible;
    float sx, sy, theta, s1, s2, detCov, depth;
    int tb[4];
};

// projectToEye (DepthFirstShaders.metal:249-339).  wp: scene-transformed position; C3: the
// covariance of the scene-scaled gaussian (the same for both eyes).
__device__ __forceinline__ DfEyeOut df_project_eye(const DfEyeConst& E, const DfArgs& P, const float wp[4],
                                                   const M3& C3) {
    DfEyeOut r;
    r.visible = false;
    r.sx = r.sy = r.theta = r.s1 = r.s2 = r.detCov = 0.0f;
    r.tb[0] = 0; r.tb[1] = -1; r.tb[2] = 0; r.tb[3] = -1;
    float vp[4], clip[4];
    m4_mul_v(E.view, wp, vp);
    m4_mul_v(E.proj, vp, clip);
    r.depth = clip[3];
    if (!(clip[3] > P.nearPlane)) return r;  // isInFrontOfCameraClipW
    if (r.depth > P.farPlane) return r;      // cullByFarPlane (GaussianShared.h:732-734)
    const float ndcx = clip[0] / clip[3], ndcy = clip[1] / clip[3];
    r.sx = (ndcx + 1.0f) * 0.5f * P.width;   // ndcToScreen (GaussianShared.h:150-155)
    r.sy = (ndcy + 1.0f) * 0.5f * P.height;
    Cov2 cov = project_cov2d(C3, vp, E.view, E.limX, E.limY, E.focalX, E.focalY);
    cov = stabilize_cov2d(cov, P.maxEig);
    float th, s1, s2;
    if (!theta_sigmas(cov, &th, &s1, &s2)) return r;
    r.theta = th;
    r.s1 = s1;
    r.s2 = s2;
    {
        const float a = cov.a, b = 0.5f * (cov.b + cov.c), d = cov.d;
        r.detCov = __builtin_fmaxf(a * d - b * b, 0.0f);
    }
    if (3.0f * __builtin_fmaxf(s1, s2) < 0.5f) return r;  // cullByRadius
    float ex, ey;
    obb_extents(cov, &ex, &ey);
    if (r.sx + ex < 0.0f || r.sx - ex > P.width || r.sy + ey < 0.0f || r.sy - ey > P.height) return r;
    // computeTileBounds (GaussianShared.h:791-828) on 16x16 tiles: x / 16 == x * (1/16) exactly
    const float maxW = P.width - 1.0f, maxH = P.height - 1.0f;
    const float xmin = clampf(r.sx - ex, 0.0f, maxW), xmax = clampf(r.sx + ex, 0.0f, maxW);
    const float ymin = clampf(r.sy - ey, 0.0f, maxH), ymax = clampf(r.sy + ey, 0.0f, maxH);
    int minTX = (int)__builtin_floorf(xmin * (1.0f / 16.0f));
    int maxTX = (int)__builtin_ceilf(xmax * (1.0f / 16.0f)) - 1;
    int minTY = (int)__builtin_floorf(ymin * (1.0f / 16.0f));
    int maxTY = (int)__builtin_ceilf(ymax * (1.0f / 16.0f)) - 1;
    r.tb[0] = max(minTX, 0);
    r.tb[1] = min(maxTX, (int)P.tilesX - 1);
    r.tb[2] = max(minTY, 0);
    r.tb[3] = min(maxTY, (int)P.tilesY - 1);
    r.visible = true;
    return r;
}

// float_to_sortable_uint (DepthFirstShaders.metal:33-37)
__device__ __forceinline__ uint32_t df_sortable(float v) {
    const uint32_t b = __builtin_bit_cast(uint32_t, v);
    return b ^ ((b & 0x80000000u) ? 0xFFFFFFFFu : 0x80000000u);
}

// the six fp16 fields of one eye in StereoTiledRenderData (DepthFirstShaders.metal:452-480):
// mean, conicFromThetaSigmas of the unquantised angle (GaussianShared.h:490-510; sin/cos of the
// numeric contract, det_sincos_theta), depth; an eye the gaussian misses gets mean -1e10 (-inf)
__device__ __forceinline__ void df_pack_eye(const DfEyeOut& e, uint32_t w[3]) {
    if (!e.visible) {
        const uint32_t hneg = f_to_hbits(-1e10f);
        w[0] = hneg | (hneg << 16);
        w[1] = 0;
        w[2] = 0;
        return;
    }
    float s, c;
    det_sincos_theta(e.theta, &s, &c);
    const float sig1 = __builtin_fmaxf(e.s1, 1e-4f), sig2 = __builtin_fmaxf(e.s2, 1e-4f);
    const float iv1 = 1.0f / (sig1 * sig1), iv2 = 1.0f / (sig2 * sig2);
    const float cc = c * c, ss = s * s, cs = c * s;
    const float A = cc * iv1 + ss * iv2;
    const float B = cs * (iv1 - iv2);
    const float C = ss * iv1 + cc * iv2;
    w[0] = (uint32_t)f_to_hbits(e.sx) | ((uint32_t)f_to_hbits(e.sy) << 16);
    w[1] = (uint32_t)f_to_hbits(A) | ((uint32_t)f_to_hbits(C) << 16);
    w[2] = (uint32_t)f_to_hbits(2.0f * B) | ((uint32_t)f_to_hbits(e.depth) << 16);
}

template <bool HALF, int DEG>
__global__ __launch_bounds__(kDfBlock) void k_df_project(const void* __restrict__ world,
                                                         const void* __restrict__ harm, DfArgs P,
                                                         StereoTiledRenderData* __restrict__ outRD,
                                                         short4* __restrict__ outBounds,
                                                         uint32_t* __restrict__ touchedOut,
                                                         uint32_t* __restrict__ depthKeys,
                                                         uint32_t* __restrict__ blockSums,
                                                         const uint16_t* __restrict__ unitCost,
                                                         uint32_t* __restrict__ unitOrder,
                                                         uint32_t* __restrict__ costMax) {
    __shared__ uint32_t lds[kDfBlock / 64];
    // block 0 of a scheduled launch orders the blend's (tile, eye) units from the previous frame's
    // walks while the other blocks project (unit_order_block; no side stream, no join)
    if (P.schedUnits) {
        if (blockIdx.x == 0) {
            __shared__ uint32_t uoBase[kUoBuckets], uoMax[kDfBlock / 64];
            unit_order_block<kDfBlock>(unitCost, unitOrder, P.schedUnits, uoBase, uoMax, costMax);
            return;
        }
    }
    const uint32_t blk = blockIdx.x - (P.schedUnits ? 1u : 0u);
    const uint32_t gid = blk * kDfBlock + threadIdx.x;
    uint32_t vis = 0;
    if (gid < P.count) {
        float pos[3], scale[3], rot[4], opacity;
        if constexpr (HALF) {
            const uint4* wq = (const uint4*)((const PackedWorldGaussianHalf*)world + gid);
            const uint4 w0 = wq[0], w1 = wq[1];
            pos[0] = __builtin_bit_cast(float, w0.x);
            pos[1] = __builtin_bit_cast(float, w0.y);
            pos[2] = __builtin_bit_cast(float, w0.z);
            opacity = hbits_to_f((uint16_t)(w0.w & 0xFFFFu));
            scale[0] = hbits_to_f((uint16_t)(w0.w >> 16));
            scale[1] = hbits_to_f((uint16_t)(w1.x & 0xFFFFu));
            scale[2] = hbits_to_f((uint16_t)(w1.x >> 16));
            rot[0] = hbits_to_f((uint16_t)(w1.y & 0xFFFFu));
            rot[1] = hbits_to_f((uint16_t)(w1.y >> 16));
            rot[2] = hbits_to_f((uint16_t)(w1.z & 0xFFFFu));
            rot[3] = hbits_to_f((uint16_t)(w1.z >> 16));
        } else {
            const float4* wq = (const float4*)((const PackedWorldGaussian*)world + gid);
            const float4 w0 = wq[0], w1 = wq[1], w2 = wq[2];
            pos[0] = w0.x; pos[1] = w0.y; pos[2] = w0.z; opacity = w0.w;
            scale[0] = w1.x; scale[1] = w1.y; scale[2] = w1.z;
            rot[0] = w2.x; rot[1] = w2.y; rot[2] = w2.z; rot[3] = w2.w;
        }
        // cullByScale (GaussianShared.h:719-722), alpha threshold (TileBinningParams 0.005)
        bool ok = !(__builtin_fmaxf(scale[0], __builtin_fmaxf(scale[1], scale[2])) < 0.0005f) &&
                  !(opacity < 0.005f);
        DfEyeOut L, R;
        L.visible = R.visible = false;
        if (ok) {
            const float p4[4] = {pos[0], pos[1], pos[2], 1.0f};
            float wp[4];
            m4_mul_v(P.scene, p4, wp);
            const float ss[3] = {scale[0] * P.sceneScale, scale[1] * P.sceneScale, scale[2] * P.sceneScale};
            const M3 C3 = build_cov3d(ss, rot);
            L = df_project_eye(P.eye[0], P, wp, C3);
            R = df_project_eye(P.eye[1], P, wp, C3);
            ok = L.visible || R.visible;
        }
        float checkDepth = 0.0f;
        if (ok) {
            checkDepth = L.visible ? L.depth : R.depth;
            if (L.visible && R.visible) checkDepth = (L.depth + R.depth) * 0.5f;
            float detCov = L.visible ? L.detCov : R.detCov;
            if (L.visible && R.visible) detCov = __builtin_fmaxf(L.detCov, R.detCov);
            // cullByTotalInk (GaussianShared.h:739-751) + computeDepthFactor (:275-278)
            const float ink = opacity * 6.283185f * __builtin_sqrtf(__builtin_fmaxf(detCov, 1e-12f));
            const float s = clampf((P.adjFar - checkDepth) / P.adjDen, 0.0f, 1.0f);
            const float depthFactor = 1.0f - s * s;
            if (ink < depthFactor * 2.0f) ok = false;
        }
        int ub[4] = {0, -1, 0, -1};
        uint32_t touched = 0;
        if (ok) {
            if (L.visible && R.visible) {
                ub[0] = min(L.tb[0], R.tb[0]);
                ub[1] = max(L.tb[1], R.tb[1]);
                ub[2] = min(L.tb[2], R.tb[2]);
                ub[3] = max(L.tb[3], R.tb[3]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) ub[q] = L.visible ? L.tb[q] : R.tb[q];
            }
            const int ux = max(ub[1] - ub[0] + 1, 0), uy = max(ub[3] - ub[2] + 1, 0);
            touched = (uint32_t)(ux * uy);
            if (touched == 0) ok = false;
        }
        if (ok) {
            float col[3];
            sh_color<HALF, DEG>(harm, gid, pos, P.mid, P.shComponents, col);
            col[0] = __builtin_fmaxf(col[0] + 0.5f, 0.0f);
            col[1] = __builtin_fmaxf(col[1] + 0.5f, 0.0f);
            col[2] = __builtin_fmaxf(col[2] + 0.5f, 0.0f);
            if (P.inputIsSRGB > 0.5f) {
                col[0] = srgb_to_linear(col[0]);
                col[1] = srgb_to_linear(col[1]);
                col[2] = srgb_to_linear(col[2]);
            }
            uint32_t wl[3], wr[3];
            df_pack_eye(L, wl);
            df_pack_eye(R, wr);
            const uint32_t cR = (uint32_t)(uint8_t)clampf(col[0] * 255.0f, 0.0f, 255.0f);
            const uint32_t cG = (uint32_t)(uint8_t)clampf(col[1] * 255.0f, 0.0f, 255.0f);
            const uint32_t cB = (uint32_t)(uint8_t)clampf(col[2] * 255.0f, 0.0f, 255.0f);
            const uint32_t cO = (uint32_t)(uint8_t)clampf(opacity * 255.0f, 0.0f, 255.0f);
            uint4* o = (uint4*)(outRD + gid);
            o[0] = make_uint4(wl[0], wl[1], wl[2], wr[0]);
            o[1] = make_uint4(wr[1], wr[2], cR | (cG << 8) | (cB << 16) | (cO << 24),
                              (uint32_t)f_to_hbits(checkDepth));
            outBounds[gid] = make_short4((short)ub[0], (short)ub[1], (short)ub[2], (short)ub[3]);
            touchedOut[gid] = touched;
            depthKeys[gid] = df_sortable(checkDepth);
            vis = 1;
        } else {
            outBounds[gid] = make_short4(0, -1, 0, -1);
            touchedOut[gid] = 0;
            depthKeys[gid] = 0xFFFFFFFFu;
        }
    }
    const uint32_t s = block_reduce_add<kDfBlock>(vis, lds);
    if (threadIdx.x == 0) blockSums[blk] = s;
}

// ---------------------------------------------------------------------------
// 2. compaction (visibilityScatterCompactKernel, DepthFirstShaders.metal:589-621): ascending id
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kDfBlock) void k_df_compact(uint32_t count, const uint32_t* __restrict__ touched,
                                                         const uint32_t* __restrict__ depthKeys,
                                                         const uint32_t* __restrict__ blockOffsets,
                                                         uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    __shared__ uint32_t lds[kDfBlock / 64];
    const uint32_t gid = blockIdx.x * kDfBlock + threadIdx.x;
    const uint32_t v = (gid < count && touched[gid] > 0u) ? 1u : 0u;
    uint32_t total;
    const uint32_t off = block_exclusive_scan<kDfBlock>(v, lds, &total);
    if (v) {
        const uint32_t o = blockOffsets[blockIdx.x] + off;
        keys[o] = depthKeys[gid];
        vals[o] = gid;
    }
}

// ---------------------------------------------------------------------------
// 3. instances in depth order (applyDepthOrderingKernel :623-640, prefix sum, then
//    createInstancesStereoKernel :790-826): gaussian i of the depth order writes its union rect's
//    tiles ty-major, tx-minor from its exclusive offset while below maxInstances
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kDfBlock) void k_df_icount(const TileAssignmentHeader* __restrict__ visHdr,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ touched,
                                                        uint32_t* __restrict__ sums) {
    __shared__ uint32_t lds[kDfBlock / 64];
    const uint32_t i = blockIdx.x * kDfBlock + threadIdx.x;
    const uint32_t V = visHdr->totalAssignments;
    const uint32_t c = i < V ? touched[order[i]] : 0u;
    const uint32_t s = block_reduce_add<kDfBlock>(c, lds);
    if (threadIdx.x == 0) sums[blockIdx.x] = s;
}

// DepthFirst skip flags: eye e of an entry provably contributes nothing to the 16x16 tile (x0, y0)
// -- every pixel has p in (9, +inf], where the stereo alpha is 0 (stereo_exp_table_entry), so the
// entry is an identity step of the blend for that eye (C + c * (0 * T) = C, T * (1 - 0) = T).  The
// rounding-error bound is quad_exceeds' (gsm_device.h).
typedef QuadBound DfEyeSkip;
__device__ __forceinline__ DfEyeSkip df_eye_skip_setup(uint32_t meanW, uint32_t ccW, uint32_t cxyW) {
    return quad_bound_setup(meanW, ccW, cxyW, true);
}
__device__ __forceinline__ bool df_eye_misses_tile(const DfEyeSkip& e, int x0, int y0) {
    return quad_exceeds(e, x0, y0, (int)kDfTile - 1, (int)kDfTile - 1, 9.0f);
}

// k_df_expand: the instances of the union rects (ty-major, tx-minor, DepthFirstShaders.metal:790-826),
// expanded cooperatively: the block's 256 gaussians (in depth order) get their offsets from one
// block scan, then thread t writes the block's instances t, t + 256, ... (consecutive threads,
// consecutive slots: coalesced stores, no thread walks a long rect alone), clamped to
// maxInstances.  Each instance also gets the blend's skip flags: bit kDfSkipShift + e of the
// gaussian id is set when eye e provably adds nothing to the instance's tile
// (df_eye_misses_tile, with each gaussian's per-eye setup computed once into LDS).
__global__ __launch_bounds__(kDfBlock) void k_df_expand(const TileAssignmentHeader* __restrict__ visHdr,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ touched,
                                                        const short4* __restrict__ bounds,
                                                        const uint32_t* __restrict__ blockOffsets,
                                                        const StereoTiledRenderData* __restrict__ rd,
                                                        uint32_t maxInstances, uint32_t tilesX,
                                                        uint32_t* __restrict__ tiles, uint32_t* __restrict__ gids) {
    __shared__ uint32_t lds[kDfBlock / 64];
    __shared__ uint32_t sOff[kDfBlock];
    __shared__ uint32_t sG[kDfBlock];
    __shared__ short4 sR[kDfBlock];
    __shared__ DfEyeSkip sE[2][kDfBlock];
    // the block's first kCandCap instances: owner << 8 | local index for rects of <= kCandRect
    // tiles, kSearch for the instances of larger rects (their owner comes from a binary search)
    constexpr uint32_t kCandCap = 4096, kCandRect = 64;
    constexpr uint16_t kSearch = 0xFFFFu;
    __shared__ uint16_t sCand[kCandCap];
    const uint32_t tid = threadIdx.x;
    const uint32_t i = blockIdx.x * kDfBlock + tid;
    const uint32_t V = visHdr->totalAssignments;
    const uint32_t g = i < V ? order[i] : 0u;
    const uint32_t c = i < V ? touched[g] : 0u;
    uint32_t total;
    const uint32_t off = block_exclusive_scan<kDfBlock>(c, lds, &total);
    sOff[tid] = off;
    sG[tid] = g;
    if (c > 0) {
        sR[tid] = bounds[g];
        const uint4 w0 = ((const uint4*)(rd + g))[0];
        const uint2 w1 = ((const uint2*)(rd + g))[2];
        sE[0][tid] = df_eye_skip_setup(w0.x, w0.y, w0.z);
        sE[1][tid] = df_eye_skip_setup(w0.w, w1.x, w1.y);
    }
    const uint32_t nCand = min(total, kCandCap);
    for (uint32_t j = tid; j < nCand; j += kDfBlock) sCand[j] = kSearch;
    __syncthreads();
    if (total == 0) return;
    if (c <= kCandRect)
        for (uint32_t j = 0; j < c && off + j < kCandCap; ++j) sCand[off + j] = (uint16_t)((tid << 8) | j);
    __syncthreads();
    const uint64_t base = (uint64_t)blockOffsets[blockIdx.x];
    for (uint32_t k = tid; k < total; k += kDfBlock) {
        const uint64_t wp = base + k;
        if (wp >= maxInstances) break;
        uint32_t lo, local;
        const uint32_t cv = k < kCandCap ? (uint32_t)sCand[k] : (uint32_t)kSearch;
        if (cv != kSearch) {
            lo = cv >> 8;
            local = cv & 0xFFu;
        } else {
            // owner: the last gaussian whose offset is <= k (gaussians without instances share an
            // offset with the next one, so the last of equal offsets is the one with instances)
            lo = 0;
            uint32_t hi = kDfBlock;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (sOff[mid] <= k) lo = mid; else hi = mid;
            }
            local = k - sOff[lo];
        }
        const short4 r = sR[lo];
        const uint32_t w = (uint32_t)(r.y - r.x + 1);
        // local / w from the hardware reciprocal (within one of the quotient), corrected exactly
        uint32_t dy = (uint32_t)((float)local * __builtin_amdgcn_rcpf((float)w));
        if (dy * w > local) dy--;
        else if ((dy + 1u) * w <= local) dy++;
        const uint32_t dx = local - dy * w;
        const int tx = r.x + (int)dx, ty = r.z + (int)dy;
        tiles[wp] = (uint32_t)(ty * (int)tilesX + tx) & 0xFFFFu;  // ushort tile id
        const int x0 = tx * (int)kDfTile, y0 = ty * (int)kDfTile;
        const uint32_t fl = (df_eye_misses_tile(sE[0][lo], x0, y0) ? 1u : 0u) |
                            (df_eye_misses_tile(sE[1][lo], x0, y0) ? 2u : 0u);
        gids[wp] = sG[lo] | (fl << kDfSkipShift);
    }
}

// ---------------------------------------------------------------------------
// 4. tile ranges (extractTileRangesKernel, DepthFirstShaders.metal:1258-1313): the reference's two
//    binary searches per tile become the tile starts the sort's last pass writes (radix_sort_tiles,
//    gsm_sort.hip); header t is {starts[t], starts[t + 1] - starts[t]} -- the lower bound for an
//    empty tile, {0, 0} for an empty frame (the debug copy rebuilds the reference's GaussianHeader
//    array from them)
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// 5. blend (clearStereoRenderTextureKernel :1813-1823, depthFirstStereoRender :1825-1982) and the
//    side-by-side copy (DepthFirstStereoCopyEncoder.swift:29-99, DepthFirstShaders.metal:1990-2018)
//
// Persistent workgroups, one per CU: the 128 KiB stereo alpha table sits in LDS and the waves
// pull (tile, eye) units from a device counter.  A lane is one reference thread: a 2x2 pixel
// group of one eye, held as packed fp16 pairs (row 0 = {x, x+1}, row 1).  The tile's list is
// walked in batches of records staged in the wave's LDS (the u8 colour and opacity turned into
// fp16 c/255 on the way), every entry read back as a uniform-address broadcast.  Per lane and
// entry the reference's control flow -- the
// joint break when both eyes' max transmittance < 1/255, the per-eye test, the all-zero skip and
// the r^2 > 9 cutoff -- is applied as data: an eye that is done, or a pixel past the cutoff
// (folded into the table, stereo_exp_table_entry), gets alpha 0, which leaves its colour and
// transmittance bit-identical (C + c * (0 * T) = C, T * (1 - 0) = T), and a dead lane stays
// dead (T never grows).  The wave leaves the list once every lane is done.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void df_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ h2 df_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t df_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2 df_lo(h2 v) { return h2{v.x, v.x}; }
__device__ __forceinline__ h2 df_hi(h2 v) { return h2{v.y, v.y}; }
typedef unsigned short df_u16x2 __attribute__((ext_vector_type(2)));
// `color += gColor * (a * trans)` (DepthFirstShaders.metal:1783-1786, 1909-1953): one fused
// multiply-add, a single rounding per channel (the numeric contract; the oracle's hfma)
__device__ __forceinline__ h2 df_acc(h2 acc, h2 c, h2 w) { return __builtin_elementwise_fma(c, w, acc); }

struct DfEyeState {
    h2 T[2], Cr[2], Cg[2], Cb[2];  // [row]: {x, x + 1}
};

// p = ((dx*dx)*cxx + (dy*dy)*cyy) + (dx*dy)*cxy2 for the lane's 2x2 pixels of one eye
// (DepthFirstShaders.metal:1881-1884); the x terms are shared by the rows, the y terms by the columns
__device__ __forceinline__ void df_quadform(h2 mean, h2 cc, h2 cxy, h2 PX, h2 PY, h2& p0, h2& p1) {
    const h2 dx = PX - df_lo(mean);
    const h2 dy = PY - df_hi(mean);
    const h2 ax = (dx * dx) * df_lo(cc);
    const h2 by = (dy * dy) * df_hi(cc);
    const h2 c2 = df_lo(cxy);
    p0 = (ax + df_lo(by)) + (dx * df_lo(dy)) * c2;
    p1 = (ax + df_hi(by)) + (dx * df_hi(dy)) * c2;
}

// some p of the 2x2 group is <= 9, negative or NaN (not every alpha is 0: the r^2 cutoff).  p > 9 holds
// exactly for the bits in [0x4881, 0x7C00]; IEEE-754-2019 minimum (v_pk_minimum3_f16) keeps NaN, so
// min(p0, p1) > 9 in both halves <=> all four p > 9 (one packed min and two ordered compares)
// -- as the wave's lane mask: one ballot per compare, so each compare's mask is used as it is
__device__ __forceinline__ uint64_t df_some_uncut_mask(h2 p0, h2 p1) {
    const h2 m = __builtin_elementwise_minimum(p0, p1);
    const h1 nine = (h1)9.0f;
    return __builtin_amdgcn_ballot_w64(!(m.x > nine)) | __builtin_amdgcn_ballot_w64(!(m.y > nine));
}

// one list entry for one eye of a lane (depthFirstStereoRender :1872-1913 / :1915-1956) from the
// quadratic forms: alpha = min(opacity * exp(-0.5 p), 0.99) with the r^2 cutoff folded into the
// table, forced to 0 for a lane whose eye is done, then C += c * (a * T), T *= 1 - a
__device__ __forceinline__ void df_blend_eye(DfEyeState& st, bool alive, h2 p0, h2 p1, h2 opr, h2 gb,
                                             const uint16_t* tbl) {
    const h2 ONE = {(h1)1.0f, (h1)1.0f};
    const h1 c099 = (h1)0.99;
    const h2 C099 = {c099, c099};
    const uint32_t b0 = df_u32(p0), b1 = df_u32(p1);
    df_u16x2 e0, e1;  // d16 loads straight into the halves
    e0.x = tbl[b0 & 0xFFFFu];
    e0.y = tbl[b0 >> 16];
    e1.x = tbl[b1 & 0xFFFFu];
    e1.y = tbl[b1 >> 16];
    const h2 op = df_lo(opr);
    h2 a0 = __builtin_elementwise_min(op * __builtin_bit_cast(h2, e0), C099);
    h2 a1 = __builtin_elementwise_min(op * __builtin_bit_cast(h2, e1), C099);
    if (!alive) {
        a0 = df_h2(0u);
        a1 = df_h2(0u);
    }
    const h2 w0 = a0 * st.T[0], w1 = a1 * st.T[1];
    const h2 r = df_hi(opr), g = df_lo(gb), b = df_hi(gb);
    st.Cr[0] = df_acc(st.Cr[0], r, w0);
    st.Cr[1] = df_acc(st.Cr[1], r, w1);
    st.Cg[0] = df_acc(st.Cg[0], g, w0);
    st.Cg[1] = df_acc(st.Cg[1], g, w1);
    st.Cb[0] = df_acc(st.Cb[0], b, w0);
    st.Cb[1] = df_acc(st.Cb[1], b, w1);
    st.T[0] = st.T[0] * (ONE - a0);
    st.T[1] = st.T[1] * (ONE - a1);
}

// the same step from the staged words of k_df_blend_eye: opacity = hi(zw), r = lo(rg), g = hi(rg),
// b = lo(bw), each used in place through op_sel
__device__ __forceinline__ void df_blend_eye_w(DfEyeState& st, bool alive, h2 p0, h2 p1, uint32_t zw, uint32_t rg,
                                               uint32_t bw, const uint16_t* tbl) {
    const h2 ONE = {(h1)1.0f, (h1)1.0f};
    const h1 c099 = (h1)0.99;
    const h2 C099 = {c099, c099};
    // a lane whose eye is done keeps C and T (alpha 0 would leave the same bits: C + c * 0 == C,
    // T * 1 == T): its updates run under an EXEC mask of the live lanes instead of zeroing its alphas
    if (!alive) return;
    const uint32_t b0 = df_u32(p0), b1 = df_u32(p1);
    df_u16x2 e0, e1;
    e0.x = tbl[b0 & 0xFFFFu];
    e0.y = tbl[b0 >> 16];
    e1.x = tbl[b1 & 0xFFFFu];
    e1.y = tbl[b1 >> 16];
    const h2 op = df_hi(df_h2(zw));
    h2 a0 = __builtin_elementwise_min(op * __builtin_bit_cast(h2, e0), C099);
    h2 a1 = __builtin_elementwise_min(op * __builtin_bit_cast(h2, e1), C099);
    const h2 w0 = a0 * st.T[0], w1 = a1 * st.T[1];
    const h2 r = df_lo(df_h2(rg)), g = df_hi(df_h2(rg)), b = df_lo(df_h2(bw));
    st.Cr[0] = df_acc(st.Cr[0], r, w0);
    st.Cr[1] = df_acc(st.Cr[1], r, w1);
    st.Cg[0] = df_acc(st.Cg[0], g, w0);
    st.Cg[1] = df_acc(st.Cg[1], g, w1);
    st.Cb[0] = df_acc(st.Cb[0], b, w0);
    st.Cb[1] = df_acc(st.Cb[1], b, w1);
    st.T[0] = st.T[0] * (ONE - a0);
    st.T[1] = st.T[1] * (ONE - a1);
}

// max transmittance of a lane's 4 pixels >= fp16(1/255); T >= 0, so fp16 order is bit order
__device__ __forceinline__ bool df_alive(const DfEyeState& st, uint32_t thrBits) {
    const df_u16x2 m = __builtin_elementwise_max(__builtin_bit_cast(df_u16x2, st.T[0]),
                                                 __builtin_bit_cast(df_u16x2, st.T[1]));
    return max((uint32_t)m.x, (uint32_t)m.y) >= thrBits;
}

// k_df_blend_eye: one wave per (tile, eye) unit.  An eye's updates only depend on its own
// transmittance (the per-eye test maxTrans >= 1/255 of :1872 and :1915 is monotone, and the joint
// break of :1866 fires only once both eyes' tests fail), so the two eyes of a tile are independent
// walks: each stops when its own lanes are all done, and 2 x tiles units balance better than tiles.
// Lane l stages record l of the 64-entry batch: the eye's mean and conic and the fp16 opacity and
// colour (uint4 + uint), read back per entry as uniform-address broadcasts.
constexpr uint32_t kDfEyeBatch = 64;
template <int NW, bool STATS>
__global__ __launch_bounds__(NW * 64) void k_df_blend_eye(const uint32_t* __restrict__ starts,
                                                          const uint32_t* __restrict__ gids,
                                                          const StereoTiledRenderData* __restrict__ rd,
                                                          const uint16_t* __restrict__ expTable,
                                                          uint32_t* __restrict__ queue, uint32_t tilesX,
                                                          uint32_t tileCount, uint32_t W, uint32_t H,
                                                          uint8_t* __restrict__ color, size_t pitch, int fmt,
                                                          const uint32_t* __restrict__ order,
                                                          uint16_t* __restrict__ unitCost, int flags,
                                                          unsigned long long* __restrict__ stats,
                                                          uint32_t* __restrict__ costMax) {
    __shared__ __attribute__((aligned(16))) uint16_t tbl[65536];
    __shared__ __attribute__((aligned(16))) uint4 stageA[NW][kDfEyeBatch];
    __shared__ __attribute__((aligned(16))) uint32_t stageB[NW][kDfEyeBatch];
    __shared__ uint16_t div255[256];
    {
        // (a loop of load / wait / store per 16 B here: GSM_EXP_TABLE_TO_LDS's batched fill measured slower
        // for this kernel, 333.5 -> 340.5 us at config 5, profiles/r06_exp_table_fill_ab.txt)
        const uint4* src = (const uint4*)expTable;
        uint4* dst = (uint4*)tbl;
        for (int i = threadIdx.x; i < 65536 * 2 / 16; i += NW * 64) dst[i] = src[i];
        if (threadIdx.x < 256) div255[threadIdx.x] = f_to_hbits((float)threadIdx.x / 255.0f);  // getColor
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t thrBits = (uint32_t)f_to_hbits(1.0f / 255.0f);  // half(1.0h / 255.0h)
    const uint32_t bpp = fmt == GSM_COLOR_FORMAT_RGBA16F ? 8u : (fmt == GSM_COLOR_FORMAT_RGBA32F ? 16u : 4u);
    const h2 ONE = {(h1)1.0f, (h1)1.0f};
    uint4* sA = stageA[wave];
    uint32_t* sB = stageB[wave];
    const uint32_t units = 2u * tileCount;
    // First unit static, then the queue.  With the schedule on (flags bit 1) one wave per SIMD
    // takes one of the gridDim.x * 4 longest units first and runs it at the top priority, so each
    // SIMD pairs its longest walk with shorter ones (the makespan is the longest walk's); with
    // flags bit 0 a walk's priority rises with its age.
    constexpr uint32_t NTOP = 4;
    const bool split = (flags & 2) != 0 && order != nullptr, agePrio = (flags & 1) != 0;
    uint32_t qi = !split ? blockIdx.x * NW + wave
                         : (wave < NTOP ? blockIdx.x * NTOP + wave
                                        : gridDim.x * NTOP + blockIdx.x * (NW - NTOP) + (wave - NTOP));
    bool topPrio = split && wave < NTOP;
    uint32_t waveMax = 0;  // this wave's longest walk, for the next frame's schedule (costMax)
    // dynamic units from the workgroup's stripe of the queue (kQueueStripes, gsm_internal.h)
    const uint32_t stripes = (gridDim.x % kQueueStripes) == 0 ? kQueueStripes : 1u;
    const uint32_t stripe = blockIdx.x % stripes;
    for (;; topPrio = false) {
        if (qi >= units) break;
        uint32_t u = order ? __builtin_amdgcn_readfirstlane(order[qi]) : qi;
        if (u >= units) u = qi;  // a schedule is a permutation of [0, units); never trust it further
        const uint32_t t = u >> 1, eye = u & 1u;
        const uint32_t st0 = starts[t];
        const uint2 hd = make_uint2(st0, starts[t + 1] - st0);
        const uint32_t tileX = t % tilesX, tileY = t / tilesX;
        const uint32_t bx = tileX * kDfTile + (lane & 7u) * 2u, by = tileY * kDfTile + (lane >> 3) * 2u;
        const h2 PX = {(h1)(float)bx, (h1)(float)(bx + 1u)};
        const h2 PY = {(h1)(float)by, (h1)(float)(by + 1u)};
        DfEyeState E;
        E.T[0] = E.T[1] = ONE;
        E.Cr[0] = E.Cr[1] = E.Cg[0] = E.Cg[1] = E.Cb[0] = E.Cb[1] = df_h2(0u);
        bool done = false;
        bool alive = true;  // the lane's max T >= 1/255 (df_alive; T = 1 at the start)
        uint64_t aliveM = __builtin_amdgcn_ballot_w64(true);  // ... as the wave's lane mask
        uint32_t walked = hd.y;  // entries this unit walked (its cost for the next frame's order)
        uint32_t nValid = 0, nBlend = 0;  // STATS: entries with a real mean / with a blend step
        // Loads run one batch ahead: while batch k blends, the records of batch k + 1 and the ids of
        // batch k + 2 are in flight.  They are unpredicated (index clamped to the list, so every lane
        // holds a valid id) -- a predicated load would merge with the old register and force its
        // wait into the loop.
        const uint32_t* lst = gids + hd.x;
        const uint32_t last = hd.y > 0 ? hd.y - 1u : 0u;
        uint32_t gwA = 0, gwB = 0;
        uint4 rcA = make_uint4(0u, 0u, 0u, 0u);
        if (hd.y > 0) {
            gwA = lst[min(lane, last)];
            const uint32_t* w = (const uint32_t*)(rd + (gwA & kDfGidMask));
            rcA = make_uint4(w[3 * eye], w[3 * eye + 1], w[3 * eye + 2], w[6]);
            gwB = lst[min(kDfEyeBatch + lane, last)];
        }
        for (uint32_t b0 = 0; b0 < hd.y && !done; b0 += kDfEyeBatch) {
            const uint32_t n = min(kDfEyeBatch, hd.y - b0);
            if (topPrio) {
                if (b0 == 0) __builtin_amdgcn_s_setprio(3);
            } else if (agePrio) {
                if (b0 == 0) __builtin_amdgcn_s_setprio(1);
                else if (b0 == 128u) __builtin_amdgcn_s_setprio(2);
                else if (b0 == 320u && !split) __builtin_amdgcn_s_setprio(3);
            }
            // the batch's entries not flagged for this eye (k_df_expand), compacted in list order (the
            // flagged ones are identity steps)
            const uint32_t gw = gwA;
            const uint4 rc = rcA;
            const bool keep = lane < n && !((gw >> (kDfSkipShift + eye)) & 1u);
            const uint64_t km = __builtin_amdgcn_ballot_w64(keep);
            // (two 32-bit counts: the batch-end tests below then stay scalar compares)
            const uint32_t nk = (uint32_t)__builtin_popcount((uint32_t)km) + (uint32_t)__builtin_popcount((uint32_t)(km >> 32));
            // next batch's records, and the ids of the one after
            {
                const uint32_t* w = (const uint32_t*)(rd + (gwB & kDfGidMask));
                rcA = make_uint4(w[3 * eye], w[3 * eye + 1], w[3 * eye + 2], w[6]);
                gwA = gwB;
                gwB = lst[min(b0 + 2u * kDfEyeBatch + lane, last)];
            }
            if (keep) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u));
                const uint32_t c = rc.w;  // colorR, G, B, opacity (bytes 24..27)
                sA[pos] = make_uint4(rc.x, rc.y, (rc.z & 0xFFFFu) | ((uint32_t)div255[c >> 24] << 16),
                                     (uint32_t)div255[c & 0xFFu] | ((uint32_t)div255[(c >> 8) & 0xFFu] << 16));
                sB[pos] = (uint32_t)div255[(c >> 16) & 0xFFu];
            }
            df_wave_sync();
            for (uint32_t j0 = 0; j0 < nk; j0 += 4) {
#pragma unroll
                for (uint32_t jj = 0; jj < 4; ++jj) {
                    const uint32_t j = j0 + jj;
                    const uint4 ra = sA[j];
                    // a kept entry's mean passes the reference's mean test (gMean.x >= -60000): an
                    // eye whose mean fails it is flagged by k_df_expand (quad_bound_setup mode 1), so
                    // the only test left is the batch's end (uniform, no pad records)
                    const uint32_t mw = ra.x;
                    if (j < nk) {
                        h2 p0, p1;
                        df_quadform(df_h2(mw), df_h2(ra.y), df_h2(ra.z), PX, PY, p0, p1);
                        if (STATS) nValid++;
                        const uint64_t some = df_some_uncut_mask(p0, p1);
                        if ((some & aliveM) != 0) {
                            df_blend_eye_w(E, alive, p0, p1, ra.z, ra.w, sB[j], tbl);
                            // T changes only here, so the per-eye test (:1872 / :1915) of the next
                            // entry is the test of the updated T (a done lane's T is unchanged and
                            // stays below 1/255); the wave leaves once every lane is done
                            alive = df_alive(E, thrBits);
                            aliveM = __builtin_amdgcn_ballot_w64(alive);
                            if (STATS) nBlend++;
                            if (aliveM == 0) {
                                done = true;
                                break;
                            }
                        }
                    }
                }
                if (done) {
                    walked = b0 + n;  // list entries traversed (a cost estimate for the schedule)
                    break;
                }
            }
            df_wave_sync();  // the stage is rewritten by the next batch
        }
        if (agePrio || topPrio) __builtin_amdgcn_s_setprio(0);
        uint32_t nq = 0;
        if (lane == 0) nq = atomicAdd(queue + stripe * kQueueStride, 1u);
        qi = gridDim.x * NW + stripe + stripes * __builtin_amdgcn_readfirstlane(nq);
        if (unitCost && lane == 0) unitCost[u] = (uint16_t)min(walked, 65535u);
        waveMax = max(waveMax, min(walked, 65535u));
        if (STATS && lane == 0) {
            atomicAdd(&stats[0], (unsigned long long)walked);
            atomicAdd(&stats[1], (unsigned long long)nValid);
            atomicAdd(&stats[2], (unsigned long long)nBlend);
            atomicAdd(&stats[3], (unsigned long long)hd.y);
        }
        // (C, 1 - T) of the eye's pixel (x, y) lands in target row H - 1 - y, column eye * W + x; a
        // tile with an empty list is not an active tile and keeps the clear value (0, 0, 0, 1)
        const uint32_t clearA = hd.y == 0 ? 0x3C003C00u : 0u;
#pragma unroll
        for (int row = 0; row < 2; ++row) {
            const uint32_t y = by + (uint32_t)row;
            if (y >= H) continue;
            uint8_t* trow = color + (size_t)(H - 1u - y) * pitch + (size_t)eye * W * bpp;
            const uint32_t ur = df_u32(E.Cr[row]), ug = df_u32(E.Cg[row]);
            const uint32_t ub = df_u32(E.Cb[row]), ua = df_u32(ONE - E.T[row]) | clearA;
            if (bx < W)
                store_color_px(fmt, (char*)(trow + (size_t)bx * bpp), (ur & 0xFFFFu) | (ug << 16),
                               (ub & 0xFFFFu) | (ua << 16));
            if (bx + 1u < W)
                store_color_px(fmt, (char*)(trow + (size_t)(bx + 1u) * bpp), (ur >> 16) | (ug & 0xFFFF0000u),
                               (ub >> 16) | (ua & 0xFFFF0000u));
        }
    }
    if (unitCost && lane == 0 && waveMax) atomicMax(&costMax[(blockIdx.x * NW + wave) % kCostMaxSlots], waveMax);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <bool HALF>
static void df_launch_project_t(uint32_t deg, const void* world, const void* harm, const DfArgs& a,
                                const DfArena& A, hipStream_t s) {
    const uint32_t blocks = (a.count + kDfBlock - 1) / kDfBlock;
    if (blocks == 0 && a.schedUnits == 0) return;  // (an empty frame still orders its blend units)
#define GSM_DF_PROJ(D)                                                                                   \
    hipLaunchKernelGGL((k_df_project<HALF, D>), dim3(blocks + (a.schedUnits ? 1u : 0u)), dim3(kDfBlock), 0, s,  \
                       world, harm, a, A.renderData, A.bounds, A.touched, A.depthKeys, A.blockSums, A.unitCost, \
                       A.unitOrder, A.costMax)
    switch (deg) {
        case 0: GSM_DF_PROJ(0); break;
        case 1: GSM_DF_PROJ(1); break;
        case 2: GSM_DF_PROJ(2); break;
        default: GSM_DF_PROJ(3); break;
    }
#undef GSM_DF_PROJ
}

void df_launch_project(bool halfInput, uint32_t deg, const void* world, const void* harm, const DfArgs& a,
                       const DfArena& A, hipStream_t s) {
    if (halfInput) df_launch_project_t<true>(deg, world, harm, a, A, s);
    else df_launch_project_t<false>(deg, world, harm, a, A, s);
}

void df_launch_compact(const DfArgs& a, const DfArena& A, hipStream_t s) {
    const uint32_t blocks = (a.count + kDfBlock - 1) / kDfBlock;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_df_compact, dim3(blocks), dim3(kDfBlock), 0, s, a.count, A.touched, A.depthKeys,
                       A.blockSums, A.dkeys[0], A.dvals[0]);
}

void df_launch_instance_counts(const uint32_t* order, const DfArgs& a, const DfArena& A, hipStream_t s) {
    const uint32_t blocks = (a.count + kDfBlock - 1) / kDfBlock;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_df_icount, dim3(blocks), dim3(kDfBlock), 0, s, A.visHdr, order, A.touched, A.instSums);
}

void df_launch_instances(const uint32_t* order, const DfArgs& a, const DfArena& A, hipStream_t s) {
    const uint32_t blocks = (a.count + kDfBlock - 1) / kDfBlock;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_df_expand, dim3(blocks), dim3(kDfBlock), 0, s, A.visHdr, order, A.touched, A.bounds,
                       A.instSums, A.renderData, a.maxInstances, a.tilesX, A.ikeys[0], A.ivals[0]);
}

constexpr int kDfBlendWaves = 16;
void df_launch_blend(const uint32_t* sortedGids, const DfArgs& a, const DfArena& A, void* color, size_t pitch,
                     int colorFormat, int numCUs, bool costOrder, hipStream_t s) {
    uint32_t grid = (uint32_t)(numCUs > 0 ? numCUs : 256);
    const uint32_t need = (2u * a.tileCount + kDfBlendWaves - 1) / kDfBlendWaves;
    if (grid > need) grid = need;
    if (grid == 0) return;
    // one wave per (tile, eye); age-raised priority (bit 0) and the longest first units on one
    // top-priority wave per SIMD (bit 1), as the Global blend
    const int flags = 1 | 2;
    if (A.blendStats)
        hipLaunchKernelGGL((k_df_blend_eye<kDfBlendWaves, true>), dim3(grid), dim3(kDfBlendWaves * 64), 0, s,
                           A.starts, sortedGids, A.renderData, A.expTable, A.queue, a.tilesX, a.tileCount,
                           (uint32_t)a.width, (uint32_t)a.height, (uint8_t*)color, pitch, colorFormat,
                           costOrder ? (const uint32_t*)A.unitOrder : nullptr, A.unitCost, flags, A.blendStats,
                           A.costMax);
    else
        hipLaunchKernelGGL((k_df_blend_eye<kDfBlendWaves, false>), dim3(grid), dim3(kDfBlendWaves * 64), 0, s,
                           A.starts, sortedGids, A.renderData, A.expTable, A.queue, a.tilesX, a.tileCount,
                           (uint32_t)a.width, (uint32_t)a.height, (uint8_t*)color, pitch, colorFormat,
                           costOrder ? (const uint32_t*)A.unitOrder : nullptr, A.unitCost, flags, nullptr,
                           A.costMax);
}

}  // namespace gsm
