// gsm_kernels.hip -- gfx950 kernels of the GlobalRenderer frame (except the sort).
//
// Reference: Sources/Renderer/GlobalRenderer/GlobalShaders.metal and
// Sources/Renderer/Shared/GaussianShared.h (paths relative to the reference root).
// Numeric contract: DESIGN.md (built with -ffp-contract=off, IEEE div/sqrt).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "gsm_device.h"
#include "gsm_detmath.h"
#include "gsm_internal.h"
#include "gsm_types.h"



namespace gsm {

// ---------------------------------------------------------------------------
// 1. project + cull + SH colour + tile count  (globalProjectCull, GlobalShaders.metal:19-123;
//    tileCountIndirectKernel, :563-616)
// ---------------------------------------------------------------------------
// Per-gaussian projection (globalProjectCull, GlobalShaders.metal:19-123, and the per-gaussian
// values of globalRender): everything one gaussian contributes before tile assignment.
struct ProjOut {
    uint4 rd;          // GaussianRenderData
    BlendRecordA ra;   // blend record (mean, conic, opacity, r, g)
    uint32_t rb;       // blend record (b, depth)
    short4 bounds;     // tile rect, (0,-1,0,-1) when culled
    float cmx, cmy, w; // fp16-rounded mean, intersection level
    Conic k;
    bool vis, countable;
};

// The per-block byte table: fp16(float(c) / 255) (getColor/getOpacity, GlobalShaders.metal:9-15) and the
// tile-test level 2 computePower(c) (tileCountIndirectKernel, GlobalShaders.metal:563-616) of every u8
// channel value c, one entry per thread of the block, copied from the host-built entries behind the sincos
// table (det_byte_lut_entry; r06: the per-gaussian division and log2 they replace were ~3% of k_project's
// VALU).  Callers use it after the barrier.
static_assert(kProjectBlock == 256, "one byte-table entry per thread");
struct ByteLut {
    uint16_t div255[256];
    float level[256];
};
// fp16 input: the gaussian's 32-B world record loaded before the byte table's load and barrier, so the
// two memory round trips overlap (r06)
template <bool HALF>
__device__ __forceinline__ void preload_world(const void* __restrict__ world, uint32_t gid, uint32_t count, uint4 (&w)[2]) {
    w[0] = w[1] = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (HALF) {
        if (gid < count) {
            const uint4* wp = (const uint4*)((const PackedWorldGaussianHalf*)world + gid);
            w[0] = wp[0];
            w[1] = wp[1];
        }
    }
}
__device__ __forceinline__ void fill_byte_lut(ByteLut& L, const float2* __restrict__ sincos) {
    const uint2 e = ((const uint2*)(sincos + kSincosEntries))[threadIdx.x];
    L.level[threadIdx.x] = __uint_as_float(e.x);
    L.div255[threadIdx.x] = (uint16_t)e.y;
    __syncthreads();
}


template <bool HALF, int DEG>
__device__ __forceinline__ ProjOut project_gaussian(const void* __restrict__ world,
                                                    const void* __restrict__ harm, uint32_t gid,
                                                    const ProjectArgs& P,
                                                    const float2* __restrict__ sincos,
                                                    const ByteLut& lut, const uint4* preWorld = nullptr) {
    ProjOut o;
    o.vis = false;
    o.countable = false;
    o.bounds = make_short4(0, -1, 0, -1);
    {
        const CameraUniforms& cam = P.cam;
        float pos[3], scale[3], rot[4], opacity;
        if constexpr (HALF) {
            uint4 w0, w1;
            if (preWorld) {  // loaded by the kernel before the byte table's barrier
                w0 = preWorld[0];
                w1 = preWorld[1];
            } else {
                const uint4* wp = (const uint4*)((const PackedWorldGaussianHalf*)world + gid);
                w0 = wp[0];
                w1 = wp[1];
            }
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
            const float4* wp = (const float4*)((const PackedWorldGaussian*)world + gid);
            float4 w0 = wp[0], w1 = wp[1], w2 = wp[2];
            pos[0] = w0.x; pos[1] = w0.y; pos[2] = w0.z; opacity = w0.w;
            scale[0] = w1.x; scale[1] = w1.y; scale[2] = w1.z;
            rot[0] = w2.x; rot[1] = w2.y; rot[2] = w2.z; rot[3] = w2.w;
        }
        bool vis = true;
        // cullByScale (GaussianShared.h:719-722)
        if (__builtin_fmaxf(scale[0], __builtin_fmaxf(scale[1], scale[2])) < 0.0005f) vis = false;
        float vp[4], clip[4];
        if (vis) {
            const float p4[4] = {pos[0], pos[1], pos[2], 1.0f};
            m4_mul_v(cam.view, p4, vp);
            m4_mul_v(cam.proj, vp, clip);
            if (!(clip[3] > cam.nearPlane)) vis = false;  // isInFrontOfCameraClipW
        }
        float sx = 0.f, sy = 0.f;
        if (vis) {
            float ndc[2] = {clip[0], clip[1]};
            div_many(ndc, clip[3]);  // clip / w, each correctly rounded (w > near > 0)
            const float ndcx = ndc[0], ndcy = ndc[1];
            sx = ((ndcx + 1.0f) * cam.width - 1.0f) * 0.5f;  // ndcToScreenCentered
            sy = ((ndcy + 1.0f) * cam.height - 1.0f) * 0.5f;
            if (opacity < P.bin.alphaThreshold) vis = false;
        }
        Cov2 cov;
        float theta = 0.f, s1 = 0.f, s2 = 0.f;
        if (vis) {
            // buildCovariance3D, projectCovariance2D, stabilizeCovariance2D, covarianceToThetaSigmas
            // (GaussianShared.h:289-324, 326-375, 655-714, 446-488; gsm_device.h)
            const M3 C3 = build_cov3d(scale, rot);
            cov = project_cov2d(C3, vp, cam.view, P.limX, P.limY, P.focalX, P.focalY);
            cov = stabilize_cov2d(cov, P.maxEig);
            if (!theta_sigmas(cov, &theta, &s1, &s2)) vis = false;
        }
        if (vis) {
            float radius = 3.0f * __builtin_fmaxf(s1, s2);
            if (radius < 0.5f) vis = false;  // cullByRadius
        }
        if (vis && P.bin.totalInkThreshold > 0.0f) {  // cullByTotalInkFromCov
            float a = cov.a, b = 0.5f * (cov.b + cov.c), d = cov.d;
            float det = a * d - b * b;
            float ink = opacity * 6.283185f * sqrt_cr(__builtin_fmaxf(det, 1e-12f));
            float s = clampf((P.adjFar - clip[3]) / P.adjDen, 0.0f, 1.0f);
            float depthFactor = 1.0f - s * s;
            if (ink < depthFactor * P.bin.totalInkThreshold) vis = false;
        }
        float ex = 0.f, ey = 0.f;
        if (vis) {  // computeOBBExtents (GaussianShared.h:402-427)
            obb_extents(cov, &ex, &ey);
            // cullByScreenBounds (GaussianShared.h:771-781)
            if (sx + ex < 0.0f || sx - ex > cam.width || sy + ey < 0.0f || sy - ey > cam.height)
                vis = false;
        }
        if (vis) {
            float col[3];
            sh_color<HALF, DEG>(harm, gid, pos, cam.cameraCenter, cam.shComponents, col);
            col[0] = __builtin_fmaxf(col[0] + 0.5f, 0.0f);
            col[1] = __builtin_fmaxf(col[1] + 0.5f, 0.0f);
            col[2] = __builtin_fmaxf(col[2] + 0.5f, 0.0f);
            if (cam.inputIsSRGB > 0.5f) {
                col[0] = srgb_to_linear(col[0]);
                col[1] = srgb_to_linear(col[1]);
                col[2] = srgb_to_linear(col[2]);
            }
            // pack GaussianRenderData (GlobalShaders.metal:106-117), packThetaPi (GaussianShared.h:434-440)
            float th = fmod_pi(theta);
            if (th < 0.0f) th = th + kPiF;
            float u = th * (65535.0f / kPiF);
            uint16_t thq = (uint16_t)clampf(u + 0.5f, 0.0f, 65535.0f);
            uint16_t hmx = f_to_hbits(sx), hmy = f_to_hbits(sy);
            uint16_t hs1 = f_to_hbits(s1), hs2 = f_to_hbits(s2), hd = f_to_hbits(clip[3]);
            uint32_t cR = (uint32_t)(uint8_t)clampf(col[0] * 255.0f, 0.0f, 255.0f);
            uint32_t cG = (uint32_t)(uint8_t)clampf(col[1] * 255.0f, 0.0f, 255.0f);
            uint32_t cB = (uint32_t)(uint8_t)clampf(col[2] * 255.0f, 0.0f, 255.0f);
            uint32_t cO = (uint32_t)(uint8_t)clampf(opacity * 255.0f, 0.0f, 255.0f);
            uint4 rdw;
            rdw.x = (uint32_t)hmx | ((uint32_t)hmy << 16);
            rdw.y = (uint32_t)thq | ((uint32_t)hs1 << 16);
            rdw.z = (uint32_t)hs2 | ((uint32_t)hd << 16);
            rdw.w = cR | (cG << 8) | (cB << 16) | (cO << 24);
            o.rd = rdw;

            // computeTileBounds (GaussianShared.h:791-828)
            float maxW = cam.width - 1.0f, maxH = cam.height - 1.0f;
            float xmin = clampf(sx - ex, 0.0f, maxW), xmax = clampf(sx + ex, 0.0f, maxW);
            float ymin = clampf(sy - ey, 0.0f, maxH), ymax = clampf(sy + ey, 0.0f, maxH);
            // x / 32 and y / 16: division by a power of two equals the product with its inverse
            static_assert(kTileWidth == 32 && kTileHeight == 16, "tile size");
            int minTX = (int)__builtin_floorf(xmin * (1.0f / 32.0f));
            int maxTX = (int)__builtin_ceilf(xmax * (1.0f / 32.0f)) - 1;
            int minTY = (int)__builtin_floorf(ymin * (1.0f / 16.0f));
            int maxTY = (int)__builtin_ceilf(ymax * (1.0f / 16.0f)) - 1;
            minTX = max(minTX, 0);
            minTY = max(minTY, 0);
            maxTX = min(maxTX, (int)P.bin.tilesX - 1);
            maxTY = min(maxTY, (int)P.bin.tilesY - 1);
            o.bounds = make_short4((short)minTX, (short)maxTX, (short)minTY, (short)maxTY);

            // per-gaussian values of globalRender (GlobalShaders.metal:1094-1105; getColor/getOpacity :9-15)
            float cmx = hbits_to_f(hmx), cmy = hbits_to_f(hmy);
            Conic k = conic_from_quant(sincos, thq, hbits_to_f(hs1), hbits_to_f(hs2));
            uint16_t hcxx = f_to_hbits(k.A), hcyy = f_to_hbits(k.C), hcxy2 = f_to_hbits(2.0f * k.B);
            // fp16(float(c) / 255) for the u8 channels: the block's byte table
            uint16_t hop = lut.div255[cO];
            uint16_t hr = lut.div255[cR], hg = lut.div255[cG];
            uint16_t hb = lut.div255[cB];
            BlendRecordA ra;
            ra.x = rdw.x;
            ra.y = (uint32_t)hcxx | ((uint32_t)hcyy << 16);
            ra.z = (uint32_t)hcxy2 | ((uint32_t)hop << 16);
            ra.w = (uint32_t)hr | ((uint32_t)hg << 16);
            o.ra = ra;
            o.rb = (uint32_t)hb | ((uint32_t)hd << 16);
            o.vis = true;
            o.cmx = cmx;
            o.cmy = cmy;
            o.k = k;

            // tileCountIndirectKernel (GlobalShaders.metal:563-616): alpha is the u8 opacity
            const float alpha = (float)cO;
            o.countable = alpha >= 1e-4f && minTX <= maxTX && minTY <= maxTY;
            o.w = o.countable ? lut.level[cO] : 0.0f;  // = 2 computePower(alpha)
        }
    }
    return o;
}

// The renderer's tile rows (ProjectArgs::rowBegin / rowEnd / rowStride): rows b, b + s, ... < e,
// row index k = (ty - b) / s; a contiguous slab has s = 1, a multi-GPU rank's interleaved rows s = W.
struct RowSet {
    int b, e, s;
};
__device__ __forceinline__ RowSet rows_of(const ProjectArgs& P) {
    return RowSet{(int)P.rowBegin, (int)P.rowEnd, P.rowStride > 1u ? (int)P.rowStride : 1};
}
// row indices [*k0, *k1] of the set inside tile rows [y0, y1] (empty when *k0 > *k1)
__device__ __forceinline__ void rows_within(const RowSet& R, int y0, int y1, int* k0, int* k1) {
    const int lo = max(y0, R.b), hi = min(y1, R.e - 1);
    if (R.s == 1) {  // contiguous rows (one GPU, contiguous slabs): no integer divisions (r06)
        *k0 = lo - R.b;
        *k1 = hi < R.b ? -1 : hi - R.b;
        return;
    }
    *k0 = (lo - R.b + R.s - 1) / R.s;
    *k1 = hi < R.b ? -1 : (hi - R.b) / R.s;
}

// tiles of a projected gaussian's rect in the renderer's rows that its ellipse meets
// (tileCountIndirectKernel, GlobalShaders.metal:563-616).  For rects of at most 32 tiles the
// answers are also returned as a bit mask in scan order (bit (k - k0) * width + (tx - tx0) for
// row index k), so the scatter reuses them instead of repeating the tests.
constexpr int kMaskTiles = 32;
__device__ __forceinline__ uint32_t count_tiles(const ProjOut& o, const RowSet& R, uint32_t* maskOut) {
    uint32_t n = 0, mask = 0;
    *maskOut = 0;
    if (!o.countable) return 0;
    int k0, k1;
    rows_within(R, (int)o.bounds.z, (int)o.bounds.w, &k0, &k1);
    uint32_t bit = 0;
    for (int k = k0; k <= k1; ++k)
        for (int tx = (int)o.bounds.x, ty = R.b + k * R.s; tx <= (int)o.bounds.y; ++tx, ++bit)
            if (intersects_tile(tx, ty, o.cmx, o.cmy, o.k, o.w)) {
                n++;
                if (bit < (uint32_t)kMaskTiles) mask |= 1u << bit;
            }
    *maskOut = mask;
    return n;
}

// The blend's half-tile skip band of a projected gaussian (BandSkip of its fp16 blend record),
// checked once against its tile rect within the renderer's rows (from its first to its last row in
// the rect: a superset for interleaved rows): (mean x, half width), or a negative width when the
// band may not be used.  Stored in the blend record's padding for k_scatter.
__device__ __forceinline__ bool band_rect_ok(const BandSkip& b, int x0, int x1, int y0, int y1) {
    if (!b.valid) return false;
    const int mxm = fp16_coord_margin(x1), mym = fp16_coord_margin(y1);
    if (mxm < 0 || mym < 0) return false;
    const float ax = __builtin_fmaxf(__builtin_fabsf((float)(x0 - mxm) - b.mx), __builtin_fabsf((float)(x1 + mxm) - b.mx));
    const float ay = __builtin_fmaxf(__builtin_fabsf((float)(y0 - mym) - b.my), __builtin_fabsf((float)(y1 + mym) - b.my));
    return ax <= 200.0f && ay <= 200.0f && b.cxx * (ax * ax) + b.cyy * (ay * ay) <= 16000.0f;
}
__device__ __forceinline__ float2 band_of(const BlendRecordA& ra, short4 r, const RowSet& R) {
    const BandSkip b = band_skip_setup(ra.x, ra.y, ra.z, kBlendZeroP);
    int k0, k1;
    rows_within(R, (int)r.z, (int)r.w, &k0, &k1);
    const int by0 = R.b + k0 * R.s, by1 = R.b + k1 * R.s;
    if (band_rect_ok(b, (int)r.x * (int)kTileWidth, (int)r.y * (int)kTileWidth + (int)kTileWidth - 1,
                     by0 * (int)kTileHeight, by1 * (int)kTileHeight + (int)kTileHeight - 1))
        return make_float2(b.mx, b.ex);
    return make_float2(0.0f, -1.0f);
}

// The tile tests (count_tiles' loop) are shared out over the block: every (gaussian, tile of its
// rect) candidate of the block's 256 gaussians goes to one thread, consecutive candidates to
// consecutive threads (owner by binary search over the block's exclusive candidate offsets), and
// the answers meet in LDS (mask bits for rects of <= 32 tiles, a counter beyond).  A thread no
// longer walks its own rect while the rest of its wave waits, so one large rect costs its wave
// nothing extra.  Candidate k of a gaussian is bit k of count_tiles' mask (ty-major, tx-minor).
template <bool HALF, int DEG>
__global__ __launch_bounds__(kProjectBlock) void k_project(
    const void* __restrict__ world, const void* __restrict__ harm, ProjectArgs P,
    GaussianRenderData* __restrict__ outRD, short4* __restrict__ outBounds,
    BlendRecord* __restrict__ outRec, uint32_t* __restrict__ counts,
    uint32_t* __restrict__ masks, uint32_t* __restrict__ blockSums, const float2* __restrict__ sincos,
    const uint16_t* __restrict__ unitCost, uint32_t* __restrict__ unitOrder, uint32_t* __restrict__ costMax) {
    __shared__ uint32_t lds[kProjectBlock / 64];
    __shared__ ByteLut lut;
    // block 0 of a scheduled launch orders the blend's units from the previous frame's walks while
    // the other blocks project (no launch, no second stream, no join before the blend)
    if (P.schedUnits) {
        if (blockIdx.x == 0) {
            __shared__ uint32_t uoBase[kUoBuckets], uoMax[kProjectBlock / 64];
            unit_order_block<kProjectBlock>(unitCost, unitOrder, P.schedUnits, uoBase, uoMax, costMax, P.pairBucket);
            return;
        }
    }
    const uint32_t blk = blockIdx.x - (P.schedUnits ? 1u : 0u);
    __shared__ float4 sEll[kProjectBlock];   // cmx, cmy, conic A, conic B
    __shared__ float2 sEll2[kProjectBlock];  // conic C, level w
    __shared__ uint32_t sOff[kProjectBlock];  // exclusive candidate offsets
    __shared__ uint32_t sRect[kProjectBlock]; // x0 | rw << 16
    __shared__ int sTy0[kProjectBlock];
    __shared__ uint32_t sMask[kProjectBlock];
    __shared__ uint32_t sMore[kProjectBlock];  // hits among candidates >= 32 (large rects)
    // the block's first kCandCap candidates: owner << 8 | k for rects of <= kCandRect tiles,
    // kSearch for the candidates of larger rects (their owner comes from a binary search).  (r06: 8 waves
    // per SIMD -- 3072 candidates and a 64-VGPR cap -- measured no faster than 7, profiles/r06_proj_ab.txt)
    constexpr uint32_t kCandCap = 4096, kCandRect = 64;
    constexpr uint16_t kSearch = 0xFFFFu;
    __shared__ uint16_t sCand[kCandCap];
    uint4 preW[2];
    preload_world<HALF>(world, blk * kProjectBlock + threadIdx.x, P.count, preW);
    fill_byte_lut(lut, sincos);
    const uint32_t tid = threadIdx.x;
    const uint32_t gid = blk * kProjectBlock + tid;
    ProjOut o;
    o.vis = false;
    o.countable = false;
    o.bounds = make_short4(0, -1, 0, -1);
    uint32_t area = 0;
    int ty0 = 0;
    if (gid < P.count) {
        o = project_gaussian<HALF, DEG>(world, harm, gid, P, sincos, lut, HALF ? preW : nullptr);
        outBounds[gid] = o.bounds;
        if (o.vis) {
            // GaussianRenderData: the frame itself only reads it for rects the scatter re-tests
            const int ry0 = max((int)o.bounds.z, (int)P.rowBegin), ry1 = min((int)o.bounds.w, (int)P.rowEnd - 1);
            if (P.keepRenderData || (ry1 - ry0 + 1) * ((int)o.bounds.y - (int)o.bounds.x + 1) > kMaskTiles)
                *(uint4*)(outRD + gid) = o.rd;
            if (o.countable && ry1 >= ry0) {  // rows limited to the slab
                area = (uint32_t)((ry1 - ry0 + 1) * ((int)o.bounds.y - (int)o.bounds.x + 1));
                ty0 = ry0;
            }
        }
    }
    sEll[tid] = make_float4(o.cmx, o.cmy, o.k.A, o.k.B);
    sEll2[tid] = make_float2(o.k.C, o.w);
    sRect[tid] = ((uint32_t)(int)o.bounds.x & 0xFFFFu) | ((uint32_t)((int)o.bounds.y - (int)o.bounds.x + 1) << 16);
    sTy0[tid] = ty0;
    sMask[tid] = 0;
    sMore[tid] = 0;
    uint32_t total;
    const uint32_t coff = block_exclusive_scan<kProjectBlock>(area, lds, &total);
    sOff[tid] = coff;
    const uint32_t nCand = min(total, kCandCap);
    for (uint32_t i = tid; i < nCand; i += kProjectBlock) sCand[i] = kSearch;
    __syncthreads();
    if (area <= kCandRect)
        for (uint32_t k = 0; k < area && coff + k < kCandCap; ++k) sCand[coff + k] = (uint16_t)((tid << 8) | k);
    __syncthreads();
    for (uint32_t c = tid; c < total; c += kProjectBlock) {
        uint32_t lo, k;
        const uint32_t v = c < kCandCap ? (uint32_t)sCand[c] : (uint32_t)kSearch;
        if (v != kSearch) {
            lo = v >> 8;
            k = v & 0xFFu;
        } else {
            lo = 0;
            uint32_t hi = kProjectBlock - 1;  // owner: the largest g with sOff[g] <= c
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (sOff[mid] <= c) lo = mid;
                else hi = mid - 1;
            }
            k = c - sOff[lo];
        }
        const uint32_t rect = sRect[lo], rw = rect >> 16;
        // k / rw from the hardware reciprocal (within one of the quotient), then corrected exactly
        uint32_t row = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)rw));
        if (row * rw > k) row--;
        else if ((row + 1u) * rw <= k) row++;
        const int ty = sTy0[lo] + (int)row, tx = (int)(rect & 0xFFFFu) + (int)(k - row * rw);
        const float4 e = sEll[lo];
        const float2 e2 = sEll2[lo];
        Conic kk;
        kk.A = e.z;
        kk.B = e.w;
        kk.C = e2.x;
        if (intersects_tile(tx, ty, e.x, e.y, kk, e2.y)) {
            if (k < (uint32_t)kMaskTiles) atomicOr(&sMask[lo], 1u << k);
            else atomicAdd(&sMore[lo], 1u);
        }
    }
    __syncthreads();
    uint32_t ntiles = 0;
    if (gid < P.count && o.vis) {
        const uint32_t mask = sMask[tid];
        ntiles = (uint32_t)__builtin_popcount(mask) + sMore[tid];
        masks[gid] = mask;
        const float2 band = ntiles ? band_of(o.ra, o.bounds, rows_of(P)) : make_float2(0.f, -1.f);
        uint4* rp = (uint4*)(outRec + gid);
        rp[0] = make_uint4(o.ra.x, o.ra.y, o.ra.z, o.ra.w);
        rp[1] = make_uint4(o.rb, __float_as_uint(band.x), __float_as_uint(band.y), 0u);
    }
    if (gid < P.count) counts[gid] = ntiles;
    uint32_t s = block_reduce_add<kProjectBlock>(ntiles, lds);
    if (threadIdx.x == 0) blockSums[blk] = s;
}

// ---------------------------------------------------------------------------
// 1b. multi-GPU partition: a rank projects its range of gaussians once,
//     keeps every projected gaussian whose ellipse meets a tile of slab s, and sends its
//     48-byte splat record to slab s's owner in ascending id order.  The record's last word
//     carries the tile answers of the slab's part of the rect (rects of <= 32 tiles), so the
//     owner rebuilds keys from it (k_records_in + the usual scatter) without repeating the
//     tile tests; a record crosses the fabric once per (gaussian, slab), not once per tile.
// ---------------------------------------------------------------------------
// The tile tests of a block's gaussians shared out over its threads (as in k_project): every
// (gaussian, tile of its rect) candidate on one thread, consecutive candidates on consecutive
// threads, owner from an LDS table for rects of <= kCandRect tiles, by binary search beyond.
// hit(lo, k, ty) is called for every candidate k (ty-major, tx-minor over the rect) of gaussian
// lo whose ellipse meets tile row ty.  Ends with a barrier.
struct TileTestLds {
    // (2560: k_project_part's LDS under 20 KiB; its 72 VGPRs then allow 7 waves per SIMD, r06)
    static constexpr uint32_t kCandCap = 2560, kCandRect = 64;
    static constexpr uint16_t kSearch = 0xFFFFu;
    float4 ell[kProjectBlock];   // cmx, cmy, conic A, conic B
    float2 ell2[kProjectBlock];  // conic C, level w
    uint32_t off[kProjectBlock];  // exclusive candidate offsets
    uint32_t rect[kProjectBlock]; // x0 | rw << 16
    int ty0[kProjectBlock];
    uint16_t cand[kCandCap];
    uint32_t scan[kProjectBlock / 64];
};
template <class Hit>
__device__ __forceinline__ void block_tile_tests(TileTestLds& L, const ProjOut& o, uint32_t area, int ty0, Hit&& hit) {
    const uint32_t tid = threadIdx.x;
    L.ell[tid] = make_float4(o.cmx, o.cmy, o.k.A, o.k.B);
    L.ell2[tid] = make_float2(o.k.C, o.w);
    L.rect[tid] = ((uint32_t)(int)o.bounds.x & 0xFFFFu) | ((uint32_t)((int)o.bounds.y - (int)o.bounds.x + 1) << 16);
    L.ty0[tid] = ty0;
    uint32_t total;
    const uint32_t coff = block_exclusive_scan<kProjectBlock>(area, L.scan, &total);
    L.off[tid] = coff;
    const uint32_t nCand = min(total, TileTestLds::kCandCap);
    for (uint32_t i = tid; i < nCand; i += kProjectBlock) L.cand[i] = TileTestLds::kSearch;
    __syncthreads();
    if (area <= TileTestLds::kCandRect)
        for (uint32_t k = 0; k < area && coff + k < TileTestLds::kCandCap; ++k) L.cand[coff + k] = (uint16_t)((tid << 8) | k);
    __syncthreads();
    for (uint32_t c = tid; c < total; c += kProjectBlock) {
        uint32_t lo, k;
        const uint32_t v = c < TileTestLds::kCandCap ? (uint32_t)L.cand[c] : (uint32_t)TileTestLds::kSearch;
        if (v != TileTestLds::kSearch) {
            lo = v >> 8;
            k = v & 0xFFu;
        } else {
            lo = 0;
            uint32_t hi = kProjectBlock - 1;  // owner: the largest g with off[g] <= c
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (L.off[mid] <= c) lo = mid;
                else hi = mid - 1;
            }
            k = c - L.off[lo];
        }
        const uint32_t rect = L.rect[lo], rw = rect >> 16;
        // k / rw from the hardware reciprocal (within one of the quotient), then corrected exactly
        uint32_t row = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)rw));
        if (row * rw > k) row--;
        else if ((row + 1u) * rw <= k) row++;
        const int ty = L.ty0[lo] + (int)row, tx = (int)(rect & 0xFFFFu) + (int)(k - row * rw);
        const float4 e = L.ell[lo];
        const float2 e2 = L.ell2[lo];
        Conic kk;
        kk.A = e.z;
        kk.B = e.w;
        kk.C = e2.x;
        if (intersects_tile(tx, ty, e.x, e.y, kk, e2.y)) hit(lo, k, ty);
    }
    __syncthreads();
}

// the rows of slab sl (SlabTable: contiguous blocks or interleaved rows)
__device__ __forceinline__ RowSet slab_rows(const SlabTable& t, const uint32_t* rows, uint32_t sl) {
    return t.interleave ? RowSet{(int)sl, (int)rows[t.n], (int)t.n} : RowSet{(int)rows[sl], (int)rows[sl + 1], 1};
}

// the slab's part of a record's tile answers: the slab's rows of the rect, scan order (k - k0) * rw
// + tx - tx0 over the slab's row indices k -- k_scatter's mask order for the slab -- when the whole
// rect has <= 32 tiles (full = the rect's answers, bit (ty - ty0) * rw + tx - tx0); 0 otherwise (the
// owner re-tests)
__device__ __forceinline__ uint32_t slab_tile_mask(short4 b, uint32_t full, const RowSet& R) {
    const int rw = (int)b.y - (int)b.x + 1;
    if (((int)b.w - (int)b.z + 1) * rw > kMaskTiles) return 0u;
    int k0, k1;
    if (R.s == 1) {  // contiguous slab (wave-uniform): rows_within without its divisions
        k0 = max((int)b.z, R.b) - R.b;
        k1 = min((int)b.w, R.e - 1) - R.b;
    } else {
        rows_within(R, (int)b.z, (int)b.w, &k0, &k1);
    }
    if (k1 < k0) return 0u;
    const uint32_t rowBits = rw >= 32 ? 0xFFFFFFFFu : ((1u << rw) - 1u);
    uint32_t out = 0, at = 0;
    for (int k = k0; k <= k1; ++k, at += (uint32_t)rw)  // (<= 32 rows: the rect has <= 32 tiles)
        out |= ((full >> (uint32_t)((R.b + k * R.s - (int)b.z) * rw)) & rowBits) << at;
    return out;
}

template <bool HALF, int DEG>
__global__ __launch_bounds__(kProjectBlock) void k_project_part(
    const void* __restrict__ world, const void* __restrict__ harm, ProjectArgs P, SlabTable slabs,
    SplatRecord* __restrict__ runs, uint32_t runStride,
    uint32_t* __restrict__ blockSlabCounts, const float2* __restrict__ sincos, const uint16_t* __restrict__ unitCost,
    uint32_t* __restrict__ unitOrder, uint32_t* __restrict__ costMax) {
    // block 0 of a scheduled launch orders the blend units of the rank's own slab (the owner renders
    // it later in the frame) while the other blocks project -- as k_project's block 0 does
    if (P.schedUnits) {
        if (blockIdx.x == 0) {
            __shared__ uint32_t uoBase[kUoBuckets], uoMax[kProjectBlock / 64];
            unit_order_block<kProjectBlock>(unitCost, unitOrder, P.schedUnits, uoBase, uoMax, costMax, P.pairBucket);
            return;
        }
    }
    const uint32_t blk = blockIdx.x - (P.schedUnits ? 1u : 0u);
    __shared__ uint32_t wcnt[kProjectBlock / 64][kMaxSlabs];
    __shared__ uint64_t wbal[kProjectBlock / 64][kMaxSlabs];  // the wave's ballot of each slab
    __shared__ ByteLut lut;
    __shared__ TileTestLds L;
    __shared__ uint32_t sTile[kProjectBlock];  // answers of candidates < 32
    __shared__ uint32_t sSlab[kProjectBlock];  // slabs with a hit
    __shared__ uint32_t sRows[kMaxSlabs + 1];
    // the slab of tile row ty < kRowTab (0xFF: none), so a hit costs one LDS byte instead of a search
    // over the slab bounds (contiguous) or a division (interleaved)
    constexpr uint32_t kRowTab = 512;
    __shared__ uint8_t sRowSlab[kRowTab];
    uint4 preW[2];
    preload_world<HALF>(world, blk * kProjectBlock + threadIdx.x, P.count, preW);
    fill_byte_lut(lut, sincos);
    const uint32_t tid = threadIdx.x;
    const uint32_t gid = blk * kProjectBlock + tid;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const uint32_t nSlabs = slabs.n;
    if (tid <= nSlabs) sRows[tid] = slabs.rows[tid];
    sTile[tid] = 0;
    sSlab[tid] = 0;
    auto slabOf = [&](uint32_t ty) -> uint32_t {  // (reads sRows)
        if (ty >= sRows[nSlabs]) return 0xFFu;
        if (slabs.interleave) return ty % nSlabs;
        uint32_t sl = 0;  // slabs.rows is non-decreasing, at most 16 slabs
        while (sl + 1u < nSlabs && ty >= sRows[sl + 1u]) ++sl;
        return ty >= sRows[sl] ? sl : 0xFFu;
    };
    __syncthreads();
    for (uint32_t r = tid; r < kRowTab; r += kProjectBlock) sRowSlab[r] = (uint8_t)slabOf(r);
    ProjOut o;
    o.vis = false;
    o.countable = false;
    o.bounds = make_short4(0, -1, 0, -1);
    uint32_t area = 0;
    if (gid < P.count) {
        o = project_gaussian<HALF, DEG>(world, harm, gid, P, sincos, lut, HALF ? preW : nullptr);
        if (o.vis && o.countable)
            area = (uint32_t)(((int)o.bounds.w - (int)o.bounds.z + 1) * ((int)o.bounds.y - (int)o.bounds.x + 1));
    }
    block_tile_tests(L, o, area, (int)o.bounds.z, [&](uint32_t lo, uint32_t k, int ty) {
        if (k < (uint32_t)kMaskTiles) atomicOr(&sTile[lo], 1u << k);
        // the slab of row ty: row ty mod n (interleaved), or the block holding it
        const uint32_t sl = (uint32_t)ty < kRowTab ? (uint32_t)sRowSlab[ty] : slabOf((uint32_t)ty);
        if (sl != 0xFFu) atomicOr(&sSlab[lo], 1u << sl);
    });
    const uint32_t mask = gid < P.count ? sSlab[tid] : 0u;  // (only visible gaussians meet a tile)
    for (uint32_t sl = 0; sl < nSlabs; ++sl) {
        const uint64_t b = __ballot((mask >> sl) & 1u);
        if (lane == 0) {
            wcnt[wave][sl] = (uint32_t)__popcll(b);
            wbal[wave][sl] = b;
        }
    }
    __syncthreads();
    const uint32_t nb = gridDim.x - (P.schedUnits ? 1u : 0u);
    if (tid < nSlabs) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kProjectBlock / 64; ++w) t += wcnt[w][tid];
        blockSlabCounts[(size_t)tid * nb + blk] = t;
    }
    // the block's run of slab sl: records [sl * runStride + blk * 256, + count), ascending id (lane
    // order within a wave, wave order within the block), stored from the threads (assembling the runs
    // in LDS first measured slower: 60.8 against 56.3 us at config 4 / W = 8); the record's last word
    // is the slab's part of the rect's tile answers (slab_tile_mask)
    // each lane walks only its own slabs (one or two for most gaussians; a wave-uniform loop over all
    // slabs ran the store body once per slab any lane of the wave had -- every slab, for scattered ids)
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint2 bw = __builtin_bit_cast(uint2, o.bounds);
    const uint32_t tileBits = sTile[tid];
    for (uint32_t m = mask; m != 0u; m &= m - 1u) {
        const uint32_t sl = (uint32_t)__builtin_ctz(m);
        uint32_t at = (uint32_t)__popcll(wbal[wave][sl] & lt);
        for (uint32_t w = 0; w < wave; ++w) at += wcnt[w][sl];
        uint4* d = (uint4*)(runs + (size_t)sl * runStride + (size_t)blk * kProjectBlock + at);
        d[0] = o.rd;
        d[1] = make_uint4(o.ra.x, o.ra.y, o.ra.z, o.ra.w);
        d[2] = make_uint4(bw.x, bw.y, o.rb, slab_tile_mask(o.bounds, tileBits, slab_rows(slabs, sRows, sl)));
    }
}

// one workgroup per slab: exclusive scan of the slab's block counts (in place) and its total.
// Multi-GPU frame (pub.arrive.done != null): the total also goes into column `slab` of row `rank` of
// every rank's count matrix (pub.row[p], peer mappings), and the workgroups arrive at barrier 0 --
// the count publication needs no kernel of its own (gsm_multigpu.hip)
__global__ __launch_bounds__(1024) void k_part_scan(uint32_t* __restrict__ blockSlabCounts, uint32_t numBlocks,
                                                    uint32_t* __restrict__ sendCounts, CountPublish pub) {
    __shared__ uint32_t lds[1024 / 64];
    const uint32_t sl = blockIdx.x;
    uint32_t* row = blockSlabCounts + (size_t)sl * numBlocks;
    uint32_t carry = 0;
    // IT consecutive counts per thread: one pass (one load latency) up to 4096 blocks (config 4's ranks
    // have 2442), where one count per thread took three dependent passes
    constexpr uint32_t IT = 4;
    for (uint32_t base = 0; base < numBlocks; base += 1024u * IT) {
        const uint32_t i0 = base + threadIdx.x * IT;
        uint32_t v[IT], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k) v[k] = row[min(i0 + k, numBlocks - 1u)];  // (unpredicated: Tail4 note)
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k) {
            v[k] = i0 + k < numBlocks ? v[k] : 0u;
            sum += v[k];
        }
        uint32_t tot;
        uint32_t run = carry + block_exclusive_scan<1024>(sum, lds, &tot);
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k) {
            if (i0 + k < numBlocks) row[i0 + k] = run;
            run += v[k];
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) sendCounts[sl] = carry;
    if (pub.arrive.done && threadIdx.x < 64u) {  // (carry is uniform over the workgroup)
        if (threadIdx.x < pub.arrive.world)
            __hip_atomic_store(pub.row[threadIdx.x] + sl, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        mg_arrive_wave(pub.arrive);  // wave 0 made every store of the workgroup that crosses ranks
    }
}

// The block runs of every slab copied to their destination: one wave per (block, slab) run (waves
// over runs, workgroups gridDim.x blocks apart), 16-B words, the run's records contiguous at both
// ends.  The run of block b for slab s starts at blockSlabOffsets[s * nb + b] (k_part_scan) within
// the slab's records; its length is the next block's offset less its own (the slab total after the
// last block).
//  PUSH (the multi-GPU frame, gsm_multigpu.hip): into slab s's owner's receive buffer, after the
//    records of the ranks before this one (the count matrix: counts[r * world + s], system-coherent
//    loads; row `rank` is this rank's totals), write-through stores; block 0 leaves the rank's receive
//    count in *recvCount; every workgroup arrives (arrive.done) after its stores.
//  !PUSH (gsm_global_project_partition): into the caller's send buffer, slab after slab.
template <bool PUSH>
__global__ __launch_bounds__(kProjectBlock) void k_part_copy(
    const SplatRecord* __restrict__ runs, uint32_t runStride, uint32_t nb, uint32_t numSlabs,
    const uint32_t* __restrict__ blockSlabOffsets, const uint32_t* __restrict__ totals, uint32_t rank,
    const uint32_t* __restrict__ counts, SlabPeers peers, uint32_t* __restrict__ recvCount, MgArrive arrive,
    SplatRecord* __restrict__ send, uint64_t capacity) {
    __shared__ uint32_t sBase[kMaxSlabs], sTotal[kMaxSlabs];
    // the count matrix (PUSH: world x world words, system-coherent loads) or the slab totals, one word per
    // thread in a single round of loads (r06: each thread summed its column in a loop -- one load round
    // trip after another, up to world of them for the last rank, and world more for block 0's receive count)
    __shared__ uint32_t sCnt[kMaxSlabs * kMaxSlabs];
    // (PUSH: the peers' receive buffers and capacities too -- indexed by slab, the kernel-argument arrays
    // were two dependent memory round trips per run)
    __shared__ SplatRecord* sRecv[kMaxSlabs];
    __shared__ uint32_t sCap[kMaxSlabs];
    const uint32_t nCnt = PUSH ? numSlabs * numSlabs : numSlabs;
    static_assert(kMaxSlabs * kMaxSlabs <= kProjectBlock, "one count-matrix word per thread");
    {  // (loads unpredicated at clamped indices, all before the first LDS store: one round trip)
        const uint32_t tc = min((uint32_t)threadIdx.x, nCnt - 1u), ts = min((uint32_t)threadIdx.x, numSlabs - 1u);
        const uint32_t cv = PUSH ? ld_sys32(counts + tc) : totals[tc];
        SplatRecord* const rv = PUSH ? peers.recv[ts] : nullptr;
        const uint32_t capv = PUSH ? peers.cap[ts] : 0u;
        if (threadIdx.x < nCnt) sCnt[threadIdx.x] = cv;
        if (PUSH && threadIdx.x < numSlabs) {
            sRecv[threadIdx.x] = rv;
            sCap[threadIdx.x] = capv;
        }
    }
    __syncthreads();
    if (threadIdx.x < numSlabs) {
        const uint32_t sl = threadIdx.x;
        uint32_t base = 0;
        if constexpr (PUSH) {
            for (uint32_t r = 0; r < rank; ++r) base += sCnt[r * numSlabs + sl];
            sTotal[sl] = sCnt[rank * numSlabs + sl];
        } else {
            for (uint32_t t = 0; t < sl; ++t) base += sCnt[t];
            sTotal[sl] = sCnt[sl];
        }
        sBase[sl] = base;
    }
    if constexpr (PUSH) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            uint32_t mine = 0;
            for (uint32_t r = 0; r < numSlabs; ++r) mine += sCnt[r * numSlabs + rank];
            *recvCount = min(mine, sCap[rank]);
        }
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = kProjectBlock / 64;
    const uint32_t runsTotal = nb * numSlabs;
    // the wave's runs k0, k0 + S, k0 + 2S, ...: lane j loads the bounds of its j-th run up front (one
    // load round trip for up to 64 runs instead of one per run), the copy loop reads them by readlane
    const uint32_t S = gridDim.x * kWaves, k0 = blockIdx.x * kWaves + wave;
    const uint32_t nRuns = k0 < runsTotal ? (runsTotal - k0 + S - 1u) / S : 0u;
    for (uint32_t c0 = 0; c0 < nRuns; c0 += 64u) {
        uint32_t offL = 0, nL = 0;
        if (c0 + lane < nRuns) {
            const uint32_t kL = k0 + (c0 + lane) * S;
            const uint32_t bL = kL / numSlabs, slL = kL - bL * numSlabs;
            offL = blockSlabOffsets[(size_t)slL * nb + bL];
            const uint32_t endL = bL + 1u < nb ? blockSlabOffsets[(size_t)slL * nb + bL + 1u] : sTotal[slL];
            nL = endL - offL;
        }
        const uint32_t cnt = min(64u, nRuns - c0);
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)nL, (int)j);
            if (n == 0) continue;
            const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)offL, (int)j);
            const uint32_t k = k0 + (c0 + j) * S;
            const uint32_t b = k / numSlabs, sl = k - b * numSlabs;
            const uint4* src = (const uint4*)(runs + (size_t)sl * runStride + (size_t)b * kProjectBlock);
            const uint64_t at = (uint64_t)sBase[sl] + off;  // the run's first record at the destination
            // four 16-B words per lane in flight before the stores (unpredicated loads at clamped indices;
            // a load-store pair per word was one round trip per 1 KiB of the run, r06)
            const uint64_t cap = PUSH ? (uint64_t)sCap[sl] : capacity;
            const uint32_t m = at >= cap ? 0u : (uint32_t)min((uint64_t)n, cap - at);  // never past it
            // Stores at clamped indices too: a word past the run rewrites the run's last word with its own
            // value, so no store (and no load sunk into it) sits under a condition.  The destination is
            // made wave-uniform explicitly (a buffer descriptor from VGPRs costs a waterfall loop per store).
            const uint32_t words = (uint32_t)__builtin_amdgcn_readfirstlane((int)(3u * m));
            const uint64_t dA = (uint64_t)(uintptr_t)(PUSH ? (void*)(sRecv[sl] + at) : (void*)(send + at));
            uint4* d = (uint4*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(dA >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)dA));
            for (uint32_t w0 = lane; w0 < words; w0 += 256u) {
                uint4 v[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) v[q] = src[min(w0 + 64u * q, words - 1u)];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t w = min(w0 + 64u * q, words - 1u);
                    if constexpr (PUSH) st_sys128(d, words * 16u, w, v[q]);
                    else d[w] = v[q];
                }
            }
        }
    }
    if constexpr (PUSH) {
        // every workgroup arrives once (barrier 1) after all its waves' record stores
        if (arrive.done) mg_arrive_block_unit(arrive, blockIdx.x);
    }
}

// slab owner: received records -> the renderer's per-gaussian arrays + tile counts for its rows.
// devCount (may be null): the record count on the device (multi-GPU exchange); P.count is then the
// capacity the grid covers, and blocks past the count leave at once (the scan and the scatter read
// the count too).  The block's records (256 x 48 B, contiguous) are loaded as 16-B words by
// consecutive threads and exchanged through LDS (whole segments of the receive buffer).
__global__ __launch_bounds__(kProjectBlock) void k_records_in(
    const SplatRecord* __restrict__ in, ProjectArgs P, GaussianRenderData* __restrict__ outRD,
    short4* __restrict__ outBounds, BlendRecord* __restrict__ outRec,
    uint32_t* __restrict__ counts, uint32_t* __restrict__ masks, uint32_t* __restrict__ blockSums,
    const float2* __restrict__ sincos, const uint32_t* __restrict__ devCount, const uint16_t* __restrict__ unitCost,
    uint32_t* __restrict__ unitOrder, uint32_t* __restrict__ costMax) {
    __shared__ uint32_t lds[kProjectBlock / 64];
    __shared__ uint4 sIn[kProjectBlock * 3];
    // block 0 of a scheduled launch orders the blend's units (as k_project's: no k_unit_order launch)
    if (P.schedUnits) {
        if (blockIdx.x == 0) {
            __shared__ uint32_t uoBase[kUoBuckets], uoMax[kProjectBlock / 64];
            unit_order_block<kProjectBlock>(unitCost, unitOrder, P.schedUnits, uoBase, uoMax, costMax, P.pairBucket);
            return;
        }
    }
    uint32_t blk = blockIdx.x - (P.schedUnits ? 1u : 0u);
    const uint32_t n = devCount ? min(*devCount, P.count) : P.count;
    // blocks of 256 records, gridDim (less the schedule block) apart: the grid is capped when the count
    // lives on the device (launch_records_in), so few blocks find nothing to do
    const uint32_t stride = gridDim.x - (P.schedUnits ? 1u : 0u);
    for (; blk * kProjectBlock < n; blk += stride) {  // (uniform)
    const uint32_t gid = blk * kProjectBlock + threadIdx.x;
    {
        // system-coherent 16-B loads (ld_sys128): on the multi-GPU path the records were stored by the
        // peers' k_part_copy over xGMI; no L1 / L2 line of an earlier frame may answer
        const uint32_t words = 3u * (min(n - blk * kProjectBlock, (uint32_t)kProjectBlock));
        const SplatRecord* src = in + (size_t)blk * kProjectBlock;
        // (unconditional: a word past the block's records is outside the buffer descriptor's range and
        // reads as 0 -- a load under `i < words` went out alone with its own wait, r06)
        uint4 t[3];
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) t[j] = ld_sys128(src, words * 16u, threadIdx.x + j * kProjectBlock);
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) sIn[threadIdx.x + j * kProjectBlock] = t[j];
    }
    __syncthreads();
    uint32_t ntiles = 0;
    if (gid < n) {
        const uint4 w0 = sIn[3 * threadIdx.x], w1 = sIn[3 * threadIdx.x + 1], w2 = sIn[3 * threadIdx.x + 2];
        SplatRecord r;
        r.rd = w0;
        r.ra.x = w1.x;
        r.ra.y = w1.y;
        r.ra.z = w1.z;
        r.ra.w = w1.w;
        r.bounds = __builtin_bit_cast(short4, make_uint2(w2.x, w2.y));
        r.rb = w2.z;
        r.pad = w2.w;
        // a received record addresses only the frame's tile grid (r06): computeTileBounds already clamps a
        // projected gaussian's rect to it, so this changes nothing for a valid record, and a corrupt one --
        // e.g. words that never arrived over a stale mapping -- cannot send the scatter or the sort outside it
        r.bounds.x = (short)max((int)r.bounds.x, 0);
        r.bounds.y = (short)min((int)r.bounds.y, (int)P.bin.tilesX - 1);
        r.bounds.z = (short)max((int)r.bounds.z, 0);
        r.bounds.w = (short)min((int)r.bounds.w, (int)P.bin.tilesY - 1);
        const int rw = max((int)r.bounds.y - (int)r.bounds.x + 1, 0);
        const RowSet R = rows_of(P);
        int k0, k1;
        rows_within(R, (int)r.bounds.z, (int)r.bounds.w, &k0, &k1);
        if (P.keepRenderData || (k1 - k0 + 1) * rw > kMaskTiles) *(uint4*)(outRD + gid) = r.rd;
        outBounds[gid] = r.bounds;
        uint4* rp = (uint4*)(outRec + gid);
        rp[0] = make_uint4(r.ra.x, r.ra.y, r.ra.z, r.ra.w);
        uint32_t mask;
        const int area = max((int)r.bounds.w - (int)r.bounds.z + 1, 0) * rw;
        if (area <= kMaskTiles) {
            // the sender's answers for this slab's rows (slab_tile_mask), never past the rect
            mask = area >= kMaskTiles ? r.pad : (r.pad & ((1u << area) - 1u));
            ntiles = (uint32_t)__builtin_popcount(mask);
        } else {
            // a rect of more than 32 tiles: the values k_project had in registers, rebuilt from the
            // record exactly as k_scatter does, and the tests of the slab's rows repeated
            ProjOut o;
            o.bounds = r.bounds;
            o.cmx = hbits_to_f((uint16_t)(r.rd.x & 0xFFFFu));
            o.cmy = hbits_to_f((uint16_t)(r.rd.x >> 16));
            o.k = conic_from_quant(sincos, (uint16_t)(r.rd.y & 0xFFFFu), hbits_to_f((uint16_t)(r.rd.y >> 16)),
                                   hbits_to_f((uint16_t)(r.rd.z & 0xFFFFu)));
            const float alpha = (float)(r.rd.w >> 24);
            o.countable = alpha >= 1e-4f && r.bounds.x <= r.bounds.y && r.bounds.z <= r.bounds.w;
            o.w = o.countable ? 2.0f * compute_power(alpha) : 0.0f;
            ntiles = count_tiles(o, R, &mask);
        }
        counts[gid] = ntiles;
        masks[gid] = mask;
        const float2 band = ntiles ? band_of(r.ra, r.bounds, R) : make_float2(0.f, -1.f);
        rp[1] = make_uint4(r.rb, __float_as_uint(band.x), __float_as_uint(band.y), 0u);
    }
    uint32_t s = block_reduce_add<kProjectBlock>(ntiles, lds);
    if (threadIdx.x == 0) blockSums[blk] = s;
    __syncthreads();  // (sIn and lds of the next block)
    }
}

// ---------------------------------------------------------------------------
// 2. exclusive scan of block sums (single workgroup) + clamp
//    (prefix sum: TwoPassTileAssignEncoder.swift:91-196; clamp GlobalShaders.metal:694-712)
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 1024;
// Exclusive scan of one 64-bit value per thread (< 2^37 each) over the workgroup, exact: one 32-bit
// block scan while every value is < 2^22 (1024 of them stay below 2^32), otherwise two 32-bit scans of
// the high (>> 16, < 2^21 each) and low 16-bit parts.  A frame far over its capacity thus never wraps
// its total below maxAssignments, and the overflow flag is raised.  Ends with the lds free.
__device__ __forceinline__ uint64_t scan_exact64(uint64_t v, uint32_t* lds, uint64_t* total) {
    if (!__syncthreads_or(v >= (1ull << 22))) {
        uint32_t t32;
        const uint32_t off = block_exclusive_scan<kScanThreads>((uint32_t)v, lds, &t32);
        *total = t32;
        return off;
    }
    uint32_t hiTot, loTot;
    const uint32_t hiOff = block_exclusive_scan<kScanThreads>((uint32_t)(v >> 16), lds, &hiTot);
    const uint32_t loOff = block_exclusive_scan<kScanThreads>((uint32_t)(v & 0xFFFFu), lds, &loTot);
    *total = ((uint64_t)hiTot << 16) + loTot;
    return ((uint64_t)hiOff << 16) + loOff;
}
// sums[i, i + 4) with zeros at and past nb, from unpredicated loads (Tail4, gsm_internal.h: conditional
// loads made config 3's 19.5K sums five memory round trips, r06)
__device__ __forceinline__ uint4 pick_sums4(uint4 q, uint32_t i, uint32_t nb, const Tail4& T) {
    if (i >= nb) return make_uint4(0u, 0u, 0u, 0u);
    if (i != T.n4) return q;
    return make_uint4(T.t[0], i + 1u < nb ? T.t[1] : 0u, i + 2u < nb ? T.t[2] : 0u, 0u);
}
__global__ __launch_bounds__(kScanThreads) void k_scan_blocks(uint32_t* __restrict__ sums,
                                                              uint32_t nb, uint32_t maxAssignments,
                                                              TileAssignmentHeader* __restrict__ hdr,
                                                              uint32_t* __restrict__ blendQueue,
                                                              const uint32_t* __restrict__ devCount) {
    __shared__ uint32_t lds[kScanThreads / 64];
    if (devCount) nb = min(nb, (*devCount + (uint32_t)kProjectBlock - 1u) / (uint32_t)kProjectBlock);
    // rows of 4 * kScanThreads block sums, kScanRows rows in flight: thread t holds sums
    // [row * 4096 + 4t, +4) as one 16-byte load, so every load of a pass is issued before the
    // first scan (the sums are read once and written once)
    constexpr uint32_t kRow = 4u * kScanThreads, kScanRows = 8;
    const uint32_t t4 = threadIdx.x * 4u;
    uint64_t carry = 0;
    // up to 32 sums per thread (nb <= 32768: config 3's 19.5K blocks): thread t scans its own
    // contiguous run of `per` sums (16-byte loads, all in flight), then ONE block scan of the run
    // totals -- instead of one block scan per 4096-sum row (config 3: 5)
    const uint32_t per = ((nb + kScanThreads - 1) / kScanThreads + 3u) & ~3u;
    if (nb > kRow && per <= 32u) {
        constexpr uint32_t kV = 8;
        uint4 v[kV];
        const uint32_t b0 = threadIdx.x * per;
        const Tail4 T = tail4_load(sums, nb);
#pragma unroll
        for (uint32_t r = 0; r < kV; ++r) v[r] = load4_clamped(sums, b0 + 4u * r, T);
#pragma unroll
        for (uint32_t r = 0; r < kV; ++r) {
            const uint32_t i = b0 + 4u * r;
            v[r] = 4u * r < per ? pick_sums4(v[r], i, nb, T) : make_uint4(0u, 0u, 0u, 0u);
        }
        uint64_t local = 0;
#pragma unroll
        for (uint32_t r = 0; r < kV; ++r) local += (uint64_t)v[r].x + v[r].y + v[r].z + v[r].w;
        uint64_t tot;
        uint64_t run = scan_exact64(local, lds, &tot);
#pragma unroll
        for (uint32_t r = 0; r < kV; ++r) {
            const uint32_t i = b0 + 4u * r;
            if (4u * r >= per || i >= nb) break;
            const uint32_t in[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[j] = run > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)run;
                run += in[j];
            }
            if (i + 3u < nb) {
                *(uint4*)(sums + i) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (i + (uint32_t)j < nb) sums[i + j] = o[j];
            }
        }
        carry = tot;
        nb = 0;  // (the row loop below has nothing left)
    }
    const Tail4 T = tail4_load(sums, nb > 0u ? nb : 1u);
    for (uint32_t base = 0; base < nb; base += kScanRows * kRow) {
        uint4 v[kScanRows];
#pragma unroll
        for (uint32_t r = 0; r < kScanRows; ++r) v[r] = load4_clamped(sums, base + r * kRow + t4, T);
#pragma unroll
        for (uint32_t r = 0; r < kScanRows; ++r) v[r] = pick_sums4(v[r], base + r * kRow + t4, nb, T);
#pragma unroll
        for (uint32_t r = 0; r < kScanRows; ++r) {
            const uint32_t row0 = base + r * kRow;
            if (row0 >= nb) break;
            uint64_t tot;
            uint64_t run = carry + scan_exact64((uint64_t)v[r].x + v[r].y + v[r].z + v[r].w, lds, &tot);
            const uint32_t in[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[j] = run > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)run;
                run += in[j];
            }
            const uint32_t i = row0 + t4;
            if (i + 3u < nb) {
                *(uint4*)(sums + i) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (i + (uint32_t)j < nb) sums[i + j] = o[j];
            }
            carry += tot;
        }
    }
    const uint32_t total = carry > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)carry;
    if (threadIdx.x == 0) {
        uint32_t tot = total;
        uint32_t ovf = 0;
        if (tot > maxAssignments) {
            tot = maxAssignments;
            ovf = 1;
        }
        hdr->totalAssignments = tot;
        hdr->maxCapacity = maxAssignments;
        hdr->paddedCount = ((tot + 1023u) / 1024u) * 1024u;
        hdr->overflow = ovf;
        // the blend's work counters for this frame (saves a memset launch)
        for (uint32_t q = 0; q < kQueueStripes; ++q) blendQueue[q * kQueueStride] = 0;
    }
}

// ---------------------------------------------------------------------------
// 3. duplicate with keys (tileScatterIndirectKernel GlobalShaders.metal:623-678 +
//    computeSortKeysKernel :266-295): key = tile<<16 | (fp16 depth ^ 0x8000), value = gid
// ---------------------------------------------------------------------------
// Small rects (<= kMaskTiles tiles, the projection's answer mask) are written cooperatively: the
// block's slots [0, total) are handed out to consecutive threads, each finding its gaussian by a
// binary search over the block's exclusive offsets in LDS and its tile as the k-th set bit of the
// mask -- consecutive threads write consecutive keys (coalesced) and a gaussian with many tiles
// no longer serialises its wave.  Large rects keep one thread looping over their rect.  Slot
// order is the reference's (ascending gid, then ty-major, tx-minor).
// Every value also carries the blend's half-tile skip flags (kHalfSkipShift, gsm_internal.h): the
// projection left each gaussian's column band in its blend record (band_of), so a (gaussian, tile)
// slot only compares the two 16-column halves of its tile with [mx - ex, mx + ex] (half_skip_flags).
// ex < 0: no skipping for this gaussian; otherwise the band test (BandSkip) on the two halves of tile tx
__device__ __forceinline__ uint32_t half_skip_flags(float mx, float ex, int tx) {
    if (ex < 0.0f) return 0u;
    const int x0 = tx * (int)kTileWidth;
    constexpr int hw = (int)kTileWidth / 2;
    const int m0 = fp16_coord_margin(x0 + hw - 1), m1 = fp16_coord_margin(x0 + 2 * hw - 1);
    const bool l = (float)(x0 - m0) - mx > ex || (float)(x0 + hw - 1 + m0) - mx < -ex;
    const bool r = (float)(x0 + hw - m1) - mx > ex || (float)(x0 + 2 * hw - 1 + m1) - mx < -ex;
    return (l ? 1u : 0u) | (r ? 2u : 0u);
}

// Sum of sums[0, n) over the workgroup, exact in 64 bits (16-B loads where the array allows).
__device__ __forceinline__ uint64_t block_sum_prefix(const uint32_t* __restrict__ sums, uint32_t n,
                                                     unsigned long long* lds64) {
    uint64_t v = 0;
    const uint32_t n4 = n & ~3u;
    constexpr uint32_t kStep = kProjectBlock * 4u;
    // up to 8 * kStep sums (the fused scan's kFusedScanMaxBlocks): 1, 2, 4 or 8 unpredicated 16-B loads per
    // thread, up to four in flight at once, the ragged end from Tail4 and the words past n masked (r06: the
    // loop below waited for each of its tail loads in turn -- up to four round trips before a scatter
    // workgroup knew its base)
    // (whole groups below n & ~3 from the clamped loads, the ragged end -- uniform loads -- added by thread 0;
    // at most 4 loads in flight, so k_scatter keeps its 58 VGPRs and 8 waves per SIMD)
    auto sum_groups = [&](auto ng) {
        constexpr uint32_t NG = decltype(ng)::value, NR = NG < 4u ? NG : 4u;
        const Tail4 T = tail4_load(sums, n);
#pragma unroll
        for (uint32_t r = 0; r < NG; r += NR) {
            uint4 q[NR];
#pragma unroll
            for (uint32_t k = 0; k < NR; ++k) q[k] = load4_clamped(sums, threadIdx.x * 4u + (r + k) * kStep, T);
#pragma unroll
            for (uint32_t k = 0; k < NR; ++k)
                if (threadIdx.x * 4u + (r + k) * kStep < T.n4) v += (uint64_t)q[k].x + q[k].y + q[k].z + q[k].w;
        }
        if (threadIdx.x == 0)
            v += (uint64_t)(T.n4 < n ? T.t[0] : 0u) + (T.n4 + 1u < n ? T.t[1] : 0u) + (T.n4 + 2u < n ? T.t[2] : 0u);
    };
    if (n == 0u) {
    } else if (n <= kStep) {
        sum_groups(std::integral_constant<uint32_t, 1>{});
    } else if (n <= 2u * kStep) {
        sum_groups(std::integral_constant<uint32_t, 2>{});
    } else if (n <= 4u * kStep) {
        sum_groups(std::integral_constant<uint32_t, 4>{});
    } else if (n <= 8u * kStep) {
        sum_groups(std::integral_constant<uint32_t, 8>{});
    } else {
        uint32_t i = threadIdx.x * 4u;
        for (; i + 3u * kStep < n4; i += 4u * kStep) {  // four 16-B loads in flight per thread
            uint4 q[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) q[k] = *(const uint4*)(sums + i + k * kStep);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) v += (uint64_t)q[k].x + q[k].y + q[k].z + q[k].w;
        }
        for (; i < n4; i += kStep) {
            const uint4 q = *(const uint4*)(sums + i);
            v += (uint64_t)q.x + q.y + q.z + q.w;
        }
        if (threadIdx.x < n - n4) v += sums[n4 + threadIdx.x];
    }
    // the wave's sum exactly in two 32-bit DPP scans: v < 2^52 (< 2^20 words per thread), so the 64 lanes'
    // low 26-bit parts and their high parts each add up below 2^32
    const uint32_t lo = wave_scan_incl((uint32_t)(v & 0x3FFFFFFull)), hi = wave_scan_incl((uint32_t)(v >> 26));
    v = ((uint64_t)hi << 26) + lo;
    if ((threadIdx.x & 63u) == 63u) lds64[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (int w = 0; w < kProjectBlock / 64; ++w) t += lds64[w];
    __syncthreads();
    return t;
}

// fusedScan (frames of <= kFusedScanMaxBlocks blocks): blockOffsets holds the unscanned block counts;
// each workgroup adds up those before its own -- the offset k_scan_blocks would have written, with
// its saturation at 2^32 - 1 -- and workgroup 0 adds up all of them for the header and resets the
// blend's queue (k_scan_blocks' other duties), so the frame needs no scan launch
__global__ __launch_bounds__(kProjectBlock) void k_scatter(
    ProjectArgs P, const GaussianRenderData* __restrict__ rd, const short4* __restrict__ bounds,
    const uint32_t* __restrict__ counts, const uint32_t* __restrict__ masks,
    const uint32_t* __restrict__ blockOffsets, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
    const float2* __restrict__ sincos, const BlendRecord* __restrict__ rec, const uint32_t* __restrict__ devCount,
    uint32_t fusedScan, TileAssignmentHeader* __restrict__ hdr, uint32_t* __restrict__ blendQueue) {
    __shared__ uint32_t lds[kProjectBlock / 64];
    __shared__ unsigned long long lds64[kProjectBlock / 64];
    __shared__ uint32_t sOff[kProjectBlock];
    __shared__ uint32_t sMask[kProjectBlock];  // 0: no cooperative slots (large rect or no tiles)
    __shared__ uint32_t sRect[kProjectBlock];  // x0 | rw << 16 (rw <= 32)
    __shared__ uint32_t sInv[kProjectBlock];   // ceil(2^16 / rw): bit / rw = (bit * inv) >> 16 for bit < 32
    __shared__ int sTy0[kProjectBlock];        // first row index of the rect in the renderer's rows
    __shared__ uint32_t sD[kProjectBlock];     // depth bits of the key
    __shared__ float2 sBand[kProjectBlock];    // skip-flag band of each gaussian: mean x, half width (< 0: none)
    // the block's first kOwnCap slots: owner << 5 | tile bit of each small-rect slot, kNoOwner for the
    // slots of large rects (their own thread writes them); later slots take the binary search
    constexpr uint32_t kOwnCap = 4096;
    constexpr uint16_t kNoOwner = 0xFFFFu;
    __shared__ uint16_t sOwn[kOwnCap];
    const uint32_t gid = blockIdx.x * kProjectBlock + threadIdx.x;
    // records path: the count lives on the device and the grid covers the capacity
    const uint32_t n = devCount ? min(*devCount, P.count) : P.count;
    if (fusedScan && blockIdx.x == 0) {  // (before any exit: an empty frame still gets its header)
        const uint64_t all = block_sum_prefix(blockOffsets, (n + kProjectBlock - 1u) / kProjectBlock, lds64);
        if (threadIdx.x == 0) {
            uint32_t tot = all > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)all;
            uint32_t ovf = 0;
            if (tot > P.maxAssignments) {
                tot = P.maxAssignments;
                ovf = 1;
            }
            hdr->totalAssignments = tot;
            hdr->maxCapacity = P.maxAssignments;
            hdr->paddedCount = ((tot + 1023u) / 1024u) * 1024u;
            hdr->overflow = ovf;
            for (uint32_t q = 0; q < kQueueStripes; ++q) blendQueue[q * kQueueStride] = 0;
        }
    }
    if (blockIdx.x * kProjectBlock >= n) return;  // (uniform; the scan stopped at the count too)
    // The scatter's once-read inputs (counts, bounds, the records' band half, masks) are streaming loads
    // (nt): they no longer displace the keys and values this kernel writes from the 256 MiB infinity
    // cache, which the first tile pass reads next -- config 3: that pass 64.4-66.1 -> 59.6-61.3 us, nothing
    // else slower (r06, VERDICT r05 item 4: profiles/r06_nt_loads_ab.txt)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define GSM_SLD(p) __builtin_nontemporal_load(p)
    // every input of the block in flight at once, while the block counts are added up (r06: the bounds,
    // band and mask no longer wait for the count -- one memory round trip less per workgroup; a gaussian
    // without tiles reads 28 B it does not use)
    uint32_t c = 0u, mw = 0u;
    unsigned long long rb = 0ull;
    u32x4 r1v = {0u, 0u, 0u, 0u};
    if (gid < n) {
        c = GSM_SLD(counts + gid);
        rb = GSM_SLD((const unsigned long long*)(bounds + gid));
        r1v = GSM_SLD((const u32x4*)(rec + gid) + 1);  // the band k_project left in the padding
        mw = GSM_SLD(masks + gid);
    }
    uint32_t base;
    if (fusedScan) {
        const uint64_t before = blockIdx.x ? block_sum_prefix(blockOffsets, blockIdx.x, lds64) : 0ull;
        base = before > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)before;
    } else {
        base = blockOffsets[blockIdx.x];
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<kProjectBlock>(c, lds, &total);
    bool large = false;
    short4 r = make_short4(0, -1, 0, -1);
    uint32_t dbits = 0;
    int ty0 = 0, ty1 = -1;
    uint32_t mask = 0;
    float2 band = make_float2(0.0f, -1.0f);
    if (c != 0) {
        r = __builtin_bit_cast(short4, rb);
        const uint4 r1 = make_uint4(r1v.x, r1v.y, r1v.z, r1v.w);
        band = make_float2(__uint_as_float(r1.y), __uint_as_float(r1.z));
        // the key's depth: the fp16 depth bits of the blend record (b = colB | depth << 16, the same
        // bits as GaussianRenderData.depth), so the scatter reads one 16-B slot per gaussian
        dbits = ((r1.x >> 16) ^ 0x8000u) & 0xFFFFu;
        // row indices of the renderer's rows inside the rect (the keys carry local tile ids,
        // k * tilesX + tx: the sort, the tile starts and the blend count the renderer's rows only)
        rows_within(rows_of(P), (int)r.z, (int)r.w, &ty0, &ty1);
        const int rw = (int)r.y - (int)r.x + 1;
        large = (ty1 - ty0 + 1) * rw > kMaskTiles;
        if (!large) mask = mw;
        sRect[threadIdx.x] = ((uint32_t)(int)r.x & 0xFFFFu) | ((uint32_t)rw << 16);
        // 2^16 / rw is a power of two (v_rcp_f32 exact) or >= 1/rw >= 1/32 away from an integer, and the
        // 1-ulp reciprocal moves it by <= 2^16 * 2^-23 < 0.008: the ceiling is exact.  With inv = ceil(2^16
        // / rw), (bit * inv) >> 16 = bit / rw for every bit < 32 and rw <= 32 (checked exhaustively)
        sInv[threadIdx.x] = (uint32_t)__builtin_ceilf(65536.0f * __builtin_amdgcn_rcpf((float)rw));
    }
    sOff[threadIdx.x] = off;
    sMask[threadIdx.x] = mask;
    sD[threadIdx.x] = dbits;
    sTy0[threadIdx.x] = ty0;
    sBand[threadIdx.x] = band;
    const uint32_t nOwn = min(total, kOwnCap);
    for (uint32_t i = threadIdx.x; i < nOwn; i += kProjectBlock) sOwn[i] = kNoOwner;
    __syncthreads();
    {  // each small rect lists its slots (<= 32, one per set bit of its mask, in bit order)
        uint32_t m = mask;
        for (uint32_t i = off; m != 0 && i < kOwnCap; ++i) {
            sOwn[i] = (uint16_t)((threadIdx.x << 5) | (uint32_t)__builtin_ctz(m));
            m &= m - 1u;
        }
    }
    __syncthreads();
    for (uint32_t sl = threadIdx.x; sl < total; sl += kProjectBlock) {
        uint32_t lo, bit;
        if (sl < kOwnCap) {
            const uint32_t v = sOwn[sl];
            if (v == kNoOwner) continue;  // a large rect: its own thread writes it
            lo = v >> 5;
            bit = v & 31u;
        } else {
            // owner: the largest g with sOff[g] <= sl (zero-count gaussians share the next offset)
            lo = 0;
            uint32_t hi = kProjectBlock - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (sOff[mid] <= sl) lo = mid;
                else hi = mid - 1;
            }
            uint32_t m = sMask[lo];
            if (m == 0) continue;  // a large rect: its own thread writes it
            for (uint32_t k = sl - sOff[lo]; k > 0; --k) m &= m - 1u;
            bit = (uint32_t)__builtin_ctz(m);
        }
        const uint64_t wp = (uint64_t)base + sl;
        if (wp >= P.maxAssignments) continue;
        const uint32_t rect = sRect[lo];
        const uint32_t rwo = rect >> 16;
        const uint32_t row = (bit * sInv[lo]) >> 16;  // bit / rwo (bit < 32)
        const int k = sTy0[lo] + (int)row, tx = (int)(rect & 0xFFFFu) + (int)(bit - row * rwo);
        keys[wp] = ((uint32_t)(k * (int)P.bin.tilesX + tx) << 16) | sD[lo];
        const float2 bd = sBand[lo];
        vals[wp] = (blockIdx.x * kProjectBlock + lo) | (half_skip_flags(bd.x, bd.y, tx) << kHalfSkipShift);
    }
    if (!large) return;
    uint64_t wp = (uint64_t)base + off;
    if (wp >= P.maxAssignments) return;
    // large rects: repeat the tests (tileScatterIndirectKernel, GlobalShaders.metal:623-678)
    uint4 rdw = *(const uint4*)(rd + gid);
    uint16_t hmx = (uint16_t)(rdw.x & 0xFFFFu), hmy = (uint16_t)(rdw.x >> 16);
    uint16_t thq = (uint16_t)(rdw.y & 0xFFFFu), hs1 = (uint16_t)(rdw.y >> 16);
    uint16_t hs2 = (uint16_t)(rdw.z & 0xFFFFu);
    uint32_t opac = rdw.w >> 24;
    float cx = hbits_to_f(hmx), cy = hbits_to_f(hmy);
    Conic k = conic_from_quant(sincos, thq, hbits_to_f(hs1), hbits_to_f(hs2));
    float w = 2.0f * compute_power((float)opac);
    const RowSet R = rows_of(P);
    for (int kr = ty0; kr <= ty1; ++kr)
        for (int tx = (int)r.x, ty = R.b + kr * R.s; tx <= (int)r.y; ++tx)
            if (intersects_tile(tx, ty, cx, cy, k, w)) {
                if (wp < P.maxAssignments) {
                    uint32_t tile = (uint32_t)(kr * (int)P.bin.tilesX + tx);
                    keys[wp] = (tile << 16) | dbits;
                    vals[wp] = gid | (half_skip_flags(band.x, band.y, tx) << kHalfSkipShift);
                    wp++;
                }
            }
}

__global__ __launch_bounds__(256) void k_tile_starts(const uint32_t* __restrict__ sortedKeys,
                                                     const TileAssignmentHeader* __restrict__ hdr,
                                                     uint32_t tileBegin, uint32_t tileEnd,
                                                     uint32_t* __restrict__ tileStart) {
    const uint32_t total = hdr->totalAssignments;
    const uint32_t stride = gridDim.x * 256u * 4u;
    // 4 consecutive positions per thread and step (one 16-byte load plus the key before them)
    for (uint32_t i0 = (blockIdx.x * 256u + threadIdx.x) * 4u; i0 <= total; i0 += stride) {
        uint32_t k[5];
        k[0] = i0 == 0 ? 0u : sortedKeys[i0 - 1];
        if (i0 + 4u <= total) {
            const uint4 q = *(const uint4*)(sortedKeys + i0);
            k[1] = q.x;
            k[2] = q.y;
            k[3] = q.z;
            k[4] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) k[j + 1] = i0 + j < total ? sortedKeys[i0 + j] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t i = i0 + j;
            if (i > total) break;
            // keys hold slab tiles only (tile count and scatter are limited to [tileBegin, tileEnd))
            const uint32_t prev = i == 0 ? tileBegin - 1u : (k[j] >> 16);
            const uint32_t cur = i == total ? tileEnd : min(k[j + 1] >> 16, tileEnd);
            for (uint32_t t = prev + 1u; t <= cur; ++t) tileStart[t] = i;
        }
    }
}


// ---------------------------------------------------------------------------
// 5. the blend's half-tile lists: per tile, the sorted ids whose skip flag for half h is clear, in
//    list order, compacted to the tile's start in halfVals[h], and their counts.  One workgroup per
//    tile, 1024 entries per step (4 per thread, block scan of the keep counts).
// ---------------------------------------------------------------------------
constexpr uint32_t kHlThreads = 256;
__global__ __launch_bounds__(kHlThreads) void k_half_lists(const uint32_t* __restrict__ tileStart,
                                                           const uint32_t* __restrict__ sortedVals,
                                                           uint32_t tileBegin, uint32_t tileCount,
                                                           uint32_t* __restrict__ half0, uint32_t* __restrict__ half1,
                                                           uint32_t* __restrict__ halfCount) {
    __shared__ uint32_t part[2][kHlThreads / 64];
    const uint32_t t = tileBegin + blockIdx.x;
    const uint32_t start = tileStart[t], n = tileStart[t + 1] - start;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t base0 = 0, base1 = 0;
    for (uint32_t b = 0; b < n; b += 4 * kHlThreads) {
        const uint32_t i0 = b + threadIdx.x * 4u;
        uint32_t v[4];
        uint32_t k0 = 0, k1 = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            v[j] = i0 + j < n ? sortedVals[start + i0 + j] : (3u << kHalfSkipShift);
            k0 += ((v[j] >> kHalfSkipShift) & 1u) ^ 1u;
            k1 += ((v[j] >> (kHalfSkipShift + 1)) & 1u) ^ 1u;
        }
        // exclusive scans of the two keep counts over the block (thread order = list order)
        const uint32_t packed = k0 | (k1 << 16);
        uint32_t inc = wave_scan_incl(packed);
        if (lane == 63) {
            part[0][wave] = inc & 0xFFFFu;
            part[1][wave] = inc >> 16;
        }
        __syncthreads();
        uint32_t off0 = 0, off1 = 0, tot0 = 0, tot1 = 0;
#pragma unroll
        for (uint32_t w = 0; w < kHlThreads / 64; ++w) {
            if (w < wave) {
                off0 += part[0][w];
                off1 += part[1][w];
            }
            tot0 += part[0][w];
            tot1 += part[1][w];
        }
        uint32_t p0 = base0 + off0 + (inc & 0xFFFFu) - k0, p1 = base1 + off1 + (inc >> 16) - k1;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t g = v[j] & kGidMask;
            if (!((v[j] >> kHalfSkipShift) & 1u)) half0[start + p0++] = g;
            if (!((v[j] >> (kHalfSkipShift + 1)) & 1u)) half1[start + p1++] = g;
        }
        base0 += tot0;
        base1 += tot1;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        halfCount[t] = base0;
        halfCount[tileCount + t] = base1;
    }
}

void launch_half_lists(const uint32_t* sortedVals, uint32_t tileBegin, uint32_t numTiles, const DeviceArena& A,
                       uint32_t tileCount, hipStream_t s) {
    if (numTiles == 0) return;
    hipLaunchKernelGGL(k_half_lists, dim3(numTiles), dim3(kHlThreads), 0, s, A.tileStart, sortedVals, tileBegin,
                       tileCount, A.halfVals[0], A.halfVals[1], A.halfCount);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <bool HALF>
static void launch_project_t(uint32_t deg, const void* world, const void* harm, const ProjectArgs& a,
                             const DeviceArena& A, hipStream_t s) {
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    if (blocks == 0 && a.schedUnits == 0) return;  // (an empty frame still orders its blend units)
#define GSM_LAUNCH_PROJ(D)                                                                     \
    hipLaunchKernelGGL((k_project<HALF, D>), dim3(blocks + (a.schedUnits ? 1u : 0u)), dim3(kProjectBlock), 0, s, \
                       world, harm, a, A.renderData, A.bounds, A.rec, A.tileCounts, A.tileMasks,           \
                       A.blockSums, A.sincosTable, A.unitCost, A.unitOrder, A.costMax)
    switch (deg) {
        case 0: GSM_LAUNCH_PROJ(0); break;
        case 1: GSM_LAUNCH_PROJ(1); break;
        case 2: GSM_LAUNCH_PROJ(2); break;
        default: GSM_LAUNCH_PROJ(3); break;
    }
#undef GSM_LAUNCH_PROJ
}

void launch_project(bool halfInput, uint32_t deg, const void* world, const void* harm,
                    const ProjectArgs& a, const DeviceArena& A, hipStream_t s) {
    if (halfInput) launch_project_t<true>(deg, world, harm, a, A, s);
    else launch_project_t<false>(deg, world, harm, a, A, s);
}

template <bool HALF>
static void launch_project_part_t(uint32_t deg, const void* world, const void* harm, const ProjectArgs& a,
                                  const SlabTable& slabs, const PartitionBuffers& B, const float2* sincos,
                                  const DeviceArena* A, hipStream_t s) {
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    const uint32_t sched = (A && a.schedUnits) ? 1u : 0u;
#define GSM_LAUNCH_PPART(D)                                                                                 \
    hipLaunchKernelGGL((k_project_part<HALF, D>), dim3(blocks + sched), dim3(kProjectBlock), 0, s, world,   \
                       harm, a, slabs, B.runs, B.runStride, B.blockSlabCounts, sincos,                      \
                       sched ? A->unitCost : nullptr, sched ? A->unitOrder : nullptr, sched ? A->costMax : nullptr)
    switch (deg) {
        case 0: GSM_LAUNCH_PPART(0); break;
        case 1: GSM_LAUNCH_PPART(1); break;
        case 2: GSM_LAUNCH_PPART(2); break;
        default: GSM_LAUNCH_PPART(3); break;
    }
#undef GSM_LAUNCH_PPART
}

constexpr uint32_t kCopyMaxBlocks = 2048;  // k_part_copy<false>: workgroups loop over the runs
void launch_partition(bool halfInput, uint32_t deg, const void* world, const void* harm,
                      const ProjectArgs& a, const SlabTable& slabs, const PartitionBuffers& B,
                      const float2* sincos, void* send, uint64_t capacity, uint32_t* sendCounts,
                      hipStream_t s) {
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    if (blocks == 0) {
        hipMemsetAsync(sendCounts, 0, slabs.n * sizeof(uint32_t), s);
        return;
    }
    ProjectArgs pa = a;
    pa.schedUnits = 0;  // (the send-buffer path leaves the schedule to the receiving renderer)
    if (halfInput) launch_project_part_t<true>(deg, world, harm, pa, slabs, B, sincos, nullptr, s);
    else launch_project_part_t<false>(deg, world, harm, pa, slabs, B, sincos, nullptr, s);
    hipLaunchKernelGGL(k_part_scan, dim3(slabs.n), dim3(1024), 0, s, B.blockSlabCounts, blocks, sendCounts,
                       CountPublish{});
    hipLaunchKernelGGL(k_part_copy<false>, dim3(min(blocks, kCopyMaxBlocks)), dim3(kProjectBlock), 0, s, B.runs,
                       B.runStride, blocks, slabs.n, B.blockSlabCounts, sendCounts, 0u, nullptr, SlabPeers{},
                       nullptr, MgArrive{}, (SplatRecord*)send, capacity);
}

void launch_partition_counts(bool halfInput, uint32_t deg, const void* world, const void* harm, const ProjectArgs& a,
                             const SlabTable& slabs, const PartitionBuffers& B, const float2* sincos,
                             uint32_t* sendCounts, const DeviceArena& A, const CountPublish& pub, hipStream_t s) {
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    if (blocks > 0 || a.schedUnits > 0) {  // (no ids: the schedule block may still run)
        if (halfInput) launch_project_part_t<true>(deg, world, harm, a, slabs, B, sincos, &A, s);
        else launch_project_part_t<false>(deg, world, harm, a, slabs, B, sincos, &A, s);
    }
    // with no ids the scan still runs: zero counts, published, and the arrival at barrier 0
    CountPublish p = pub;
    if (p.arrive.done) p.arrive.total = slabs.n;
    hipLaunchKernelGGL(k_part_scan, dim3(slabs.n), dim3(1024), 0, s, B.blockSlabCounts, blocks, sendCounts, p);
}

void launch_partition_push(const ProjectArgs& a, uint32_t world, uint32_t rank, const PartitionBuffers& B,
                           const uint32_t* counts, const SlabPeers& peers, uint32_t* recvCount, const SlabTable& slabs,
                           const MgArrive& arrive, hipStream_t s, uint32_t gridCap) {
    (void)slabs;
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    // (no ids here: one workgroup still takes the receive count from the matrix and arrives)
    uint32_t grid = blocks ? blocks : 1u;
    if (gridCap && grid > gridCap) grid = gridCap;
    MgArrive ar = arrive;
    ar.total = grid;
    hipLaunchKernelGGL(k_part_copy<true>, dim3(grid), dim3(kProjectBlock), 0, s, B.runs, B.runStride, blocks, world,
                       B.blockSlabCounts, nullptr, rank, counts, peers, recvCount, ar, nullptr, 0ull);
}

// a grid covering a device-side count: 8 workgroups per CU of a 256-CU device, each looping over the
// 256-record blocks (a grid for the whole capacity spent most of its workgroups finding nothing)
constexpr uint32_t kRecordsInMaxBlocks = 2048;
void launch_records_in(const void* records, const ProjectArgs& a, const DeviceArena& A, hipStream_t s,
                       const uint32_t* devCount) {
    uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    if (blocks == 0 && a.schedUnits == 0) return;  // (an empty frame still orders its blend units)
    if (devCount && blocks > kRecordsInMaxBlocks) blocks = kRecordsInMaxBlocks;
    hipLaunchKernelGGL(k_records_in, dim3(blocks + (a.schedUnits ? 1u : 0u)), dim3(kProjectBlock), 0, s,
                       (const SplatRecord*)records, a, A.renderData, A.bounds, A.rec, A.tileCounts, A.tileMasks,
                       A.blockSums, A.sincosTable, devCount, A.unitCost, A.unitOrder, A.costMax);
}

void launch_scan_sums(uint32_t* sums, uint32_t nb, uint32_t cap, TileAssignmentHeader* hdr, uint32_t* queue,
                      hipStream_t s) {
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kScanThreads), 0, s, sums, nb, cap, hdr, queue,
                       (const uint32_t*)nullptr);
}

void launch_scan_blocks(uint32_t nb, const ProjectArgs& a, const DeviceArena& A, hipStream_t s,
                        const uint32_t* devCount) {
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kScanThreads), 0, s, A.blockSums, nb,
                       a.maxAssignments, A.header, A.tileQueue, devCount);
}

void launch_scatter(const ProjectArgs& a, const DeviceArena& A, hipStream_t s, const uint32_t* devCount,
                    bool fusedScan) {
    const uint32_t blocks = (a.count + kProjectBlock - 1) / kProjectBlock;
    if (blocks == 0) return;  // (the caller scans such a frame with launch_scan_blocks)
    hipLaunchKernelGGL(k_scatter, dim3(blocks), dim3(kProjectBlock), 0, s, a, A.renderData, A.bounds,
                       A.tileCounts, A.tileMasks, A.blockSums, A.keys[0], A.vals[0], A.sincosTable, A.rec, devCount,
                       fusedScan ? 1u : 0u, A.header, A.tileQueue);
}

void launch_headers(const uint32_t* sortedKeys, const FrameGeometry& g, const DeviceArena& A,
                    hipStream_t s) {
    const uint32_t t0 = 0, t1 = g.rowCount * g.tilesX;  // the keys hold local tile ids (k_scatter)
    if (t1 <= t0) return;
    uint32_t blocks = (g.maxAssignments + 1u + 1023u) / 1024u;  // grid-stride over the device-side total
    if (blocks > 4096u) blocks = 4096u;
    hipLaunchKernelGGL(k_tile_starts, dim3(blocks), dim3(256), 0, s, sortedKeys, A.header, t0, t1,
                       A.tileStart);
}

}  // namespace gsm
