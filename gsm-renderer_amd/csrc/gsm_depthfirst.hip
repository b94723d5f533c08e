// gsm_depthfirst.hip -- host orchestration and C ABI (include/gsm_depthfirst.h) of the
// DepthFirst stereo side-by-side path on MI355X.
//
// The C++ analogue of DepthFirstRenderer.renderStereo(target: .sideBySide) ->
// renderStereoSideBySideRaster -> encodeStereoPipeline (DepthFirstRenderer.swift:205-223,
// 469-512, 595-831) over the DepthFirstResources scratch set (DepthFirstResources.swift:380-470).
// One HIP stream replaces the command buffer; grids are capacity-sized and data-dependent
// counts are read on the device, so a frame is enqueue-only.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/gsm_depthfirst.h"
#include "gsm_detmath.h"
#include "gsm_df_internal.h"
#include "gsm_internal.h"

namespace gsm {

class DepthFirstRenderer {
   public:
    static gsm_status create(const gsm_renderer_config& cfg, int hipDevice, DepthFirstRenderer** out);
    ~DepthFirstRenderer() { release(); }
    gsm_status renderStereoSbs(hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& left,
                               const gsm_camera_params& right, const float* scene, uint32_t width, uint32_t height,
                               void* color, size_t pitch);
    gsm_status counters(gsm_depthfirst_counters* out);
    gsm_status debugCopy(int which, void* dst, size_t bytes, size_t* needed);
    gsm_status setProfiling(int flags);
    gsm_status stageTimes(float* ms, int n);
    gsm_status lastGpuTime(double* seconds);

   private:
    DepthFirstRenderer() = default;
    gsm_status alloc(void** p, size_t bytes);
    void release();
    int device_ = -1;
    int numCUs_ = 256;
    gsm_renderer_config config_{};
    Tuning tuning_{};  // A/B switches, read once at create
    uint32_t maxGaussians_ = 1, maxWidth_ = 1, maxHeight_ = 1, maxInstances_ = 4;
    uint32_t maxTiles_ = 1;
    DfArena A_;
    std::vector<void*> allocations_;
    // last frame
    uint32_t lastCount_ = 0, lastTilesX_ = 0, lastTilesY_ = 0;
    uint64_t schedKey_ = ~0ull;  // geometry the unit costs belong to
    unsigned long long* statsBuf_ = nullptr;  // blend walk statistics (profiling bit 1)
    const uint32_t* depthOrder_ = nullptr;
    const uint32_t* instTiles_ = nullptr;
    const uint32_t* instGids_ = nullptr;
    // profiling: a ring of per-stage events
    static constexpr int kRing = 64;
    std::vector<hipEvent_t> events_;  // [kRing][GSM_DF_STAGE_COUNT + 1]
    uint32_t profFrames_ = 0;
    uint32_t sampleFrame_ = 0;  // frames since setProfiling (blend-event sampling)
    int profiling_ = 0;
    hipEvent_t* frameEvents(uint32_t f) { return &events_[(f % kRing) * (GSM_DF_STAGE_COUNT + 1)]; }
};

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

void DepthFirstRenderer::release() {
    if (device_ >= 0) hipSetDevice(device_);
    for (void* p : allocations_) hipFree(p);
    allocations_.clear();
    for (auto& e : events_)
        if (e) hipEventDestroy(e);
    events_.clear();
}

gsm_status DepthFirstRenderer::alloc(void** p, size_t bytes) {
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipMalloc(p, align_up(bytes, 256)) != hipSuccess) {
        *p = nullptr;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    allocations_.push_back(*p);
    return GSM_OK;
}

gsm_status DepthFirstRenderer::create(const gsm_renderer_config& cfg, int hipDevice, DepthFirstRenderer** out) {
    *out = nullptr;
    // DepthFirstRenderer.init guard (DepthFirstRenderer.swift:51-56)
    if (cfg.max_gaussians > kMaxSupportedGaussians) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (cfg.precision != GSM_PRECISION_FLOAT32 && cfg.precision != GSM_PRECISION_FLOAT16)
        return GSM_ERR_INVALID_ARGUMENT;
    if (cfg.color_format > GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB) return GSM_ERR_INVALID_ARGUMENT;
    const uint32_t maxW = cfg.max_width ? cfg.max_width : 1u, maxH = cfg.max_height ? cfg.max_height : 1u;
    const uint64_t tiles = (uint64_t)((maxW + kDfTile - 1) / kDfTile) * ((maxH + kDfTile - 1) / kDfTile);
    if (tiles > 65535u) return GSM_ERR_INVALID_TILE_COUNT;  // 16-bit tile ids (DepthFirstResources.swift)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    int dev = hipDevice;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    if (dev >= ndev || hipSetDevice(dev) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    DepthFirstRenderer* r = new (std::nothrow) DepthFirstRenderer();
    if (!r) return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    r->device_ = dev;
    r->config_ = cfg;
    r->maxGaussians_ = cfg.max_gaussians ? cfg.max_gaussians : 1u;
    r->maxWidth_ = maxW;
    r->maxHeight_ = maxH;
    r->maxTiles_ = (uint32_t)tiles;
    const uint64_t cap64 = 4ull * r->maxGaussians_;  // DepthFirstResources.swift:399
    r->maxInstances_ = (uint32_t)(cap64 > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : cap64);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        delete r;
        return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    r->numCUs_ = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    r->tuning_ = tuning_from_env(dev);
    const size_t G = r->maxGaussians_, cap = r->maxInstances_;
    const size_t nb = (G + kDfBlock - 1) / kDfBlock;
    DfArena& A = r->A_;
    gsm_status st = GSM_OK;
#define GSM_DF_ALLOC(ptr, bytes) \
    do {                         \
        if (st == GSM_OK) st = r->alloc((void**)&(ptr), (bytes)); \
    } while (0)
    GSM_DF_ALLOC(A.renderData, G * sizeof(StereoTiledRenderData));
    GSM_DF_ALLOC(A.bounds, G * sizeof(short4));
    GSM_DF_ALLOC(A.touched, G * 4);
    GSM_DF_ALLOC(A.depthKeys, G * 4);
    GSM_DF_ALLOC(A.blockSums, (nb + 1) * 4);
    GSM_DF_ALLOC(A.instSums, (nb + 1) * 4);
    GSM_DF_ALLOC(A.visHdr, sizeof(TileAssignmentHeader));
    GSM_DF_ALLOC(A.instHdr, sizeof(TileAssignmentHeader));
    for (int i = 0; i < 2; ++i) {
        GSM_DF_ALLOC(A.dkeys[i], G * 4);
        GSM_DF_ALLOC(A.dvals[i], G * 4);
        GSM_DF_ALLOC(A.ikeys[i], cap * 4);
        GSM_DF_ALLOC(A.ivals[i], cap * 4);
    }
    A.radixHistBytes = radix_workspace_bytes(r->maxInstances_ > r->maxGaussians_ ? r->maxInstances_ : r->maxGaussians_);
    GSM_DF_ALLOC(A.radixHist, A.radixHistBytes);
    if (st == GSM_OK &&
        hipMemset(A.radixHist, 0, radix_workspace_bytes(r->maxInstances_ > r->maxGaussians_ ? r->maxInstances_ : r->maxGaussians_)) != hipSuccess)
        st = GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    GSM_DF_ALLOC(A.radixBinTotals, kSortTotalsWords * 4);  // radix_sort_tiles: totals + block table
    GSM_DF_ALLOC(A.starts, ((size_t)r->maxTiles_ + 1) * sizeof(uint32_t));
    GSM_DF_ALLOC(A.queue, kQueueStripes * kQueueStride * sizeof(uint32_t));
    GSM_DF_ALLOC(A.expTable, 65536 * 2);
    GSM_DF_ALLOC(A.unitCost, (size_t)r->maxTiles_ * 2 * sizeof(uint16_t));
    GSM_DF_ALLOC(A.unitOrder, (size_t)r->maxTiles_ * 2 * sizeof(uint32_t));
    GSM_DF_ALLOC(A.costMax, kCostMaxSlots * sizeof(uint32_t));
#undef GSM_DF_ALLOC
    if (st != GSM_OK) {
        delete r;
        return st;
    }
    std::vector<uint16_t> expt(65536);
    for (uint32_t i = 0; i < 65536; ++i) expt[i] = stereo_exp_table_entry((uint16_t)i);
    if (hipMemcpy(A.expTable, expt.data(), 65536 * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(A.visHdr, 0, sizeof(TileAssignmentHeader)) != hipSuccess ||
        hipMemset(A.instHdr, 0, sizeof(TileAssignmentHeader)) != hipSuccess ||
        hipMemset(A.costMax, 0, kCostMaxSlots * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(A.starts, 0, ((size_t)r->maxTiles_ + 1) * sizeof(uint32_t)) != hipSuccess) {
        delete r;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = r;
    return GSM_OK;
}

// per-eye projectCovariance2D terms, the same fp32 operations the reference repeats per gaussian
// (GaussianShared.h:340-355)
static void eye_const(const gsm_camera_params& c, float W, float H, DfEyeConst* e) {
    std::memcpy(e->view, c.view, sizeof(e->view));
    std::memcpy(e->proj, c.proj, sizeof(e->proj));
    const float p00 = c.proj[0], p11 = c.proj[5];
    e->limX = 1.3f * (1.0f / std::fmax(std::fabs(p00), 1e-4f));
    e->limY = 1.3f * (1.0f / std::fmax(std::fabs(p11), 1e-4f));
    e->focalX = W * std::fabs(p00) * 0.5f;
    e->focalY = H * std::fabs(p11) * 0.5f;
}

gsm_status DepthFirstRenderer::renderStereoSbs(hipStream_t s, const gsm_gaussian_input& in,
                                               const gsm_camera_params& left, const gsm_camera_params& right,
                                               const float* scene, uint32_t width, uint32_t height, void* color,
                                               size_t pitch) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    // encodeStereoPipeline guards (DepthFirstRenderer.swift:478, 607) -- errors, not a silent skip
    if (in.gaussian_count > maxGaussians_) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (width == 0 || height == 0 || width > maxWidth_ || height > maxHeight_) return GSM_ERR_INVALID_DIMENSIONS;
    if (!color) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    if (in.gaussian_count > 0 && (!in.gaussians || !in.harmonics)) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    const int fmt = (int)config_.color_format;
    const size_t bpp = fmt == GSM_COLOR_FORMAT_RGBA16F ? 8 : (fmt == GSM_COLOR_FORMAT_RGBA32F ? 16 : 4);
    if (pitch < (size_t)2 * width * bpp) return GSM_ERR_INVALID_BUFFER_SIZE;
    if ((((uintptr_t)color) & 3u) || (pitch & 3u)) return GSM_ERR_INVALID_BUFFER_SIZE;
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;

    DfArgs a;
    std::memset(&a, 0, sizeof(a));
    const float W = (float)width, H = (float)height;
    eye_const(left, W, H, &a.eye[0]);
    eye_const(right, W, H, &a.eye[1]);
    static const float kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::memcpy(a.scene, scene ? scene : kIdentity, sizeof(a.scene));
    {  // length(sceneTransform[0].xyz) (DepthFirstShaders.metal:293)
        float d = a.scene[0] * a.scene[0] + a.scene[1] * a.scene[1];
        d = d + a.scene[2] * a.scene[2];
        a.sceneScale = std::sqrt(d);
    }
    a.width = W;
    a.height = H;
    // makeStereoCameraUniforms: near/far of the left camera (DepthFirstRenderer.swift:583-584)
    a.nearPlane = left.near_plane;
    a.farPlane = left.far_plane;
    const float maxDim = std::fmax(W, H);
    const float maxEig = (maxDim * 2.0f) / 3.0f;
    a.maxEig = maxEig * maxEig;
    a.adjFar = a.farPlane * 0.02f;
    a.adjDen = a.adjFar - a.nearPlane;
    for (int i = 0; i < 3; ++i) a.mid[i] = (left.position[i] + right.position[i]) * 0.5f;
    a.inputIsSRGB = config_.gaussian_color_space == GSM_COLOR_SPACE_SRGB ? 1.0f : 0.0f;
    a.shComponents = in.sh_components;
    a.count = in.gaussian_count;
    // buildBinningParams(gaussianCount:width:height:) on 16x16 tiles (GlobalRenderer.swift:54-70)
    a.tilesX = (width + kDfTile - 1) / kDfTile;
    a.tilesY = (height + kDfTile - 1) / kDfTile;
    a.tileCount = a.tilesX * a.tilesY;
    a.maxInstances = maxInstances_;
    const uint32_t k = in.sh_components;
    const uint32_t deg = k <= 1 ? 0u : (k <= 4 ? 1u : (k <= 9 ? 2u : 3u));
    const bool half = config_.precision == GSM_PRECISION_FLOAT16;
    const uint32_t nb = (a.count + kDfBlock - 1) / kDfBlock;

    // The blend schedule only needs the previous frame's walk lengths: one extra workgroup of the
    // projection launch orders the units while the others project (no side stream, no join).
    const bool costOrder = tuning_.costOrder;
    a.schedUnits = costOrder ? 2u * a.tileCount : 0u;
    {
        const uint64_t key = ((uint64_t)a.tilesX << 32) | a.tilesY;
        if (key != schedKey_) {  // costs of another geometry: start from index order
            hipMemsetAsync(A_.unitCost, 0, (size_t)a.tileCount * 2 * sizeof(uint16_t), s);
            hipMemsetAsync(A_.costMax, 0, kCostMaxSlots * sizeof(uint32_t), s);
            schedKey_ = key;
        }
    }
    const bool prof = (profiling_ & 1) != 0;                   // every stage bracketed
    // only the blend's pair of events, on every frame or every period-th (bits 8-15)
    const uint32_t period = ((uint32_t)profiling_ >> 8) & 0xFFu;
    const bool blendOnly = !prof && (profiling_ & 8) != 0 && (period <= 1 || (sampleFrame_++ % period) == 0);
    hipEvent_t* ev = (prof || blendOnly) ? frameEvents(profFrames_) : nullptr;
    if (prof) hipEventRecord(ev[0], s);
    df_launch_project(half, deg, in.gaussians, in.harmonics, a, A_, s);
    launch_scan_sums(A_.blockSums, nb, maxGaussians_, A_.visHdr, A_.queue, s);
    df_launch_compact(a, A_, s);
    if (prof) hipEventRecord(ev[1], s);
    // DepthRadixSortEncoder, 32-bit keys (DepthFirstRenderer.swift:664-681): stable LSD
    // (3 wide passes of 11/11/10 bits unless GSM_SORT_WIDE=0: the same stable order)
    const int dc = radix_sort_bits(A_.dkeys, A_.dvals, &A_.visHdr->totalAssignments, maxGaussians_, 0, 32,
                                   sort_space(A_), s, tuning_.ballotRank, tuning_.wideSort,
                                   tuning_.sortScanless);
    if (dc == kSortNoSpace) return GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;  // (nothing of the sort launched)
    if (prof) hipEventRecord(ev[2], s);
    df_launch_instance_counts(A_.dvals[dc], a, A_, s);
    launch_scan_sums(A_.instSums, nb, maxInstances_, A_.instHdr, A_.queue, s);
    df_launch_instances(A_.dvals[dc], a, A_, s);  // with the blend's skip flags
    if (prof) hipEventRecord(ev[3], s);
    // TileSortEncoder (DepthFirstRenderer.swift:683-768): stable sort by the 16-bit tile id
    // the last pass also writes the tile ranges' starts (radix_sort_tiles: no pass over the instances)
    const int ic = radix_sort_tiles(A_.ikeys, A_.ivals, &A_.instHdr->totalAssignments, maxInstances_, 0, sort_space(A_),
                                    A_.starts, 0u, a.tileCount, a.tileCount, s, tuning_.ballotRank,
                                    tuning_.wideSort, tuning_.sortScanless);
    if (ic == kSortNoSpace) return GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;
    // Blend schedule: (tile, eye) units handed out longest first by the walk lengths the previous
    // frame of the same geometry measured (the image does not depend on the order, only the load
    // balance does).  Tuning::costOrder false (GSM_BLEND_SCHED=0 at create): index order.

    A_.blendStats = (profiling_ & 2) ? statsBuf_ : nullptr;
    if (A_.blendStats) hipMemsetAsync(statsBuf_, 0, 4 * sizeof(unsigned long long), s);
    if (prof || blendOnly) hipEventRecord(ev[4], s);
    df_launch_blend(A_.ivals[ic], a, A_, color, pitch, fmt, numCUs_, costOrder, s);
    if (prof || blendOnly) {
        hipEventRecord(ev[5], s);
        profFrames_++;
    }
    lastCount_ = a.count;
    lastTilesX_ = a.tilesX;
    lastTilesY_ = a.tilesY;
    depthOrder_ = A_.dvals[dc];
    instTiles_ = A_.ikeys[ic];
    instGids_ = A_.ivals[ic];
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status DepthFirstRenderer::counters(gsm_depthfirst_counters* out) {
    hipSetDevice(device_);
    TileAssignmentHeader v, i;
    if (hipMemcpy(&v, A_.visHdr, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&i, A_.instHdr, sizeof(i), hipMemcpyDeviceToHost) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    out->gaussian_count = lastCount_;
    out->visible = v.totalAssignments;
    out->total_instances = i.totalAssignments;
    out->max_instances = maxInstances_;
    out->overflow = i.overflow;
    out->tiles_x = lastTilesX_;
    out->tiles_y = lastTilesY_;
    out->tile_count = lastTilesX_ * lastTilesY_;
    return GSM_OK;
}

gsm_status DepthFirstRenderer::debugCopy(int which, void* dst, size_t bytes, size_t* needed) {
    gsm_depthfirst_counters c;
    gsm_status st = counters(&c);
    if (st != GSM_OK) return st;
    const size_t n = lastCount_;
    const void* src = nullptr;
    size_t full = 0;
    switch (which) {
        case GSM_DF_BUF_RENDER_DATA: src = A_.renderData; full = n * 32; break;
        case GSM_DF_BUF_BOUNDS: full = n * 16; break;
        case GSM_DF_BUF_TOUCHED: src = A_.touched; full = n * 4; break;
        case GSM_DF_BUF_DEPTH_KEYS: src = A_.depthKeys; full = n * 4; break;
        case GSM_DF_BUF_DEPTH_ORDER: src = depthOrder_; full = (size_t)c.visible * 4; break;
        case GSM_DF_BUF_INSTANCE_TILES: src = instTiles_; full = (size_t)c.total_instances * 4; break;
        case GSM_DF_BUF_INSTANCE_GAUSSIANS: src = instGids_; full = (size_t)c.total_instances * 4; break;
        case GSM_DF_BUF_HEADERS: full = (size_t)c.tile_count * 8; break;
        case GSM_DF_BUF_BLEND_STATS: src = (profiling_ & 2) ? statsBuf_ : nullptr; full = 32; break;
        default: return GSM_ERR_INVALID_ARGUMENT;
    }
    if (needed) *needed = full;
    if (!dst || bytes == 0 || full == 0) return GSM_OK;
    const size_t cpy = bytes < full ? bytes : full;
    if (which == GSM_DF_BUF_BOUNDS) {  // short4 on the device, int4 in the reference buffer
        std::vector<short4> b(n);
        if (hipMemcpy(b.data(), A_.bounds, n * sizeof(short4), hipMemcpyDeviceToHost) != hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        std::vector<int32_t> w(n * 4);
        for (size_t i = 0; i < n; ++i) {
            w[4 * i] = b[i].x;
            w[4 * i + 1] = b[i].y;
            w[4 * i + 2] = b[i].z;
            w[4 * i + 3] = b[i].w;
        }
        std::memcpy(dst, w.data(), cpy);
        return GSM_OK;
    }
    if (which == GSM_DF_BUF_HEADERS) {  // GaussianHeader {offset, count} from the run starts
        std::vector<uint32_t> st((size_t)c.tile_count + 1);
        if (hipMemcpy(st.data(), A_.starts, st.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        std::vector<uint32_t> h((size_t)c.tile_count * 2);
        for (size_t t = 0; t < c.tile_count; ++t) {
            h[2 * t] = st[t];
            h[2 * t + 1] = st[t + 1] - st[t];
        }
        std::memcpy(dst, h.data(), cpy);
        return GSM_OK;
    }
    if (!src) return GSM_ERR_RENDER_FAILED;
    if (hipMemcpy(dst, src, cpy, hipMemcpyDeviceToHost) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    if (which == GSM_DF_BUF_INSTANCE_GAUSSIANS) {  // drop the blend's skip flags (kDfSkipShift)
        uint32_t* v = (uint32_t*)dst;
        for (size_t i = 0; i < cpy / 4; ++i) v[i] &= kDfGidMask;
    }
    return GSM_OK;
}

gsm_status DepthFirstRenderer::setProfiling(int flags) {
    hipSetDevice(device_);
    if ((flags & 2) && !statsBuf_) {
        gsm_status st = alloc((void**)&statsBuf_, 4 * sizeof(unsigned long long));
        if (st != GSM_OK) return st;
    }
    if ((flags & 9) && events_.empty()) {  // bit 0: every stage, bit 3: the blend only
        events_.assign((size_t)kRing * (GSM_DF_STAGE_COUNT + 1), nullptr);
        for (auto& e : events_)
            if (hipEventCreate(&e) != hipSuccess) return GSM_ERR_ENCODER_CREATION_FAILED;
    }
    profiling_ = flags;
    profFrames_ = 0;
    sampleFrame_ = 0;
    return GSM_OK;
}

gsm_status DepthFirstRenderer::stageTimes(float* ms, int n) {
    if (profFrames_ == 0 || events_.empty()) return GSM_ERR_RENDER_FAILED;
    hipSetDevice(device_);
    if (hipEventSynchronize(frameEvents(profFrames_ - 1)[GSM_DF_STAGE_COUNT]) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    const uint32_t frames = profFrames_ < (uint32_t)kRing ? profFrames_ : (uint32_t)kRing;
    const bool blendOnly = (profiling_ & 1) == 0;
    for (int i = 0; i < n && i < GSM_DF_STAGE_COUNT; ++i) {
        if (blendOnly && i != GSM_DF_STAGE_BLEND) {
            ms[i] = 0.0f;
            continue;
        }
        double acc = 0.0;
        for (uint32_t f = profFrames_ - frames; f < profFrames_; ++f) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, frameEvents(f)[i], frameEvents(f)[i + 1]) != hipSuccess)
                return GSM_ERR_RENDER_FAILED;
            acc += t;
        }
        ms[i] = (float)(acc / frames);
    }
    return GSM_OK;
}

gsm_status DepthFirstRenderer::lastGpuTime(double* seconds) {
    if (profFrames_ == 0 || events_.empty() || (profiling_ & 1) == 0) return GSM_ERR_RENDER_FAILED;
    hipSetDevice(device_);
    hipEvent_t* ev = frameEvents(profFrames_ - 1);
    if (hipEventSynchronize(ev[GSM_DF_STAGE_COUNT]) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    float t = 0.f;
    if (hipEventElapsedTime(&t, ev[0], ev[GSM_DF_STAGE_COUNT]) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    *seconds = (double)t * 1e-3;
    return GSM_OK;
}

}  // namespace gsm

struct gsm_depthfirst {
    gsm::DepthFirstRenderer* impl;
};

extern "C" {

gsm_status gsm_depthfirst_create(const gsm_renderer_config* config, int hip_device, gsm_depthfirst** out) {
    if (!config || !out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    gsm::DepthFirstRenderer* impl = nullptr;
    gsm_status st = gsm::DepthFirstRenderer::create(*config, hip_device, &impl);
    if (st != GSM_OK) return st;
    gsm_depthfirst* h = new (std::nothrow) gsm_depthfirst;
    if (!h) {
        delete impl;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    h->impl = impl;
    *out = h;
    return GSM_OK;
}

void gsm_depthfirst_destroy(gsm_depthfirst* r) {
    if (!r) return;
    delete r->impl;
    delete r;
}

gsm_status gsm_depthfirst_render_stereo_sbs(gsm_depthfirst* r, void* stream, const gsm_gaussian_input* input,
                                            const gsm_camera_params* left, const gsm_camera_params* right,
                                            const float* scene_transform, uint32_t width, uint32_t height,
                                            void* color, size_t color_pitch_bytes) {
    if (!r || !input || !left || !right) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->renderStereoSbs((hipStream_t)stream, *input, *left, *right, scene_transform, width, height,
                                    color, color_pitch_bytes);
}

gsm_status gsm_depthfirst_debug_counters(gsm_depthfirst* r, gsm_depthfirst_counters* out) {
    if (!r || !out) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->counters(out);
}

gsm_status gsm_depthfirst_debug_copy(gsm_depthfirst* r, int which, void* host_dst, size_t bytes, size_t* needed) {
    if (!r) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->debugCopy(which, host_dst, bytes, needed);
}

gsm_status gsm_depthfirst_set_profiling(gsm_depthfirst* r, int enable) {
    if (!r) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->setProfiling(enable);
}

gsm_status gsm_depthfirst_stage_times(gsm_depthfirst* r, float* ms, int n) {
    if (!r || !ms) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->stageTimes(ms, n);
}

gsm_status gsm_depthfirst_last_gpu_time(gsm_depthfirst* r, double* seconds) {
    if (!r || !seconds) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->lastGpuTime(seconds);
}

}  // extern "C"
