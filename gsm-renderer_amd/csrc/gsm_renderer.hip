// gsm_renderer.hip -- host orchestration of one GlobalRenderer frame on MI355X.
//
// The C++ analogue of GlobalRenderer.swift (frame orchestration, :110-572) and
// GlobalResources.swift (up-front scratch arena, :58-361).  One HIP stream replaces
// the Metal command buffer; every grid size is a host constant (capacity-sized) and
// data-dependent counts are read on the device, so a frame is enqueue-only and can
// be captured into a hipGraph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/gsm_debug.h"
#include "../../include/gsm_renderer.h"
#include "gsm_detmath.h"
#include "gsm_internal.h"
#include "gsm_renderer_impl.h"

namespace gsm {

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

GlobalRenderer::~GlobalRenderer() { release(); }

void GlobalRenderer::release() {
    if (device_ >= 0) hipSetDevice(device_);
    for (void* p : allocations_) hipFree(p);
    allocations_.clear();
    for (auto& e : events_)
        if (e) hipEventDestroy(e);
    events_.clear();
}

gsm_status GlobalRenderer::alloc(void** p, size_t bytes) {
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipMalloc(p, bytes) != hipSuccess) {
        *p = nullptr;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    allocations_.push_back(*p);
    return GSM_OK;
}

gsm_status GlobalRenderer::create(const gsm_renderer_config& cfg, int hipDevice, GlobalRenderer** out) {
    *out = nullptr;
    // GlobalRenderer.init guard (GlobalRenderer.swift:111-113)
    if (cfg.max_gaussians > kMaxSupportedGaussians) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (cfg.precision != GSM_PRECISION_FLOAT32 && cfg.precision != GSM_PRECISION_FLOAT16)
        return GSM_ERR_INVALID_ARGUMENT;
    if (cfg.color_format > GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB) return GSM_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    int dev = hipDevice;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    if (dev >= ndev) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    if (hipSetDevice(dev) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;

    GlobalRenderer* r = new (std::nothrow) GlobalRenderer();
    if (!r) return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    r->device_ = dev;
    r->config_ = cfg;
    // RendererLimits (GlobalRenderer.swift:6-23)
    r->maxGaussians_ = cfg.max_gaussians ? cfg.max_gaussians : 1u;
    r->maxWidth_ = cfg.max_width ? cfg.max_width : 1u;
    r->maxHeight_ = cfg.max_height ? cfg.max_height : 1u;
    r->tilesX_ = (r->maxWidth_ + kTileWidth - 1) / kTileWidth;
    r->tilesY_ = (r->maxHeight_ + kTileHeight - 1) / kTileHeight;
    r->tileCount_ = r->tilesX_ * r->tilesY_;
    if (r->tileCount_ > 65536u) {  // 16-bit tile field of the sort key (GlobalShaders.metal:288)
        delete r;
        return GSM_ERR_INVALID_TILE_COUNT;
    }
    r->rowBegin_ = 0;
    r->rowEnd_ = r->tilesY_;
    const uint64_t cap64 = 4ull * r->maxGaussians_;  // GlobalResources.swift:79
    r->maxAssignments_ = (uint32_t)(cap64 > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : cap64);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        delete r;
        return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    r->numCUs_ = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    r->tuning_ = tuning_from_env(dev);

    const size_t G = r->maxGaussians_;
    const size_t cap = r->maxAssignments_;
    const size_t nb = (G + kProjectBlock - 1) / kProjectBlock;
    DeviceArena& A = r->arena_;
    gsm_status st = GSM_OK;
#define GSM_ALLOC(ptr, bytes)                                              \
    do {                                                                   \
        if (st == GSM_OK) st = r->alloc((void**)&(ptr), align_up((bytes), 256)); \
    } while (0)
    GSM_ALLOC(A.renderData, G * sizeof(GaussianRenderData));
    GSM_ALLOC(A.bounds, G * sizeof(short4));
    GSM_ALLOC(A.rec, G * sizeof(BlendRecord));
    GSM_ALLOC(A.tileCounts, G * sizeof(uint32_t));
    GSM_ALLOC(A.tileMasks, G * sizeof(uint32_t));
    GSM_ALLOC(A.blockSums, (nb + 1) * sizeof(uint32_t));
    GSM_ALLOC(A.header, sizeof(TileAssignmentHeader));
    GSM_ALLOC(A.keys[0], cap * sizeof(uint32_t));
    GSM_ALLOC(A.keys[1], cap * sizeof(uint32_t));
    GSM_ALLOC(A.vals[0], cap * sizeof(uint32_t));
    GSM_ALLOC(A.vals[1], cap * sizeof(uint32_t));
    A.radixHistBytes = radix_workspace_bytes(r->maxAssignments_);
    GSM_ALLOC(A.radixHist, A.radixHistBytes);
    if (st == GSM_OK && hipMemset(A.radixHist, 0, radix_workspace_bytes(r->maxAssignments_)) != hipSuccess)
        st = GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    GSM_ALLOC(A.radixBinTotals, kSortTotalsWords * sizeof(uint32_t));  // radix_sort_tiles: totals + block table
    GSM_ALLOC(A.tileStart, ((size_t)r->tileCount_ + 1) * sizeof(uint32_t));
    GSM_ALLOC(A.tileQueue, kQueueStripes * kQueueStride * sizeof(uint32_t));
    GSM_ALLOC(A.unitCost, (size_t)r->tileCount_ * 4 * sizeof(uint16_t));
    GSM_ALLOC(A.unitOrder, (size_t)r->tileCount_ * 4 * sizeof(uint32_t));
    GSM_ALLOC(A.costMax, (kCostMaxSlots + 2) * sizeof(uint32_t));
    GSM_ALLOC(A.halfVals[0], cap * sizeof(uint32_t));
    GSM_ALLOC(A.halfVals[1], cap * sizeof(uint32_t));
    GSM_ALLOC(A.halfCount, (size_t)r->tileCount_ * 2 * sizeof(uint32_t));
    GSM_ALLOC(A.expTable, 65536 * sizeof(uint16_t));
    GSM_ALLOC(A.sincosTable, (kSincosEntries + 256) * sizeof(float2));
#undef GSM_ALLOC
    if (st != GSM_OK) {
        delete r;
        return st;
    }
    r->sched_[0] = {A.unitCost, A.unitOrder, A.costMax};
    // numeric-contract tables (gsm_detmath.h)
    std::vector<uint16_t> expt(65536);
    for (uint32_t i = 0; i < 65536; ++i) expt[i] = blend_exp_table_entry((uint16_t)i);
    std::vector<float2> sc(kSincosEntries + 256);
    for (uint32_t i = 0; i < kSincosEntries; ++i) det_sincos_table_entry(i, &sc[i].x, &sc[i].y);
    for (uint32_t c = 0; c < 256; ++c) {
        uint32_t d;
        det_byte_lut_entry(c, &sc[kSincosEntries + c].x, &d);
        std::memcpy(&sc[kSincosEntries + c].y, &d, 4);  // (bits, not a value)
    }
    if (hipMemcpy(A.expTable, expt.data(), 65536 * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(A.sincosTable, sc.data(), sc.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(A.header, 0, sizeof(TileAssignmentHeader)) != hipSuccess ||
        hipMemset(A.tileStart, 0, ((size_t)r->tileCount_ + 1) * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(A.unitCost, 0, (size_t)r->tileCount_ * 4 * sizeof(uint16_t)) != hipSuccess ||
        hipMemset(A.costMax, 0, (kCostMaxSlots + 2) * sizeof(uint32_t)) != hipSuccess ||
        // every entry of the value buffers is a valid gaussian id at all times (the blend's
        // clamped, unpredicated gathers may read entry 0 of an empty frame)
        hipMemset(A.vals[0], 0, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(A.vals[1], 0, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(A.halfVals[0], 0, cap * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(A.halfVals[1], 0, cap * sizeof(uint32_t)) != hipSuccess) {
        delete r;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = r;
    return GSM_OK;
}

int GlobalRenderer::sortPassCount() const {
    // RadixSortEncoder.swift:52-63: depth bytes (2) + bytes of (tileCount-1), max 4.
    int tileBytes = 1;
    uint32_t remaining = tileCount_ > 0 ? tileCount_ - 1 : 0;
    while (remaining >= 256) {
        tileBytes++;
        remaining >>= 8;
    }
    int p = 2 + tileBytes;
    return p > 4 ? 4 : p;
}

ProjectArgs GlobalRenderer::frameArgs(const gsm_camera_params& camp, uint32_t width, uint32_t height,
                                      uint32_t count, uint32_t shComponents) const {
    ProjectArgs a;
    std::memset(&a, 0, sizeof(a));
    // CameraUniforms(from: camera, ...) (KernelTypes.swift:107-123)
    std::memcpy(a.cam.view, camp.view, sizeof(a.cam.view));
    std::memcpy(a.cam.proj, camp.proj, sizeof(a.cam.proj));
    std::memcpy(a.cam.cameraCenter, camp.position, sizeof(a.cam.cameraCenter));
    a.cam.pixelFactor = 1.0f;
    a.cam.focalX = camp.focal_x;
    a.cam.focalY = camp.focal_y;
    a.cam.width = (float)width;
    a.cam.height = (float)height;
    a.cam.nearPlane = camp.near_plane;
    a.cam.farPlane = camp.far_plane;
    a.cam.shComponents = shComponents;
    a.cam.gaussianCount = count;
    a.cam.inputIsSRGB = config_.gaussian_color_space == GSM_COLOR_SPACE_SRGB ? 1.0f : 0.0f;
    // buildBinningParams (GlobalRenderer.swift:38-51)
    a.bin.gaussianCount = count;
    a.bin.tilesX = tilesX_;
    a.bin.tilesY = tilesY_;
    a.bin.tileWidth = kTileWidth;
    a.bin.tileHeight = kTileHeight;
    a.bin.surfaceWidth = maxWidth_;
    a.bin.surfaceHeight = maxHeight_;
    a.bin.maxCapacity = count;
    a.bin.alphaThreshold = 0.005f;
    a.bin.totalInkThreshold = 2.0f;
    a.rowBegin = rowBegin_;
    a.rowEnd = rowEnd_;
    a.rowStride = rowStride_;
    a.count = count;
    a.maxAssignments = maxAssignments_;
    // uniform terms of the projection, same operation order as the per-gaussian code
    const float p00 = a.cam.proj[0], p11 = a.cam.proj[5];
    a.limX = 1.3f * (1.0f / std::fmax(std::fabs(p00), 1e-4f));
    a.limY = 1.3f * (1.0f / std::fmax(std::fabs(p11), 1e-4f));
    a.focalX = a.cam.width * std::fabs(p00) * 0.5f;
    a.focalY = a.cam.height * std::fabs(p11) * 0.5f;
    const float maxDim = std::fmax(a.cam.width, a.cam.height);
    const float maxEig = (maxDim * 2.0f) / 3.0f;
    a.maxEig = maxEig * maxEig;
    a.adjFar = a.cam.farPlane * 0.02f;
    a.adjDen = a.adjFar - a.cam.nearPlane;

    return a;
}

gsm_status GlobalRenderer::validateFrame(uint32_t count, bool inputMissing, uint32_t width, uint32_t height,
                                         const void* color, size_t colorPitch, const void* depth,
                                         size_t depthPitch) const {
    // validateLimits (GlobalRenderer.swift:372-376) -- errors instead of a silent skip
    if (count > maxGaussians_) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (width == 0 || height == 0 || width > maxWidth_ || height > maxHeight_)
        return GSM_ERR_INVALID_DIMENSIONS;
    if (!color) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    if (count > 0 && inputMissing) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    const size_t bpp = config_.color_format == GSM_COLOR_FORMAT_RGBA16F ? 8
                       : (config_.color_format == GSM_COLOR_FORMAT_RGBA32F ? 16 : 4);
    if (colorPitch < (size_t)width * bpp) return GSM_ERR_INVALID_BUFFER_SIZE;
    // the blend stores at least 4-byte words of colour and 2-byte depth values
    if ((((uintptr_t)color) & 3u) || (colorPitch & 3u)) return GSM_ERR_INVALID_BUFFER_SIZE;
    if (depth && ((((uintptr_t)depth) & 1u) || (depthPitch & 1u))) return GSM_ERR_INVALID_BUFFER_SIZE;
    if (depth && depthPitch < (size_t)width * 2) return GSM_ERR_INVALID_BUFFER_SIZE;
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    return GSM_OK;
}

gsm_status GlobalRenderer::render(hipStream_t s, const gsm_gaussian_input& in,
                                  const gsm_camera_params& camp, uint32_t width, uint32_t height,
                                  void* color, size_t colorPitch, void* depth, size_t depthPitch) {
    gsm_status st = validateFrame(in.gaussian_count, !in.gaussians || !in.harmonics, width, height, color,
                                  colorPitch, depth, depthPitch);
    if (st != GSM_OK) return st;
    // the projection's tile tests walk contiguous rows; interleaved row sets come from the records
    // path only (gsm_multigpu)
    if (rowStride_ != 1) return GSM_ERR_INVALID_ARGUMENT;
    const ProjectArgs a = frameArgs(camp, width, height, in.gaussian_count, in.sh_components);
    // GlobalProjectCullEncoder.swift:19-26 SH_DEGREE selection
    const uint32_t k = in.sh_components;
    const uint32_t deg = k <= 1 ? 0u : (k <= 4 ? 1u : (k <= 9 ? 2u : 3u));
    const bool half = config_.precision == GSM_PRECISION_FLOAT16;
    return runFrame(s, a, width, height, color, colorPitch, depth, depthPitch,
                    [&](const ProjectArgs& pa) {
                        launch_project(half, deg, in.gaussians, in.harmonics, pa, arena_, s);
                    });
}

gsm_status GlobalRenderer::renderRecords(hipStream_t s, const void* records, uint32_t count, uint32_t width,
                                         uint32_t height, void* color, size_t colorPitch, void* depth,
                                         size_t depthPitch, const uint32_t* devCount, bool preOrdered,
                                         const MgArrive* blendArrive) {
    // devCount: the count lives on the device (multi-GPU exchange, gsm_multigpu_render); `count` is
    // then the capacity the grids cover
    gsm_status st = validateFrame(count, !records, width, height, color, colorPitch, depth, depthPitch);
    if (st != GSM_OK) return st;
    gsm_camera_params cam;
    std::memset(&cam, 0, sizeof(cam));
    const ProjectArgs a = frameArgs(cam, width, height, count, 1);
    return runFrame(s, a, width, height, color, colorPitch, depth, depthPitch,
                    [&](const ProjectArgs& pa) {
                        launch_records_in(records, pa, arena_, s, devCount);
                    }, devCount, preOrdered, blendArrive);
}

gsm_status GlobalRenderer::preparePartition(const gsm_gaussian_input& in, const gsm_camera_params& camp,
                                            uint32_t width, uint32_t height, uint32_t first, uint32_t count,
                                            const uint32_t* slabRows, uint32_t numSlabs, bool needSend,
                                            const void* send, const uint32_t* sendCounts, PartitionFrame* f,
                                            bool interleave) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    if ((uint64_t)first + count > in.gaussian_count || count > maxGaussians_)
        return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (width == 0 || height == 0 || width > maxWidth_ || height > maxHeight_)
        return GSM_ERR_INVALID_DIMENSIONS;
    if (!slabRows || numSlabs == 0 || numSlabs > kMaxSlabs) return GSM_ERR_INVALID_ARGUMENT;
    if (!sendCounts || (count > 0 && ((needSend && !send) || !in.gaussians || !in.harmonics)))
        return GSM_ERR_MISSING_REQUIRED_BUFFER;
    std::memset(&f->slabs, 0, sizeof(f->slabs));
    f->slabs.n = numSlabs;
    f->slabs.interleave = interleave ? 1u : 0u;  // slab s = rows s, s + n, ... < slabRows[n]
    for (uint32_t i = 0; i <= numSlabs; ++i) {
        if (slabRows[i] > tilesY_ || (!interleave && i > 0 && slabRows[i] < slabRows[i - 1]))
            return GSM_ERR_INVALID_ARGUMENT;
        f->slabs.rows[i] = slabRows[i];
    }
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    gsm_status st = ensurePartitionBuffers(numSlabs);
    if (st != GSM_OK) return st;
    f->half = config_.precision == GSM_PRECISION_FLOAT16;
    f->a = frameArgs(camp, width, height, count, in.sh_components);
    f->a.rowBegin = 0;  // the rank's ids are projected against the whole frame
    f->a.rowEnd = tilesY_;
    f->a.rowStride = 1;
    const size_t ws = f->half ? sizeof(PackedWorldGaussianHalf) : sizeof(PackedWorldGaussian);
    const size_t hs = (size_t)in.sh_components * 3 * (f->half ? 2 : 4);
    f->world = (const char*)in.gaussians + (size_t)first * ws;
    f->harm = (const char*)in.harmonics + (size_t)first * hs;
    const uint32_t k = in.sh_components;
    f->deg = k <= 1 ? 0u : (k <= 4 ? 1u : (k <= 9 ? 2u : 3u));
    return GSM_OK;
}

gsm_status GlobalRenderer::ensurePartitionBuffers(uint32_t numSlabs) {
    // lazily: only ranks of a partitioned frame need these (the multi-GPU frame: at prepare)
    if (part_.runs && part_.runSlabs >= numSlabs) return GSM_OK;
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    const size_t blocks = ((size_t)maxGaussians_ + kProjectBlock - 1) / kProjectBlock;
    PartitionBuffers b = part_;
    b.runStride = (uint32_t)(blocks * kProjectBlock);
    b.runSlabs = numSlabs;
    // (a buffer for fewer slabs stays allocated until the renderer is destroyed)
    gsm_status st = alloc((void**)&b.runs, (size_t)numSlabs * b.runStride * sizeof(SplatRecord));
    if (st == GSM_OK && !b.blockSlabCounts) st = alloc((void**)&b.blockSlabCounts, kMaxSlabs * (blocks + 1) * 4);
    if (st == GSM_OK) part_ = b;
    if (st == GSM_OK && !sched_[1].unitOrder) {
        ScheduleSet t;
        st = alloc((void**)&t.unitCost, (size_t)tileCount_ * 4 * sizeof(uint16_t));
        if (st == GSM_OK) st = alloc((void**)&t.unitOrder, (size_t)tileCount_ * 4 * sizeof(uint32_t));
        if (st == GSM_OK) st = alloc((void**)&t.costMax, (kCostMaxSlots + 2) * sizeof(uint32_t));
        if (st == GSM_OK && (hipMemset(t.unitCost, 0, (size_t)tileCount_ * 4 * sizeof(uint16_t)) != hipSuccess ||
                             hipMemset(t.costMax, 0, (kCostMaxSlots + 2) * sizeof(uint32_t)) != hipSuccess ||
                             hipDeviceSynchronize() != hipSuccess))
            st = GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
        if (st == GSM_OK) sched_[1] = t;
    }
    return st;
}

void GlobalRenderer::selectSchedule(uint32_t parity) {
    const ScheduleSet& t = sched_[(parity & 1u) && sched_[1].unitOrder ? 1 : 0];
    arena_.unitCost = t.unitCost;
    arena_.unitOrder = t.unitOrder;
    arena_.costMax = t.costMax;
}

gsm_status GlobalRenderer::projectPartition(hipStream_t s, const gsm_gaussian_input& in,
                                            const gsm_camera_params& camp, uint32_t width, uint32_t height,
                                            uint32_t first, uint32_t count, const uint32_t* slabRows,
                                            uint32_t numSlabs, void* send, uint64_t capacity,
                                            uint32_t* sendCounts, bool interleave) {
    PartitionFrame f;
    gsm_status st = preparePartition(in, camp, width, height, first, count, slabRows, numSlabs, true, send,
                                     sendCounts, &f, interleave);
    if (st != GSM_OK) return st;
    launch_partition(f.half, f.deg, f.world, f.harm, f.a, f.slabs, part_, arena_.sincosTable, send, capacity,
                     sendCounts, s);
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status GlobalRenderer::partitionCounts(hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& camp,
                                           uint32_t width, uint32_t height, uint32_t first, uint32_t count,
                                           const uint32_t* slabRows, uint32_t numSlabs, uint32_t* sendCounts,
                                           bool orderUnits, bool interleave, const CountPublish* publish) {
    PartitionFrame f;
    gsm_status st = preparePartition(in, camp, width, height, first, count, slabRows, numSlabs, false, nullptr,
                                     sendCounts, &f, interleave);
    if (st != GSM_OK) return st;
    // the blend units of this renderer's rows (its slab), ordered by one extra workgroup of the launch
    f.a.schedUnits = orderUnits ? scheduleUnits(s, width, height) : 0u;
    f.a.pairBucket = tuning_.blendPairs ? (uint32_t)std::max(1, tuning_.pairBucket) : kUoBuckets;
    launch_partition_counts(f.half, f.deg, f.world, f.harm, f.a, f.slabs, part_, arena_.sincosTable, sendCounts,
                            arena_, publish ? *publish : CountPublish{}, s);
    partCount_ = count;
    partSlabs_ = f.slabs;
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status GlobalRenderer::partitionPush(hipStream_t s, uint32_t world, uint32_t rank, const uint32_t* counts,
                                         const SlabPeers& peers, uint32_t* recvCount, const MgArrive& arrive) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    ProjectArgs a;
    std::memset(&a, 0, sizeof(a));
    a.count = partCount_;
    if (world != partSlabs_.n) return GSM_ERR_INVALID_ARGUMENT;  // one slab per rank, as partitionCounts split
    launch_partition_push(a, world, rank, part_, counts, peers, recvCount, partSlabs_, arrive, s,
                          (uint32_t)(4 * numCUs_));  // 4 workgroups per CU looping over the runs
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

uint32_t GlobalRenderer::scheduleUnits(hipStream_t s, uint32_t width, uint32_t height) {
    const uint32_t upt = blend_units_per_tile(rowCount() * tilesX_, numCUs_);
    const uint32_t units = rowCount() * tilesX_ * upt;
    const uint64_t key = ((uint64_t)upt << 60) ^ ((uint64_t)width << 40) ^ ((uint64_t)height << 20) ^
                         ((uint64_t)rowStride_ << 30) ^ ((uint64_t)rowBegin_ << 10) ^ rowEnd_;
    if (key != schedKey_) {  // new geometry: no walks to order by yet (either schedule set)
        for (const ScheduleSet& t : sched_) {
            if (!t.unitCost) continue;
            hipMemsetAsync(t.unitCost, 0, (size_t)units * sizeof(uint16_t), s);
            hipMemsetAsync(t.costMax, 0, (kCostMaxSlots + 2) * sizeof(uint32_t), s);
        }
        schedKey_ = key;
    }
    return tuning_.costOrder ? units : 0u;
}

template <class Front>
gsm_status GlobalRenderer::runFrame(hipStream_t s, const ProjectArgs& a, uint32_t width, uint32_t height,
                                    void* color, size_t colorPitch, void* depth, size_t depthPitch,
                                    Front&& front, const uint32_t* devCount, bool preOrdered,
                                    const MgArrive* blendArrive) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    const bool prof = (profiling_ & 1) != 0;         // every stage bracketed by events
    // only the blend (2 events per frame), on every frame or every period-th (bits 8-15)
    const uint32_t period = ((uint32_t)profiling_ >> 8) & 0xFFu;
    const bool blendOnly = !prof && (profiling_ & 8) != 0 && (period <= 1 || (sampleFrame_++ % period) == 0);
    const bool keep = (profiling_ & 2) != 0;
    // captured frame: the reference's intermediates (render data, sorted keys / values) are kept
    // for readback; the product path writes neither (the blend reads its records and half lists)
    const bool capture = (profiling_ & (2 | 16)) != 0;
    const uint32_t nb = (a.count + kProjectBlock - 1) / kProjectBlock;
    // GaussianRenderData for readback only when profiling (bits 0, 1), gsm_debug.h
    ProjectArgs fa = a;
    fa.keepRenderData = capture ? 1u : 0u;
    keptRenderData_ = fa.keepRenderData != 0;
    lastCount_ = a.count;
    lastWidth_ = width;
    lastHeight_ = height;
    // Blend schedule: the units ordered by the walk lengths the previous frame of the same
    // geometry measured (the image does not depend on the order, only the load balance does).
    // The ordering only needs those costs: one extra workgroup of the projection launch does it
    // (unit_order_block) while the others project (k_project, or k_records_in on the records path;
    // the multi-GPU frame orders them earlier, in its partition projection: preOrdered).
    const uint32_t units = preOrdered ? 0u : scheduleUnits(s, width, height);
    const bool costOrder = preOrdered ? tuning_.costOrder : units > 0;
    fa.schedUnits = units;
    // (written on every scheduled frame: the blend's remaining-walk priorities read the longest walk too)
    fa.pairBucket = tuning_.blendPairs ? (uint32_t)std::max(1, tuning_.pairBucket) : kUoBuckets;

    hipEvent_t* ev = (prof || blendOnly) ? frameEvents(profFrames_) : nullptr;
    if (prof) hipEventRecord(ev[0], s);
    front(fa);  // the projection (or records) launch; its block 0 orders the blend units (fa.schedUnits)
    if (prof) hipEventRecord(ev[1], s);
    // (a frame of few blocks: the scatter's workgroups add up the block counts themselves).  The records path
    // (devCount: a multi-GPU slab) sizes its grids for the receive capacity but adds up only the blocks of
    // the records received -- at 8 ranks ~1/8 of a frame's gaussians -- so it takes the fused scan up to 4x
    // the block count (a slab that receives more than 2M records pays a longer prefix instead of the launch)
    const bool fusedScan = tuning_.fusedScan && nb > 0 && nb <= (devCount ? 4u : 1u) * kFusedScanMaxBlocks;
    if (!fusedScan) launch_scan_blocks(nb, a, arena_, s, devCount);
    if (prof) hipEventRecord(ev[2], s);
    launch_scatter(a, arena_, s, devCount, fusedScan);
    if (keep) {  // preserve the unsorted assignment arrays for readback
        hipMemcpyAsync(arena_.keysKeep, arena_.keys[0], (size_t)maxAssignments_ * 4, hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(arena_.valsKeep, arena_.vals[0], (size_t)maxAssignments_ * 4, hipMemcpyDeviceToDevice, s);
    }
    if (prof) hipEventRecord(ev[3], s);
    uint32_t* kb[2] = {arena_.keys[0], arena_.keys[1]};
    uint32_t* vb[2] = {arena_.vals[0], arena_.vals[1]};
    FrameGeometry g;
    g.tilesX = tilesX_;
    g.tilesY = tilesY_;
    g.tileCount = tileCount_;
    g.rowBegin = rowBegin_;
    g.rowEnd = rowEnd_;
    g.rowStride = rowStride_;
    g.rowCount = rowCount();
    g.width = width;
    g.height = height;
    g.maxAssignments = maxAssignments_;
    // Frame sort.  Default: a stable LSD sort by the tile field only
    // (ceil(tileBits / 8) passes, the last one writing the tile starts), then each tile's run sorted
    // stably by depth by one wave in LDS -- the same order as the reference's 4-pass sort of
    // (tile << 16 | depth) keys.  Tuning::fullRadix keeps the 4 full 8-bit passes (A/B).
    const bool fullRadix = tuning_.fullRadix;
    const bool ballot = tuning_.ballotRank;
    if (!fullRadix) {
        // the last tile pass also writes the tile starts (radix_sort_tiles: no pass over the keys); the
        // keys hold local tile ids of the renderer's rows (k_scatter): a slab of <= 2048 tiles
        // (multi-GPU) takes one wide pass
        const uint32_t localTiles = rowCount() * tilesX_;
        const int res = radix_sort_tiles(kb, vb, &arena_.header->totalAssignments, maxAssignments_, 16,
                                         sort_space(arena_), arena_.tileStart, 0u, localTiles,
                                         tileCount_, s, ballot, tuning_.wideSort, tuning_.sortScanless);
        if (res == kSortNoSpace) return GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;  // (nothing of the sort launched)
        tile_depth_sort(kb[res], vb[res], kb[res ^ 1], vb[res ^ 1], arena_.tileStart, 0u, localTiles, s, ballot,
                        arena_.halfVals[0], arena_.halfVals[1],
                        arena_.halfCount, tileCount_, capture, numCUs_);
        sortedKeys_ = capture ? kb[res ^ 1] : nullptr;
        sortedVals_ = capture ? vb[res ^ 1] : nullptr;
    } else {
        const int res = radix_sort_pairs(kb, vb, &arena_.header->totalAssignments, maxAssignments_, 0,
                                         sortPassCount(), sort_space(arena_), s, ballot,
                                         tuning_.sortScanless);
        if (res == kSortNoSpace) return GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;
        sortedKeys_ = kb[res];
        sortedVals_ = vb[res];
    }
    unsortedKeys_ = keep ? arena_.keysKeep : nullptr;
    unsortedVals_ = keep ? arena_.valsKeep : nullptr;
    if (prof) hipEventRecord(ev[4], s);
    if (fullRadix) launch_headers(sortedKeys_, g, arena_, s);  // else done inside the sort
    // the blend walks per-half lists without the entries its half provably skips (k_scatter flags);
    // the tile sort writes them, the 4-pass sort needs the separate pass
    if (fullRadix)
        launch_half_lists(sortedVals_, 0u, rowCount() * tilesX_, arena_, tileCount_, s);
    arena_.blendTrace = (profiling_ & 4) ? traceBuf_ : nullptr;
    // the schedule from the walks the previous frame's blend recorded (same stream: no join)
    if (prof || blendOnly) hipEventRecord(ev[5], s);
    lastBlendKernel_ = launch_blend(g, arena_, color, colorPitch, depth, depthPitch, numCUs_, costOrder,
                 (int)config_.color_format, s, tuning_.blendWaves, tuning_.blendClaim, blendArrive,
                 tuning_.blendPairs);
    if (prof || blendOnly) hipEventRecord(ev[6], s);
    if (prof || blendOnly) profFrames_++;
    haveTimes_ = profFrames_ > 0;
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status GlobalRenderer::stageTimes(float* ms, int n) {
    // Average of every profiled frame still in the ring (the last kEventRing frames).
    if (!haveTimes_ || profFrames_ == 0) return GSM_ERR_RENDER_FAILED;
    hipSetDevice(device_);
    if (hipEventSynchronize(frameEvents(profFrames_ - 1)[GSM_STAGE_COUNT]) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    const uint32_t frames = profFrames_ < (uint32_t)kEventRing ? profFrames_ : (uint32_t)kEventRing;
    const uint32_t first = profFrames_ - frames;
    const bool blendOnly = (profiling_ & 1) == 0;  // bit 3: only the blend's pair of events exists
    for (int i = 0; i < n && i < GSM_STAGE_COUNT; ++i) {
        if (blendOnly && i != GSM_STAGE_BLEND) {
            ms[i] = 0.0f;
            continue;
        }
        double acc = 0.0;
        for (uint32_t f = first; f < profFrames_; ++f) {
            float t = 0.f;
            hipEvent_t* ev = frameEvents(f);
            if (hipEventElapsedTime(&t, ev[i], ev[i + 1]) != hipSuccess) return GSM_ERR_RENDER_FAILED;
            acc += t;
        }
        ms[i] = (float)(acc / frames);
    }
    return GSM_OK;
}

gsm_status GlobalRenderer::lastGpuTime(double* seconds) {
    // the whole-frame span needs ev[0], which only the every-stage mode records
    if (!haveTimes_ || profFrames_ == 0 || (profiling_ & 1) == 0) return GSM_ERR_RENDER_FAILED;
    hipSetDevice(device_);
    hipEvent_t* ev = frameEvents(profFrames_ - 1);
    if (hipEventSynchronize(ev[GSM_STAGE_COUNT]) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    float t = 0.f;
    if (hipEventElapsedTime(&t, ev[0], ev[GSM_STAGE_COUNT]) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    *seconds = (double)t * 1e-3;
    return GSM_OK;
}

gsm_status GlobalRenderer::counters(gsm_debug_counters* out) {
    hipSetDevice(device_);
    TileAssignmentHeader h;
    if (hipMemcpy(&h, arena_.header, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    out->total_assignments = h.totalAssignments;
    out->max_capacity = h.maxCapacity;
    out->padded_count = h.paddedCount;
    out->overflow = h.overflow;
    out->tiles_x = tilesX_;
    out->tiles_y = tilesY_;
    out->tile_count = tileCount_;
    out->gaussian_count = lastCount_;
    return GSM_OK;
}

gsm_status GlobalRenderer::debugCopy(int which, void* dst, size_t bytes, size_t* needed) {
    hipSetDevice(device_);
    gsm_debug_counters c;
    gsm_status st = counters(&c);
    if (st != GSM_OK) return st;
    const size_t n = lastCount_, tot = c.total_assignments;
    const void* src = nullptr;
    size_t full = 0;
    std::vector<short4> tmpBounds;
    switch (which) {
        case GSM_BUF_RENDER_DATA:
            if (!keptRenderData_) return GSM_ERR_MISSING_REQUIRED_BUFFER;  // frame not profiled (gsm_debug.h)
            src = arena_.renderData;
            full = n * 16;
            break;
        case GSM_BUF_BOUNDS: full = n * 16; break;
        case GSM_BUF_TILE_COUNTS: src = arena_.tileCounts; full = n * 4; break;
        case GSM_BUF_KEYS: src = unsortedKeys_; full = tot * 4; break;
        case GSM_BUF_VALUES: src = unsortedVals_; full = tot * 4; break;
        case GSM_BUF_SORTED_KEYS:  // kept by captured frames only (gsm_debug.h)
            if (!sortedKeys_) return GSM_ERR_MISSING_REQUIRED_BUFFER;
            src = sortedKeys_;
            full = tot * 4;
            break;
        case GSM_BUF_SORTED_VALUES:
            if (!sortedVals_) return GSM_ERR_MISSING_REQUIRED_BUFFER;
            src = sortedVals_;
            full = tot * 4;
            break;
        case GSM_BUF_HEADERS: full = (size_t)tileCount_ * 8; break;
        case GSM_BUF_EXP_TABLE: src = arena_.expTable; full = 65536 * 2; break;
        case GSM_BUF_BLEND_TRACE: src = (profiling_ & 4) ? traceBuf_ : nullptr; full = (size_t)tileCount_ * 4 * 4 * 8; break;
        default: return GSM_ERR_INVALID_ARGUMENT;
    }
    if (needed) *needed = full;
    if (!dst || bytes == 0) return GSM_OK;
    size_t cpy = bytes < full ? bytes : full;
    if (which == GSM_BUF_BOUNDS) {
        tmpBounds.resize(n ? n : 1);
        if (n && hipMemcpy(tmpBounds.data(), arena_.bounds, n * sizeof(short4), hipMemcpyDeviceToHost) != hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        std::vector<int32_t> b(n * 4);
        for (size_t i = 0; i < n; ++i) {
            b[4 * i + 0] = tmpBounds[i].x;
            b[4 * i + 1] = tmpBounds[i].y;
            b[4 * i + 2] = tmpBounds[i].z;
            b[4 * i + 3] = tmpBounds[i].w;
        }
        std::memcpy(dst, b.data(), cpy);
        return GSM_OK;
    }
    if (which == GSM_BUF_HEADERS) {  // {offset = lower_bound, count} per tile, as the reference
        std::vector<uint32_t> ts((size_t)tileCount_ + 1);
        if (hipMemcpy(ts.data(), arena_.tileStart, ts.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        std::vector<uint32_t> h((size_t)tileCount_ * 2);
        for (uint32_t t = 0; t < tileCount_; ++t) {
            h[2 * t] = ts[t];
            h[2 * t + 1] = ts[t + 1] >= ts[t] ? ts[t + 1] - ts[t] : 0u;
        }
        std::memcpy(dst, h.data(), cpy);
        return GSM_OK;
    }
    if (!src) return full == 0 ? GSM_OK : GSM_ERR_MISSING_REQUIRED_BUFFER;
    if (cpy && hipMemcpy(dst, src, cpy, hipMemcpyDeviceToHost) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    if (which == GSM_BUF_VALUES || which == GSM_BUF_SORTED_VALUES) {  // the reference's ids: no skip flags
        uint32_t* v = (uint32_t*)dst;
        for (size_t i = 0; i < cpy / 4; ++i) v[i] &= kGidMask;
    }
    return GSM_OK;
}

gsm_status GlobalRenderer::setTileRows(uint32_t b, uint32_t e, uint32_t stride) {
    if (b == 0 && e == 0) {
        rowBegin_ = 0;
        rowEnd_ = tilesY_;
        rowStride_ = 1;
        return GSM_OK;
    }
    if (b >= e || e > tilesY_ || stride == 0) return GSM_ERR_INVALID_ARGUMENT;
    rowBegin_ = b;
    rowEnd_ = e;
    rowStride_ = stride;
    return GSM_OK;
}

}  // namespace gsm

namespace gsm {
gsm_status GlobalRenderer::setProfiling(int flags) {
    hipSetDevice(device_);
    if ((flags & 2) && !arena_.keysKeep) {
        gsm_status st = alloc((void**)&arena_.keysKeep, (size_t)maxAssignments_ * 4);
        if (st == GSM_OK) st = alloc((void**)&arena_.valsKeep, (size_t)maxAssignments_ * 4);
        if (st != GSM_OK) return st;
    }
    if ((flags & 4) && !traceBuf_) {
        gsm_status st = alloc((void**)&traceBuf_, (size_t)tileCount_ * 4 * 4 * 8);
        if (st != GSM_OK) return st;
    }
    if ((flags & 9) && events_.empty()) {  // bit 0 (every stage) or bit 3 (blend only)
        events_.assign((size_t)kEventRing * (GSM_STAGE_COUNT + 1), nullptr);
        for (auto& e : events_)
            if (hipEventCreate(&e) != hipSuccess) return GSM_ERR_ENCODER_CREATION_FAILED;
    }
    profiling_ = flags;
    profFrames_ = 0;  // restart the averaging window
    sampleFrame_ = 0;
    haveTimes_ = false;
    return GSM_OK;
}
}  // namespace gsm
