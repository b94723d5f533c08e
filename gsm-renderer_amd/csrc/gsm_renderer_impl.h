// gsm_renderer_impl.h -- C++ GlobalRenderer behind the C ABI (include/gsm_renderer.h).
// Mirrors the reference class GlobalRenderer (GlobalRenderer.swift:72-572).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/gsm_debug.h"
#include "../../include/gsm_renderer.h"
#include "gsm_internal.h"

namespace gsm {

class GlobalRenderer {
   public:
    // GlobalRenderer.init(device:config:) (GlobalRenderer.swift:110-193)
    static gsm_status create(const gsm_renderer_config& cfg, int hipDevice, GlobalRenderer** out);
    ~GlobalRenderer();

    // GlobalRenderer.render (GlobalRenderer.swift:201-238)
    gsm_status render(hipStream_t stream, const gsm_gaussian_input& input,
                      const gsm_camera_params& camera, uint32_t width, uint32_t height, void* color,
                      size_t colorPitch, void* depth, size_t depthPitch);

    // multi-GPU partition: project ids [first, first+count) and pack the splat
    // records of every tile-row slab they meet; render a slab from the records it received
    gsm_status projectPartition(hipStream_t stream, const gsm_gaussian_input& input,
                                const gsm_camera_params& camera, uint32_t width, uint32_t height,
                                uint32_t first, uint32_t count, const uint32_t* slabRows, uint32_t numSlabs,
                                void* send, uint64_t capacity, uint32_t* sendCounts, bool interleave = false);
    // the same projection for the direct exchange: per-slab counts first, then the records written
    // into every slab owner's receive buffer once the count matrix is on the device (gsm_multigpu.hip)
    // orderUnits: the launch also orders the blend units of the renderer's own rows (set_tile_rows) for a
    // later renderRecords(..., preOrdered = true) of the same frame
    // publish (multi-GPU frame): the per-slab totals also go into every rank's count matrix and the
    // scan's workgroups arrive at barrier 0 (gsm_multigpu.hip); null: counts only
    gsm_status partitionCounts(hipStream_t stream, const gsm_gaussian_input& input, const gsm_camera_params& camera,
                               uint32_t width, uint32_t height, uint32_t first, uint32_t count,
                               const uint32_t* slabRows, uint32_t numSlabs, uint32_t* sendCounts,
                               bool orderUnits = false, bool interleave = false, const CountPublish* publish = nullptr);
    // the push's workgroups arrive at `arrive`'s barrier after their record stores
    gsm_status partitionPush(hipStream_t stream, uint32_t world, uint32_t rank, const uint32_t* counts,
                             const SlabPeers& peers, uint32_t* recvCount, const MgArrive& arrive);
    // blendArrive (nullable): the blend's waves arrive at that barrier after their pixel stores
    gsm_status renderRecords(hipStream_t stream, const void* records, uint32_t count, uint32_t width,
                             uint32_t height, void* color, size_t colorPitch, void* depth, size_t depthPitch,
                             const uint32_t* devCount = nullptr, bool preOrdered = false,
                             const MgArrive* blendArrive = nullptr);
    // what renderRecords / the multi-GPU frame would refuse, checked before anything is enqueued
    gsm_status validateFrame(uint32_t count, bool inputMissing, uint32_t width, uint32_t height,
                             const void* color, size_t colorPitch, const void* depth, size_t depthPitch) const;
    // the partition buffers (allocated lazily by the first partition frame; the multi-GPU frame
    // allocates them at prepare so that no frame can fail on an allocation)
    gsm_status ensurePartitionBuffers(uint32_t numSlabs);
    // The multi-GPU frame's two sets of blend-schedule buffers (unit costs, order, longest walk):
    // frame f uses set f & 1 in its projection (ordering) and in its blend, so with frame f + 1's
    // projection running beside frame f's blend (gsm_multigpu pipelined) neither reads what the other
    // writes; the ordering then follows the walks of frame f - 2.  Set 1 is allocated by
    // ensurePartitionBuffers.
    void selectSchedule(uint32_t parity);
    uint32_t maxGaussians() const { return maxGaussians_; }
    uint32_t tilesY() const { return tilesY_; }
    uint32_t maxWidth() const { return maxWidth_; }
    uint32_t maxHeight() const { return maxHeight_; }
    uint32_t colorBytesPerPixel() const {
        return config_.color_format == GSM_COLOR_FORMAT_RGBA16F ? 8u
               : (config_.color_format == GSM_COLOR_FORMAT_RGBA32F ? 16u : 4u);
    }
    bool halfPrecision() const { return config_.precision == GSM_PRECISION_FLOAT16; }

    gsm_status counters(gsm_debug_counters* out);
    int lastBlendKernel() const { return lastBlendKernel_; }
    gsm_status debugCopy(int which, void* dst, size_t bytes, size_t* needed);
    gsm_status setProfiling(int flags);  // bit0: stage events, bit1: keep unsorted keys
    gsm_status stageTimes(float* ms, int n);
    gsm_status lastGpuTime(double* seconds);
    // the renderer's tile rows: begin, begin + stride, ... < end (0, 0: the whole frame)
    gsm_status setTileRows(uint32_t begin, uint32_t end, uint32_t stride = 1);
    uint32_t rowCount() const { return rowEnd_ > rowBegin_ ? (rowEnd_ - rowBegin_ + rowStride_ - 1) / rowStride_ : 0u; }
    int device() const { return device_; }

   private:
    GlobalRenderer() = default;
    gsm_status alloc(void** p, size_t bytes);
    ProjectArgs frameArgs(const gsm_camera_params& camera, uint32_t width, uint32_t height, uint32_t count,
                          uint32_t shComponents) const;
    // scan, scatter, sort, headers and blend after `front` filled the per-gaussian arrays
    template <class Front>
    gsm_status runFrame(hipStream_t s, const ProjectArgs& a, uint32_t width, uint32_t height, void* color,
                        size_t colorPitch, void* depth, size_t depthPitch, Front&& front,
                        const uint32_t* devCount = nullptr, bool preOrdered = false,
                        const MgArrive* blendArrive = nullptr);
    // the blend schedule's unit count for the current rows (0 when cost order is off), its cost
    // arrays cleared when the geometry changed
    uint32_t scheduleUnits(hipStream_t s, uint32_t width, uint32_t height);
    PartitionBuffers part_;
    uint32_t partCount_ = 0;  // ids of the last partitionCounts
    SlabTable partSlabs_{};
    struct ScheduleSet {
        uint16_t* unitCost = nullptr;
        uint32_t* unitOrder = nullptr;
        uint32_t* costMax = nullptr;
    } sched_[2];   // its slab table (partitionPush cuts each record's tile answers by it)
    struct PartitionFrame {
        ProjectArgs a;
        SlabTable slabs;
        const void* world;
        const void* harm;
        uint32_t deg;
        bool half;
    };
    gsm_status preparePartition(const gsm_gaussian_input& in, const gsm_camera_params& camera, uint32_t width,
                                uint32_t height, uint32_t first, uint32_t count, const uint32_t* slabRows,
                                uint32_t numSlabs, bool needSend, const void* send, const uint32_t* sendCounts,
                                PartitionFrame* f, bool interleave = false);
    void release();
    int sortPassCount() const;

    int device_ = -1;
    int numCUs_ = 256;
    gsm_renderer_config config_{};
    Tuning tuning_{};  // A/B switches, read once at create
    uint32_t maxGaussians_ = 1, maxWidth_ = 1, maxHeight_ = 1;
    uint32_t tilesX_ = 1, tilesY_ = 1, tileCount_ = 1;
    uint32_t rowBegin_ = 0, rowEnd_ = 1, rowStride_ = 1;
    uint32_t maxAssignments_ = 4;
    DeviceArena arena_;
    std::vector<void*> allocations_;
    static constexpr int kEventRing = 128;  // frames of stage events kept for averaging
    std::vector<hipEvent_t> events_;       // [kEventRing][GSM_STAGE_COUNT + 1]
    uint32_t profFrames_ = 0;
    uint32_t sampleFrame_ = 0;  // frames since setProfiling (blend-event sampling)
    hipEvent_t* frameEvents(uint32_t frame) { return &events_[(frame % kEventRing) * (GSM_STAGE_COUNT + 1)]; }
    int profiling_ = 0;
    int lastBlendKernel_ = 0;  // gsm_blend_kernel of the last enqueued frame (gsm_global_debug_blend_kernel)
    bool keptRenderData_ = false;  // the last frame wrote GaussianRenderData for readback
    bool haveTimes_ = false;
    uint32_t lastCount_ = 0, lastWidth_ = 0, lastHeight_ = 0;
    const uint32_t* sortedKeys_ = nullptr;
    const uint32_t* sortedVals_ = nullptr;
    const uint32_t* unsortedKeys_ = nullptr;
    const uint32_t* unsortedVals_ = nullptr;
    unsigned long long* traceBuf_ = nullptr;  // blend unit trace (profiling bit 2)
    uint64_t schedKey_ = ~0ull;               // geometry the unit costs belong to
};

}  // namespace gsm

struct gsm_renderer {
    gsm::GlobalRenderer* impl;
};
