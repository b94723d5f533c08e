// gsm_multigpu.hip -- one frame partitioned across the GPUs of a node by screen slab, behind the
// C ABI (include/gsm_multigpu.h).
//
// One process and one GlobalRenderer per GPU; the caller hands over its RCCL communicator.  Per
// frame, enqueue-only on the caller's stream, no host synchronisation:
//   1. project the rank's id range once and count its records per destination slab
//      (GlobalRenderer::partitionCounts: k_project_part, k_part_scan);
//   2. ncclAllGather of the per-slab counts: every rank holds the world x world count matrix on
//      the device;
//   3. k_part_push: every record goes straight from the projection into its slab owner's receive
//      buffer over xGMI (peer pointers opened once from IPC handles), at the offset the count matrix
//      gives -- rank order, so the receiver's records are in ascending id order (the stable sort's
//      tie order); no send buffer, no copy pass;
//   4. ncclAllReduce of one word orders every rank's pushes before every rank's render;
//   5. the owner renders its tile rows from the received records, their count read on the device;
//   6. the bands are gathered into rank 0's frame with grouped ncclSend / ncclRecv (fixed sizes:
//      the slab rows are fixed by the frame height).
// RCCL is loaded at run time (dlopen, reusing the copy the process already has loaded, e.g. the one
// torch bundles), so libgsm_amd.so has no link-time RCCL dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/gsm_multigpu.h"
#include "gsm_internal.h"
#include "gsm_renderer_impl.h"

namespace gsm {

namespace {
struct Rccl {
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclCommCount) commCount = nullptr;
    decltype(&ncclCommUserRank) userRank = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static std::once_flag once;
    static Rccl R;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the process's own RCCL first
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        R.allGather = (decltype(R.allGather))dlsym(h, "ncclAllGather");
        R.allReduce = (decltype(R.allReduce))dlsym(h, "ncclAllReduce");
        R.send = (decltype(R.send))dlsym(h, "ncclSend");
        R.recv = (decltype(R.recv))dlsym(h, "ncclRecv");
        R.groupStart = (decltype(R.groupStart))dlsym(h, "ncclGroupStart");
        R.groupEnd = (decltype(R.groupEnd))dlsym(h, "ncclGroupEnd");
        R.commCount = (decltype(R.commCount))dlsym(h, "ncclCommCount");
        R.userRank = (decltype(R.userRank))dlsym(h, "ncclCommUserRank");
        R.ok = R.allGather && R.allReduce && R.send && R.recv && R.groupStart && R.groupEnd && R.commCount &&
               R.userRank;
    });
    return R;
}

}  // namespace

class MultiGpu {
   public:
    static gsm_status create(GlobalRenderer* r, void* comm, int rank, int world, MultiGpu** out);
    ~MultiGpu() { release(); }
    gsm_status render(hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam, uint32_t width,
                      uint32_t height, void* color, size_t colorPitch, void* depth, size_t depthPitch,
                      void* gatherColor);
    gsm_status counts(uint32_t* hostCounts);  // world x world, after the frame's stream work

   private:
    void release();
    GlobalRenderer* r_ = nullptr;
    ncclComm_t comm_ = nullptr;
    int rank_ = 0, world_ = 1, device_ = 0;
    uint32_t* sendCounts_ = nullptr;
    uint32_t* countsAll_ = nullptr;
    SplatRecord* recv_ = nullptr;
    uint32_t* recvCount_ = nullptr;
    int* order_ = nullptr;  // the ordering collective's word
    SlabPeers peers_{};
    std::vector<void*> opened_;
};

void MultiGpu::release() {
    hipSetDevice(device_);
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    for (void* p : {(void*)sendCounts_, (void*)countsAll_, (void*)recv_, (void*)recvCount_, (void*)order_})
        if (p) hipFree(p);
    recv_ = nullptr;
    sendCounts_ = countsAll_ = recvCount_ = nullptr;
    order_ = nullptr;
}

gsm_status MultiGpu::create(GlobalRenderer* r, void* comm, int rank, int world, MultiGpu** out) {
    *out = nullptr;
    const Rccl& R = rccl();
    if (!R.ok) return GSM_ERR_UNSUPPORTED;
    if (!comm || world < 1 || world > (int)kMaxSlabs || rank < 0 || rank >= world) return GSM_ERR_INVALID_ARGUMENT;
    int n = 0, me = -1;
    if (R.commCount((ncclComm_t)comm, &n) != ncclSuccess || R.userRank((ncclComm_t)comm, &me) != ncclSuccess ||
        n != world || me != rank)
        return GSM_ERR_INVALID_ARGUMENT;
    if (hipSetDevice(r->device()) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    MultiGpu* m = new (std::nothrow) MultiGpu();
    if (!m) return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    m->r_ = r;
    m->comm_ = (ncclComm_t)comm;
    m->rank_ = rank;
    m->world_ = world;
    m->device_ = r->device();
    const uint64_t G = r->maxGaussians();
    bool ok = hipMalloc(&m->sendCounts_, kMaxSlabs * 4) == hipSuccess &&
              hipMalloc(&m->countsAll_, kMaxSlabs * kMaxSlabs * 4) == hipSuccess &&
              // a slab receives each id at most once; uncached, so peers' xGMI stores (k_part_push, no
              // fence: they are complete when the kernel is, and the ordering collective on every
              // stream follows it) and the owner's reads meet in HBM without any L2 holding a stale
              // line of the previous frame
              hipExtMallocWithFlags((void**)&m->recv_, G * sizeof(SplatRecord), hipDeviceMallocUncached) ==
                  hipSuccess &&
              hipMalloc(&m->recvCount_, 4) == hipSuccess && hipMalloc(&m->order_, 4) == hipSuccess &&
              hipMemset(m->order_, 0, 4) == hipSuccess && hipMemset(m->recvCount_, 0, 4) == hipSuccess;
    // receive buffers of every rank, opened once from their IPC handles (gathered over RCCL)
    hipStream_t s = nullptr;
    hipIpcMemHandle_t* dHandles = nullptr;
    std::vector<hipIpcMemHandle_t> handles((size_t)world);
    if (ok) {
        hipIpcMemHandle_t mine;
        ok = hipIpcGetMemHandle(&mine, m->recv_) == hipSuccess && hipStreamCreate(&s) == hipSuccess &&
             hipMalloc(&dHandles, sizeof(hipIpcMemHandle_t) * (size_t)world) == hipSuccess &&
             hipMemcpy(dHandles + rank, &mine, sizeof(mine), hipMemcpyHostToDevice) == hipSuccess &&
             R.allGather(dHandles + rank, dHandles, sizeof(mine), ncclUint8, m->comm_, s) == ncclSuccess &&
             hipStreamSynchronize(s) == hipSuccess &&
             hipMemcpy(handles.data(), dHandles, sizeof(mine) * (size_t)world, hipMemcpyDeviceToHost) == hipSuccess;
    }
    for (int p = 0; ok && p < world; ++p) {
        if (p == rank) {
            m->peers_.recv[p] = m->recv_;
            continue;
        }
        void* ptr = nullptr;
        ok = hipIpcOpenMemHandle(&ptr, handles[(size_t)p], hipIpcMemLazyEnablePeerAccess) == hipSuccess;
        if (ok) {
            m->opened_.push_back(ptr);
            m->peers_.recv[p] = (SplatRecord*)ptr;
        }
    }
    if (dHandles) hipFree(dHandles);
    if (s) hipStreamDestroy(s);
    if (!ok) {
        (void)hipGetLastError();
        delete m;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = m;
    return GSM_OK;
}

gsm_status MultiGpu::render(hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam,
                            uint32_t width, uint32_t height, void* color, size_t colorPitch, void* depth,
                            size_t depthPitch, void* gatherColor) {
    const Rccl& R = rccl();
    const uint32_t world = (uint32_t)world_, rank = (uint32_t)rank_;
    if (!color || (rank == 0 && gatherColor && gatherColor != color)) return GSM_ERR_INVALID_ARGUMENT;
    if (gatherColor && colorPitch != (size_t)width * 8) return GSM_ERR_INVALID_BUFFER_SIZE;  // contiguous bands
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    // slabs: contiguous tile rows, ceil(tilesY / world) each (gsm_amd.slabs.partition)
    const uint32_t tilesY = r_->tilesY();
    const uint32_t perRows = (tilesY + world - 1) / world;
    uint32_t rows[kMaxSlabs + 1];
    for (uint32_t i = 0; i <= world; ++i) rows[i] = i * perRows < tilesY ? i * perRows : tilesY;
    // the rank's id range (gsm_amd.exchange.id_range)
    const uint32_t N = in.gaussian_count;
    const uint32_t perIds = (N + world - 1) / world;
    const uint32_t first = rank * perIds < N ? rank * perIds : N;
    const uint32_t cnt = perIds < N - first ? perIds : N - first;

    gsm_status st = r_->partitionCounts(s, in, cam, width, height, first, cnt, rows, world, sendCounts_);
    if (st != GSM_OK) return st;
    if (R.allGather(sendCounts_, countsAll_, world, ncclUint32, comm_, s) != ncclSuccess) return GSM_ERR_RENDER_FAILED;
    if ((st = r_->partitionPush(s, world, rank, countsAll_, peers_, recvCount_)) != GSM_OK) return st;
    if (R.allReduce(order_, order_, 1, ncclInt32, ncclSum, comm_, s) != ncclSuccess) return GSM_ERR_RENDER_FAILED;
    const uint32_t y0 = rows[rank] * kTileHeight < height ? rows[rank] * kTileHeight : height;
    const uint32_t y1 = rows[rank + 1] * kTileHeight < height ? rows[rank + 1] * kTileHeight : height;
    if (rows[rank] < rows[rank + 1]) {
        if ((st = r_->setTileRows(rows[rank], rows[rank + 1])) != GSM_OK) return st;
        st = r_->renderRecords(s, recv_, r_->maxGaussians(), width, height, color, colorPitch, depth, depthPitch,
                               recvCount_);
        if (st != GSM_OK) return st;
    }
    if (gatherColor || rank != 0) {  // bands -> rank 0's frame
        if (R.groupStart() != ncclSuccess) return GSM_ERR_RENDER_FAILED;
        ncclResult_t e = ncclSuccess;
        if (rank != 0) {
            if (y1 > y0) e = R.send((const char*)color + (size_t)y0 * colorPitch, (size_t)(y1 - y0) * colorPitch,
                                    ncclUint8, 0, comm_, s);
        } else {
            for (uint32_t p = 1; p < world && e == ncclSuccess; ++p) {
                const uint32_t a = rows[p] * kTileHeight < height ? rows[p] * kTileHeight : height;
                const uint32_t b = rows[p + 1] * kTileHeight < height ? rows[p + 1] * kTileHeight : height;
                if (b > a) e = R.recv((char*)gatherColor + (size_t)a * colorPitch, (size_t)(b - a) * colorPitch,
                                      ncclUint8, (int)p, comm_, s);
            }
        }
        if (R.groupEnd() != ncclSuccess || e != ncclSuccess) return GSM_ERR_RENDER_FAILED;
    }
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status MultiGpu::counts(uint32_t* hostCounts) {
    hipSetDevice(device_);
    if (hipMemcpy(hostCounts, countsAll_, (size_t)world_ * world_ * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

}  // namespace gsm

struct gsm_multigpu {
    gsm::MultiGpu* impl;
};

extern "C" {

gsm_status gsm_multigpu_create(gsm_renderer* renderer, void* nccl_comm, int rank, int world_size,
                               gsm_multigpu** out) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!renderer || !renderer->impl) return GSM_ERR_INVALID_ARGUMENT;
    gsm::MultiGpu* m = nullptr;
    gsm_status st = gsm::MultiGpu::create(renderer->impl, nccl_comm, rank, world_size, &m);
    if (st != GSM_OK) return st;
    gsm_multigpu* h = new (std::nothrow) gsm_multigpu{m};
    if (!h) {
        delete m;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = h;
    return GSM_OK;
}

void gsm_multigpu_destroy(gsm_multigpu* m) {
    if (!m) return;
    delete m->impl;
    delete m;
}

gsm_status gsm_multigpu_render(gsm_multigpu* m, void* stream, const gsm_gaussian_input* input,
                               const gsm_camera_params* camera, uint32_t width, uint32_t height, void* color,
                               size_t color_pitch_bytes, void* depth, size_t depth_pitch_bytes, void* gather_color) {
    if (!m || !m->impl || !input || !camera) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->render((hipStream_t)stream, *input, *camera, width, height, color, color_pitch_bytes, depth,
                           depth_pitch_bytes, gather_color);
}

gsm_status gsm_multigpu_debug_counts(gsm_multigpu* m, uint32_t* host_counts) {
    if (!m || !m->impl || !host_counts) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->counts(host_counts);
}

}  // extern "C"
