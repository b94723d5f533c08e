// gsm_multigpu.hip -- one frame partitioned across the GPUs of a node by screen slab, behind the
// C ABI (include/gsm_multigpu.h).
//
// One process and one GlobalRenderer per GPU.  Every rank owns one uncached "exchange"
// allocation; at set-up the ranks open each other's (IPC handles exchanged by the caller, or over
// an RCCL communicator).  Per frame, enqueue-only on the caller's stream, no host synchronisation
// and no collective library:
//   phase 0  project the rank's id range once and count its records per destination slab
//            (GlobalRenderer::partitionCounts: k_project_part, k_part_scan); k_mg_sync writes the
//            counts into row `rank` of every rank's count matrix and arrives at barrier 0;
//   phase 1  wait at barrier 0; k_part_push: every record goes straight from the projection into
//            its slab owner's receive buffer, at the offset the count matrix gives -- rank order, so
//            the receiver's records are in ascending id order (the stable sort's tie order); arrive
//            at barrier 1;
//   phase 2  wait at barrier 1; the owner renders its tile rows from the received records, their
//            count read on the device; when gathering, the blend writes its pixels straight into
//            rank 0's frame, and the rank arrives at barrier 2;
//   phase 3  rank 0 waits at barrier 2 for every slab (then copies the frame to the caller's
//            gather target unless the caller renders into the library frame itself).
// A barrier is an arrival and a wait, each one 64-lane workgroup: the arrival is a system-scope
// release and one flag word per peer written with the frame number (lane p -> rank p's flag of this
// rank); the wait is lane p spinning, bounded by a timeout, on this rank's flag of rank p, and a
// system-scope acquire.  Flags, counts, records and the
// gathered frame all live in uncached memory, so the owner's reads never meet a stale L2 line of
// a peer's write.  Ordering across frames: a rank arrives at frame k + 1's barrier 0 only after
// its stream finished frame k, so no record or pixel of frame k + 1 is written into a rank before
// it is done reading frame k; the count matrix is double-buffered by frame parity.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <cstdlib>
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
        R.commCount = (decltype(R.commCount))dlsym(h, "ncclCommCount");
        R.userRank = (decltype(R.userRank))dlsym(h, "ncclCommUserRank");
        R.ok = R.allGather && R.commCount && R.userRank;
    });
    return R;
}

// exchange allocation layout (bytes from its base)
constexpr uint32_t kBarriers = 3;
constexpr size_t kFlagWords = 0;      // u32 flag[kBarriers][kMaxSlabs]: [b][src] = last frame src reached b
constexpr size_t kStatusWord = 64;    // u32: this rank's barrier timeouts
constexpr size_t kCountsWord = 256;   // u32 counts[2][kMaxSlabs * kMaxSlabs] (frame parity; row = source)
constexpr size_t kRecordsOff = 4096;  // SplatRecord[capacity]
static_assert(kFlagWords + kBarriers * kMaxSlabs <= kStatusWord, "flags before the status word");
constexpr uint32_t kHandleMagic = 0x58534D47u;  // "GMSX"
constexpr uint32_t kHandleVersion = 1;

struct ExchangeFields {
    uint32_t magic, version;
    int32_t rank, world;
    uint32_t capacity;  // records of the receive buffer (the renderer's max_gaussians)
    uint32_t maxWidth, maxHeight, bytesPerPixel;
    int32_t pid, device;
    uint64_t base;      // device address in the owner's process (a same-process peer uses it directly)
    uint64_t bytes;
    uint64_t frameOff;  // rank 0: the gathered frame; 0 elsewhere
    char busId[32];
    hipIpcMemHandle_t ipc;
};
struct ExchangeHandle : ExchangeFields {
    uint8_t pad[GSM_MULTIGPU_HANDLE_BYTES - sizeof(ExchangeFields)];
};
static_assert(sizeof(ExchangeHandle) == GSM_MULTIGPU_HANDLE_BYTES, "handle size is ABI");

struct SyncPeers {
    uint32_t* ctl[kMaxSlabs];  // base of every rank's exchange allocation (peer mappings)
};

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

// One barrier of the multi-GPU frame (header comment).  publish (nullable): this rank's per-slab
// record counts, written into row `rank` of every rank's count matrix before the arrival.
__global__ __launch_bounds__(64) void k_mg_sync(SyncPeers peers, uint32_t* __restrict__ mine, uint32_t rank,
                                                uint32_t world, uint32_t barrier, uint32_t epoch,
                                                const uint32_t* __restrict__ publish, uint32_t parity, int arrive,
                                                int wait, unsigned long long timeoutTicks) {
    const uint32_t lane = threadIdx.x;
    if (publish && lane < world) {
        uint32_t* row = peers.ctl[lane] + kCountsWord + parity * kMaxSlabs * kMaxSlabs + rank * world;
        for (uint32_t s = 0; s < world; ++s) row[s] = publish[s];
    }
    if (arrive) {
        // every store of this rank's earlier kernels (records, pixels) and of this wave (counts)
        // is visible at system scope before any peer can see the flag
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        if (lane < world)
            __hip_atomic_store(peers.ctl[lane] + kFlagWords + barrier * kMaxSlabs + rank, epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!wait) return;
    uint32_t* status = mine + kStatusWord;
    // after a timeout every later wait is skipped: a missing peer costs one timeout, not one per barrier
    const bool skip = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    if (!skip && lane < world) {
        const uint32_t* flag = mine + kFlagWords + barrier * kMaxSlabs + lane;
        const unsigned long long t0 = wall_clock64();
        while ((int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
            if (wall_clock64() - t0 > timeoutTicks) {
                __hip_atomic_fetch_add(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

class MultiGpu {
   public:
    static gsm_status prepare(GlobalRenderer* r, int rank, int world, MultiGpu** out, void* handle);
    gsm_status connect(const void* all);
    ~MultiGpu() { release(); }
    gsm_status phase(int p, hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam, uint32_t width,
                     uint32_t height, void* color, size_t colorPitch, void* depth, size_t depthPitch,
                     void* gatherColor);
    gsm_status frame(void** color, size_t* pitch) const {
        *color = rank_ == 0 ? frame0_ : nullptr;
        *pitch = rank_ == 0 ? framePitch_ : 0;
        return GSM_OK;
    }
    gsm_status status(uint32_t* timeouts, bool clear);
    gsm_status setTimeout(uint32_t ms) {
        if (ms == 0) return GSM_ERR_INVALID_ARGUMENT;
        timeoutTicks_ = (unsigned long long)ms * wallKHz_;
        return GSM_OK;
    }
    gsm_status counts(uint32_t* hostCounts);  // world x world, after the frame's stream work
    gsm_status copyExchange(void* dst, size_t bytes) {
        hipSetDevice(device_);
        return hipMemcpy(dst, mem_, bytes < memBytes_ ? bytes : memBytes_, hipMemcpyDeviceToHost) == hipSuccess
                   ? GSM_OK
                   : GSM_ERR_RENDER_FAILED;
    }
    gsm_status copyFrame(void* dst, size_t pitch, uint32_t width, uint32_t height) {
        if (rank_ != 0 || !frame0_ || !dst || width > r_->maxWidth() || height > r_->maxHeight() ||
            pitch < (size_t)width * bpp_)
            return GSM_ERR_INVALID_ARGUMENT;
        hipSetDevice(device_);
        if (hipMemcpy2D(dst, pitch, frame0_, framePitch_, (size_t)width * bpp_, height, hipMemcpyDeviceToHost) !=
            hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        return GSM_OK;
    }

   private:
    void release();
    gsm_status check(const gsm_gaussian_input& in, uint32_t width, uint32_t height, void* color, size_t colorPitch,
                     void* gatherColor) const;
    uint32_t* ctl() const { return (uint32_t*)mem_; }
    void sync(hipStream_t s, uint32_t barrier, const uint32_t* publish, bool arrive, bool wait) {
        hipLaunchKernelGGL(k_mg_sync, dim3(1), dim3(64), 0, s, sync_, ctl(), (uint32_t)rank_, (uint32_t)world_,
                           barrier, frame_, publish, frame_ & 1u, arrive ? 1 : 0, wait ? 1 : 0, timeoutTicks_);
    }

    GlobalRenderer* r_ = nullptr;
    int rank_ = 0, world_ = 1, device_ = 0;
    char* mem_ = nullptr;  // this rank's exchange allocation (uncached)
    size_t memBytes_ = 0, frameOff_ = 0, framePitch_ = 0;
    uint32_t bpp_ = 8, capacity_ = 0, minCap_ = 0;
    uint32_t* sendCounts_ = nullptr;  // this rank's per-slab counts (k_part_scan)
    uint32_t* recvCount_ = nullptr;   // records this rank receives (k_part_push, block 0)
    SyncPeers sync_{};
    SlabPeers recs_{};
    char* frame0_ = nullptr;  // rank 0's gathered frame (peer mapping on the other ranks)
    bool connected_ = false;
    uint32_t frame_ = 0;  // frames begun (phase 0); the barriers' epoch
    bool interleave_ = false;  // slab rows interleaved (GSM_MG_ROWS=interleaved at prepare)
    uint32_t wallKHz_ = 100000;
    unsigned long long timeoutTicks_ = 0;
    std::vector<void*> opened_;  // IPC mappings of peer allocations
};

void MultiGpu::release() {
    hipSetDevice(device_);
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    for (void* p : {(void*)mem_, (void*)sendCounts_, (void*)recvCount_})
        if (p) hipFree(p);
    mem_ = nullptr;
    sendCounts_ = recvCount_ = nullptr;
}

gsm_status MultiGpu::prepare(GlobalRenderer* r, int rank, int world, MultiGpu** out, void* handle) {
    *out = nullptr;
    if (!handle || world < 1 || world > (int)kMaxSlabs || rank < 0 || rank >= world) return GSM_ERR_INVALID_ARGUMENT;
    if (hipSetDevice(r->device()) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    MultiGpu* m = new (std::nothrow) MultiGpu();
    if (!m) return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    m->r_ = r;
    m->rank_ = rank;
    m->world_ = world;
    m->device_ = r->device();
    m->capacity_ = r->maxGaussians();
    m->bpp_ = r->colorBytesPerPixel();
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, m->device_) == hipSuccess && khz > 0)
        m->wallKHz_ = (uint32_t)khz;
    m->timeoutTicks_ = 10000ull * m->wallKHz_;
    const char* rv = getenv("GSM_MG_ROWS");  // every rank must agree (the same environment)
    m->interleave_ = rv && std::strcmp(rv, "interleaved") == 0;
    const size_t recBytes = (size_t)m->capacity_ * sizeof(SplatRecord);
    m->framePitch_ = (size_t)r->maxWidth() * m->bpp_;
    m->frameOff_ = rank == 0 ? align_up(kRecordsOff + recBytes, 4096) : 0;
    m->memBytes_ = rank == 0 ? m->frameOff_ + m->framePitch_ * r->maxHeight() : kRecordsOff + recBytes;
    // fine-grained device memory (GSM_MG_MEM=uncached|cached: the A/B of DESIGN.md 7, create-time only):
    // uncached exchange memory rendered wrong slabs on MI355X (tools/dbg/mg_ab2.sh: 30 of 36 virtual-rank
    // frames, fine-grained and ordinary memory 0 of 36)
    const char* mode = getenv("GSM_MG_MEM");
    hipError_t ae = mode && !strcmp(mode, "cached")
                        ? hipMalloc((void**)&m->mem_, m->memBytes_)
                        : hipExtMallocWithFlags((void**)&m->mem_, m->memBytes_,
                                                mode && !strcmp(mode, "uncached") ? hipDeviceMallocUncached
                                                                                  : hipDeviceMallocFinegrained);
    bool ok = ae == hipSuccess &&
              (!getenv("GSM_MG_POISON") || hipMemset(m->mem_, 0xAB, m->memBytes_) == hipSuccess) &&
              hipMemset(m->mem_, 0, kRecordsOff) == hipSuccess &&
              hipMalloc(&m->sendCounts_, kMaxSlabs * 4) == hipSuccess && hipMalloc(&m->recvCount_, 4) == hipSuccess &&
              hipMemset(m->sendCounts_, 0, kMaxSlabs * 4) == hipSuccess && hipMemset(m->recvCount_, 0, 4) == hipSuccess;
    ExchangeHandle h;
    std::memset(&h, 0, sizeof(h));
    if (ok) ok = hipIpcGetMemHandle(&h.ipc, m->mem_) == hipSuccess;
    if (ok) ok = hipDeviceGetPCIBusId(h.busId, (int)sizeof(h.busId) - 1, m->device_) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        delete m;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    h.magic = kHandleMagic;
    h.version = kHandleVersion;
    h.rank = rank;
    h.world = world;
    h.capacity = m->capacity_;
    h.maxWidth = r->maxWidth();
    h.maxHeight = r->maxHeight();
    h.bytesPerPixel = m->bpp_;
    h.pid = (int32_t)getpid();
    h.device = m->device_;
    h.base = (uint64_t)(uintptr_t)m->mem_;
    h.bytes = m->memBytes_;
    h.frameOff = m->frameOff_;
    std::memcpy(handle, &h, sizeof(h));
    *out = m;
    return GSM_OK;
}

gsm_status MultiGpu::connect(const void* all) {
    if (connected_) return GSM_ERR_INVALID_ARGUMENT;
    if (!all) return GSM_ERR_INVALID_ARGUMENT;
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    std::vector<ExchangeHandle> hs((size_t)world_);
    std::memcpy(hs.data(), all, sizeof(ExchangeHandle) * (size_t)world_);
    uint32_t minCap = 0xFFFFFFFFu;
    for (int p = 0; p < world_; ++p) {
        const ExchangeHandle& h = hs[(size_t)p];
        if (h.magic != kHandleMagic || h.version != kHandleVersion || h.rank != p || h.world != world_ ||
            h.maxWidth != r_->maxWidth() || h.maxHeight != r_->maxHeight() || h.bytesPerPixel != bpp_)
            return GSM_ERR_INVALID_ARGUMENT;
        if (p == 0 && h.frameOff == 0) return GSM_ERR_INVALID_ARGUMENT;
        if (h.capacity < minCap) minCap = h.capacity;
    }
    if (hs[(size_t)rank_].base != (uint64_t)(uintptr_t)mem_) return GSM_ERR_INVALID_ARGUMENT;  // not our handle
    const int32_t pid = (int32_t)getpid();
    char* base[kMaxSlabs] = {};
    for (int p = 0; p < world_; ++p) {
        const ExchangeHandle& h = hs[(size_t)p];
        if (p == rank_) {
            base[p] = mem_;
        } else if (h.pid == pid) {  // a rank of this process (virtual ranks): the pointer itself
            if (h.device != device_) {
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, device_, h.device) != hipSuccess || !can) return GSM_ERR_UNSUPPORTED;
                hipError_t e = hipDeviceEnablePeerAccess(h.device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return GSM_ERR_UNSUPPORTED;
                (void)hipGetLastError();
            }
            base[p] = (char*)(uintptr_t)h.base;
        } else {
            void* ptr = nullptr;
            if (hipIpcOpenMemHandle(&ptr, h.ipc, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
            }
            opened_.push_back(ptr);
            base[p] = (char*)ptr;
        }
        sync_.ctl[p] = (uint32_t*)base[p];
        recs_.recv[p] = (SplatRecord*)(base[p] + kRecordsOff);
        recs_.cap[p] = h.capacity;
    }
    frame0_ = base[0] + hs[0].frameOff;
    minCap_ = minCap;
    connected_ = true;
    return GSM_OK;
}

gsm_status MultiGpu::check(const gsm_gaussian_input& in, uint32_t width, uint32_t height, void* color,
                           size_t colorPitch, void* gatherColor) const {
    if (!connected_) return GSM_ERR_INVALID_ARGUMENT;
    // the same answer on every rank (same N, size and limits): no rank is left waiting at a barrier
    if (in.gaussian_count > minCap_) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (width == 0 || height == 0 || width > r_->maxWidth() || height > r_->maxHeight())
        return GSM_ERR_INVALID_DIMENSIONS;
    if (in.gaussian_count > 0 && (!in.gaussians || !in.harmonics)) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    if (rank_ == 0 && gatherColor && gatherColor != frame0_) {
        if (colorPitch < (size_t)width * bpp_) return GSM_ERR_INVALID_BUFFER_SIZE;
    } else if (!gatherColor && !color) {
        return GSM_ERR_MISSING_REQUIRED_BUFFER;
    }
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    return GSM_OK;
}

gsm_status MultiGpu::phase(int p, hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam,
                           uint32_t width, uint32_t height, void* color, size_t colorPitch, void* depth,
                           size_t depthPitch, void* gatherColor) {
    if (p < 0 || p > 3) return GSM_ERR_INVALID_ARGUMENT;
    gsm_status st = check(in, width, height, color, colorPitch, gatherColor);
    if (st != GSM_OK) return st;
    const uint32_t world = (uint32_t)world_, rank = (uint32_t)rank_;
    // slabs: contiguous blocks of ceil(tilesY / world) tile rows (default: each record travels to the
    // fewest ranks -- interleaving sends a gaussian to every rank one of its rect rows maps to, +71 %
    // records at 1080p / W = 8, device frame +3.5-5 % on the benchmark's uniform cloud), or interleaved
    // rows r, r + W, r + 2W, ... (GSM_MG_ROWS=interleaved at prepare), which keep an off-centre scene's
    // row loads within 1.1x of the mean where contiguous blocks reach 2.8x
    const uint32_t tilesY = r_->tilesY();
    const uint32_t perRows = (tilesY + world - 1) / world;
    uint32_t rows[kMaxSlabs + 1];
    for (uint32_t i = 0; i <= world; ++i)
        rows[i] = interleave_ ? (i < world ? (i < tilesY ? i : tilesY) : tilesY) : (i * perRows < tilesY ? i * perRows : tilesY);
    const bool mine = interleave_ ? rank < tilesY : rows[rank] < rows[rank + 1];
    auto setRows = [&]() {
        return interleave_ ? r_->setTileRows(rank, tilesY, world) : r_->setTileRows(rows[rank], rows[rank + 1]);
    };
    const bool gather = gatherColor != nullptr;
    // every phase ends with an arrival and the next begins with the matching wait, so a barrier
    // only ever waits for work enqueued in an earlier phase (virtual ranks on one stream)
    switch (p) {
        case 0: {
            // the rank's id range (gsm_amd.exchange.id_range)
            const uint32_t N = in.gaussian_count;
            const uint32_t perIds = (N + world - 1) / world;
            const uint32_t first = rank * perIds < N ? rank * perIds : N;
            const uint32_t cnt = perIds < N - first ? perIds : N - first;
            // the slab's blend units are ordered inside this launch (the long kernel of the frame's
            // first half), not in the short records-in launch of phase 2
            if (mine && (st = setRows()) != GSM_OK) return st;
            st = r_->partitionCounts(s, in, cam, width, height, first, cnt, rows, world, sendCounts_, mine, interleave_);
            if (st != GSM_OK) return st;
            ++frame_;
            sync(s, 0, sendCounts_, true, false);  // counts into every rank's matrix, then arrive
            break;
        }
        case 1: {
            sync(s, 0, nullptr, false, true);  // every rank's counts are in my matrix
            const uint32_t* counts = ctl() + kCountsWord + (frame_ & 1u) * kMaxSlabs * kMaxSlabs;
            if ((st = r_->partitionPush(s, world, rank, counts, recs_, recvCount_)) != GSM_OK) return st;
            sync(s, 1, nullptr, true, false);
            break;
        }
        case 2: {
            sync(s, 1, nullptr, false, true);  // every record of my slab has arrived
            if (mine) {
                if ((st = setRows()) != GSM_OK) return st;
                void* target = gather ? (void*)frame0_ : color;
                const size_t pitch = gather ? framePitch_ : colorPitch;
                st = r_->renderRecords(s, mem_ + kRecordsOff, capacity_, width, height, target, pitch, depth,
                                       depthPitch, recvCount_, /*preOrdered=*/true);
                if (st != GSM_OK) return st;
            }
            if (gather && world > 1) sync(s, 2, nullptr, true, false);  // my band is in rank 0's frame
            break;
        }
        case 3: {
            if (gather && rank == 0) {
                if (world > 1) sync(s, 2, nullptr, false, true);  // every band is in my frame
                if (gatherColor != frame0_ &&
                    hipMemcpy2DAsync(gatherColor, colorPitch, frame0_, framePitch_, (size_t)width * bpp_, height,
                                     hipMemcpyDeviceToDevice, s) != hipSuccess)
                    return GSM_ERR_RENDER_FAILED;
            }
            break;
        }
    }
    if (hipGetLastError() != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status MultiGpu::status(uint32_t* timeouts, bool clear) {
    hipSetDevice(device_);
    if (hipMemcpy(timeouts, ctl() + kStatusWord, 4, hipMemcpyDeviceToHost) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    if (clear && hipMemset(ctl() + kStatusWord, 0, 4) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

gsm_status MultiGpu::counts(uint32_t* hostCounts) {
    hipSetDevice(device_);
    const uint32_t* c = ctl() + kCountsWord + (frame_ & 1u) * kMaxSlabs * kMaxSlabs;
    if (hipMemcpy(hostCounts, c, (size_t)world_ * world_ * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

}  // namespace gsm

struct gsm_multigpu {
    gsm::MultiGpu* impl;
};

extern "C" {

gsm_status gsm_multigpu_prepare(gsm_renderer* renderer, int rank, int world_size, gsm_multigpu** out, void* handle) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!renderer || !renderer->impl) return GSM_ERR_INVALID_ARGUMENT;
    gsm::MultiGpu* m = nullptr;
    gsm_status st = gsm::MultiGpu::prepare(renderer->impl, rank, world_size, &m, handle);
    if (st != GSM_OK) return st;
    gsm_multigpu* h = new (std::nothrow) gsm_multigpu{m};
    if (!h) {
        delete m;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = h;
    return GSM_OK;
}

gsm_status gsm_multigpu_connect(gsm_multigpu* m, const void* all_handles) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->connect(all_handles);
}

gsm_status gsm_multigpu_create(gsm_renderer* renderer, void* nccl_comm, int rank, int world_size,
                               gsm_multigpu** out) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!renderer || !renderer->impl) return GSM_ERR_INVALID_ARGUMENT;
    const gsm::Rccl& R = gsm::rccl();
    if (!R.ok) return GSM_ERR_UNSUPPORTED;
    if (!nccl_comm || world_size < 1 || world_size > (int)gsm::kMaxSlabs || rank < 0 || rank >= world_size)
        return GSM_ERR_INVALID_ARGUMENT;
    int n = 0, me = -1;
    if (R.commCount((ncclComm_t)nccl_comm, &n) != ncclSuccess || R.userRank((ncclComm_t)nccl_comm, &me) != ncclSuccess ||
        n != world_size || me != rank)
        return GSM_ERR_INVALID_ARGUMENT;
    std::vector<uint8_t> all((size_t)world_size * GSM_MULTIGPU_HANDLE_BYTES);
    gsm_multigpu* h = nullptr;
    gsm_status st = gsm_multigpu_prepare(renderer, rank, world_size, &h, all.data() + (size_t)rank * GSM_MULTIGPU_HANDLE_BYTES);
    if (st != GSM_OK) return st;
    // the handles over the communicator (once, at set-up; the frame itself uses no collective)
    uint8_t* d = nullptr;
    hipStream_t s = nullptr;
    bool ok = hipStreamCreate(&s) == hipSuccess && hipMalloc(&d, all.size()) == hipSuccess &&
              hipMemcpy(d + (size_t)rank * GSM_MULTIGPU_HANDLE_BYTES, all.data() + (size_t)rank * GSM_MULTIGPU_HANDLE_BYTES,
                        GSM_MULTIGPU_HANDLE_BYTES, hipMemcpyHostToDevice) == hipSuccess &&
              R.allGather(d + (size_t)rank * GSM_MULTIGPU_HANDLE_BYTES, d, GSM_MULTIGPU_HANDLE_BYTES, ncclUint8,
                          (ncclComm_t)nccl_comm, s) == ncclSuccess &&
              hipStreamSynchronize(s) == hipSuccess &&
              hipMemcpy(all.data(), d, all.size(), hipMemcpyDeviceToHost) == hipSuccess;
    if (d) hipFree(d);
    if (s) hipStreamDestroy(s);
    if (!ok) {
        (void)hipGetLastError();
        gsm_multigpu_destroy(h);
        return GSM_ERR_RENDER_FAILED;
    }
    if ((st = h->impl->connect(all.data())) != GSM_OK) {
        gsm_multigpu_destroy(h);
        return st;
    }
    *out = h;
    return GSM_OK;
}

void gsm_multigpu_destroy(gsm_multigpu* m) {
    if (!m) return;
    delete m->impl;
    delete m;
}

gsm_status gsm_multigpu_render_phase(gsm_multigpu* m, int phase, void* stream, const gsm_gaussian_input* input,
                                     const gsm_camera_params* camera, uint32_t width, uint32_t height, void* color,
                                     size_t color_pitch_bytes, void* depth, size_t depth_pitch_bytes,
                                     void* gather_color) {
    if (!m || !m->impl || !input || !camera) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->phase(phase, (hipStream_t)stream, *input, *camera, width, height, color, color_pitch_bytes, depth,
                          depth_pitch_bytes, gather_color);
}

gsm_status gsm_multigpu_render(gsm_multigpu* m, void* stream, const gsm_gaussian_input* input,
                               const gsm_camera_params* camera, uint32_t width, uint32_t height, void* color,
                               size_t color_pitch_bytes, void* depth, size_t depth_pitch_bytes, void* gather_color) {
    for (int p = 0; p < 4; ++p) {
        gsm_status st = gsm_multigpu_render_phase(m, p, stream, input, camera, width, height, color, color_pitch_bytes,
                                                  depth, depth_pitch_bytes, gather_color);
        if (st != GSM_OK) return st;
    }
    return GSM_OK;
}

gsm_status gsm_multigpu_frame(gsm_multigpu* m, void** color, size_t* pitch_bytes) {
    if (!m || !m->impl || !color || !pitch_bytes) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->frame(color, pitch_bytes);
}

gsm_status gsm_multigpu_status(gsm_multigpu* m, uint32_t* timeouts, int clear) {
    if (!m || !m->impl || !timeouts) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->status(timeouts, clear != 0);
}

gsm_status gsm_multigpu_set_timeout_ms(gsm_multigpu* m, uint32_t ms) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->setTimeout(ms);
}

gsm_status gsm_multigpu_debug_copy_frame(gsm_multigpu* m, void* host_dst, size_t dst_pitch_bytes, uint32_t width,
                                         uint32_t height) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->copyFrame(host_dst, dst_pitch_bytes, width, height);
}

gsm_status gsm_multigpu_debug_copy_exchange(gsm_multigpu* m, void* host_dst, size_t bytes) {
    if (!m || !m->impl || !host_dst) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->copyExchange(host_dst, bytes);
}

gsm_status gsm_multigpu_debug_counts(gsm_multigpu* m, uint32_t* host_counts) {
    if (!m || !m->impl || !host_counts) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->counts(host_counts);
}

}  // extern "C"
