// gsm_multigpu.hip -- one frame partitioned across the GPUs of a node by screen slab, behind the
// C ABI (include/gsm_multigpu.h).
//
// One process and one GlobalRenderer per GPU.  Every rank owns one fine-grained "exchange"
// allocation; at set-up the ranks open each other's (IPC handles exchanged by the caller, or over
// an RCCL communicator).  Per frame, enqueue-only on the caller's stream, no host synchronisation
// and no collective library:
//   phase 0  project the rank's id range once and count its records per destination slab
//            (GlobalRenderer::partitionCounts: k_project_part, k_part_scan); k_part_scan's workgroup
//            for slab s stores its total into column s of row `rank` of every rank's count matrix and
//            arrives at barrier 0;
//   phase 1  wait at barrier 0; k_part_copy: every block run of the projection (staged per slab) goes into
//            its slab owner's receive buffer, at the offset the count matrix gives -- rank order, so
//            the receiver's records are in ascending id order (the stable sort's tie order); its
//            workgroups arrive at barrier 1;
//   phase 2  wait at barrier 1; the owner renders its tile rows from the received records, their
//            count read on the device; when gathering, the blend writes its pixels (colour, and
//            depth when asked) straight into rank 0's frame and its waves arrive at barrier 2;
//   phase 3  rank 0 waits at barrier 2 for every slab (then copies the frame to the caller's
//            targets unless the caller renders into the library frame itself).
//
// Memory model (gsm_internal.h MgArrive): the records and counts are system-coherent
// write-through stores (sc0 sc1); the gathered pixels are plain stores that the blend's workgroups
// write back at system scope (their XCD's L2) before arriving.  The kernels that make them arrive at
// the barrier themselves -- every storing unit drains its stores, then adds to the rank's arrival
// counter, and the last unit raises the rank's flag in every rank's control block.  A wait is k_mg_sync: lane p polls
// the flag of rank p (relaxed system-scope loads, bounded by a timeout), then an acquire at system
// scope; every consumer load of exchange data is system-coherent (ld_sys32 / ld_sys128), and before
// the caller may read rank 0's gathered frame, kSyncWaitBlocks workgroups acquire so that every XCD's
// L2 drops its lines of it.  Nothing relies on the fence scope HIP puts between two kernels.
// Errors: a rank whose frame is refused (check: validated before anything is enqueued) still
// performs every barrier of the frame, arriving with the failure bit set and zero counts, so the
// epochs of all ranks stay aligned; a peer waiting on such an arrival counts it (peer_errors) and
// the next frame is unaffected.  A wait that times out skips the remaining waits of that frame only.
// Ordering across frames: a rank arrives at frame k + 1's barrier 0 only after its stream finished
// frame k, so no record or pixel of frame k + 1 is written into a rank before it is done reading
// frame k; the count matrix is double-buffered by frame parity.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
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
    decltype(&ncclSend) send = nullptr;  // the RCCL transport's frame (GSM_MG_TRANSPORT_RCCL)
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    bool ok = false;
    bool p2p = false;
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
        R.send = (decltype(R.send))dlsym(h, "ncclSend");
        R.recv = (decltype(R.recv))dlsym(h, "ncclRecv");
        R.groupStart = (decltype(R.groupStart))dlsym(h, "ncclGroupStart");
        R.groupEnd = (decltype(R.groupEnd))dlsym(h, "ncclGroupEnd");
        R.p2p = R.ok && R.send && R.recv && R.groupStart && R.groupEnd;
    });
    return R;
}

// exchange allocation layout (bytes from its base)
constexpr uint32_t kBarriers = 3;
constexpr size_t kFlagWords = 0;      // u32 flag[kBarriers][kMaxSlabs]: [b][src] = last frame src reached b
constexpr size_t kStatusWord = 64;    // u32 [0] barrier timeouts, [1] failed peer arrivals, [2] epoch of the last timeout
constexpr size_t kCountsWord = 256;   // u32 counts[2][kMaxSlabs * kMaxSlabs] (frame parity; row = source)
constexpr size_t kRecordsOff = 4096;  // SplatRecord[2][capacity] (frame parity)
constexpr size_t kProbeWord = 768;    // u32 probe[kMaxSlabs][8]: words 8 src .. 8 src + 7 of the connect-time check
                                      // (MultiGpu::probe); in every later page of an allocation the same words
                                      // from its start
constexpr size_t kCtlZeroWords = kProbeWord;  // control words zeroed at prepare (flags, status, counts)
static_assert(kCountsWord + 2 * kMaxSlabs * kMaxSlabs <= kProbeWord, "counts before the probe words");
static_assert(kProbeWord + 8 * kMaxSlabs <= 1024, "probe words inside the control page");
static_assert(kFlagWords + kBarriers * kMaxSlabs <= kStatusWord, "flags before the status word");
constexpr uint32_t kFailBit = 0x80000000u;  // a flag's epoch with this bit: that rank's frame failed
constexpr uint32_t kEpochMask = 0x7FFFFFFFu;
constexpr uint32_t kSyncWaitBlocks = 32;    // workgroups of a wait: >= 4 per XCD (blocks are dealt round robin)
constexpr uint32_t kHandleMagic = 0x58534D47u;  // "GMSX"
constexpr uint32_t kHandleVersion = 4;

struct ExchangeFields {
    uint32_t magic, version;
    int32_t rank, world;
    uint32_t capacity;  // records of the receive buffer (the renderer's max_gaussians)
    uint32_t maxWidth, maxHeight, bytesPerPixel;
    int32_t pid, device;
    uint64_t base;      // device address in the owner's process (a same-process peer uses it directly)
    uint64_t bytes;
    uint64_t frameOff;  // rank 0: the gathered colour frame; 0 elsewhere
    uint64_t depthOff;  // rank 0: the gathered r16f depth frame; 0 elsewhere
    uint32_t interleave;  // slab rows interleaved (GSM_MG_ROWS=interleaved): every rank must agree
    uint32_t memKind;     // exchange memory kind (0 fine-grained, 2 device)
    uint32_t pipelined;   // options.pipelined (rank 0 holds two gathered frames): every rank must agree
    uint32_t transport;   // gsm_multigpu_transport: every rank must agree
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
// bytes of one frame parity of a receive buffer of `capacity` records
size_t recv_parity_bytes(uint32_t capacity) { return align_up((size_t)capacity * sizeof(SplatRecord), 4096); }
}  // namespace

// A barrier step outside the producing kernels:
//  * wait (kSyncWaitBlocks workgroups of 64): lane p of every workgroup spins on this rank's flag of
//    rank p (relaxed system-scope loads, s_sleep, bounded by timeoutTicks), then the workgroup acquires
//    at system scope (its CU's L1 and its XCD's L2 drop their lines of the exchange memory).  Block 0
//    counts a timeout (status[0], and the frame's epoch in status[2]: the frame's later waits skip)
//    and every arrival carrying the failure bit (status[1]).
//  * arrive (one workgroup; a rank that renders nothing, or one whose frame failed): zero counts
//    into row `rank` of every count matrix when `publishZero`, a system-scope release, then this
//    rank's flag in every rank's control block (with kFailBit when `fail`).
__global__ __launch_bounds__(64) void k_mg_sync(SyncPeers peers, uint32_t* __restrict__ mine, uint32_t rank,
                                                uint32_t world, uint32_t barrier, uint32_t epoch, int publishZero,
                                                uint32_t parity, int arrive, int fail, unsigned long long timeoutTicks) {
    const uint32_t lane = threadIdx.x;
    if (arrive) {
        if (publishZero && lane < world) {
            uint32_t* row = peers.ctl[lane] + kCountsWord + parity * kMaxSlabs * kMaxSlabs + rank * world;
            for (uint32_t s = 0; s < world; ++s) __hip_atomic_store(row + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (write-through stores, drained)
        if (lane < world)
            __hip_atomic_store(peers.ctl[lane] + kFlagWords + barrier * kMaxSlabs + rank, epoch | (fail ? kFailBit : 0u),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    uint32_t* status = mine + kStatusWord;
    // after a timeout the frame's remaining waits are skipped (a missing peer costs one timeout per
    // frame, and the next frame waits again)
    const bool skip = ld_sys32(status + 2) == epoch;
    bool failed = false;
    if (!skip && lane < world) {
        const uint32_t* flag = mine + kFlagWords + barrier * kMaxSlabs + lane;
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            const uint32_t f = ld_sys32(flag);
            // f at or after epoch, modulo 2^31 (epochs wrap from 2^31 - 1 to 1)
            if ((int)(((f & kEpochMask) - epoch) << 1) >= 0) {
                failed = (f & kFailBit) != 0u && (f & kEpochMask) == epoch;
                break;
            }
            if (wall_clock64() - t0 > timeoutTicks) {
                if (blockIdx.x == 0) {
                    __hip_atomic_fetch_add(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(status + 2, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (failed && blockIdx.x == 0) __hip_atomic_fetch_add(status + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// The control words of a fresh exchange allocation zeroed with system-coherent write-through stores
// (at prepare, before any peer can hold a handle): no dirty line of a cached memset can linger in an
// XCD's L2 and be written back over a flag or a count later (r06).
__global__ __launch_bounds__(256) void k_mg_zero_ctl(uint32_t* __restrict__ mem, uint32_t words) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < words) __hip_atomic_store(mem + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The mapping check (r06) of every mapping this rank stores into or polls:
// one word per 4 KiB page of each mapping -- page 0: probe word 8 src + j of the control page (no peer
// writes it), page g > 0: word 8 src + j of the page (records / frames: scratch until the first frame's
// barrier 0, which needs this rank's arrival).  Workgroups 8c .. 8c + 7 take pages 64c .. 64c + 63 (lane =
// page), workgroup 8c + j (dealt round robin to the eight XCDs) on word j: stored with the flags' store
// form (a relaxed system-scope atomic store: write-through) or, with `check`, polled with the barrier's
// load form (ld_sys32) on word (j + 3) & 7 -- stored from another XCD -- until it holds value + that index
// or `spinTicks` pass (then counted in *fails).  So every page is stored from all eight XCDs and checked
// across XCDs, as a frame's flags and records are.
struct ProbeMaps {
    uint32_t* base[kMaxSlabs];
    uint32_t pages[kMaxSlabs];
    uint32_t n;
};
__device__ __forceinline__ uint32_t* probe_word(const ProbeMaps& maps, uint32_t t, uint32_t src, uint32_t j) {
    uint32_t i = t, m = 0;
    while (m + 1u < maps.n && i >= maps.pages[m]) i -= maps.pages[m++];
    return maps.base[m] + (size_t)i * 1024u + (i == 0 ? kProbeWord : 0) + 8u * src + j;
}
__global__ __launch_bounds__(64) void k_mg_probe(ProbeMaps maps, uint32_t total, uint32_t src, uint32_t value, int check,
                                                 uint32_t* __restrict__ fails, unsigned long long spinTicks) {
    const uint32_t j = check ? ((blockIdx.x + 3u) & 7u) : (blockIdx.x & 7u);
    for (uint32_t t = (blockIdx.x >> 3) * 64u + threadIdx.x; t < total; t += (gridDim.x >> 3) * 64u) {
        uint32_t* w = probe_word(maps, t, src, j);
        if (!check) {
            __hip_atomic_store(w, value + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        const unsigned long long t0 = wall_clock64();
        while (ld_sys32(w) != value + j) {
            if (wall_clock64() - t0 > spinTicks) {
                atomicAdd(fails, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// The same words written with the gathered pixels' store form: plain stores, then each workgroup's
// system-scope release (the blend's L2 write-back, gsm_blend.hip) -- read back by the host.  Workgroups
// 8c .. 8c + 7 take pages 64c .. 64c + 63 (lane = page), workgroup 8c + j writing word 8 src + j of each,
// so that every page is stored from workgroups of all eight XCDs (dealt round robin).
__global__ __launch_bounds__(64) void k_mg_probe_plain(ProbeMaps maps, uint32_t total, uint32_t src, uint32_t value) {
    const uint32_t j = blockIdx.x & 7u;
    for (uint32_t t = (blockIdx.x >> 3) * 64u + threadIdx.x; t < total; t += (gridDim.x >> 3) * 64u)
        *probe_word(maps, t, src, j) = value + j;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (as a gathering blend workgroup at its exit)
}

// rank 0's copy of the gathered frame into the caller's target (rows of `rowBytes`, a multiple of 2):
// system-coherent loads (the peers stored the frame over xGMI), 4-byte words where aligned
__global__ __launch_bounds__(256) void k_mg_copy2d(uint8_t* __restrict__ dst, size_t dpitch, const uint8_t* src,
                                                   size_t spitch, uint32_t rowBytes, uint32_t rows) {
    const uint32_t y = blockIdx.y;
    if (y >= rows) return;
    const uint8_t* s = src + (size_t)y * spitch;
    uint8_t* d = dst + (size_t)y * dpitch;
    const bool w4 = ((((uintptr_t)s) | ((uintptr_t)d) | rowBytes) & 3u) == 0;
    if (w4) {
        for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < rowBytes / 4u; i += gridDim.x * 256u)
            ((uint32_t*)d)[i] = ld_sys32((const uint32_t*)s + i);
    } else {
        for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < rowBytes / 2u; i += gridDim.x * 256u)
            ((uint16_t*)d)[i] = __hip_atomic_load((const uint16_t*)s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

class MultiGpu {
   public:
    static gsm_status prepare(GlobalRenderer* r, int rank, int world, const gsm_multigpu_options& o, MultiGpu** out,
                              void* handle);
    gsm_status connect(const void* all);
    ~MultiGpu() { release(); }
    gsm_status phase(int p, hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam, uint32_t width,
                     uint32_t height, void* color, size_t colorPitch, void* depth, size_t depthPitch,
                     void* gatherColor);
    // gsm_multigpu_finish_frame: the remaining phases of a frame left unfinished (barrier steps only
    // from the slab render on; phase 1's push still runs when phase 0 published this rank's counts)
    gsm_status finishFrame(hipStream_t s);
    // gsm_multigpu_wait_event: the next phase 0 waits for `ev` on the stream its projection runs on
    // gsm_multigpu_debug_set_epoch: the barrier epoch of the next frame - 1 (every rank alike, no frame
    // pending or in flight): this rank's flag words are set to it, as if every peer had reached it
    gsm_status debugSetEpoch(uint32_t epoch) {
        if (nextPhase_ != 0) return GSM_ERR_PHASE_ORDER;
        if (!mem_) return GSM_ERR_UNSUPPORTED;  // (no flag words with the RCCL transport)
        epoch &= kEpochMask;
        if (epoch == 0) epoch = 1;
        if (hipSetDevice(device_) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return GSM_ERR_RENDER_FAILED;
        uint32_t f[kBarriers * kMaxSlabs];
        for (uint32_t& w : f) w = epoch;
        if (hipMemcpy(ctl() + kFlagWords, f, sizeof(f), hipMemcpyHostToDevice) != hipSuccess) return GSM_ERR_RENDER_FAILED;
        frame_ = epoch;
        return GSM_OK;
    }
    gsm_status waitEvent(hipEvent_t ev) {
        inputEvent_ = ev;
        return GSM_OK;
    }
    gsm_status frame(void** color, size_t* pitch) const {
        *color = rank_ == 0 ? frameBuf(par_) : nullptr;
        *pitch = rank_ == 0 ? framePitch_ : 0;
        return GSM_OK;
    }
    gsm_status frameDepth(void** depth, size_t* pitch) const {
        *depth = rank_ == 0 ? depthBuf(par_) : nullptr;
        *pitch = rank_ == 0 ? depthPitch0_ : 0;
        return GSM_OK;
    }
    gsm_status status(uint32_t* timeouts, uint32_t* peerErrors, bool clear);
    gsm_status setTimeout(uint32_t ms) {
        if (ms == 0) return GSM_ERR_INVALID_ARGUMENT;
        timeoutTicks_ = (unsigned long long)ms * wallKHz_;
        return GSM_OK;
    }
    gsm_status counts(uint32_t* hostCounts);  // world x world, after the frame's stream work
    gsm_status copyExchange(void* dst, size_t bytes) {
        if (!mem_) return GSM_ERR_UNSUPPORTED;  // (the RCCL transport has no exchange allocation)
        hipSetDevice(device_);
        return hipMemcpy(dst, mem_, bytes < memBytes_ ? bytes : memBytes_, hipMemcpyDeviceToHost) == hipSuccess
                   ? GSM_OK
                   : GSM_ERR_RENDER_FAILED;
    }
    gsm_status copyFrame(void* dst, size_t pitch, uint32_t width, uint32_t height, bool depth) {
        const char* src = depth ? depthBuf(par_) : frameBuf(par_);
        const size_t bpp = depth ? 2u : bpp_;
        if (rank_ != 0 || !src || !dst || width > r_->maxWidth() || height > r_->maxHeight() || pitch < (size_t)width * bpp)
            return GSM_ERR_INVALID_ARGUMENT;
        hipSetDevice(device_);
        if (hipMemcpy2D(dst, pitch, src, depth ? depthPitch0_ : framePitch_, (size_t)width * bpp, height,
                        hipMemcpyDeviceToHost) != hipSuccess)
            return GSM_ERR_RENDER_FAILED;
        return GSM_OK;
    }

   private:
    // the targets phase 2 renders into and what phase 3 copies (one frame's call arguments)
    struct Targets {
        bool gather = false, gatherDepth = false;
        void* color = nullptr;  // the blend's colour target
        size_t colorPitch = 0;
        void* depth = nullptr;  // the blend's depth target (nullable)
        size_t depthPitch = 0;
    };
    void release();
    gsm_status check(const gsm_gaussian_input& in, uint32_t width, uint32_t height, void* color, size_t colorPitch,
                     void* depth, size_t depthPitch, void* gatherColor, Targets* t) const;
    uint32_t* ctl() const { return (uint32_t*)mem_; }
    // rank 0's gathered frames of a frame of parity `par`: one pair, or (pipelined) two alternating
    char* frameBuf(uint32_t par) const { return frame0_ ? frame0_ + (pipelined_ ? par * frameStride_ : 0) : nullptr; }
    char* depthBuf(uint32_t par) const { return depth0_ ? depth0_ + (pipelined_ ? par * depthStride_ : 0) : nullptr; }
    gsm_status run(int p, hipStream_t s, const gsm_gaussian_input* in, const gsm_camera_params* cam, uint32_t width,
                   uint32_t height, Targets t, size_t colorPitch, void* depth, size_t depthPitch, void* gatherColor);
    // the same phases over RCCL (GSM_MG_TRANSPORT_RCCL): no exchange memory, no device barrier
    gsm_status runRccl(int p, hipStream_t s, const gsm_gaussian_input* in, const gsm_camera_params* cam, uint32_t width,
                       uint32_t height, Targets t, size_t colorPitch, void* depth, size_t depthPitch, void* gatherColor);
    // the mapping check of n mappings (peer-stores transport): GSM_OK or GSM_ERR_DEVICE_NOT_AVAILABLE
    gsm_status probe(char* const* base, const size_t* bytes, int n, const char* who);
    // slab rows [*y0, *y1) of pixel rows of tile-row index k of rank q's slab (contiguous: k = 0 only)
    bool slabPixelRows(uint32_t q, uint32_t k, uint32_t height, uint32_t* y0, uint32_t* y1) const;
    bool libraryFrame(const void* p) const {
        return p && (p == frame0_ || p == depth0_ || (pipelined_ && (p == frame0_ + frameStride_ || p == depth0_ + depthStride_)));
    }
    uint32_t* done(uint32_t barrier) const { return done_ + barrier * kArriveWordsPerBarrier; }
    MgArrive arrival(uint32_t barrier) const {
        MgArrive a{};
        for (int p = 0; p < world_; ++p) a.flag[p] = sync_.ctl[p] + kFlagWords + barrier * kMaxSlabs + rank_;
        a.done = done(barrier);
        a.epoch = frame_;
        a.world = (uint32_t)world_;
        return a;
    }
    // barriers 0 and 1: the consumers' loads of exchange data are system-coherent, one workgroup
    // waits; barrier 2: the caller may read rank 0's library frame with plain loads next, so
    // kSyncWaitBlocks workgroups acquire (every XCD's L2 drops its lines of the frame)
    void wait(hipStream_t s, uint32_t barrier) {
        hipLaunchKernelGGL(k_mg_sync, dim3(barrier == 2 ? kSyncWaitBlocks : 1u), dim3(64), 0, s, sync_, ctl(),
                           (uint32_t)rank_, (uint32_t)world_, barrier, frame_, 0, par_, 0, 0, timeoutTicks_);
    }
    void arrive(hipStream_t s, uint32_t barrier, bool publishZero, bool fail) {
        hipLaunchKernelGGL(k_mg_sync, dim3(1), dim3(64), 0, s, sync_, ctl(), (uint32_t)rank_, (uint32_t)world_, barrier,
                           frame_, publishZero ? 1 : 0, par_, 1, fail ? 1 : 0, timeoutTicks_);
    }

    GlobalRenderer* r_ = nullptr;
    int rank_ = 0, world_ = 1, device_ = 0;
    char* mem_ = nullptr;  // this rank's exchange allocation (fine-grained)
    size_t memBytes_ = 0, frameOff_ = 0, framePitch_ = 0, depthOff_ = 0, depthPitch0_ = 0;
    size_t frameStride_ = 0, depthStride_ = 0;  // rank 0: bytes of one gathered colour / depth frame
    uint32_t bpp_ = 8, capacity_ = 0, minCap_ = 0;
    uint32_t* sendCounts_ = nullptr;  // this rank's per-slab counts (k_part_scan)
    uint32_t* recvCount_ = nullptr;   // [2] records this rank receives, by frame parity (k_part_copy, block 0)
    uint32_t* done_ = nullptr;        // arrival counters per barrier: main + shards (own device memory)
    SyncPeers sync_{};
    SlabPeers recs_{};
    char* frame0_ = nullptr;  // rank 0's gathered colour frame (peer mapping on the other ranks)
    char* depth0_ = nullptr;  // rank 0's gathered depth frame
    bool connected_ = false;
    uint32_t frame_ = 0;       // frames begun (phase 0); the barriers' epoch: 1 .. 2^31 - 1, then 1 again
    uint32_t par_ = 0;         // the frame's parity, alternating every frame (also across the epoch's wrap)
    int nextPhase_ = 0;        // phases run in order 0..3
    Targets frameT_{};         // phase 0's targets (gathering or not: the barrier steps of finishFrame)
    uint32_t frameW_ = 0, frameH_ = 0;  // phase 0's frame size (the RCCL transport's gather rows)
    hipEvent_t inputEvent_ = nullptr;  // gsm_multigpu_wait_event (one-shot, the next phase 0)
    gsm_status frameErr_ = GSM_OK;  // this rank's error of the current frame (barrier-only phases after it)
    bool launchFailed_ = false;     // the last run() saw a failed launch (finishFrame's status)
    bool interleave_ = false;  // slab rows interleaved (options.rows)
    // GSM_MG_TRANSPORT_RCCL: the communicator, this rank's packed send records (slab after slab), its
    // receive buffer, the W x W count matrix (device, and pinned host), the records received this frame,
    // and (ranks != 0, gathering) the full-frame colour / depth targets the slab renders into
    uint32_t transport_ = GSM_MG_TRANSPORT_PEER_STORES;
    void* comm_ = nullptr;
    SplatRecord* sendRec_ = nullptr;
    SplatRecord* recvRec_ = nullptr;
    uint64_t sendCap_ = 0;
    uint32_t* countMat_ = nullptr;
    uint32_t* hostCounts_ = nullptr;
    uint32_t recvTotal_ = 0;
    char* ownFrame_ = nullptr;  // the RCCL transport's frames: rank 0's gathered frame, or a rank's staging
    char* ownDepth_ = nullptr;
    // Pipelined (GSM_MG_PIPELINE=1 at prepare, every rank alike): phases 0-1 on the library's own stream
    // (front_), phases 2-3 on the caller's, joined by events -- frame f + 1's projection and push run
    // beside frame f's slab render.  front_ starts frame f only after the caller's stream finished frame
    // f - 2 (evEnd_[f & 1]): the receive buffer, receive count, blend schedule and rank 0's gathered
    // frames of parity f & 1 are then free.
    bool pipelined_ = false;
    hipStream_t front_ = nullptr;
    hipEvent_t evFront_[2] = {nullptr, nullptr}, evEnd_[2] = {nullptr, nullptr};
    uint32_t memKind_ = 0;
    uint32_t wallKHz_ = 100000;
    unsigned long long timeoutTicks_ = 0;
    std::vector<void*> opened_;  // IPC mappings of peer allocations
    // exchange allocations that failed the prepare-time mapping check, kept until destroy so that their
    // ranges are not handed out again (r06)
    std::vector<char*> heldBack_;
    uint32_t heldBackCount_ = 0;
    static constexpr int kAllocAttempts = 4;

   public:
    uint32_t heldBack() const { return heldBackCount_; }
};

void MultiGpu::release() {
    hipSetDevice(device_);
    // pipelined: the library's stream may still run a frame's projection or push into peer memory
    if (front_) hipStreamSynchronize(front_);
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    for (char* p : heldBack_) hipFree(p);
    heldBack_.clear();
    for (void* p : {(void*)mem_, (void*)sendCounts_, (void*)recvCount_, (void*)done_, (void*)sendRec_, (void*)recvRec_,
                    (void*)countMat_, (void*)ownFrame_, (void*)ownDepth_})
        if (p) hipFree(p);
    if (hostCounts_) hipHostFree(hostCounts_);
    sendRec_ = recvRec_ = nullptr;
    countMat_ = hostCounts_ = nullptr;
    ownFrame_ = ownDepth_ = nullptr;
    for (hipEvent_t& e : evFront_)
        if (e) hipEventDestroy(e), e = nullptr;
    for (hipEvent_t& e : evEnd_)
        if (e) hipEventDestroy(e), e = nullptr;
    if (front_) hipStreamDestroy(front_), front_ = nullptr;
    mem_ = nullptr;
    sendCounts_ = recvCount_ = done_ = nullptr;
}

gsm_status MultiGpu::prepare(GlobalRenderer* r, int rank, int world, const gsm_multigpu_options& o, MultiGpu** out,
                             void* handle) {
    *out = nullptr;
    if (!handle || world < 1 || world > (int)kMaxSlabs || rank < 0 || rank >= world) return GSM_ERR_INVALID_ARGUMENT;
    if (o.struct_bytes != sizeof(gsm_multigpu_options) || (o.rows != GSM_MG_ROWS_CONTIGUOUS && o.rows != GSM_MG_ROWS_INTERLEAVED) ||
        (o.transport != GSM_MG_TRANSPORT_PEER_STORES && o.transport != GSM_MG_TRANSPORT_RCCL) || (o.pipelined & ~1))
        return GSM_ERR_INVALID_ARGUMENT;
    const bool rcclT = o.transport == GSM_MG_TRANSPORT_RCCL;
    if (rcclT && (o.pipelined || !o.nccl_comm)) return o.pipelined ? GSM_ERR_UNSUPPORTED : GSM_ERR_INVALID_ARGUMENT;
    if (rcclT && !rccl().p2p) return GSM_ERR_UNSUPPORTED;
    if (hipSetDevice(r->device()) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    // exchange memory kind: fine-grained device memory; GSM_MG_MEM=cached (ordinary device
    // memory, one GPU only) is an A/B override of the environment
    const char* mode = getenv("GSM_MG_MEM");
    // uncached exchange memory renders wrong slabs on MI355X: refused; the A/B script
    // (tools/exp/mg_memkind_ab.py) reaches it as "uncached-ab"
    if (mode && !strcmp(mode, "uncached")) return GSM_ERR_UNSUPPORTED;
    MultiGpu* m = new (std::nothrow) MultiGpu();
    if (!m) return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    m->r_ = r;
    m->rank_ = rank;
    m->world_ = world;
    m->device_ = r->device();
    m->capacity_ = r->maxGaussians();
    m->bpp_ = r->colorBytesPerPixel();
    m->memKind_ = mode && !strcmp(mode, "cached") ? 2u : (mode && !strcmp(mode, "uncached-ab") ? 1u : 0u);
    m->transport_ = (uint32_t)o.transport;
    m->comm_ = o.nccl_comm;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, m->device_) == hipSuccess && khz > 0)
        m->wallKHz_ = (uint32_t)khz;
    m->timeoutTicks_ = (unsigned long long)(o.timeout_ms ? o.timeout_ms : 10000u) * m->wallKHz_;
    m->interleave_ = o.rows == GSM_MG_ROWS_INTERLEAVED;  // every rank must agree: checked at connect (the handle)
    m->pipelined_ = o.pipelined != 0;
    m->framePitch_ = align_up((size_t)r->maxWidth() * m->bpp_, 16);
    m->depthPitch0_ = align_up((size_t)r->maxWidth() * 2u, 16);
    m->frameStride_ = align_up(m->framePitch_ * r->maxHeight(), 4096);
    m->depthStride_ = align_up(m->depthPitch0_ * r->maxHeight(), 4096);
    gsm_status failSt = GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    bool ok = r->ensurePartitionBuffers((uint32_t)world) == GSM_OK &&
              hipMalloc(&m->sendCounts_, kMaxSlabs * 4) == hipSuccess && hipMalloc(&m->recvCount_, 8) == hipSuccess &&
              hipMalloc(&m->done_, kBarriers * kArriveWordsPerBarrier * 4) == hipSuccess &&
              hipMemset(m->sendCounts_, 0, kMaxSlabs * 4) == hipSuccess && hipMemset(m->recvCount_, 0, 8) == hipSuccess &&
              hipMemset(m->done_, 0, kBarriers * kArriveWordsPerBarrier * 4) == hipSuccess;
    if (ok && rcclT) {
        // RCCL transport: ordinary device memory only -- packed send records (a rank's ceil(N / W) ids, each
        // in at most W slabs: at most N + W - 1 records), the receive buffer (a slab receives every id at most
        // once), the count matrix, and full-frame colour / depth targets (rank 0: the gathered frame)
        m->sendCap_ = (uint64_t)m->capacity_ + kMaxSlabs;
        ok = hipMalloc((void**)&m->sendRec_, m->sendCap_ * sizeof(SplatRecord)) == hipSuccess &&
             hipMalloc((void**)&m->recvRec_, ((size_t)m->capacity_ + 1) * sizeof(SplatRecord)) == hipSuccess &&
             hipMalloc((void**)&m->countMat_, kMaxSlabs * kMaxSlabs * 4) == hipSuccess &&
             hipHostMalloc((void**)&m->hostCounts_, kMaxSlabs * kMaxSlabs * 4, hipHostMallocDefault) == hipSuccess &&
             hipMalloc((void**)&m->ownFrame_, m->frameStride_) == hipSuccess &&
             hipMalloc((void**)&m->ownDepth_, m->depthStride_) == hipSuccess;
        if (ok) std::memset(m->hostCounts_, 0, kMaxSlabs * kMaxSlabs * 4);
        if (ok && rank == 0) {
            m->frame0_ = m->ownFrame_;
            m->depth0_ = m->ownDepth_;
        }
    } else if (ok) {
        // two frame parities of the receive buffer (a source pushes frame f + 2 into the parity of frame f
        // only after its barrier 0 of frame f + 2, which needs this rank's arrival there -- made after this
        // rank finished reading frame f's records: in stream order, or, pipelined, after evEnd_)
        const size_t recBytes = 2 * recv_parity_bytes(m->capacity_);
        const size_t nFrames = m->pipelined_ ? 2 : 1;
        m->frameOff_ = rank == 0 ? align_up(kRecordsOff + recBytes, 4096) : 0;
        m->depthOff_ = rank == 0 ? m->frameOff_ + nFrames * m->frameStride_ : 0;
        m->memBytes_ = rank == 0 ? m->depthOff_ + nFrames * m->depthStride_ : kRecordsOff + recBytes;
        // The allocation passes the mapping check before its handle exists (MultiGpu::probe): an allocation
        // that fails it -- r06: one that reused the range of a freed uncached allocation -- is kept (so its
        // range is not handed out again) and another is made; connect checks the peers' mappings the same way
        for (int attempt = 0; ok; ++attempt) {
            hipError_t ae = m->memKind_ == 2u ? hipMalloc((void**)&m->mem_, m->memBytes_)
                                              : hipExtMallocWithFlags((void**)&m->mem_, m->memBytes_,
                                                                      m->memKind_ == 1u ? hipDeviceMallocUncached
                                                                                        : hipDeviceMallocFinegrained);
            ok = ae == hipSuccess && (!getenv("GSM_MG_POISON") || hipMemset(m->mem_, 0xAB, m->memBytes_) == hipSuccess) &&
                 hipDeviceSynchronize() == hipSuccess;
            if (ok) {  // the control words: write-through zeros, not a cached memset (k_mg_zero_ctl)
                (void)hipGetLastError();  // (only this launch's error counts below)
                hipLaunchKernelGGL(k_mg_zero_ctl, dim3((kCtlZeroWords + 255) / 256), dim3(256), 0, 0, (uint32_t*)m->mem_,
                                   (uint32_t)kCtlZeroWords);
                ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess;
            }
            if (!ok) break;
            const gsm_status pst = m->probe(&m->mem_, &m->memBytes_, 1, "gsm_multigpu_prepare");
            if (pst == GSM_OK) break;
            if (pst != GSM_ERR_DEVICE_NOT_AVAILABLE || attempt + 1 >= kAllocAttempts) {
                ok = false;
                failSt = pst;
                break;
            }
            fprintf(stderr, "gsm_multigpu_prepare: rank %d: exchange allocation %p (%zu B) held back, allocating another\n",
                    rank, (void*)m->mem_, m->memBytes_);
            m->heldBack_.push_back(m->mem_);
            m->mem_ = nullptr;
            ++m->heldBackCount_;
        }
    }
    if (ok) ok = hipDeviceSynchronize() == hipSuccess;
    if (ok && m->pipelined_)
        ok = hipStreamCreateWithFlags(&m->front_, hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&m->evFront_[0], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&m->evFront_[1], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&m->evEnd_[0], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&m->evEnd_[1], hipEventDisableTiming) == hipSuccess;
    ExchangeHandle h;
    std::memset(&h, 0, sizeof(h));
    if (ok && !rcclT) ok = hipIpcGetMemHandle(&h.ipc, m->mem_) == hipSuccess;
    if (ok) ok = hipDeviceGetPCIBusId(h.busId, (int)sizeof(h.busId) - 1, m->device_) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        delete m;
        return failSt;
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
    h.depthOff = m->depthOff_;
    h.interleave = m->interleave_ ? 1u : 0u;
    h.memKind = m->memKind_;
    h.pipelined = m->pipelined_ ? 1u : 0u;
    h.transport = m->transport_;
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
    const bool rcclT = transport_ == GSM_MG_TRANSPORT_RCCL;
    for (int p = 0; p < world_; ++p) {
        const ExchangeHandle& h = hs[(size_t)p];
        // the ranks agree on the world, the frame limits and the options (a rank with another row layout
        // would send records with the wrong slab masks: refused here)
        if (h.magic != kHandleMagic || h.version != kHandleVersion || h.rank != p || h.world != world_ ||
            h.maxWidth != r_->maxWidth() || h.maxHeight != r_->maxHeight() || h.bytesPerPixel != bpp_ ||
            h.interleave != (interleave_ ? 1u : 0u) || h.pipelined != (pipelined_ ? 1u : 0u) || h.transport != transport_)
            return GSM_ERR_INVALID_ARGUMENT;
        if (!rcclT && p == 0 && (h.frameOff == 0 || h.depthOff == 0)) return GSM_ERR_INVALID_ARGUMENT;
        if (h.capacity < minCap) minCap = h.capacity;
    }
    if (hs[(size_t)rank_].base != (uint64_t)(uintptr_t)mem_) return GSM_ERR_INVALID_ARGUMENT;  // not our handle
    if (rcclT) {  // no mappings: every frame's data moves through the communicator
        minCap_ = minCap;
        connected_ = true;
        return GSM_OK;
    }
    const int32_t pid = (int32_t)getpid();
    char* base[kMaxSlabs] = {};
    size_t bytes[kMaxSlabs] = {};
    for (int p = 0; p < world_; ++p) {
        const ExchangeHandle& h = hs[(size_t)p];
        bytes[p] = h.bytes;
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
            // ordinary device memory is coherent only inside one GPU: refused across processes
            if (h.memKind == 2u) return GSM_ERR_UNSUPPORTED;
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
    // every mapping this rank will store into or poll, checked before the first frame relies on it
    const gsm_status pst = probe(base, bytes, world_, "gsm_multigpu_connect");
    if (pst != GSM_OK) return pst;
    frame0_ = base[0] + hs[0].frameOff;
    depth0_ = base[0] + hs[0].depthOff;
    minCap_ = minCap;
    connected_ = true;
    return GSM_OK;
}

// The mapping check (r06).  r05: the first frame whose exchange allocation
// reused the address range of a freed *uncached* allocation lost flag stores (every wait of that frame timed
// out) or read wrong record words.  r06 (profiles/r06_mg_uc_reuse.log): on such a range, words stored by
// some workgroups are not seen by others nor by the host -- the accesses of different CUs / XCDs and of the
// host go to different memory, as through stale translations of the freed range.  So before a frame relies
// on a mapping, this rank makes the frame's own accesses to one word of every 4 KiB page of it: stored with
// the flags' write-through store from all eight XCDs and polled across XCDs with the barrier's load (a
// bounded spin of 50 ms), then stored with the gathered pixels' plain stores and release and read back by
// the host -- twice.  GSM_OK, or GSM_ERR_DEVICE_NOT_AVAILABLE with the evidence on stderr (`who`).
gsm_status MultiGpu::probe(char* const* base, const size_t* bytes, int n, const char* who) {
    ProbeMaps maps{};
    uint32_t total = 0;
    for (int p = 0; p < n; ++p) {
        maps.base[p] = (uint32_t*)base[p];
        maps.pages[p] = (uint32_t)((bytes[p] + 4095) / 4096);
        total += maps.pages[p];
    }
    maps.n = (uint32_t)n;
    // an error left by an earlier call of the process (another library's, or the caller's) is not this
    // check's: only the calls below decide (r06: a failed call of the reuse test's own once read as a refusal)
    (void)hipGetLastError();
    uint32_t* fails = nullptr;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipMalloc(&fails, 4) != hipSuccess ||
        hipMemsetAsync(fails, 0, 4, s) != hipSuccess) {
        if (fails) hipFree(fails);
        if (s) hipStreamDestroy(s);
        (void)hipGetLastError();
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    const uint32_t grid = 8u * std::min<uint32_t>(512u, (total + 63u) / 64u);
    const unsigned long long spin = 50ull * wallKHz_;
    uint32_t maxPages = 0;
    for (int p = 0; p < n; ++p) maxPages = std::max(maxPages, maps.pages[p]);
    std::vector<uint32_t> host((size_t)maxPages * 8);
    bool ok = true;
    uint32_t nf = 0, badPlain = 0, firstMap = 0, firstPage = 0, firstGot = 0, firstWant = 0;
    for (uint32_t round = 0; round < 2 && ok; ++round) {
        // (a) the counts' / records' / flags' forms: write-through stores, polled with system-coherent loads
        //     by workgroups of other XCDs
        const uint32_t value = 0x5EED0000u | ((uint32_t)rank_ << 8) | ((round + 1u) << 4);
        hipLaunchKernelGGL(k_mg_probe, dim3(grid), dim3(64), 0, s, maps, total, (uint32_t)rank_, value, 0, fails, spin);
        hipLaunchKernelGGL(k_mg_probe, dim3(grid), dim3(64), 0, s, maps, total, (uint32_t)rank_, value, 1, fails, spin);
        nf = 1;
        ok = hipMemcpyAsync(&nf, fails, 4, hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess &&
             nf == 0;
        // (b) the gathered pixels' form: plain stores from every XCD released at the workgroups' exit, read
        //     back by the host (one 32-B run per page)
        const uint32_t pv = 0x9A5E0000u | ((uint32_t)rank_ << 8) | ((round + 1u) << 4);
        hipLaunchKernelGGL(k_mg_probe_plain, dim3(grid), dim3(64), 0, s, maps, total, (uint32_t)rank_, pv);
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        for (int p = 0; ok && p < n; ++p) {
            const char* b = (const char*)maps.base[p];
            const size_t off = 32u * (uint32_t)rank_;
            ok = hipMemcpy(host.data(), b + kProbeWord * 4 + off, 32, hipMemcpyDeviceToHost) == hipSuccess;
            if (ok && maps.pages[p] > 1)
                ok = hipMemcpy2D(host.data() + 8, 32, b + 4096 + off, 4096, 32, maps.pages[p] - 1, hipMemcpyDeviceToHost) ==
                     hipSuccess;
            for (size_t i = 0; ok && i < (size_t)maps.pages[p] * 8; ++i)
                if (host[i] != pv + (uint32_t)(i & 7u)) {
                    if (badPlain++ == 0) {
                        firstMap = (uint32_t)p;
                        firstPage = (uint32_t)(i / 8);
                        firstGot = host[i];
                        firstWant = pv + (uint32_t)(i & 7u);
                    }
                }
            ok = ok && badPlain == 0;
        }
        if (!ok)  // (the evidence, on stderr)
            fprintf(stderr,
                    "%s: rank %d: mapping check failed (round %u): %u polled words not seen in 50 ms, %u plain-stored "
                    "words wrong through the host (first: mapping %u page %u holds 0x%08x, stored 0x%08x)\n",
                    who, rank_, round, nf, badPlain, firstMap, firstPage, firstGot, firstWant);
    }
    const hipError_t launchErr = hipGetLastError();  // (the probe kernels' launches)
    hipFree(fails);
    hipStreamDestroy(s);
    if (launchErr != hipSuccess) {
        fprintf(stderr, "%s: rank %d: mapping check failed to run (%s)\n", who, rank_, hipGetErrorString(launchErr));
        ok = false;
    }
    return ok ? GSM_OK : GSM_ERR_DEVICE_NOT_AVAILABLE;
}

gsm_status MultiGpu::check(const gsm_gaussian_input& in, uint32_t width, uint32_t height, void* color,
                           size_t colorPitch, void* depth, size_t depthPitch, void* gatherColor, Targets* t) const {
    // which barrier steps the frame has (gather, and so barrier 2) follows from the arguments alone:
    // a refused frame still performs them
    t->gather = gatherColor != nullptr;
    t->gatherDepth = t->gather && depth != nullptr;
    // the frame capacity is the smallest rank's: the same answer on every rank for the same frame
    if (in.gaussian_count > minCap_) return GSM_ERR_INVALID_GAUSSIAN_COUNT;
    if (width == 0 || height == 0 || width > r_->maxWidth() || height > r_->maxHeight())
        return GSM_ERR_INVALID_DIMENSIONS;
    if (in.gaussian_count > 0 && (!in.gaussians || !in.harmonics)) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    if (t->gather) {
        // the slab render's targets: rank 0's gathered frame (peer stores: every rank's blend writes into it
        // through the mapping; RCCL: each rank renders into its own frame, sent to rank 0 in phase 3)
        const bool rcclT = transport_ == GSM_MG_TRANSPORT_RCCL;
        t->color = rcclT ? ownFrame_ : frame0_;
        t->colorPitch = framePitch_;
        t->depth = t->gatherDepth ? (void*)(rcclT ? ownDepth_ : depth0_) : nullptr;
        t->depthPitch = depthPitch0_;
        if (rank_ == 0) {  // the copies of phase 3 into the caller's targets
            // pipelined: the library frames alternate and a peer may be writing the other one
            if (pipelined_ && (libraryFrame(gatherColor) || (t->gatherDepth && libraryFrame(depth))))
                return GSM_ERR_INVALID_ARGUMENT;
            if (gatherColor != frame0_ && colorPitch < (size_t)width * bpp_) return GSM_ERR_INVALID_BUFFER_SIZE;
            if (t->gatherDepth && depth != depth0_ && (depthPitch < (size_t)width * 2u || (depthPitch & 1u) ||
                                                       (((uintptr_t)depth) & 1u)))
                return GSM_ERR_INVALID_BUFFER_SIZE;
        }
    } else {
        t->color = color;
        t->colorPitch = colorPitch;
        t->depth = depth;
        t->depthPitch = depthPitch;
    }
    // what the slab render (GlobalRenderer::renderRecords) would refuse
    return r_->validateFrame(0, false, width, height, t->color, t->colorPitch, t->depth, t->depthPitch);
}

gsm_status MultiGpu::phase(int p, hipStream_t s, const gsm_gaussian_input& in, const gsm_camera_params& cam,
                           uint32_t width, uint32_t height, void* color, size_t colorPitch, void* depth,
                           size_t depthPitch, void* gatherColor) {
    if (p < 0 || p > 3) return GSM_ERR_INVALID_ARGUMENT;
    if (!connected_) return GSM_ERR_INVALID_ARGUMENT;  // no peers to stay in step with
    // phases in order, nothing enqueued otherwise (a frame left unfinished: gsm_multigpu_finish_frame)
    if (p != nextPhase_) return GSM_ERR_PHASE_ORDER;
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    Targets t;
    gsm_status cst = check(in, width, height, color, colorPitch, depth, depthPitch, gatherColor, &t);
    if (p == 0) {
        ++frame_;
        frame_ &= kEpochMask;
        if (frame_ == 0) frame_ = 1;  // (epoch 0 is the flags' initial value)
        par_ ^= 1u;
        frameErr_ = cst;
        frameT_ = t;
    } else if (frameErr_ == GSM_OK) {
        frameErr_ = cst;  // (the same arguments as phase 0's for a caller that follows the protocol)
    }
    if (p == 0) {
        frameW_ = width;
        frameH_ = height;
    }
    if (transport_ == GSM_MG_TRANSPORT_RCCL)
        return runRccl(p, s, &in, &cam, width, height, t, colorPitch, depth, depthPitch, gatherColor);
    return run(p, s, &in, &cam, width, height, t, colorPitch, depth, depthPitch, gatherColor);
}

gsm_status MultiGpu::finishFrame(hipStream_t s) {
    if (!connected_) return GSM_ERR_INVALID_ARGUMENT;
    if (nextPhase_ == 0) return GSM_OK;  // no frame pending
    if (hipSetDevice(device_) != hipSuccess) return GSM_ERR_DEVICE_NOT_AVAILABLE;
    gsm_status first = GSM_OK;
    while (nextPhase_ != 0) {
        const int p = nextPhase_;
        // phase 1 needs no caller argument: the push runs when phase 0 published this rank's counts (the
        // owners expect those records); from phase 2 on the frame is abandoned -- barrier steps only,
        // a failed arrival at barrier 2 when gathering.  The first real failure of any phase is returned
        // (phase 1's push status, or a launch that failed in any phase: ADVICE r05), not the abandonment.
        if (p >= 2 && frameErr_ == GSM_OK) frameErr_ = GSM_ERR_RENDER_FAILED;
        launchFailed_ = false;
        const gsm_status st = transport_ == GSM_MG_TRANSPORT_RCCL
                                  ? runRccl(p, s, nullptr, nullptr, frameW_, frameH_, frameT_, 0, nullptr, 0, nullptr)
                                  : run(p, s, nullptr, nullptr, 0, 0, frameT_, 0, nullptr, 0, nullptr);
        if (first == GSM_OK && (launchFailed_ || p == 1)) first = launchFailed_ ? GSM_ERR_RENDER_FAILED : st;
    }
    return first;
}

gsm_status MultiGpu::run(int p, hipStream_t s, const gsm_gaussian_input* in, const gsm_camera_params* cam,
                         uint32_t width, uint32_t height, Targets t, size_t colorPitch, void* depth,
                         size_t depthPitch, void* gatherColor) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    nextPhase_ = (p + 1) & 3;
    const uint32_t world = (uint32_t)world_, rank = (uint32_t)rank_;
    const uint32_t par = par_;  // the frame's parity: count matrix, receive buffer, schedule set
    if (t.gather) {  // rank 0's gathered frames of this frame (two alternating ones when pipelined)
        t.color = frameBuf(par);
        t.depth = t.gatherDepth ? (void*)depthBuf(par) : nullptr;
    }
    // pipelined: phases 0-1 on front_ after the caller's stream finished frame f - 2, phases 2-3 on the
    // caller's stream after this frame's phase 1
    const hipStream_t cs = s;
    if (pipelined_ && p <= 1) s = front_;
    if (pipelined_ && p == 0) hipStreamWaitEvent(front_, evEnd_[par], 0);
    if (p == 0 && inputEvent_) {  // the caller's inputs of this frame are complete (gsm_multigpu_wait_event)
        hipStreamWaitEvent(s, inputEvent_, 0);
        inputEvent_ = nullptr;
    }
    if (pipelined_ && p == 2) hipStreamWaitEvent(cs, evFront_[par], 0);
    SlabPeers recv = recs_;  // this frame's parity of every owner's receive buffer
    for (uint32_t q = 0; q < world; ++q)
        recv.recv[q] = (SplatRecord*)((char*)recs_.recv[q] + par * recv_parity_bytes(recs_.cap[q]));
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
    gsm_status st = GSM_OK;
    // Every phase performs its barrier steps whatever happened before in this frame on this rank: a
    // failed frame arrives with the failure bit (and zero counts), so every rank's epochs stay equal.
    switch (p) {
        case 0: {
            if (frameErr_ == GSM_OK) {
                // the rank's id range (gsm_amd.exchange.id_range)
                const uint32_t N = in->gaussian_count;
                const uint32_t perIds = (N + world - 1) / world;
                const uint32_t first = rank * perIds < N ? rank * perIds : N;
                const uint32_t cnt = perIds < N - first ? perIds : N - first;
                CountPublish pub{};
                for (uint32_t q = 0; q < world; ++q)
                    pub.row[q] = sync_.ctl[q] + kCountsWord + par * kMaxSlabs * kMaxSlabs + rank * world;
                pub.arrive = arrival(0);
                // the slab's blend units are ordered inside this launch (the long kernel of the frame's
                // first half), not in the short records-in launch of phase 2
                if (mine && (st = setRows()) != GSM_OK) frameErr_ = st;
                r_->selectSchedule(par);
                if (frameErr_ == GSM_OK &&
                    (st = r_->partitionCounts(s, *in, *cam, width, height, first, cnt, rows, world, sendCounts_, mine,
                                              interleave_, &pub)) != GSM_OK)
                    frameErr_ = st;  // (refused before any launch)
            }
            if (frameErr_ != GSM_OK) arrive(s, 0, /*publishZero=*/true, /*fail=*/true);
            break;
        }
        case 1: {
            wait(s, 0);  // every rank's counts are in my matrix
            if (frameErr_ == GSM_OK) {
                const uint32_t* counts = ctl() + kCountsWord + par * kMaxSlabs * kMaxSlabs;
                if ((st = r_->partitionPush(s, world, rank, counts, recv, recvCount_ + par, arrival(1))) != GSM_OK)
                    frameErr_ = st;
            }
            if (frameErr_ != GSM_OK) arrive(s, 1, false, true);
            if (pipelined_) hipEventRecord(evFront_[par], front_);
            break;
        }
        case 2: {
            wait(s, 1);  // every record of my slab has arrived
            const bool signal = t.gather && world > 1;  // rank 0 waits for every slab's pixels
            bool arrived = false;
            if (frameErr_ == GSM_OK && mine) {
                if ((st = setRows()) == GSM_OK) {
                    const MgArrive ba = arrival(2);
                    r_->selectSchedule(par);
                    st = r_->renderRecords(s, mem_ + kRecordsOff + par * recv_parity_bytes(capacity_), capacity_, width,
                                           height, t.color, t.colorPitch, t.depth, t.depthPitch, recvCount_ + par,
                                           /*preOrdered=*/true, signal ? &ba : nullptr);
                    arrived = signal && st == GSM_OK;  // the blend's waves arrive
                }
                if (st != GSM_OK) frameErr_ = st;
            }
            if (signal && !arrived) arrive(s, 2, false, frameErr_ != GSM_OK);
            break;
        }
        case 3: {
            if (t.gather && rank == 0) {
                if (world > 1) wait(s, 2);  // every band is in my frame
                if (frameErr_ == GSM_OK) {
                    const uint32_t gy = height;
                    if (gatherColor != t.color) {
                        const uint32_t rowBytes = width * bpp_;
                        hipLaunchKernelGGL(k_mg_copy2d, dim3((rowBytes / 4u + 255u) / 256u, gy), dim3(256), 0, s,
                                           (uint8_t*)gatherColor, colorPitch, (const uint8_t*)t.color, framePitch_,
                                           rowBytes, gy);
                    }
                    if (t.gatherDepth && depth != t.depth) {
                        const uint32_t rowBytes = width * 2u;
                        hipLaunchKernelGGL(k_mg_copy2d, dim3((rowBytes / 4u + 255u) / 256u, gy), dim3(256), 0, s,
                                           (uint8_t*)depth, depthPitch, (const uint8_t*)t.depth, depthPitch0_, rowBytes,
                                           gy);
                    }
                }
            }
            if (pipelined_) hipEventRecord(evEnd_[par], s);
            break;
        }
    }
    if (hipGetLastError() != hipSuccess) {
        launchFailed_ = true;
        return GSM_ERR_RENDER_FAILED;
    }
    return frameErr_;
}

gsm_status MultiGpu::status(uint32_t* timeouts, uint32_t* peerErrors, bool clear) {
    if (!mem_) {  // the RCCL transport has no device barrier: nothing times out
        if (timeouts) *timeouts = 0;
        if (peerErrors) *peerErrors = 0;
        return GSM_OK;
    }
    hipSetDevice(device_);
    uint32_t w[2] = {0, 0};
    if (hipMemcpy(w, ctl() + kStatusWord, 8, hipMemcpyDeviceToHost) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    if (timeouts) *timeouts = w[0];
    if (peerErrors) *peerErrors = w[1];
    if (clear && hipMemset(ctl() + kStatusWord, 0, 12) != hipSuccess) return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

bool MultiGpu::slabPixelRows(uint32_t q, uint32_t k, uint32_t height, uint32_t* y0, uint32_t* y1) const {
    const uint32_t tilesY = r_->tilesY(), W = (uint32_t)world_;
    uint32_t t0, t1;
    if (interleave_) {  // tile row q + k W
        t0 = q + k * W;
        t1 = t0 + 1u;
    } else {  // rows [q p, (q + 1) p) in one piece
        if (k > 0) return false;
        const uint32_t per = (tilesY + W - 1u) / W;
        t0 = std::min(q * per, tilesY);
        t1 = std::min(t0 + per, tilesY);
    }
    if (t0 >= tilesY || t0 >= t1) return false;
    *y0 = std::min(t0 * 16u, height);
    *y1 = std::min(t1 * 16u, height);
    return *y1 > *y0;
}

// The frame over RCCL (GSM_MG_TRANSPORT_RCCL; SURVEY.md 8e's exchange): the same
// projection and per-slab runs as the peer-stores frame, moved by the communicator instead of the producing
// kernels' peer stores.  Every rank performs every collective of every phase -- a refused frame with zero
// counts -- so the ranks' collectives always match.
//   0  projection of the rank's ids, runs packed slab after slab into sendRec_ (k_part_copy), the per-slab
//      counts into sendCounts_ (gsm_global_project_partition's path);
//   1  ncclAllGather of the count rows -> the W x W matrix, copied to the host (the frame's one host
//      synchronisation), then one group of ncclSend / ncclRecv: slab q's records to rank q, rank q's records
//      for this slab into recvRec_ at the offset of the ranks before q (source-rank order = ascending id,
//      the stable sort's tie order); this rank's own records by a device copy;
//   2  the slab render from the received records (count known on the host), into rank 0's gathered frame
//      (rank 0), this rank's staging frame (gathering) or the caller's targets;
//   3  gathering: one group of sends of every slab's pixel rows (colour, and depth when gathered) to rank 0,
//      which receives them in place; then rank 0's copy into the caller's targets.
gsm_status MultiGpu::runRccl(int p, hipStream_t s, const gsm_gaussian_input* in, const gsm_camera_params* cam,
                             uint32_t width, uint32_t height, Targets t, size_t colorPitch, void* depth,
                             size_t depthPitch, void* gatherColor) {
    (void)hipGetLastError();  // (an error left by an earlier call of the process is not this call's: the launches below are checked)
    nextPhase_ = (p + 1) & 3;
    const Rccl& R = rccl();
    const ncclComm_t comm = (ncclComm_t)comm_;
    const uint32_t world = (uint32_t)world_, rank = (uint32_t)rank_;
    const uint32_t tilesY = r_->tilesY();
    const uint32_t perRows = (tilesY + world - 1) / world;
    uint32_t rows[kMaxSlabs + 1];
    for (uint32_t i = 0; i <= world; ++i)
        rows[i] = interleave_ ? (i < world ? (i < tilesY ? i : tilesY) : tilesY) : (i * perRows < tilesY ? i * perRows : tilesY);
    const bool mine = interleave_ ? rank < tilesY : rows[rank] < rows[rank + 1];
    auto setRows = [&]() {
        return interleave_ ? r_->setTileRows(rank, tilesY, world) : r_->setTileRows(rows[rank], rows[rank + 1]);
    };
    // the slab render's targets: rank 0's gathered frame, this rank's staging frame, or the caller's
    char* const colorT = t.gather ? ownFrame_ : (char*)t.color;
    char* const depthT = t.gather ? (t.gatherDepth ? ownDepth_ : nullptr) : (char*)t.depth;
    const size_t colorP = t.gather ? framePitch_ : t.colorPitch, depthP = t.gather ? depthPitch0_ : t.depthPitch;
    gsm_status st = GSM_OK;
    bool collOk = true;
    switch (p) {
        case 0: {
            if (frameErr_ == GSM_OK) {
                const uint32_t N = in->gaussian_count;
                const uint32_t perIds = (N + world - 1) / world;
                const uint32_t first = rank * perIds < N ? rank * perIds : N;
                const uint32_t cnt = perIds < N - first ? perIds : N - first;
                r_->selectSchedule(0);
                if ((st = r_->projectPartition(s, *in, *cam, width, height, first, cnt, rows, world, sendRec_, sendCap_,
                                               sendCounts_, interleave_)) != GSM_OK)
                    frameErr_ = st;  // (refused before any launch)
            }
            if (frameErr_ != GSM_OK) hipMemsetAsync(sendCounts_, 0, world * sizeof(uint32_t), s);
            break;
        }
        case 1: {
            collOk = R.allGather(sendCounts_, countMat_, world, ncclUint32, comm, s) == ncclSuccess &&
                     hipMemcpyAsync(hostCounts_, countMat_, (size_t)world * world * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                     hipStreamSynchronize(s) == hipSuccess;
            if (!collOk) break;
            // (recvTotal <= N <= the smallest capacity: a slab receives every id at most once)
            uint64_t sendOff = 0, recvOff = 0;
            uint32_t recvTotal = 0;
            for (uint32_t q = 0; q < world; ++q) recvTotal += hostCounts_[q * world + rank];
            // this rank's own records first (a device copy), then one group for every peer
            for (uint32_t q = 0; q < rank; ++q) sendOff += hostCounts_[rank * world + q];
            for (uint32_t q = 0; q < rank; ++q) recvOff += hostCounts_[q * world + rank];
            const uint32_t self = hostCounts_[rank * world + rank];
            if (self)
                hipMemcpyAsync(recvRec_ + recvOff, sendRec_ + sendOff, (size_t)self * sizeof(SplatRecord),
                               hipMemcpyDeviceToDevice, s);
            collOk = R.groupStart() == ncclSuccess;
            sendOff = recvOff = 0;
            for (uint32_t q = 0; q < world && collOk; ++q) {
                const uint32_t ns = hostCounts_[rank * world + q], nr = hostCounts_[q * world + rank];
                if (q != rank) {
                    if (ns) collOk = R.send(sendRec_ + sendOff, (size_t)ns * sizeof(SplatRecord), ncclUint8, (int)q, comm, s) == ncclSuccess;
                    if (nr && collOk)
                        collOk = R.recv(recvRec_ + recvOff, (size_t)nr * sizeof(SplatRecord), ncclUint8, (int)q, comm, s) ==
                                 ncclSuccess;
                }
                sendOff += ns;
                recvOff += nr;
            }
            if (R.groupEnd() != ncclSuccess) collOk = false;
            recvTotal_ = recvTotal;
            break;
        }
        case 2: {
            if (frameErr_ == GSM_OK && mine) {
                if ((st = setRows()) == GSM_OK) {
                    r_->selectSchedule(0);
                    st = r_->renderRecords(s, recvRec_, recvTotal_, width, height, colorT, colorP, depthT, depthP);
                }
                if (st != GSM_OK) frameErr_ = st;
            }
            break;
        }
        case 3: {
            if (t.gather && world > 1) {  // every slab's pixel rows to rank 0 (sent even by a failed rank)
                collOk = R.groupStart() == ncclSuccess;
                for (uint32_t q = 1; q < world && collOk; ++q) {
                    if (rank != 0 && rank != q) continue;
                    uint32_t y0, y1;
                    for (uint32_t k = 0; collOk && slabPixelRows(q, k, height, &y0, &y1); ++k) {
                        const size_t cOff = (size_t)y0 * framePitch_, cBytes = (size_t)(y1 - y0) * framePitch_;
                        const size_t dOff = (size_t)y0 * depthPitch0_, dBytes = (size_t)(y1 - y0) * depthPitch0_;
                        if (rank == 0) {
                            collOk = R.recv(ownFrame_ + cOff, cBytes, ncclUint8, (int)q, comm, s) == ncclSuccess &&
                                     (!t.gatherDepth || R.recv(ownDepth_ + dOff, dBytes, ncclUint8, (int)q, comm, s) == ncclSuccess);
                        } else {
                            collOk = R.send(ownFrame_ + cOff, cBytes, ncclUint8, 0, comm, s) == ncclSuccess &&
                                     (!t.gatherDepth || R.send(ownDepth_ + dOff, dBytes, ncclUint8, 0, comm, s) == ncclSuccess);
                        }
                    }
                }
                if (R.groupEnd() != ncclSuccess) collOk = false;
            }
            if (t.gather && rank == 0 && frameErr_ == GSM_OK && gatherColor) {  // the caller's targets
                const size_t rowBytes = (size_t)width * bpp_;
                if (gatherColor != ownFrame_)
                    hipMemcpy2DAsync(gatherColor, colorPitch, ownFrame_, framePitch_, rowBytes, height, hipMemcpyDeviceToDevice, s);
                if (t.gatherDepth && depth && depth != ownDepth_)
                    hipMemcpy2DAsync(depth, depthPitch, ownDepth_, depthPitch0_, (size_t)width * 2u, height,
                                     hipMemcpyDeviceToDevice, s);
            }
            break;
        }
    }
    if (!collOk) {
        if (frameErr_ == GSM_OK) frameErr_ = GSM_ERR_RENDER_FAILED;
        launchFailed_ = true;
        return GSM_ERR_RENDER_FAILED;
    }
    if (hipGetLastError() != hipSuccess) {
        launchFailed_ = true;
        return GSM_ERR_RENDER_FAILED;
    }
    return frameErr_;
}

gsm_status MultiGpu::counts(uint32_t* hostCounts) {
    if (transport_ == GSM_MG_TRANSPORT_RCCL) {  // (the last frame's matrix, copied to the host in its phase 1)
        std::memcpy(hostCounts, hostCounts_, (size_t)world_ * world_ * 4);
        return GSM_OK;
    }
    hipSetDevice(device_);
    const uint32_t* c = ctl() + kCountsWord + par_ * kMaxSlabs * kMaxSlabs;
    if (hipMemcpy(hostCounts, c, (size_t)world_ * world_ * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return GSM_ERR_RENDER_FAILED;
    return GSM_OK;
}

}  // namespace gsm

struct gsm_multigpu {
    gsm::MultiGpu* impl;
};

extern "C" {

void gsm_multigpu_default_options(gsm_multigpu_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->struct_bytes = sizeof(gsm_multigpu_options);
    o->rows = GSM_MG_ROWS_CONTIGUOUS;
    o->transport = GSM_MG_TRANSPORT_PEER_STORES;
    o->timeout_ms = 10000;
}

// the options of the entry points without them: the defaults with the environment's test overrides
static gsm_multigpu_options env_options() {
    gsm_multigpu_options o;
    gsm_multigpu_default_options(&o);
    const char* rv = getenv("GSM_MG_ROWS");
    if (rv && std::strcmp(rv, "interleaved") == 0) o.rows = GSM_MG_ROWS_INTERLEAVED;
    const char* pv = getenv("GSM_MG_PIPELINE");
    if (pv && pv[0] == '1') o.pipelined = 1;
    return o;
}

gsm_status gsm_multigpu_prepare_with_options(gsm_renderer* renderer, int rank, int world_size,
                                             const gsm_multigpu_options* options, gsm_multigpu** out, void* handle) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!renderer || !renderer->impl || !options) return GSM_ERR_INVALID_ARGUMENT;
    gsm::MultiGpu* m = nullptr;
    gsm_status st = gsm::MultiGpu::prepare(renderer->impl, rank, world_size, *options, &m, handle);
    if (st != GSM_OK) return st;
    gsm_multigpu* h = new (std::nothrow) gsm_multigpu{m};
    if (!h) {
        delete m;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    *out = h;
    return GSM_OK;
}

gsm_status gsm_multigpu_prepare(gsm_renderer* renderer, int rank, int world_size, gsm_multigpu** out, void* handle) {
    const gsm_multigpu_options o = env_options();
    return gsm_multigpu_prepare_with_options(renderer, rank, world_size, &o, out, handle);
}

gsm_status gsm_multigpu_connect(gsm_multigpu* m, const void* all_handles) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->connect(all_handles);
}

gsm_status gsm_multigpu_create_with_options(gsm_renderer* renderer, void* nccl_comm, int rank, int world_size,
                                            const gsm_multigpu_options* options, gsm_multigpu** out) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!renderer || !renderer->impl || !options) return GSM_ERR_INVALID_ARGUMENT;
    const gsm::Rccl& R = gsm::rccl();
    if (!R.ok) return GSM_ERR_UNSUPPORTED;
    if (!nccl_comm || world_size < 1 || world_size > (int)gsm::kMaxSlabs || rank < 0 || rank >= world_size)
        return GSM_ERR_INVALID_ARGUMENT;
    int n = 0, me = -1;
    if (R.commCount((ncclComm_t)nccl_comm, &n) != ncclSuccess || R.userRank((ncclComm_t)nccl_comm, &me) != ncclSuccess ||
        n != world_size || me != rank)
        return GSM_ERR_INVALID_ARGUMENT;
    gsm_multigpu_options o = *options;
    if (o.struct_bytes != sizeof(gsm_multigpu_options)) return GSM_ERR_INVALID_ARGUMENT;
    if (o.transport == GSM_MG_TRANSPORT_RCCL) o.nccl_comm = nccl_comm;  // the frames' collectives run on it
    std::vector<uint8_t> all((size_t)world_size * GSM_MULTIGPU_HANDLE_BYTES);
    gsm_multigpu* h = nullptr;
    gsm_status st = gsm_multigpu_prepare_with_options(renderer, rank, world_size, &o, &h,
                                                      all.data() + (size_t)rank * GSM_MULTIGPU_HANDLE_BYTES);
    if (st != GSM_OK) return st;
    // the handles over the communicator (once, at set-up; the peer-stores frame itself uses no collective)
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

gsm_status gsm_multigpu_create(gsm_renderer* renderer, void* nccl_comm, int rank, int world_size,
                               gsm_multigpu** out) {
    const gsm_multigpu_options o = env_options();
    return gsm_multigpu_create_with_options(renderer, nccl_comm, rank, world_size, &o, out);
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

gsm_status gsm_multigpu_finish_frame(gsm_multigpu* m, void* stream) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->finishFrame((hipStream_t)stream);
}

gsm_status gsm_multigpu_debug_set_epoch(gsm_multigpu* m, uint32_t epoch) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->debugSetEpoch(epoch);
}

gsm_status gsm_multigpu_wait_event(gsm_multigpu* m, void* event) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->waitEvent((hipEvent_t)event);
}

gsm_status gsm_multigpu_render(gsm_multigpu* m, void* stream, const gsm_gaussian_input* input,
                               const gsm_camera_params* camera, uint32_t width, uint32_t height, void* color,
                               size_t color_pitch_bytes, void* depth, size_t depth_pitch_bytes, void* gather_color) {
    // every phase runs even after a refusal: its barrier steps keep the ranks' epochs in step
    gsm_status first = GSM_OK;
    for (int p = 0; p < 4; ++p) {
        gsm_status st = gsm_multigpu_render_phase(m, p, stream, input, camera, width, height, color, color_pitch_bytes,
                                                  depth, depth_pitch_bytes, gather_color);
        if (first == GSM_OK) first = st;
    }
    return first;
}

gsm_status gsm_multigpu_frame(gsm_multigpu* m, void** color, size_t* pitch_bytes) {
    if (!m || !m->impl || !color || !pitch_bytes) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->frame(color, pitch_bytes);
}

gsm_status gsm_multigpu_frame_depth(gsm_multigpu* m, void** depth, size_t* pitch_bytes) {
    if (!m || !m->impl || !depth || !pitch_bytes) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->frameDepth(depth, pitch_bytes);
}

gsm_status gsm_multigpu_status(gsm_multigpu* m, uint32_t* timeouts, int clear) {
    if (!m || !m->impl || !timeouts) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->status(timeouts, nullptr, clear != 0);
}

gsm_status gsm_multigpu_errors(gsm_multigpu* m, uint32_t* timeouts, uint32_t* failed_peer_arrivals, int clear) {
    if (!m || !m->impl || !timeouts || !failed_peer_arrivals) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->status(timeouts, failed_peer_arrivals, clear != 0);
}

gsm_status gsm_multigpu_set_timeout_ms(gsm_multigpu* m, uint32_t ms) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->setTimeout(ms);
}

gsm_status gsm_multigpu_debug_copy_frame(gsm_multigpu* m, void* host_dst, size_t dst_pitch_bytes, uint32_t width,
                                         uint32_t height) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->copyFrame(host_dst, dst_pitch_bytes, width, height, false);
}

gsm_status gsm_multigpu_debug_copy_depth(gsm_multigpu* m, void* host_dst, size_t dst_pitch_bytes, uint32_t width,
                                         uint32_t height) {
    if (!m || !m->impl) return GSM_ERR_INVALID_ARGUMENT;
    return m->impl->copyFrame(host_dst, dst_pitch_bytes, width, height, true);
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
