// gsm_internal.h -- host-side launchers for the gfx950 kernels (gsm_kernels.hip) and
// the radix sort (gsm_sort.hip).  Every launcher only enqueues on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "gsm_types.h"

namespace gsm {

// Scalars the projection/assignment kernels read (kernel argument, by value).
struct ProjectArgs {
    CameraUniforms cam;
    TileBinningParams bin;
    // the renderer's tile rows: rowBegin, rowBegin + rowStride, ... < rowEnd -- a
    // contiguous slab (stride 1; full frame [0, tilesY)) or a multi-GPU rank's interleaved rows
    // (stride = world).  Tile ids of keys, tile starts and blend units count the set's rows only:
    // local tile = k * tilesX + tx for row rowBegin + k * rowStride.
    uint32_t rowBegin, rowEnd, rowStride;
    uint32_t count;
    uint32_t maxAssignments;
    uint32_t keepRenderData;  // write GaussianRenderData of every visible gaussian (debug readback);
                              // otherwise only where the scatter needs it (rects over kMaskTiles tiles)
    uint32_t schedUnits;      // > 0: the projection launch also orders this many blend units
    uint32_t pairBucket;      // the pair-walk blend (k_blend_pw): units of the schedule's walk buckets below this
                              // one (walk > (256 - pairBucket) / 256 of the longest) run alone, the rest in pairs;
                              // the split position goes to costMax[kCostMaxSlots] (0: not written)
                              // (unit_order_block in one extra workgroup, block 0)
    // per-frame constants of projectCovariance2D / stabilizeCovariance2D / computeDepthFactor,
    // evaluated once on the host with the same IEEE fp32 operations the kernels would repeat
    // per gaussian (GaussianShared.h:326-375, 655-714, 275-278)
    float limX, limY, focalX, focalY, maxEig, adjFar, adjDen;
};

// Multi-GPU partition: tile-row boundaries of the slabs, and the 48-byte
// record a slab owner receives per gaussian (GaussianRenderData + blend record + tile rect).
constexpr uint32_t kMaxSlabs = 16;
struct SlabTable {
    uint32_t rows[kMaxSlabs + 1];  // contiguous: slab s = rows [rows[s], rows[s + 1])
    uint32_t n;
    uint32_t interleave;  // 1: slab s = rows s, s + n, s + 2n, ... < rows[n] (rows[n] = tilesY)
};
struct SplatRecord {
    uint4 rd;         // GaussianRenderData
    BlendRecordA ra;  // mean, conic, opacity, r, g
    short4 bounds;    // tile rect
    uint32_t rb;      // b, depth
    uint32_t pad;
};
static_assert(sizeof(SplatRecord) == 48, "SplatRecord must be 48 B");
// the receive buffer of every slab owner (peer device pointers; the multi-GPU exchange)
struct SlabPeers {
    SplatRecord* recv[kMaxSlabs];
    uint32_t cap[kMaxSlabs];  // records each receive buffer holds (k_part_copy writes no further)
};
struct PartitionBuffers {
    SplatRecord* runs = nullptr;        // [slabs][runStride]: the projection's block runs, block b of
                                        // slab s at s * runStride + b * 256 (k_project_part)
    uint32_t runStride = 0;             // records per slab: the blocks of maxG ids x 256
    uint32_t runSlabs = 0;              // slabs `runs` holds
    uint32_t* blockSlabCounts = nullptr;  // [kMaxSlabs * blocks]
};

// ---------------------------------------------------------------------------
// Multi-GPU frame (gsm_multigpu.hip): memory model of the exchange.
// Every store of exchange data (counts, records, the gathered pixels) is a SYSTEM-coherent
// write-through store (`sc0 sc1`: st_sys* below) -- it leaves no dirty line in any L2 and is
// acknowledged only once it is visible at system scope.  A producing kernel arrives at a barrier
// itself: every storing unit (a wave, or a workgroup after a barrier) drains its stores
// (`s_waitcnt vmcnt(0)`), then makes one device-scope add to the rank's arrival counter; the unit
// whose add completes the count raises this rank's flag word of the barrier in every rank's control
// block (system-coherent stores) and re-arms the counter.  Every consumer load of exchange data is
// system-coherent (`sc0 sc1`: ld_sys*), so no L1 or L2 line that predates the flag can serve it, on
// any XCD of any GPU.  (r04: a system-scope release -- buffer_wbl2 sc0 sc1 -- in every storing unit
// instead of write-through stores cost the config-4 virtual-rank frame 0.272 -> 0.372 ms.)
// ---------------------------------------------------------------------------
struct MgArrive {
    uint32_t* flag[kMaxSlabs];  // this rank's word of the barrier in rank p's control block (peer mappings)
    uint32_t* done;             // this rank's arrival counter of the barrier (own memory, 0 between frames)
    uint32_t total;             // arriving units of the launch
    uint32_t epoch;             // the frame number the flags receive
    uint32_t world;
};

// One arriving unit: called by every lane of ONE wave, after every exchange store the unit signals
// for (a workgroup arriving as one unit: every wave's `s_waitcnt vmcnt(0)`, then a workgroup
// barrier, then one wave calls this).
// (total: the arriving units, a.total unless the caller counts them otherwise)
__device__ __forceinline__ void mg_arrive_wave(const MgArrive& a, uint32_t total) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through stores are acknowledged
    uint32_t last = 0;
    if ((threadIdx.x & 63u) == 0)
        last = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1u ? 1u : 0u;
    if (__builtin_amdgcn_readfirstlane(last)) {
        // every other unit drained its stores before its add: the flags go out after all of them
        const uint32_t lane = threadIdx.x & 63u;
        if (lane == 0) __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane < a.world) __hip_atomic_store(a.flag[lane], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__device__ __forceinline__ void mg_arrive_wave(const MgArrive& a) { mg_arrive_wave(a, a.total); }
// a workgroup arriving as one unit (see mg_arrive_wave); ends the kernel's use of it
__device__ __forceinline__ void mg_arrive_block(const MgArrive& a) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64u) mg_arrive_wave(a);
}
// Arrivals of many units (thousands of workgroups) spread over kArriveShards counters, each on its
// own 128-B line after the barrier's main counter (a.done[0]): unit u adds to shard u % kArriveShards;
// the add completing a shard (its unit count is known from a.total) re-arms that shard and arrives at
// the main counter for it, whose last add raises the flags (mg_arrive_wave).  Same-address atomics
// serialize in one L2 channel: 2442 adds to one word cost more than the projection's tail.
constexpr uint32_t kArriveShards = 16, kArriveLineWords = 32;
constexpr uint32_t kArriveWordsPerBarrier = (1 + kArriveShards) * kArriveLineWords;
// called by every lane of ONE wave, after every exchange store of the unit (as mg_arrive_wave)
__device__ __forceinline__ void mg_arrive_unit(const MgArrive& a, uint32_t unit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t sh = unit % kArriveShards;
    const uint32_t shTotal = (a.total - sh + kArriveShards - 1u) / kArriveShards;  // (unit < total)
    uint32_t* c = a.done + (1u + sh) * kArriveLineWords;
    uint32_t last = 0;
    if ((threadIdx.x & 63u) == 0)
        last = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shTotal - 1u ? 1u : 0u;
    if (__builtin_amdgcn_readfirstlane(last)) {
        if ((threadIdx.x & 63u) == 0) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mg_arrive_wave(a, a.total < kArriveShards ? a.total : kArriveShards);  // (the shards that have units)
    }
}
__device__ __forceinline__ void mg_arrive_block_unit(const MgArrive& a, uint32_t unit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64u) mg_arrive_unit(a, unit);
}
// k_part_scan's count publication: row `rank` of rank p's count matrix (this frame's parity), and
// the arrival at barrier 0 (arrive.done == null: no publication, the send-buffer path)
struct CountPublish {
    uint32_t* row[kMaxSlabs];
    MgArrive arrive;
};
// system-coherent access to exchange data (sc0 sc1): loads no cached copy can answer, write-through
// stores; `base` wave-uniform, `bytes` its extent (the buffer descriptor's range), i in elements
constexpr int kSysCoherent = 17;  // cache-policy bits sc0 | sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t ld_sys32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint4 ld_sys128(const void* base, uint32_t bytes, uint32_t i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(sys_rsrc(base, bytes), (int)(i * 16u), 0, kSysCoherent);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_sys128(void* base, uint32_t bytes, uint32_t i, uint4 v) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, sys_rsrc(base, bytes), (int)(i * 16u), 0, kSysCoherent);
}
// byte offset `off` from a wave-uniform base
__device__ __forceinline__ void st_sys32_at(void* base, uint32_t bytes, uint32_t off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, sys_rsrc(base, bytes), (int)off, 0, kSysCoherent);
}
__device__ __forceinline__ void st_sys16_at(void* base, uint32_t bytes, uint32_t off, uint16_t v) {
    __builtin_amdgcn_raw_buffer_store_b16(v, sys_rsrc(base, bytes), (int)off, 0, kSysCoherent);
}
__device__ __forceinline__ void st_sys128_at(void* base, uint32_t bytes, uint32_t off, uint4 v) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, sys_rsrc(base, bytes), (int)off, 0, kSysCoherent);
}

// A sort's device workspace and its sizes.  Every sort below plans its passes first and launches
// nothing (returns kSortNoSpace) when one pass's per-block digit counts, super-group rows or digit
// totals would not fit -- a knob or a grid rule changed without the allocation (the r05 wide-pass
// A/B fault class); callers report GSM_ERR_INVALID_ASSIGNMENT_CAPACITY.
struct SortSpace {
    uint32_t* hist = nullptr;      // radix_workspace_bytes(capacity) bytes, zeroed once at allocation
    size_t histBytes = 0;
    uint32_t* binTotals = nullptr;  // digit totals (+ the tile passes' bucket starts)
    size_t binWords = 0;
};
constexpr int kSortNoSpace = -1;

// Device buffers of one renderer (the GlobalViewResources analogue, GlobalResources.swift:6-362).
struct DeviceArena {
    GaussianRenderData* renderData = nullptr;  // [maxG]
    short4* bounds = nullptr;                  // [maxG]
    BlendRecord* rec = nullptr;                // [maxG] blend records, 32 B each
    uint32_t* tileCounts = nullptr;            // [maxG]
    uint32_t* tileMasks = nullptr;             // [maxG] tile tests of rects <= 32 tiles, scan order
    uint32_t* blockSums = nullptr;             // [ceil(maxG/256) + 1]
    TileAssignmentHeader* header = nullptr;    // [1]
    uint32_t* keys[2] = {nullptr, nullptr};    // [cap] ping-pong
    uint32_t* vals[2] = {nullptr, nullptr};    // [cap]
    uint32_t* keysKeep = nullptr;              // [cap] unsorted copy (profiling/debug only)
    uint32_t* valsKeep = nullptr;
    unsigned long long* blendTrace = nullptr;  // [4 * tiles * 4] (profiling bit 2 only)
    uint32_t* costMax = nullptr;               // [kCostMaxSlots] longest walk of the last blend
    uint32_t* radixHist = nullptr;             // radix_workspace_bytes(maxAssignments) bytes
    size_t radixHistBytes = 0;
    uint32_t* radixBinTotals = nullptr;        // [kSortTotalsWords] (radix_sort_tiles)
    uint32_t* tileStart = nullptr;             // [tileCount + 1] first sorted entry of each tile
    uint32_t* tileQueue = nullptr;             // [kQueueStripes * kQueueStride] blend work counters
    uint16_t* unitCost = nullptr;              // [4 * tileCount] list entries each blend unit walked
    uint32_t* unitOrder = nullptr;             // [4 * tileCount] blend units, longest last-frame walk first
    uint32_t* halfVals[2] = {nullptr, nullptr};  // [cap] per half tile: the tile's sorted gaussian ids whose
                                                 // skip flag for that half is clear, from the tile's start
    uint32_t* halfCount = nullptr;             // [2 * tileCount] entries of each half list (half-major)
    uint16_t* expTable = nullptr;              // [65536]
    float2* sincosTable = nullptr;             // [kSincosEntries + 256]: sin/cos, then the byte table (det_byte_lut_entry)
};

// A/B switches of the frame pipeline.  Read ONCE, when a renderer is created (tuning_from_env),
// never per frame; every setting renders the same image, only the schedule differs.
struct Tuning {
    bool fullRadix = false;   // GSM_SORT=radix4: 4 x 8-bit passes over (tile << 16 | depth) keys instead
                              // of the tile passes + per-tile depth sort
    bool ballotRank = false;  // stable ranks from ballot matches instead of lane-ordered LDS atomics:
                              // set when the create-time device probe (sort_lane_ordered_atomics) fails,
                              // or forced by GSM_SORT_RANK=ballot
    bool costOrder = true;    // GSM_BLEND_SCHED=0: blend units in index order instead of last frame's walks
    int blendWaves = 0;       // GSM_BLEND_WAVES=8|12|16: waves per blend workgroup (0: by frame size)
    int blendClaim = 1;       // GSM_BLEND_CLAIM=early|late|auto (0/1/2): when a blend wave claims its next unit
    bool wideSort = true;     // GSM_SORT_WIDE=0: narrow passes only (no wide 9..11-bit tile or depth passes)
    bool sortScanless = true; // GSM_SORT_SCAN=kernel: narrow passes with the k_radix_scan launch (r05 default: none)
    bool blendPairs = true;   // half-tile frames on one GPU: two units per blend wave (k_blend_pw, r05);
                              // GSM_BLEND_PAIRS=0: one unit per wave (k_blend_px)
    int pairBucket = 128;     // GSM_BLEND_PAIR_SPLIT=b (0..256): the units whose last walk exceeds (256 - b) / 256
                              // of the longest run alone, the others in pairs (ProjectArgs::pairBucket)
    bool fusedScan = true;    // frames of <= kFusedScanMaxBlocks projection blocks: every scatter workgroup
                              // sums the block counts before its own (no k_scan_blocks launch);
                              // GSM_SCAN_FUSED=0: the separate scan
};
constexpr uint32_t kFusedScanMaxBlocks = 8192;
// the environment's settings plus the device probe; `device` is a HIP device id
Tuning tuning_from_env(int device);
// Create-time probe of the one undocumented hardware property the default sort ranks rely on:
// the lanes of one ds_add_rtn_u32 that hit the same LDS address receive their old values in lane
// order.  Runs a small kernel once per device and process (cached); false -> ballot ranks.
bool sort_lane_ordered_atomics(int device);

// Half-tile skip flags of an assignment (the value word's two top bits, set by k_scatter): bit
// kHalfSkipShift + h when every pixel of half h (16 px columns [16h, 16h + 16) of the 32x16 tile)
// provably gets alpha 0 from the gaussian -- its fp16 quadratic form p exceeds kBlendZeroP there
// (quad_exceeds, gsm_device.h), and the blend's exp table is 0 for every fp16 p above it
// (tests/golden/exp_h_table.npy: 34.65625 is the largest p with a nonzero entry), so alpha =
// min(op * 0, 0.99) = 0 and the pixel's colour and transmittance stay bit-identical.
constexpr uint32_t kHalfSkipShift = 30;
constexpr uint32_t kGidMask = (1u << kHalfSkipShift) - 1u;
constexpr float kBlendZeroP = 34.65625f;

constexpr int kProjectBlock = 256;
// entries of the sincos table (one per quantised angle); the 256 byte-table entries follow (gsm_detmath.h)
constexpr uint32_t kSincosEntries = 65536;
constexpr int kRadixBlock = 256;
constexpr int kRadixItems = 16;  // keys per thread per chunk (4096-key chunks)
constexpr int kRadixChunk = kRadixBlock * kRadixItems;
// wide radix digits (gsm_sort.hip): up to 11 bits, 2048 bins
constexpr uint32_t kWideMaxBits = 11, kWideBins = 1u << kWideMaxBits;
// radix_sort_tiles' workspace beside the histogram: two passes' digit totals + the bucket starts
// (narrow passes, 768 words), or one wide pass's 2048 digit totals
constexpr size_t kSortTotalsWords = kWideBins;
inline SortSpace sort_space(const DeviceArena& A) { return SortSpace{A.radixHist, A.radixHistBytes, A.radixBinTotals, kSortTotalsWords}; }

// project + cull + SH + tile count + per-block count sums (GlobalShaders.metal:19-123, 563-616)
void launch_project(bool halfInput, uint32_t shDegree, const void* world, const void* harmonics,
                    const ProjectArgs& args, const DeviceArena& A, hipStream_t stream);
// exclusive scan of the per-block sums, total + clamp into the header (GlobalShaders.metal:685-712)
// project gaussians [0, a.count) of world/harm (already offset to the rank's range) and pack
// the records of each slab's gaussians into `send` (slab-major, ascending id), counts to sendCounts
void launch_partition(bool halfInput, uint32_t shDegree, const void* world, const void* harmonics,
                      const ProjectArgs& args, const SlabTable& slabs, const PartitionBuffers& B,
                      const float2* sincos, void* send, uint64_t capacity, uint32_t* sendCounts,
                      hipStream_t stream);
// the first half of launch_partition (projection + per-slab counts, no packing), then the records
// written straight to every slab owner from the all-gathered count matrix (gsm_multigpu.hip)
// (args.schedUnits > 0: one extra workgroup orders the blend units of the renderer's own rows, A)
void launch_partition_counts(bool halfInput, uint32_t shDegree, const void* world, const void* harmonics,
                             const ProjectArgs& args, const SlabTable& slabs, const PartitionBuffers& B,
                             const float2* sincos, uint32_t* sendCounts, const DeviceArena& A,
                             const CountPublish& publish, hipStream_t stream);
void launch_partition_push(const ProjectArgs& args, uint32_t world, uint32_t rank, const PartitionBuffers& B,
                           const uint32_t* counts, const SlabPeers& peers, uint32_t* recvCount, const SlabTable& slabs,
                           const MgArrive& arrive, hipStream_t stream, uint32_t gridCap = 0);
// received records -> per-gaussian arrays + tile counts of the renderer's rows (replaces project)
void launch_records_in(const void* records, const ProjectArgs& args, const DeviceArena& A,
                       hipStream_t stream, const uint32_t* devCount = nullptr);
// devCount (nullable): the gaussian count on the device (records path); only its blocks are scanned
void launch_scan_blocks(uint32_t numBlocks, const ProjectArgs& args, const DeviceArena& A,
                        hipStream_t stream, const uint32_t* devCount = nullptr);
// the same scan for any array of nb per-block sums: exclusive scan in place, the total clamped
// to cap into hdr (overflow flag when it exceeds cap), *queue = 0
void launch_scan_sums(uint32_t* sums, uint32_t nb, uint32_t cap, TileAssignmentHeader* hdr, uint32_t* queue,
                      hipStream_t stream);
// duplicate-with-keys (GlobalShaders.metal:623-678 fused with :266-295)
// fusedScan: A.blockSums holds the unscanned block counts (no launch_scan_blocks before it); each
// workgroup adds up the counts before its own, workgroup 0 also the total (header, blend queue)
void launch_scatter(const ProjectArgs& args, const DeviceArena& A, hipStream_t stream,
                    const uint32_t* devCount = nullptr, bool fusedScan = false);
// the blend's half-tile lists from the sorted values (skip flags, k_scatter), tiles [tileBegin, +numTiles)
void launch_half_lists(const uint32_t* sortedVals, uint32_t tileBegin, uint32_t numTiles, const DeviceArena& A,
                       uint32_t tileCount, hipStream_t stream);
// per-tile binary search headers (GlobalShaders.metal:304-363), tiles of rows [rowBegin,rowEnd)
void launch_headers(const uint32_t* sortedKeys, const FrameGeometry& geo, const DeviceArena& A,
                    hipStream_t stream);
// front-to-back fp16 blend + clear (GlobalShaders.metal:140-154, 1030-1187); returns the kernel it
// launched (gsm_blend_kernel, include/gsm_debug.h; 0 for an empty frame)
int launch_blend(const FrameGeometry& geo, const DeviceArena& A,
                  void* color, size_t colorPitch, void* depth, size_t depthPitch, int numCUs,
                  bool costOrder, int colorFormat, hipStream_t stream, int waves = 0, int claim = 1,
                  const MgArrive* arrive = nullptr, bool pairs = false);
// k_blend_pw (gsm_blend_pw.hip): two half-tile units per wave, one GPU's frame
void launch_blend_pw(const FrameGeometry& g, const DeviceArena& A, void* color, size_t colorPitch, void* depth,
                     size_t depthPitch, int numCUs, bool costOrder, int colorFormat, hipStream_t s, int waves);
// blend kernel shape: pixel pairs per lane (0 = quadrant kernel) and blend units per tile
int blend_pairs_per_lane(uint32_t numTiles, int numCUs);
uint32_t blend_units_per_tile(uint32_t numTiles, int numCUs);

// Stable LSD radix sort of (key, value) pairs; n read from device memory *nPtr.
// Returns the index (0/1) of the ping-pong buffer holding the result (or kSortNoSpace).
// ballot: ranks from ballot matches (Tuning::ballotRank) instead of lane-ordered LDS atomics.
int radix_sort_pairs(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                     int firstDigit, int numDigits, const SortSpace& ws,
                     hipStream_t stream, bool ballot, bool scanless = true);
// Stable LSD radix sort by bits [shift, shift + bits) only, in ceil(bits / 8) passes of
// near-equal digit widths (4..8 bits), or -- `wide` and where that saves a pass -- ceil(bits / 11)
// passes of 9..11 bits.  binTotals: kSortTotalsWords words.  Returns the ping-pong index of the result.
int radix_sort_bits(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                    uint32_t shift, uint32_t bits, const SortSpace& ws, hipStream_t stream,
                    bool ballot, bool wide = false, bool scanless = true);
// the frame sort's tile field (tiles [tileBase, tileBase + numTiles) of allTiles, bits <= 16) with
// the tile starts written by its last pass (tileStart[0..allTiles], lower bounds for empty tiles);
// one wide pass relative to tileBase when numTiles <= 2048 and `wide`; binTotals: kSortTotalsWords words
int radix_sort_tiles(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity, uint32_t shift,
                     const SortSpace& ws, uint32_t* tileStart, uint32_t tileBase, uint32_t numTiles,
                     uint32_t allTiles, hipStream_t stream, bool ballot, bool wide = true, bool scanless = true);
// the workspace footprint of one pass (words of `hist`, incl. the super-group rows in front), and
// whether every pass radix_sort_bits plans fits `ws` (host only: no launch)
size_t sort_pass_hist_words(bool wide, int bits, uint32_t grid);
bool sort_bits_plan_fits(uint32_t capacity, uint32_t bits, bool wide, const SortSpace& ws);
// scanless: narrow passes without the k_radix_scan launch (super-group digit rows, gsm_sort.hip;
// Tuning::sortScanless) -- the same order either way
uint32_t radix_grid_for_capacity(uint32_t capacity);
// bytes of the sort workspace (`hist` argument above) for a capacity; zero it once at allocation
size_t radix_workspace_bytes(uint32_t capacity);
// stable per-tile sort by the 16-bit depth key of runs already grouped by tile (one workgroup per
// tile), which writes the blend's half-tile lists (as launch_half_lists) and, when `full`, the sorted
// keys and values (keysOut / valsOut; the reference's sorted arrays, read back by captured frames)
void tile_depth_sort(uint32_t* keysIn, uint32_t* valsIn, uint32_t* keysOut, uint32_t* valsOut,
                     const uint32_t* tileStart, uint32_t tileBegin, uint32_t numTiles, hipStream_t stream,
                     bool ballot, uint32_t* half0, uint32_t* half1, uint32_t* halfCount, uint32_t tileCount,
                     bool full, int numCUs);

// Inclusive prefix sum over the 64 lanes of a wave by DPP (row_shr 1/2/4/8 within rows of 16, then
// row_bcast 15 / 31 across rows): six VALU adds with their operand moved by the DPP unit, where a
// __shfl_up step is a ds_bpermute (an LDS round trip; six of them per scan -- r06: the sorts' digit
// scans and the block scans).  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// Unpredicated loads of 4-word groups p[i, i + 4) (i % 4 == 0) ending at n.  A load under a condition
// whose value is used under the same condition is issued alone and waited for before the next one (the
// compiler's diamond per group: r06, every k_scan_blocks / upsweep / tile-sort / schedule load was its own
// memory round trip).  Here the 16-B load's index is clamped to the last whole group and the ragged group
// at n & ~3 comes from `t` (three uniform loads, once per thread), so all loads go out before any wait.
// Words at and past n are unspecified (callers mask them).  Needs n >= 1 and 16 readable bytes at p.
struct Tail4 {
    uint32_t n4, last4, t[3];
};
__device__ __forceinline__ Tail4 tail4_load(const uint32_t* __restrict__ p, uint32_t n) {
    Tail4 T;
    T.n4 = n & ~3u;
    T.last4 = T.n4 >= 4u ? T.n4 - 4u : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) T.t[j] = p[min(T.n4 + j, n - 1u)];
    return T;
}
__device__ __forceinline__ uint4 load4_clamped(const uint32_t* __restrict__ p, uint32_t i, const Tail4& T) {
    return *(const uint4*)(p + min(i, T.last4));
}
__device__ __forceinline__ uint4 fix4(uint4 q, uint32_t i, const Tail4& T) {
    return i == T.n4 ? make_uint4(T.t[0], T.t[1], T.t[2], 0u) : q;
}

// The blends' 128 KiB exp table from global memory into the workgroup's LDS copy: every load of a thread
// in flight at once (unpredicated, clamped), then the 16-B LDS stores.  (A `dst[i] = src[i]` loop over
// i += NT compiled to load / wait / store per iteration: 8-16 memory round trips, one after another, before
// any wave could blend -- r06.)
#define GSM_EXP_TABLE_TO_LDS(NTHREADS, expTable, tbl)                                                        \
    do {                                                                                                     \
        constexpr uint32_t kVec_ = 65536u * 2u / 16u, kPer_ = (kVec_ + (NTHREADS) - 1u) / (NTHREADS);        \
        const uint4* src_ = (const uint4*)(expTable);                                                        \
        uint4 t_[kPer_];                                                                                     \
        _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPer_; ++k_)                                            \
            t_[k_] = src_[min((uint32_t)threadIdx.x + k_ * (uint32_t)(NTHREADS), kVec_ - 1u)];                \
        _Pragma("unroll") for (uint32_t k_ = 0; k_ < kPer_; ++k_) {                                          \
            const uint32_t i_ = (uint32_t)threadIdx.x + k_ * (uint32_t)(NTHREADS);                           \
            if (i_ < kVec_) ((uint4*)(tbl))[i_] = t_[k_];                                                    \
        }                                                                                                    \
    } while (0)

// Blend schedule (the blend's unit order): the units in descending order of the walk each made
// in the previous frame (longest-processing-time-first list scheduling on the blend's persistent
// waves), as a counting sort into kUoBuckets buckets of walk length (bucket width = max walk /
// 256, so the order is exact to ~1 % of the longest walk; any order inside a bucket -- the image
// does not depend on the schedule).  One workgroup of NT threads: the longest walk, bucket sizes
// (LDS atomics), their scan, a scatter with one LDS atomic per unit; every pass keeps 8 loads per
// thread in flight.  `base` = LDS[kUoBuckets], `wmax` = LDS[NT / 64]; the longest walk comes from
// `costMax` (kCostMaxSlots words the blend's waves atomicMax into).
constexpr uint32_t kUoBuckets = 256;
// The blend's dynamic queue is striped: workgroup b draws positions of the schedule congruent to
// b % kQueueStripes from counter b % kQueueStripes (words kQueueStride apart, one 64-B line each),
// so the same-address atomics of the many waves spread over 8 lines (r02: with one counter the
// average gap between a wave's units at 4K was 7.7 us of queueing).
constexpr uint32_t kQueueStripes = 8, kQueueStride = 16;
constexpr uint32_t kCostMaxSlots = 64;  // words of the longest-walk maximum (spread atomics)
// (+ 2 words after them in the Global renderer's schedule sets: the pair walk's split position and the
// longest walk of the previous frame, which the blend's remaining-work priorities scale by)
template <int NT>
__device__ __forceinline__ void unit_order_block(const uint16_t* __restrict__ cost, uint32_t* __restrict__ order,
                                                 uint32_t n, uint32_t* base, uint32_t* wmax,
                                                 uint32_t* __restrict__ costMax, uint32_t splitBucket = 0) {
    static_assert(NT >= (int)kUoBuckets && NT % 64 == 0, "one thread per bucket");
    constexpr uint32_t UN = 8;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    auto load = [&](uint32_t b0, uint32_t (&c)[UN]) {  // (b0 < n; unpredicated, clamped: see Tail4)
#pragma unroll
        for (uint32_t k = 0; k < UN; ++k) c[k] = (uint32_t)cost[min(b0 + k * (uint32_t)NT + t, n - 1u)];
    };
    // the longest walk: the previous frame's blend left each wave's longest in one of kCostMaxSlots
    // words (atomicMax at its exit); read them and clear them for this frame's blend
    uint32_t m = t < kCostMaxSlots ? costMax[t] : 0u;
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
    if (lane == 0) wmax[w] = m;
    if (t < kUoBuckets) base[t] = 0;
    __syncthreads();
    if (t < kCostMaxSlots) costMax[t] = 0;
    uint32_t mx = 0;
    for (uint32_t k = 0; k < (uint32_t)NT / 64u; ++k) mx = max(mx, wmax[k]);
    const float scale = (float)kUoBuckets / (float)(mx + 1u);  // bucket 0 = the longest walks
    auto bucket = [&](uint32_t c) { return (kUoBuckets - 1u) - min(kUoBuckets - 1u, (uint32_t)((float)c * scale)); };
    for (uint32_t b0 = 0; b0 < n; b0 += (uint32_t)NT * UN) {
        uint32_t c[UN];
        load(b0, c);
#pragma unroll
        for (uint32_t k = 0; k < UN; ++k)
            if (b0 + k * (uint32_t)NT + t < n) atomicAdd(&base[bucket(c[k])], 1u);
    }
    __syncthreads();
    if (w == 0) {
        const uint4 c = *(const uint4*)(base + lane * 4u);
        const uint32_t local = c.x + c.y + c.z + c.w;
        const uint32_t inc = wave_scan_incl(local);
        const uint32_t e = inc - local;
        const uint4 starts = make_uint4(e, e + c.x, e + c.x + c.y, e + c.x + c.y + c.z);
        *(uint4*)(base + lane * 4u) = starts;
        // the pair walk's split: the units of buckets [0, splitBucket) -- the longest walks -- run alone.
        // Taken here, from the lane that owns bucket splitBucket's start, before the ordering loop below
        // advances base[] (read after the barrier it raced with other waves' atomics).
        if (splitBucket) {
            if (splitBucket >= kUoBuckets) {
                if (lane == 0) costMax[kCostMaxSlots] = n;
            } else if (lane == splitBucket / 4u) {
                const uint32_t q = splitBucket & 3u;
                costMax[kCostMaxSlots] = q == 0 ? starts.x : q == 1 ? starts.y : q == 2 ? starts.z : starts.w;
            }
        }
    }
    __syncthreads();

    for (uint32_t b0 = 0; b0 < n; b0 += (uint32_t)NT * UN) {
        uint32_t c[UN];
        load(b0, c);
#pragma unroll
        for (uint32_t k = 0; k < UN; ++k) {
            const uint32_t i = b0 + k * (uint32_t)NT + t;
            if (i < n) {
                const uint32_t pos = atomicAdd(&base[bucket(c[k])], 1u);
                if (pos < n) order[pos] = i;
            }
        }
    }
}

}  // namespace gsm
