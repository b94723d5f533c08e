// gsm_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs for gfx950, and the
// frame sort built from it.
//
// Replaces the reference's 5-kernel-per-digit Metal radix sort
// (RadixSortEncoder.swift:41-214, GlobalShaders.metal:768-1028) with a
// reduce-then-scan design for wave64, digits of BITS <= 8 bits:
//   upsweep   : per-block 2^BITS-bin digit histogram (wave-aggregated LDS counters)
//   scan      : one workgroup per digit scans its column over blocks
//   downsweep : per 4096-key chunk, wave64 ballot-match ranking (BITS ballots), LDS
//               staging in digit order, coalesced run writes
// The element count is read on the device (no host round trip, graph-capturable);
// every block owns a contiguous range, so the sort is stable like the reference's.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "gsm_internal.h"

namespace gsm {

constexpr int kWaves = kRadixBlock / 64;

__device__ __forceinline__ void block_range(uint32_t n, uint32_t grid, uint32_t b, uint32_t* begin,
                                            uint32_t* end) {
    uint32_t per = (n + grid - 1) / grid;
    per = (per + kRadixChunk - 1) / kRadixChunk * kRadixChunk;
    uint64_t bb = (uint64_t)per * b;
    uint64_t ee = bb + per;
    if (bb > n) bb = n;
    if (ee > n) ee = n;
    *begin = (uint32_t)bb;
    *end = (uint32_t)ee;
}

// 64-bit mask of the active lanes whose BITS-bit digit equals this lane's.
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < BITS; ++bit) {
        const bool set = (d >> bit) & 1u;
        const uint64_t m = __ballot(set);
        peers &= set ? m : ~m;
    }
    return peers;
}

// Stable rank of a lane's digit among the earlier lanes of its wave with the same digit, from
// one LDS atomic: gfx950 serves the lanes of one ds_add_rtn_u32 that hit the same address in
// lane order (tools/exp/lds_atomic_order.hip: 15M same-address lane pairs, every one in lane
// order; the GPU parity tests re-check the sorts bit for bit).  Returns the counter's old value;
// the counter ends at the count.  kBallotRank selects the ballot-match form instead (8 ballots
// per digit) for A/B measurement.
constexpr bool kBallotRank = false;
template <int BITS>
__device__ __forceinline__ uint32_t wave_rank(uint32_t* cnt, uint32_t d, bool valid, uint64_t lt) {
    if constexpr (kBallotRank) {
        const uint64_t peers = match_digit<BITS>(d, valid);
        const uint32_t before = cnt[d];
        if (valid && (peers & lt) == 0) cnt[d] = before + (uint32_t)__popcll(peers);
        return before + (uint32_t)__popcll(peers & lt);
    } else {
        uint32_t r = 0;
        if (valid) r = atomicAdd(&cnt[d], 1u);
        return r;
    }
}

template <int BITS>
__global__ __launch_bounds__(kRadixBlock) void k_radix_upsweep(const uint32_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ nPtr,
                                                               uint32_t shift,
                                                               uint32_t* __restrict__ hist) {
    constexpr uint32_t R = 1u << BITS;
    __shared__ uint32_t cnt[kWaves][R];
    const uint32_t wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * (int)R; i += kRadixBlock) (&cnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t begin, end;
    block_range(*nPtr, gridDim.x, blockIdx.x, &begin, &end);
    // a chunk's keys are all loaded before any is counted (16 loads in flight per thread);
    // order does not matter for a histogram, so they come as 16-byte vectors
    for (uint32_t cbase = begin; cbase < end; cbase += kRadixChunk) {
        uint4 q[kRadixItems / 4];
#pragma unroll
        for (int i = 0; i < kRadixItems / 4; ++i) {
            const uint32_t idx = cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u;
            q[i] = idx + 3u < end ? *(const uint4*)(keys + idx)
                                  : make_uint4(idx < end ? keys[idx] : 0u, idx + 1u < end ? keys[idx + 1u] : 0u,
                                               idx + 2u < end ? keys[idx + 2u] : 0u, 0u);
        }
#pragma unroll
        for (int i = 0; i < kRadixItems / 4; ++i) {
            const uint32_t idx = cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u;
            const uint32_t kk[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)  // per-wave LDS counters: one ds_add per key
                if (idx + (uint32_t)c < end) atomicAdd(&cnt[wave][(kk[c] >> shift) & (R - 1u)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += kRadixBlock) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += cnt[w][d];
        hist[(size_t)d * gridDim.x + blockIdx.x] = s;
    }
}

// One workgroup per digit: exclusive scan of hist[d][0..grid) in place, digit total out.
// grid <= 1024, so every thread holds at most 4 entries in registers (one read, one write).
__global__ __launch_bounds__(256) void k_radix_scan(uint32_t* __restrict__ hist, uint32_t grid,
                                                    uint32_t* __restrict__ binTotals) {
    __shared__ uint32_t part[4];
    const uint32_t d = blockIdx.x;
    uint32_t* row = hist + (size_t)d * grid;
    const uint32_t b0 = threadIdx.x * 4u;
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = b0 + i < grid ? row[b0 + i] : 0u;
    const uint32_t local = v[0] + v[1] + v[2] + v[3];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if ((uint32_t)w < wave) off += part[w];
        tot += part[w];
    }
    uint32_t run = off + inc - local;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (b0 + i < grid) {
            row[b0 + i] = run;
            run += v[i];
        }
    if (threadIdx.x == 0) binTotals[d] = tot;
}

// Digits >= 2^BITS do not exist: their counters stay 0 (thread tid owns digit tid of 256).
template <int BITS>
__global__ __launch_bounds__(kRadixBlock) void k_radix_downsweep(
    const uint32_t* __restrict__ keysIn, const uint32_t* __restrict__ valsIn,
    uint32_t* __restrict__ keysOut, uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ nPtr,
    uint32_t shift, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ binTotals) {
    constexpr uint32_t R = 1u << BITS;
    __shared__ uint32_t binBase[256];
    __shared__ uint32_t localStart[256];
    __shared__ uint32_t chunkTotal[256];
    __shared__ uint32_t waveCnt[kWaves][256];
    __shared__ uint32_t sKeys[kRadixChunk];
    __shared__ uint32_t sVals[kRadixChunk];
    __shared__ uint32_t part[kWaves];

    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = *nPtr;
    uint32_t begin, end;
    block_range(n, gridDim.x, blockIdx.x, &begin, &end);
    if (begin >= end) return;

    // global base of every digit for this block: exclusive scan over digits + block column offset
    {
        const uint32_t t = tid < R ? binTotals[tid] : 0u;
        uint32_t inc = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t v = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += v;
        }
        if (lane == 63) part[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w)
            if ((uint32_t)w < wave) off += part[w];
        binBase[tid] = off + inc - t + (tid < R ? hist[(size_t)tid * gridDim.x + blockIdx.x] : 0u);
#pragma unroll
        for (int w = 0; w < kWaves; ++w) waveCnt[w][tid] = 0;
        __syncthreads();
    }

    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t cbase = begin; cbase < end; cbase += kRadixChunk) {
        uint32_t k[kRadixItems], v[kRadixItems], rank[kRadixItems];
        // wave w owns elements [cbase + w*64*items, +64*items): item j at + j*64 + lane (index order)
#pragma unroll
        for (int j = 0; j < kRadixItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
            const bool valid = idx < end;
            k[j] = valid ? keysIn[idx] : 0xFFFFFFFFu;
            v[j] = valid ? valsIn[idx] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kRadixItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
            const bool valid = idx < end;
            const uint32_t d = (k[j] >> shift) & (R - 1u);
            rank[j] = wave_rank<BITS>(waveCnt[wave], d, valid, lt);
        }
        __syncthreads();
        // per digit: offsets of each wave, chunk total, then exclusive scan over digits
        {
            uint32_t tot = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t c = waveCnt[w][tid];
                waveCnt[w][tid] = tot;
                tot += c;
            }
            chunkTotal[tid] = tot;
            uint32_t inc = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                uint32_t x = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += x;
            }
            if (lane == 63) part[wave] = inc;
            __syncthreads();
            uint32_t off = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w)
                if ((uint32_t)w < wave) off += part[w];
            localStart[tid] = off + inc - tot;
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < kRadixItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
            if (idx < end) {
                const uint32_t d = (k[j] >> shift) & (R - 1u);
                const uint32_t pos = localStart[d] + waveCnt[wave][d] + rank[j];
                sKeys[pos] = k[j];
                sVals[pos] = v[j];
            }
        }
        __syncthreads();
        const uint32_t cn = min((uint32_t)kRadixChunk, end - cbase);
        for (uint32_t p = tid; p < cn; p += kRadixBlock) {
            const uint32_t key = sKeys[p];
            const uint32_t d = (key >> shift) & (R - 1u);
            const uint32_t dst = binBase[d] + (p - localStart[d]);
            keysOut[dst] = key;
            valsOut[dst] = sVals[p];
        }
        __syncthreads();
        binBase[tid] += chunkTotal[tid];
#pragma unroll
        for (int w = 0; w < kWaves; ++w) waveCnt[w][tid] = 0;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Onesweep variant (opt-in, GSM_RADIX=onesweep; slower here, see onesweep_enabled): one
// histogram kernel for every pass of the sort, then ONE kernel per pass (instead of upsweep +
// scan + downsweep).  A pass's workgroups take 4096-key partitions in
// dispatch order from a counter, rank their chunk exactly as k_radix_downsweep does, publish
// the chunk's per-digit counts, and find the counts of all earlier partitions by decoupled
// look-back over the published words -- a workgroup only ever waits on partitions taken before
// its own, by workgroups already running, so the chain always drains.  Same stable order as
// the reduce-then-scan passes (contiguous partitions in index order, list order inside).
//
// Workspace (after the classic hist region of the same buffer, zeroed at allocation):
//   2 regions x { u32 hist[4][256]; u32 counter[4] }   -- region = sort parity, the histogram
//                                                        kernel zeroes the other region
//   u64 status[parts][256]: epoch << 32 | flag << 30 | count (flag 1 aggregate, 2 prefix); a
//   word of an older pass has another epoch, so the status never needs clearing.
// ---------------------------------------------------------------------------
constexpr uint32_t kOsRegionWords = 4 * 256 + 4;
constexpr uint32_t kOsClassicGrid = 1024;  // the classic hist region at its largest grid: one layout for all capacities
constexpr uint64_t kOsSpinLimit = 1ull << 24;
constexpr int kOsLook = 16;  // look-back window  // a broken chain ends the kernel, not the GPU

struct OsPasses {
    uint32_t shift[4];
    uint32_t bits[4];
    uint32_t passes;
};

__global__ __launch_bounds__(256) void k_os_hist(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ nPtr,
                                                 OsPasses P, uint32_t* __restrict__ region,
                                                 uint32_t* __restrict__ other) {
    __shared__ uint32_t cnt[4][256];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) (&cnt[0][0])[i] = 0;
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < (int)kOsRegionWords; i += 256) other[i] = 0;  // next sort's region
    __syncthreads();
    const uint32_t n = *nPtr;
    const uint32_t nv = n >> 2;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i <= nv; i += gridDim.x * 256) {
        uint32_t kk[4];
        uint32_t m = 0;
        if (i < nv) {
            const uint4 q = ((const uint4*)keys)[i];
            kk[0] = q.x; kk[1] = q.y; kk[2] = q.z; kk[3] = q.w;
            m = 4;
        } else {  // the n % 4 tail
            for (uint32_t c = 0; c < (n & 3u); ++c) kk[c] = keys[(nv << 2) + c];
            m = n & 3u;
        }
        for (uint32_t c = 0; c < m; ++c)
            for (uint32_t p = 0; p < P.passes; ++p)
                atomicAdd(&cnt[p][(kk[c] >> P.shift[p]) & ((1u << P.bits[p]) - 1u)], 1u);
    }
    __syncthreads();
    for (uint32_t p = 0; p < P.passes; ++p) {
        const uint32_t c = cnt[p][threadIdx.x];
        if (c) atomicAdd(&region[p * 256 + threadIdx.x], c);
    }
}

template <int BITS>
__global__ __launch_bounds__(kRadixBlock) void k_onesweep(
    const uint32_t* __restrict__ keysIn, const uint32_t* __restrict__ valsIn,
    uint32_t* __restrict__ keysOut, uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ nPtr,
    uint32_t shift, const uint32_t* __restrict__ histPass, uint32_t* __restrict__ counter,
    unsigned long long* __restrict__ status, uint32_t epoch) {
    constexpr uint32_t R = 1u << BITS;
    __shared__ uint32_t binBase[256];
    __shared__ uint32_t localStart[256];
    __shared__ uint32_t chunkTotal[256];
    __shared__ uint32_t waveCnt[kWaves][256];
    __shared__ uint32_t sKeys[kRadixChunk];
    __shared__ uint32_t sVals[kRadixChunk];
    __shared__ uint32_t part[kWaves];
    __shared__ uint32_t sPart;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) sPart = atomicAdd(counter, 1u);
#pragma unroll
    for (int w = 0; w < kWaves; ++w) waveCnt[w][tid] = 0;
    __syncthreads();
    const uint32_t pid = sPart;
    const uint32_t n = *nPtr;
    const uint32_t cbase = pid * (uint32_t)kRadixChunk;
    if (cbase >= n) return;  // uniform: more workgroups than partitions
    const uint32_t end = min(n, cbase + (uint32_t)kRadixChunk);

    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t k[kRadixItems], v[kRadixItems], rank[kRadixItems];
#pragma unroll
    for (int j = 0; j < kRadixItems; ++j) {
        const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
        const bool valid = idx < end;
        k[j] = valid ? keysIn[idx] : 0xFFFFFFFFu;
        v[j] = valid ? valsIn[idx] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kRadixItems; ++j) {
        const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
        const bool valid = idx < end;
        const uint32_t d = (k[j] >> shift) & (R - 1u);
        rank[j] = wave_rank<BITS>(waveCnt[wave], d, valid, lt);
    }
    __syncthreads();
    // per digit: wave offsets and the chunk total; publish the total before the scans
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t c = waveCnt[w][tid];
        waveCnt[w][tid] = tot;
        tot += c;
    }
    chunkTotal[tid] = tot;
    unsigned long long* st = status + (size_t)pid * 256u;
    const unsigned long long ep = (unsigned long long)epoch << 32;
    if (tid < R)
        __hip_atomic_store(&st[tid], ep | ((pid == 0 ? 2ull : 1ull) << 30) | tot, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // exclusive scan over digits: of the chunk totals (LDS positions) and of the pass histogram
    const uint32_t g = tid < R ? histPass[tid] : 0u;
    uint32_t inc = tot, incg = g;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(inc, o, 64), y = __shfl_up(incg, o, 64);
        if (lane >= (uint32_t)o) {
            inc += x;
            incg += y;
        }
    }
    __shared__ uint32_t partG[kWaves];
    if (lane == 63) {
        part[wave] = inc;
        partG[wave] = incg;
    }
    // decoupled look-back: counts of this digit in every earlier partition
    uint32_t excl = 0;
    if (tid < R && pid > 0) {
        // kOsLook predecessors' words per round trip (independent loads), nearest first
        uint32_t q = pid;  // partitions [0, q) not yet examined
        uint64_t spins = 0;
        bool fin = false;
        while (!fin) {
            unsigned long long w[kOsLook];
#pragma unroll
            for (int i = 0; i < kOsLook; ++i) {
                const uint32_t qi = q > (uint32_t)i ? q - 1u - (uint32_t)i : 0u;
                w[i] = __hip_atomic_load(&status[(size_t)qi * 256u + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int i = 0; i < kOsLook; ++i) {
                if (fin) break;
                const uint32_t qi = q - 1u - (uint32_t)i;  // q > i: partition 0 always ends the walk
                unsigned long long x = w[i];
                while (((x >> 32) != (unsigned long long)epoch || ((x >> 30) & 3u) == 0) && spins <= kOsSpinLimit) {
                    ++spins;
                    __builtin_amdgcn_s_sleep(1);
                    x = __hip_atomic_load(&status[(size_t)qi * 256u + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                excl += (uint32_t)x & 0x3FFFFFFFu;
                if (((x >> 30) & 3u) == 2u || qi == 0u || spins > kOsSpinLimit) fin = true;
            }
            q -= kOsLook;
        }
        __hip_atomic_store(&st[tid], ep | (2ull << 30) | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    {
        uint32_t off = 0, offg = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w)
            if ((uint32_t)w < wave) {
                off += part[w];
                offg += partG[w];
            }
        localStart[tid] = off + inc - tot;
        binBase[tid] = offg + incg - g + excl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRadixItems; ++j) {
        const uint32_t idx = cbase + wave * (64 * kRadixItems) + j * 64 + lane;
        if (idx < end) {
            const uint32_t d = (k[j] >> shift) & (R - 1u);
            const uint32_t pos = localStart[d] + waveCnt[wave][d] + rank[j];
            sKeys[pos] = k[j];
            sVals[pos] = v[j];
        }
    }
    __syncthreads();
    const uint32_t cn = end - cbase;
    for (uint32_t p = tid; p < cn; p += kRadixBlock) {
        const uint32_t key = sKeys[p];
        const uint32_t d = (key >> shift) & (R - 1u);
        const uint32_t dst = binBase[d] + (p - localStart[d]);
        keysOut[dst] = key;
        valsOut[dst] = sVals[p];
    }
}

size_t radix_workspace_bytes(uint32_t capacity) {
    const size_t classic = (size_t)256 * kOsClassicGrid * sizeof(uint32_t);
    const size_t parts = ((size_t)capacity + kRadixChunk - 1) / kRadixChunk + 1;
    return classic + 2 * kOsRegionWords * sizeof(uint32_t) + 64 + parts * 256 * sizeof(unsigned long long);
}

namespace {
std::mutex gOsMutex;
std::unordered_map<const void*, uint32_t> gOsParity;  // per workspace: the region of its next sort
uint32_t gOsEpoch = 0;                                 // per pass, process-wide, never 0
// Opt-in (GSM_RADIX=onesweep), measured slower on MI355X: the look-back words need device-scope
// (cross-XCD) loads, and the prefix frontier advances one window (kOsLook partitions) per round
// trip, so a pass costs ~parts / kOsLook round trips -- config 5 tile sort 94 us per pass against
// 35 us for upsweep + scan + downsweep.
bool onesweep_enabled() {
    const char* v = getenv("GSM_RADIX");
    return v && v[0] == 'o';
}
}  // namespace

// Sort passes (shift, bits) over a workspace; returns the ping-pong index of the result.
static int onesweep_sort(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                         const OsPasses& P, uint32_t* work, hipStream_t s) {
    uint32_t parity, epoch0;
    {
        std::lock_guard<std::mutex> lk(gOsMutex);
        parity = gOsParity[work];
        gOsParity[work] = parity ^ 1u;
        if (gOsEpoch > 0xFFFFFFF0u) gOsEpoch = 0;
        epoch0 = gOsEpoch + 1;
        gOsEpoch += P.passes;
    }
    uint32_t* base = work + (size_t)256 * kOsClassicGrid;
    uint32_t* region = base + parity * kOsRegionWords;
    uint32_t* other = base + (parity ^ 1u) * kOsRegionWords;
    unsigned long long* status =
        (unsigned long long*)(((uintptr_t)(base + 2 * kOsRegionWords) + 63) & ~(uintptr_t)63);
    uint32_t hgrid = (capacity / 4u + 255u) / 256u;
    if (hgrid > 1024u) hgrid = 1024u;
    if (hgrid < 1u) hgrid = 1u;
    hipLaunchKernelGGL(k_os_hist, dim3(hgrid), dim3(256), 0, s, keys[0], nPtr, P, region, other);
    const uint32_t grid = (capacity + kRadixChunk - 1) / kRadixChunk;
    int cur = 0;
    for (uint32_t p = 0; p < P.passes; ++p) {
        uint32_t* hp = region + p * 256;
        uint32_t* ctr = region + 4 * 256 + p;
#define GSM_OS_PASS(B)                                                                                        \
    hipLaunchKernelGGL(k_onesweep<B>, dim3(grid > 0 ? grid : 1), dim3(kRadixBlock), 0, s, keys[cur], vals[cur], \
                       keys[cur ^ 1], vals[cur ^ 1], nPtr, P.shift[p], hp, ctr, status, epoch0 + p)
        switch (P.bits[p]) {
            case 4: GSM_OS_PASS(4); break;
            case 5: GSM_OS_PASS(5); break;
            case 6: GSM_OS_PASS(6); break;
            case 7: GSM_OS_PASS(7); break;
            default: GSM_OS_PASS(8); break;
        }
#undef GSM_OS_PASS
        cur ^= 1;
    }
    return cur;
}

uint32_t radix_grid_for_capacity(uint32_t capacity) {
    // <= 1024 blocks: k_radix_scan holds a digit's column in 4 registers per thread
    uint32_t g = (capacity + kRadixChunk - 1) / kRadixChunk;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    return g;
}

static void radix_pass(uint32_t* kin, uint32_t* vin, uint32_t* kout, uint32_t* vout, const uint32_t* nPtr,
                       uint32_t grid, uint32_t shift, int bits, uint32_t* hist, uint32_t* binTotals,
                       hipStream_t s) {
#define GSM_RADIX_PASS(B)                                                                                   \
    hipLaunchKernelGGL(k_radix_upsweep<B>, dim3(grid), dim3(kRadixBlock), 0, s, kin, nPtr, shift, hist);    \
    hipLaunchKernelGGL(k_radix_scan, dim3(1u << B), dim3(256), 0, s, hist, grid, binTotals);               \
    hipLaunchKernelGGL(k_radix_downsweep<B>, dim3(grid), dim3(kRadixBlock), 0, s, kin, vin, kout, vout, nPtr, \
                       shift, hist, binTotals)
    switch (bits) {
        case 4: GSM_RADIX_PASS(4); break;
        case 5: GSM_RADIX_PASS(5); break;
        case 6: GSM_RADIX_PASS(6); break;
        case 7: GSM_RADIX_PASS(7); break;
        default: GSM_RADIX_PASS(8); break;
    }
#undef GSM_RADIX_PASS
}

int radix_sort_pairs(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                     int firstDigit, int numDigits, uint32_t* hist, uint32_t* binTotals,
                     hipStream_t s) {
    if (onesweep_enabled() && numDigits >= 1 && numDigits <= 4) {
        OsPasses P{};
        P.passes = (uint32_t)numDigits;
        for (int i = 0; i < numDigits; ++i) {
            P.shift[i] = (uint32_t)(firstDigit + i) * 8u;
            P.bits[i] = 8;
        }
        return onesweep_sort(keys, vals, nPtr, capacity, P, hist, s);
    }
    const uint32_t grid = radix_grid_for_capacity(capacity);
    int cur = 0;
    for (int dgt = firstDigit; dgt < firstDigit + numDigits; ++dgt) {
        radix_pass(keys[cur], vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, grid, (uint32_t)dgt * 8u, 8, hist,
                   binTotals, s);
        cur ^= 1;
    }
    return cur;
}

int radix_sort_bits(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                    uint32_t shift, uint32_t bits, uint32_t* hist, uint32_t* binTotals, hipStream_t s) {
    const uint32_t grid = radix_grid_for_capacity(capacity);
    const uint32_t passes = (bits + 7) / 8;
    if (onesweep_enabled() && passes >= 1 && passes <= 4) {
        OsPasses P{};
        P.passes = passes;
        uint32_t dn = 0;
        for (uint32_t p = 0; p < passes; ++p) {  // the digit widths of the loop below
            uint32_t b = (bits - dn + (passes - p) - 1) / (passes - p);
            if (b < 4) b = 4;
            P.shift[p] = shift + dn;
            P.bits[p] = b;
            dn += b;
        }
        return onesweep_sort(keys, vals, nPtr, capacity, P, hist, s);
    }
    int cur = 0;
    uint32_t done = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        // near-equal digit widths; a digit wider than the bits left reads zero bits above the field
        uint32_t b = (bits - done + (passes - p) - 1) / (passes - p);
        if (b < 4) b = 4;
        radix_pass(keys[cur], vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, grid, shift + done, (int)b, hist,
                   binTotals, s);
        done += b;
        cur ^= 1;
    }
    return cur;
}

}  // namespace gsm

namespace gsm {

// ---------------------------------------------------------------------------
// Frame sort, second half.  After the tile-digit passes the assignments are grouped by tile,
// each tile's run in assignment order (ascending gaussian id, SURVEY.md 8(a) determinism
// contract); sorting every run stably by its 16-bit depth key then gives exactly the
// reference's 4-pass LSD order of (tile << 16 | depth) keys (RadixSortEncoder.swift:41-101).
//
// k_tile_sort: one workgroup per tile, runs of up to kTsCap entries held 8 per thread.  Two
// 8-bit LSD passes over the depth key.  Wave w owns a contiguous segment of the run and ranks
// its items in order against per-wave LDS digit counters (ballot match, no barrier inside the
// segment); one scan over (digit, wave) then turns the local ranks into positions -- the
// downsweep of the global sort with a single chunk, so the order is stable.  Pass 1 scatters
// (depth << 16 | position-in-run) words into LDS; pass 2 scatters the rebuilt keys and the
// values gathered by the position field into the output run.  Longer runs (rare) take the
// same passes through global memory in chunks of 256.
constexpr uint32_t kTsThreads = 256;
constexpr uint32_t kTsItems = 8;
constexpr uint32_t kTsCap = kTsThreads * kTsItems;  // 2048 entries per tile in LDS

// Lanes of one wave hand LDS words to each other below.  The hardware keeps a wave's LDS
// operations in order, but the language does not: without this (no instruction) the compiler
// may forward a lane's own earlier store past another lane's update.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Thread tid owns digit tid: exclusive scan over (digit, wave) of the counts in wcnt, in place.
__device__ __forceinline__ void ts_offsets(uint32_t (*wcnt)[256], uint32_t* part) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t c0 = wcnt[0][tid], c1 = wcnt[1][tid], c2 = wcnt[2][tid], c3 = wcnt[3][tid];
    const uint32_t tot = c0 + c1 + c2 + c3;
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w)
        if (w < wave) off += part[w];
    const uint32_t e = off + inc - tot;
    wcnt[0][tid] = e;
    wcnt[1][tid] = e + c0;
    wcnt[2][tid] = e + c0 + c1;
    wcnt[3][tid] = e + c0 + c1 + c2;
    __syncthreads();
}

// one pass: pos[j] = destination of item j (items of wave w at seg + j*64 + lane)
__device__ __forceinline__ void ts_rank_pass(const uint32_t (&x)[kTsItems], uint32_t (&pos)[kTsItems], uint32_t E,
                                             uint32_t seg, uint32_t n, uint32_t shift, uint32_t (*wcnt)[256],
                                             uint32_t* part) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t* cnt = wcnt[wave];
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        if (j < E) {
            const bool valid = seg + j * 64u + lane < n;
            const uint32_t d = (x[j] >> shift) & 0xFFu;
            pos[j] = wave_rank<8>(cnt, d, valid, lt);
            wave_sync();
        }
    }
    __syncthreads();
    ts_offsets(wcnt, part);
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j)
        if (j < E) pos[j] += cnt[(x[j] >> shift) & 0xFFu];
}

// one stable 8-bit LSD pass of a run of n (key, value) pairs by the workgroup, in -> out (global)
__device__ void ts_pass_global(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                               uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint32_t n,
                               uint32_t shift, uint32_t (*wcnt)[256], uint32_t* part, uint32_t* carry) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // digit starts over the whole run
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kTsThreads) atomicAdd(&wcnt[0][(kin[i] >> shift) & 0xFFu], 1u);
    __syncthreads();
    ts_offsets(wcnt, part);
    carry[tid] = wcnt[0][tid];
    __syncthreads();
    for (uint32_t b = 0; b < n; b += kTsThreads) {  // chunks of 256 in order: stable
        const uint32_t i = b + tid;
        const bool valid = i < n;
        const uint32_t k = valid ? kin[i] : 0u, v = valid ? vin[i] : 0u;
        const uint32_t d = (k >> shift) & 0xFFu;
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) wcnt[w][tid] = 0;
        __syncthreads();
        const uint32_t r = wave_rank<8>(wcnt[wave], d, valid, lt);
        __syncthreads();
        if (valid) {
            uint32_t before = carry[d];
            for (uint32_t w = 0; w < wave; ++w) before += wcnt[w][d];
            const uint32_t p = before + r;
            kout[p] = k;
            vout[p] = v;
        }
        __syncthreads();
        carry[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
        __syncthreads();
    }
}

__global__ __launch_bounds__(kTsThreads) void k_tile_sort(
    uint32_t* __restrict__ keysIn, uint32_t* __restrict__ valsIn, uint32_t* __restrict__ keysOut,
    uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ tileStart, uint32_t tileBegin) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[kTsCap];
    __shared__ __attribute__((aligned(16))) uint32_t wcnt[4][256];
    __shared__ uint32_t part[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t t = tileBegin + blockIdx.x;
    const uint32_t start = tileStart[t];
    const uint32_t n = tileStart[t + 1] - start;
    if (n == 0) return;  // uniform: the whole workgroup leaves
    if (n > kTsCap) {  // rare: the same two passes streamed through global memory
        ts_pass_global(keysIn + start, valsIn + start, keysOut + start, valsOut + start, n, 0, wcnt, part, buf);
        ts_pass_global(keysOut + start, valsOut + start, keysIn + start, valsIn + start, n, 8, wcnt, part, buf);
        for (uint32_t i = tid; i < n; i += kTsThreads) {
            keysOut[start + i] = keysIn[start + i];
            valsOut[start + i] = valsIn[start + i];
        }
        return;
    }
    const uint32_t* kin = keysIn + start;
    const uint32_t* vin = valsIn + start;
    const uint32_t E = (n + kTsThreads - 1) / kTsThreads;  // items per thread
    const uint32_t seg = wave * 64u * E;                    // this wave's segment of the run
    uint32_t x[kTsItems], pos[kTsItems];
    // all of the run's keys in flight at once; word = depth << 16 | position in the run
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        const uint32_t i = seg + j * 64u + lane;
        x[j] = (j < E && i < n) ? ((kin[i] & 0xFFFFu) << 16) | i : 0u;
    }
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    ts_rank_pass(x, pos, E, seg, n, 16, wcnt, part);  // low depth byte
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j)
        if (j < E && seg + j * 64u + lane < n) buf[pos[j]] = x[j];
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j)
        if (j < E) x[j] = seg + j * 64u + lane < n ? buf[seg + j * 64u + lane] : 0u;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    ts_rank_pass(x, pos, E, seg, n, 24, wcnt, part);  // high depth byte
    uint32_t* kout = keysOut + start;
    uint32_t* vout = valsOut + start;
    const uint32_t tileBits = t << 16;
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        if (j < E && seg + j * 64u + lane < n) {
            kout[pos[j]] = tileBits | (x[j] >> 16);
            vout[pos[j]] = vin[x[j] & 0xFFFFu];
        }
    }
}

void tile_depth_sort(uint32_t* keysIn, uint32_t* valsIn, uint32_t* keysOut, uint32_t* valsOut,
                     const uint32_t* tileStart, uint32_t tileBegin, uint32_t numTiles, hipStream_t s) {
    if (numTiles == 0) return;
    hipLaunchKernelGGL(k_tile_sort, dim3(numTiles), dim3(kTsThreads), 0, s, keysIn, valsIn, keysOut, valsOut,
                       tileStart, tileBegin);
}

}  // namespace gsm
