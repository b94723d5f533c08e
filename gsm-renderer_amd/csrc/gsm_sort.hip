// gsm_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs for gfx950.
//
// Replaces the reference's 5-kernel-per-digit Metal radix sort
// (RadixSortEncoder.swift:41-214, GlobalShaders.metal:768-1028) with a
// reduce-then-scan design for wave64:
//   upsweep   : per-block 256-bin digit histogram (wave-aggregated LDS counters)
//   scan      : one workgroup per digit scans its column over blocks
//   downsweep : per 2048-key chunk, wave64 ballot-match ranking (8 ballots), LDS
//               staging in digit order, coalesced run writes
// The element count is read on the device (no host round trip, graph-capturable);
// every block owns a contiguous range, so the sort is stable like the reference's.
#include <hip/hip_runtime.h>

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

// 64-bit mask of the active lanes whose 8-bit digit equals this lane's.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        const bool set = (d >> bit) & 1u;
        const uint64_t m = __ballot(set);
        peers &= set ? m : ~m;
    }
    return peers;
}

__global__ __launch_bounds__(kRadixBlock) void k_radix_upsweep(const uint32_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ nPtr,
                                                               uint32_t shift,
                                                               uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[kWaves][256];
    const uint32_t wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * 256; i += kRadixBlock) (&cnt[0][0])[i] = 0;
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
                if (idx + (uint32_t)c < end) atomicAdd(&cnt[wave][(kk[c] >> shift) & 0xFFu], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < 256; d += kRadixBlock) {
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

__global__ __launch_bounds__(kRadixBlock) void k_radix_downsweep(
    const uint32_t* __restrict__ keysIn, const uint32_t* __restrict__ valsIn,
    uint32_t* __restrict__ keysOut, uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ nPtr,
    uint32_t shift, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ binTotals) {
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
        const uint32_t t = binTotals[tid];
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
        binBase[tid] = off + inc - t + hist[(size_t)tid * gridDim.x + blockIdx.x];
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
            const uint32_t d = (k[j] >> shift) & 0xFFu;
            const uint64_t peers = match_digit(d, valid);
            const uint32_t before = valid ? waveCnt[wave][d] : 0u;
            rank[j] = before + (uint32_t)__popcll(peers & lt);
            if (valid && (peers & lt) == 0) waveCnt[wave][d] = before + (uint32_t)__popcll(peers);
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
                const uint32_t d = (k[j] >> shift) & 0xFFu;
                const uint32_t pos = localStart[d] + waveCnt[wave][d] + rank[j];
                sKeys[pos] = k[j];
                sVals[pos] = v[j];
            }
        }
        __syncthreads();
        const uint32_t cn = min((uint32_t)kRadixChunk, end - cbase);
        for (uint32_t p = tid; p < cn; p += kRadixBlock) {
            const uint32_t key = sKeys[p];
            const uint32_t d = (key >> shift) & 0xFFu;
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

uint32_t radix_grid_for_capacity(uint32_t capacity) {
    // <= 1024 blocks: k_radix_scan holds a digit's column in 4 registers per thread
    uint32_t g = (capacity + kRadixChunk - 1) / kRadixChunk;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    return g;
}

int radix_sort_pairs(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                     int firstDigit, int numDigits, uint32_t* hist, uint32_t* binTotals,
                     hipStream_t s) {
    const uint32_t grid = radix_grid_for_capacity(capacity);
    int cur = 0;
    for (int dgt = firstDigit; dgt < firstDigit + numDigits; ++dgt) {
        const uint32_t shift = (uint32_t)dgt * 8u;
        hipLaunchKernelGGL(k_radix_upsweep, dim3(grid), dim3(kRadixBlock), 0, s, keys[cur], nPtr,
                           shift, hist);
        hipLaunchKernelGGL(k_radix_scan, dim3(256), dim3(256), 0, s, hist, grid, binTotals);
        hipLaunchKernelGGL(k_radix_downsweep, dim3(grid), dim3(kRadixBlock), 0, s, keys[cur],
                           vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, shift, hist, binTotals);
        cur ^= 1;
    }
    return cur;
}

}  // namespace gsm

namespace gsm {

// ---------------------------------------------------------------------------
// Frame sort, second half: after the tile-digit passes the keys are grouped by tile, each
// tile's run in assignment order; one workgroup per tile then sorts its run stably by the
// 16-bit depth key.  Stable by construction: the LDS path sorts (depth << 16 | position)
// with a bitonic network; runs longer than the LDS capacity take two LSD byte passes over
// global memory within the workgroup.  The result equals the reference's 4-pass LSD sort of
// (tile << 16 | depth) keys (SURVEY.md 8(a) determinism contract).
// ---------------------------------------------------------------------------
constexpr uint32_t kSegThreads = 256;
constexpr uint32_t kSegCap = 8192;  // entries per tile sorted in LDS (32 KiB)

__device__ void seg_radix_pass(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                               uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint32_t n,
                               uint32_t shift, uint32_t* hist, uint32_t* wcnt) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t i = tid; i < 256; i += kSegThreads) hist[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kSegThreads) atomicAdd(&hist[(kin[i] >> shift) & 0xFFu], 1u);
    __syncthreads();
    if (tid == 0) {  // exclusive scan of the 256 digit counts
        uint32_t run = 0;
        for (int d = 0; d < 256; ++d) {
            const uint32_t c = hist[d];
            hist[d] = run;
            run += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t base = 0; base < n; base += kSegThreads) {  // chunks in order: stable
        const uint32_t i = base + tid;
        const bool valid = i < n;
        const uint32_t k = valid ? kin[i] : 0u, v = valid ? vin[i] : 0u;
        const uint32_t d = (k >> shift) & 0xFFu;
        const uint64_t peers = match_digit(d, valid);
        for (uint32_t j = tid; j < 4 * 256; j += kSegThreads) wcnt[j] = 0;
        __syncthreads();
        if (valid && (peers & lt) == 0) wcnt[wave * 256 + d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t before = 0;
            for (uint32_t w = 0; w < wave; ++w) before += wcnt[w * 256 + d];
            const uint32_t pos = hist[d] + before + (uint32_t)__popcll(peers & lt);
            kout[pos] = k;
            vout[pos] = v;
        }
        __syncthreads();
        for (uint32_t j = tid; j < 256; j += kSegThreads)
            hist[j] += wcnt[j] + wcnt[256 + j] + wcnt[512 + j] + wcnt[768 + j];
        __syncthreads();
    }
}

__global__ __launch_bounds__(kSegThreads) void k_tile_depth_sort(
    uint32_t* __restrict__ keysIn, uint32_t* __restrict__ valsIn, uint32_t* __restrict__ keysOut,
    uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ tileStart, uint32_t tileBegin) {
    __shared__ uint32_t sk[kSegCap];
    const uint32_t t = tileBegin + blockIdx.x;
    const uint32_t start = tileStart[t];
    const uint32_t n = tileStart[t + 1] - start;
    if (n == 0) return;
    const uint32_t tid = threadIdx.x;
    uint32_t* kin = keysIn + start;
    uint32_t* vin = valsIn + start;
    uint32_t* kout = keysOut + start;
    uint32_t* vout = valsOut + start;
    if (n <= kSegCap) {
        uint32_t np = 1;
        while (np < n) np <<= 1;
        for (uint32_t i = tid; i < np; i += kSegThreads)
            sk[i] = i < n ? ((kin[i] & 0xFFFFu) << 16) | i : 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t k = 2; k <= np; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < np; i += kSegThreads) {
                    const uint32_t ixj = i ^ j;
                    if (ixj > i) {
                        const uint32_t a = sk[i], b = sk[ixj];
                        if ((a > b) == ((i & k) == 0)) {
                            sk[i] = b;
                            sk[ixj] = a;
                        }
                    }
                }
                __syncthreads();
            }
        const uint32_t tileBits = t << 16;
        for (uint32_t i = tid; i < n; i += kSegThreads) {
            const uint32_t c = sk[i];
            kout[i] = tileBits | (c >> 16);
            vout[i] = vin[c & 0xFFFFu];
        }
    } else {  // long run: low then high depth byte through global memory, then back to out
        uint32_t* hist = sk;
        uint32_t* wcnt = sk + 256;
        seg_radix_pass(kin, vin, kout, vout, n, 0, hist, wcnt);
        __syncthreads();
        seg_radix_pass(kout, vout, kin, vin, n, 8, hist, wcnt);
        __syncthreads();
        for (uint32_t i = tid; i < n; i += kSegThreads) {
            kout[i] = kin[i];
            vout[i] = vin[i];
        }
    }
}

void tile_depth_sort(uint32_t* keysIn, uint32_t* valsIn, uint32_t* keysOut, uint32_t* valsOut,
                     const uint32_t* tileStart, uint32_t tileBegin, uint32_t numTiles, hipStream_t s) {
    if (numTiles == 0) return;
    hipLaunchKernelGGL(k_tile_depth_sort, dim3(numTiles), dim3(kSegThreads), 0, s, keysIn, valsIn, keysOut,
                       valsOut, tileStart, tileBegin);
}

}  // namespace gsm
