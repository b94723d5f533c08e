// gsm_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs for gfx950, and the
// frame sort built from it.
//
// Replaces the reference's 5-kernel-per-digit Metal radix sort
// (RadixSortEncoder.swift:41-214, GlobalShaders.metal:768-1028) with a
// reduce-then-scan design for wave64, digits of BITS <= 8 bits:
//   upsweep   : per-block 2^BITS-bin digit histogram (wave-aggregated LDS counters)
//   scan      : one workgroup per digit scans its column over blocks
//   downsweep : per 4096-key chunk, stable wave ranks (wave_rank), LDS staging in digit
//               order, coalesced run writes
// The element count is read on the device (no host round trip, graph-capturable);
// every block owns a contiguous range, so the sort is stable like the reference's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
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
// the counter ends at the count.  BALLOT selects the ballot-match form (BITS ballots per digit),
// which needs no such property: the renderer takes it when the create-time probe
// (sort_lane_ordered_atomics) does not see lane order, or when GSM_SORT_RANK=ballot.
template <int BITS, bool BALLOT>
__device__ __forceinline__ uint32_t wave_rank(uint32_t* cnt, uint32_t d, bool valid, uint64_t lt) {
    if constexpr (BALLOT) {
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

// Scanless narrow passes (the default; Tuning::sortScanless, GSM_SORT_SCAN=kernel restores k_radix_scan): the upsweep also
// adds each block's digit counts into its super-group's row (kSuperGroup consecutive blocks share a
// row of 256 words; device-scope atomics, at most kSuperGroup deep per word), and every downsweep
// block derives its digit bases itself -- digit totals = the sum of all rows, its prefix = the rows of
// the earlier super-groups plus the earlier blocks of its own group (< kSuperGroup + grid/kSuperGroup
// reads per digit, spread over 256 / R threads).  One launch less per pass, no extra pass over the keys.
// Two row sets: a sort call of an even number of narrow passes alternates them, pass i on set i & 1,
// and each upsweep zeroes the other set (its last reader, the previous pass, has finished), so every
// call starts and ends with set 0 zero; calls of an odd number of narrow passes keep k_radix_scan.
// (A ticket taken by the downsweep's last block to zero the rows costs more than the scan it replaces:
// a single ticket serializes at ~36 ns an atomic, and an agent-scope fence per block writes back the
// XCD's L2 -- +35 us a pass, measured.)
constexpr uint32_t kSuperGroup = 32;
constexpr uint32_t kSuperRows = 1024 / kSuperGroup;  // radix_grid_for_capacity caps the grid at 1024
constexpr size_t kSuperSetWords = (size_t)kSuperRows * 256;
constexpr size_t kSuperWords = 2 * kSuperSetWords;
static_assert(kRadixBlock == 256 && kRadixBlock / 64 == 4, "the scanless base reduction assumes 4 waves");


template <int BITS>
__global__ __launch_bounds__(kRadixBlock) void k_radix_upsweep(const uint32_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ nPtr,
                                                               uint32_t shift,
                                                               uint32_t* __restrict__ hist,
                                                               uint32_t* __restrict__ super,
                                                               uint32_t* __restrict__ superClear) {
    constexpr uint32_t R = 1u << BITS;
    // CP counter copies per wave (lane & (copies - 1) picks one), rows padded by a
    // word so one digit's copies sit in different LDS banks: fewer same-address collisions among
    // the 64 lanes of one ds_add
    constexpr uint32_t CP = 4, RS = R + (CP > 1 ? 1u : 0u);
    __shared__ uint32_t cnt[kWaves * CP][RS];
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t row = wave * CP + (threadIdx.x & (CP - 1u));
    for (int i = threadIdx.x; i < (int)(kWaves * CP * RS); i += kRadixBlock) (&cnt[0][0])[i] = 0;
    if (superClear)  // scanless: the previous pass's row set, for the next pass
        for (uint32_t i = blockIdx.x * kRadixBlock + threadIdx.x; i < (uint32_t)kSuperSetWords; i += gridDim.x * kRadixBlock)
            superClear[i] = 0u;
    __syncthreads();
    uint32_t begin, end;
    block_range(*nPtr, gridDim.x, blockIdx.x, &begin, &end);
    // a chunk's keys are all loaded before any is counted (16 loads in flight per thread), and the
    // next chunk's loads are issued before this chunk's counting starts (its LDS atomics hide them);
    // order does not matter for a histogram, so they come as 16-byte vectors
    // (unpredicated, the ragged end from T: see Tail4; keys at and past `end` are not counted)
    const Tail4 T = tail4_load(keys, end > 0u ? end : 1u);
    auto load_chunk = [&](uint32_t cbase, uint4 (&q)[kRadixItems / 4]) {
#pragma unroll
        for (int i = 0; i < kRadixItems / 4; ++i) q[i] = load4_clamped(keys, cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u, T);
#pragma unroll
        for (int i = 0; i < kRadixItems / 4; ++i) q[i] = fix4(q[i], cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u, T);
    };
    uint4 q[kRadixItems / 4];
    if (begin < end) load_chunk(begin, q);
    for (uint32_t cbase = begin; cbase < end; cbase += kRadixChunk) {
        uint4 nq[kRadixItems / 4];
        const bool more = cbase + kRadixChunk < end;
        if (more) load_chunk(cbase + kRadixChunk, nq);
#pragma unroll
        for (int i = 0; i < kRadixItems / 4; ++i) {
            const uint32_t idx = cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u;
            const uint32_t kk[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)  // per-wave LDS counters: one ds_add per key
                if (idx + (uint32_t)c < end) atomicAdd(&cnt[row][(kk[c] >> shift) & (R - 1u)], 1u);
        }
        if (more) {
#pragma unroll
            for (int i = 0; i < kRadixItems / 4; ++i) q[i] = nq[i];
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += kRadixBlock) {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t w = 0; w < kWaves * CP; ++w) s += cnt[w][d];
        hist[(size_t)d * gridDim.x + blockIdx.x] = s;
        if (super && s) atomicAdd(&super[(blockIdx.x / kSuperGroup) * 256u + d], s);
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
    uint32_t inc = wave_scan_incl(local);
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

// ---------------------------------------------------------------------------
// Tile starts from the sort itself (radix_sort_tiles).  The frame sort's keys are tile << 16 |
// depth (the DepthFirst instance keys: the tile alone); its passes sort the tile field, low digit
// first.  The first pass leaves buckets: bucket l = the run of keys whose low digit is l, starting
// at bucketStart[l] (block 0 of that pass writes these, the exclusive scan of its digit totals).
// In the last pass, the keys of bucket l that precede digit h's output are exactly those of tile
// (h << lowBits | l)'s predecessors: all keys of high digits < h and the keys of digit h in
// buckets < l.  So where a block's chunk holds the start p of bucket l, the start of tile
// (h, l) is digit h's output base at that chunk plus the chunk's keys of digit h before p -- a lower
// bound also when the tile is empty.  Those counts: the earlier waves' (the per-digit wave scan)
// plus the holding wave's counters copied when its rank loop reaches p's item (a further start
// in the same chunk, rare, recounts the chunk's keys before it from L2).  The block holding
// p = bucketStart[l] writes the
// starts of every tile of bucket l; the last block those of the empty buckets at the end
// (bucketStart = n); no separate pass over the sorted keys.  One pass: one bucket, lowBits = 0.
struct TileStarts {
    const uint32_t* bucketStart;  // [1 << lowBits] (null with one pass: the single bucket starts at 0)
    uint32_t* bucketStartOut;     // first pass: written by its block 0
    uint32_t lowBits;             // bits of the first pass (the low tile digit)
    uint32_t numTiles;
    uint32_t* tileStart;          // [numTiles + 1]
};

// Digits >= 2^BITS do not exist: their counters stay 0 (thread tid owns digit tid of 256).
// STARTS: the last pass of radix_sort_tiles (tile starts written, see TileStarts).
template <int BITS, bool BALLOT, bool STARTS>
__global__ __launch_bounds__(kRadixBlock) void k_radix_downsweep(
    const uint32_t* __restrict__ keysIn, const uint32_t* __restrict__ valsIn,
    uint32_t* __restrict__ keysOut, uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ nPtr,
    uint32_t shift, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ binTotals, TileStarts ts,
    const uint32_t* __restrict__ super) {
    constexpr uint32_t R = 1u << BITS;
    __shared__ uint32_t binBase[256];
    __shared__ uint32_t localStart[256];
    __shared__ uint32_t chunkTotal[256];
    __shared__ uint32_t waveCnt[kWaves][256];
    __shared__ uint32_t sKeys[kRadixChunk];
    __shared__ uint32_t sVals[kRadixChunk];
    __shared__ uint32_t part[kWaves];

    // STARTS: the chunk's keys per digit before a bucket start (1 << BITS words: with the arrays
    // above, 4 blocks per CU still fit for BITS <= 7 -- radix_pass limits every narrow downsweep to 3)
    __shared__ uint32_t sCntB[1u << BITS];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = *nPtr;
    uint32_t begin, end;
    block_range(n, gridDim.x, blockIdx.x, &begin, &end);
    if (STARTS && n == 0u && blockIdx.x == 0)  // no keys: every tile starts (and ends) at 0
        for (uint32_t t = tid; t <= ts.numTiles; t += kRadixBlock) ts.tileStart[t] = 0u;
    if (begin >= end) return;
    const uint32_t L = 1u << ts.lowBits;
    // STARTS: bucket l's start (uniform l: a scalar load); the first bucket not yet handled
    auto bucketAt = [&](uint32_t l) -> uint32_t { return ts.bucketStart ? ts.bucketStart[l] : 0u; };
    uint32_t nextL = 0;  // (starts are non-decreasing: the earlier blocks' buckets come first)
    if (STARTS) nextL = (uint32_t)__syncthreads_count(tid < L && bucketAt(tid) < begin);

    // global base of every digit for this block: exclusive scan over digits + block column offset
    {
        uint32_t t, pre;
        if (super) {  // scanless: totals and this block's prefix from the super-group rows
            constexpr uint32_t SPLIT = (256u / R) < 4u ? (256u / R) : 4u;
            const uint32_t d = tid % R, q = tid / R, b = blockIdx.x, g = b / kSuperGroup;
            const uint32_t rows = (gridDim.x + kSuperGroup - 1u) / kSuperGroup;
            uint32_t tq = 0, pq = 0;
            if (q < SPLIT) {  // fixed trip counts, unrolled: every load in flight at once
                constexpr uint32_t NR = kSuperRows / SPLIT, NB = kSuperGroup / SPLIT;
                uint32_t rv[NR], bv[NB];
#pragma unroll
                for (uint32_t i = 0; i < NR; ++i) {
                    const uint32_t r = q + i * SPLIT;
                    rv[i] = r < rows ? super[r * 256u + d] : 0u;
                }
#pragma unroll
                for (uint32_t i = 0; i < NB; ++i) {
                    const uint32_t bb = g * kSuperGroup + q + i * SPLIT;
                    bv[i] = bb < b ? hist[(size_t)d * gridDim.x + bb] : 0u;
                }
#pragma unroll
                for (uint32_t i = 0; i < NR; ++i) {
                    tq += rv[i];
                    pq += q + i * SPLIT < g ? rv[i] : 0u;
                }
#pragma unroll
                for (uint32_t i = 0; i < NB; ++i) pq += bv[i];
                sKeys[q * 256u + d] = tq;
                waveCnt[q][d] = pq;
            }
            __syncthreads();
            t = 0u;
            pre = 0u;
            if (tid < R)
#pragma unroll
                for (uint32_t i = 0; i < SPLIT; ++i) {
                    t += sKeys[i * 256u + tid];
                    pre += waveCnt[i][tid];
                }
        } else {
            t = tid < R ? binTotals[tid] : 0u;
            pre = tid < R ? hist[(size_t)tid * gridDim.x + blockIdx.x] : 0u;
        }
        uint32_t inc = wave_scan_incl(t);
        if (lane == 63) part[wave] = inc;
        __syncthreads();
        uint32_t off = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w)
            if ((uint32_t)w < wave) off += part[w];
        binBase[tid] = off + inc - t + pre;
        // first pass of radix_sort_tiles: its digits are the last pass's buckets
        if (!STARTS && ts.bucketStartOut && blockIdx.x == 0 && tid < R) ts.bucketStartOut[tid] = off + inc - t;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) waveCnt[w][tid] = 0;
        __syncthreads();
    }

    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t cbase = begin; cbase < end; cbase += kRadixChunk) {
        uint32_t k[kRadixItems], v[kRadixItems], rank[kRadixItems];
        // STARTS: the first bucket start p0 in this chunk, at item jp, lane lp of wave wp
        uint32_t p0 = ~0u, wp = ~0u, jp = 0, lp = 0;
        if constexpr (STARTS) {
            if (nextL < L && bucketAt(nextL) < cbase + min((uint32_t)kRadixChunk, end - cbase)) {
                p0 = bucketAt(nextL);
                const uint32_t r = p0 - cbase;
                wp = r / (64u * kRadixItems);
                jp = (r / 64u) % kRadixItems;
                lp = r % 64u;
            }
        }
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
            if (STARTS && wave == wp && (uint32_t)j == jp) {
                // the wave's digit counts before p0: its counters before item jp (LDS operations of
                // a wave complete in order) plus item jp's lanes before lp
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (uint32_t q = lane; q < R; q += 64u) sCntB[q] = waveCnt[wave][q];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (valid && lane < lp) atomicAdd(&sCntB[d], 1u);
            }
            rank[j] = wave_rank<BITS, BALLOT>(waveCnt[wave], d, valid, lt);
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
            uint32_t inc = wave_scan_incl(tot);
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
        if constexpr (STARTS) {  // buckets starting in this chunk (uniform; most chunks have none)
            if (p0 != ~0u) {  // at p0: the earlier waves' keys of digit h plus wave wp's before p0
                do {          // (empty buckets share their successor's start)
                    const uint32_t tt = (tid << ts.lowBits) | nextL;
                    if (tid < R && tt <= ts.numTiles)
                        ts.tileStart[tt] = binBase[tid] + waveCnt[wp][tid] + sCntB[tid];
                    ++nextL;
                } while (nextL < L && bucketAt(nextL) == p0);
                __syncthreads();
            }
            // further starts in the same chunk (small buckets): count the keys before them again
            while (nextL < L && bucketAt(nextL) < cbase + cn) {
                const uint32_t p = bucketAt(nextL);
                if (tid < R) sCntB[tid] = 0u;
                __syncthreads();
                // the chunk's keys before p per digit (the keys are still in L2)
                for (uint32_t i = cbase + tid; i < p; i += kRadixBlock)
                    atomicAdd(&sCntB[(keysIn[i] >> shift) & (R - 1u)], 1u);
                __syncthreads();
                do {  // every bucket starting at p (empty buckets share their successor's start)
                    const uint32_t tt = (tid << ts.lowBits) | nextL;
                    if (tid < R && tt <= ts.numTiles) ts.tileStart[tt] = binBase[tid] + sCntB[tid];
                    ++nextL;
                } while (nextL < L && bucketAt(nextL) == p);
                __syncthreads();
            }
        }
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
    if (STARTS && end == n) {  // the last block: binBase[h] = the keys of high digits <= h; the
        if (tid < R)           // buckets left start at n (empty)
            for (uint32_t l = nextL; l < L; ++l) {
                const uint32_t tt = (tid << ts.lowBits) | l;
                if (tt <= ts.numTiles) ts.tileStart[tt] = binBase[tid];
            }
        if (tid == 0) ts.tileStart[ts.numTiles] = n;
    }
}

// ---------------------------------------------------------------------------
// Wide passes take chunks of kWideChunk keys (kWideItems per thread; 8 measured slower): their per-chunk digit
// bookkeeping is heavier, so their blocks are fewer per CU.
constexpr int kWideItems = 16;
constexpr int kWideChunk = kRadixBlock * kWideItems;
static_assert(kWideItems % 4 == 0 && kWideItems <= kRadixItems, "wide chunks: 16-B loads, <= the narrow chunk");
__device__ __forceinline__ void block_range_w(uint32_t n, uint32_t grid, uint32_t b, uint32_t* begin, uint32_t* end) {
    uint32_t per = (n + grid - 1) / grid;
    per = (per + kWideChunk - 1) / kWideChunk * kWideChunk;
    uint64_t bb = (uint64_t)per * b;
    uint64_t ee = bb + per;
    if (bb > n) bb = n;
    if (ee > n) ee = n;
    *begin = (uint32_t)bb;
    *end = (uint32_t)ee;
}

// Wide digits (9..11 bits, up to 2048 bins): one pass where the narrow kernels need two -- the tile
// field of a frame with <= 2048 tiles in its rows (a multi-GPU slab, keys counted relative to the
// slab's first tile), and the DepthFirst depth sort's 32-bit keys (3 passes of 11/11/10 bits).
// Same chunks, block ranges and stable ranks as the narrow downsweep; what changes is the
// per-chunk digit bookkeeping: thread t owns the 2^BITS / 256 contiguous digits [t * DPT, +DPT)
// (registers for their running global bases), and the per-wave counters are padded one word in
// eight so those contiguous reads hit distinct LDS banks.
// digit(k) = ((k >> shift) - base) & (2^BITS - 1): base = the slab's first tile (0 otherwise).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wide_pad(uint32_t d) { return d + (d >> 3); }
// block-major count rows of 2^BITS words, padded by 256 B (rows of a power-of-two stride all start on
// the same HBM channel group)
constexpr uint32_t kWideRowPad = 64;

template <int BITS>
__global__ __launch_bounds__(kRadixBlock) void k_wide_upsweep(const uint32_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ nPtr, uint32_t shift,
                                                              uint32_t base, uint32_t* __restrict__ hist) {
    constexpr uint32_t R = 1u << BITS;
    // one counter array: a histogram needs no order, and 2^BITS bins spread the atomics
    __shared__ uint32_t cnt[R];
    uint32_t begin, end;
    block_range_w(*nPtr, gridDim.x, blockIdx.x, &begin, &end);
    if (begin >= end) return;  // no row: k_wide_scan reads the active blocks' rows only
    for (uint32_t i = threadIdx.x; i < R; i += kRadixBlock) cnt[i] = 0;
    __syncthreads();
    // (unpredicated, the ragged end from T: see Tail4; keys at and past `end` are not counted)
    const Tail4 T = tail4_load(keys, end);
    auto load_chunk = [&](uint32_t cbase, uint4 (&q)[kWideItems / 4]) {
#pragma unroll
        for (int i = 0; i < kWideItems / 4; ++i) q[i] = load4_clamped(keys, cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u, T);
#pragma unroll
        for (int i = 0; i < kWideItems / 4; ++i) q[i] = fix4(q[i], cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u, T);
    };
    uint4 q[kWideItems / 4];
    if (begin < end) load_chunk(begin, q);
    for (uint32_t cbase = begin; cbase < end; cbase += kWideChunk) {
        uint4 nq[kWideItems / 4];
        const bool more = cbase + kWideChunk < end;
        if (more) load_chunk(cbase + kWideChunk, nq);
#pragma unroll
        for (int i = 0; i < kWideItems / 4; ++i) {
            const uint32_t idx = cbase + (uint32_t)(i * kRadixBlock + threadIdx.x) * 4u;
            const uint32_t kk[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (idx + (uint32_t)c < end) atomicAdd(&cnt[((kk[c] >> shift) - base) & (R - 1u)], 1u);
        }
        if (more) {
#pragma unroll
            for (int i = 0; i < kWideItems / 4; ++i) q[i] = nq[i];
        }
    }
    __syncthreads();
    // block-major counts (hist[b][d]): coalesced here, and the downsweep reads its row contiguously
    for (uint32_t d = threadIdx.x; d < R; d += kRadixBlock) hist[(size_t)blockIdx.x * (R + kWideRowPad) + d] = cnt[d];
}

// Exclusive scan over blocks of the block-major wide counts, in place, digit totals out -- over the
// blocks that hold keys (block_range: the grid is sized for the capacity, a frame fills a part of
// it).  Workgroup g owns digits [16g, 16g + 16); thread t scans digit 16g + (t & 15) over the
// (t >> 4)-th sixteenth of those blocks: up to 32 rows loaded at once and kept in registers (one
// memory round trip; more rows loop and re-read), the 16 segment sums meet in LDS.
constexpr uint32_t kWideScanDigits = 16, kWideScanRegs = 32;
template <int BITS>
__global__ __launch_bounds__(256) void k_wide_scan(uint32_t* __restrict__ hist, uint32_t grid,
                                                   const uint32_t* __restrict__ nPtr, uint32_t* __restrict__ binTotals) {
    constexpr uint32_t R = 1u << BITS, RS = R + kWideRowPad;
    constexpr uint32_t S = 256 / kWideScanDigits;  // segments
    __shared__ uint32_t ss[S][kWideScanDigits];
    // active blocks, as block_range splits n: block b holds keys iff b * per < n
    const uint32_t n = *nPtr;
    uint32_t per = (n + grid - 1) / grid;
    per = (per + kWideChunk - 1) / kWideChunk * kWideChunk;
    const uint32_t active = per ? min(grid, (n + per - 1) / per) : 0u;
    const uint32_t j = threadIdx.x % kWideScanDigits, sg = threadIdx.x / kWideScanDigits;
    const uint32_t d = blockIdx.x * kWideScanDigits + j;
    const uint32_t q = (active + S - 1) / S;
    const uint32_t b0 = min(sg * q, active), b1 = min(b0 + q, active);
    uint32_t* col = hist + d;
    uint32_t v[kWideScanRegs];
    uint32_t sum = 0;
    if (q <= kWideScanRegs) {
#pragma unroll
        for (uint32_t i = 0; i < kWideScanRegs; ++i) v[i] = b0 + i < b1 ? col[(size_t)(b0 + i) * RS] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < kWideScanRegs; ++i) sum += v[i];
    } else {
        for (uint32_t b = b0; b < b1; ++b) sum += col[(size_t)b * RS];
    }
    ss[sg][j] = sum;
    __syncthreads();
    uint32_t run = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < S; ++w) {
        const uint32_t x = ss[w][j];
        if (w < sg) run += x;
        tot += x;
    }
    if (sg == 0) binTotals[d] = tot;
    if (q <= kWideScanRegs) {
#pragma unroll
        for (uint32_t i = 0; i < kWideScanRegs; ++i)
            if (b0 + i < b1) {
                col[(size_t)(b0 + i) * RS] = run;
                run += v[i];
            }
    } else {
        for (uint32_t b = b0; b < b1; ++b) {
            const uint32_t x = col[(size_t)b * RS];
            col[(size_t)b * RS] = run;
            run += x;
        }
    }
}

// Exclusive scan over the block of one value per thread (4 waves); returns this thread's offset.
__device__ __forceinline__ uint32_t wide_block_scan(uint32_t x, uint32_t* part, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t inc = wave_scan_incl(x);
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        if ((uint32_t)w < wave) off += part[w];
        tot += part[w];
    }
    *total = tot;
    return off + inc - x;
}

// STARTS (one pass over a frame's tile field, radix_sort_tiles): block 0 writes every tile's start
// -- the exclusive scan of the digit totals, i.e. its digit's global base -- tiles before the
// slab start at 0 and those after it at n (no keys there), tileStart[allTiles] = n.
template <int BITS, bool BALLOT, bool STARTS>
__global__ __launch_bounds__(kRadixBlock) void k_wide_downsweep(
    const uint32_t* __restrict__ keysIn, const uint32_t* __restrict__ valsIn, uint32_t* __restrict__ keysOut,
    uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ nPtr, uint32_t shift, uint32_t base,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ binTotals, uint32_t* __restrict__ tileStart,
    uint32_t numTiles, uint32_t allTiles) {
    constexpr uint32_t R = 1u << BITS;
    constexpr uint32_t DPT = R / kRadixBlock;  // digits per thread
    constexpr uint32_t RP = (R + R / 8 + 255u) / 256u * 256u;  // padded counter rows (whole uint4 zeroing rounds)
    static_assert(DPT >= 2 && DPT <= 8, "wide digits: 9..11 bits");
    __shared__ __attribute__((aligned(16))) uint32_t waveCnt[kWaves][RP];  // ranks, then each wave's LDS start per digit
    __shared__ uint32_t adj[RP];               // per digit: global destination minus LDS start
    __shared__ uint32_t sKeys[kWideChunk];
    __shared__ uint32_t sVals[kWideChunk];
    __shared__ uint32_t part[kWaves];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t n = *nPtr;
    uint32_t begin, end;
    block_range_w(n, gridDim.x, blockIdx.x, &begin, &end);
    const uint32_t d0 = tid * DPT;  // this thread's digits
    auto zero_counters = [&]() {    // 16-byte stores
        static_assert((kWaves * RP) % (4 * kRadixBlock) == 0, "counter rows in whole uint4 rounds");
        uint4* z = (uint4*)&waveCnt[0][0];
#pragma unroll
        for (uint32_t i = 0; i < kWaves * RP / 4 / kRadixBlock; ++i) z[i * kRadixBlock + tid] = make_uint4(0u, 0u, 0u, 0u);
    };

    // global base of this thread's digits: exclusive scan of the digit totals + the block's column
    uint32_t gbase[DPT];
    {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t i = 0; i < DPT; ++i) {
            gbase[i] = run;
            run += binTotals[d0 + i];
        }
        uint32_t tot;
        const uint32_t off = wide_block_scan(run, part, &tot);
#pragma unroll
        for (uint32_t i = 0; i < DPT; ++i) gbase[i] += off;
        if (STARTS && blockIdx.x == 0) {
            // tiles [base, base + numTiles) of allTiles: their digits' global bases
            for (uint32_t t = tid; t < base; t += kRadixBlock) tileStart[t] = 0u;
#pragma unroll
            for (uint32_t i = 0; i < DPT; ++i)
                if (d0 + i < numTiles) tileStart[base + d0 + i] = gbase[i];
            for (uint32_t t = base + numTiles + tid; t <= allTiles; t += kRadixBlock) tileStart[t] = n;
        }
        if (begin >= end) return;
        const uint32_t* row = hist + (size_t)blockIdx.x * (R + kWideRowPad) + d0;  // block-major (k_wide_scan)
#pragma unroll
        for (uint32_t i = 0; i < DPT; ++i) gbase[i] += row[i];
        zero_counters();
        __syncthreads();
    }

    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (uint32_t cbase = begin; cbase < end; cbase += kWideChunk) {
        uint32_t k[kWideItems], v[kWideItems], rank[kWideItems];
#pragma unroll
        for (int j = 0; j < kWideItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kWideItems) + j * 64 + lane;
            const bool valid = idx < end;
            k[j] = valid ? keysIn[idx] : 0u;
            v[j] = valid ? valsIn[idx] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kWideItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kWideItems) + j * 64 + lane;
            const bool valid = idx < end;
            const uint32_t d = ((k[j] >> shift) - base) & (R - 1u);
            if constexpr (BALLOT) {
                const uint64_t peers = match_digit<BITS>(d, valid);
                const uint32_t before = waveCnt[wave][wide_pad(d)];
                if (valid && (peers & lt) == 0) waveCnt[wave][wide_pad(d)] = before + (uint32_t)__popcll(peers);
                rank[j] = before + (uint32_t)__popcll(peers & lt);
            } else {
                rank[j] = valid ? atomicAdd(&waveCnt[wave][wide_pad(d)], 1u) : 0u;
            }
        }
        __syncthreads();
        // per digit: chunk total, its LDS start (scan over digits), each wave's start within it
        {
            uint32_t c[DPT][kWaves], tot[DPT], run = 0;
#pragma unroll
            for (uint32_t i = 0; i < DPT; ++i) {
                tot[i] = 0;
#pragma unroll
                for (int w = 0; w < kWaves; ++w) {
                    c[i][w] = waveCnt[w][wide_pad(d0 + i)];
                    tot[i] += c[i][w];
                }
                run += tot[i];
            }
            uint32_t all;
            uint32_t ls = wide_block_scan(run, part, &all);
#pragma unroll
            for (uint32_t i = 0; i < DPT; ++i) {
                const uint32_t pd = wide_pad(d0 + i);
                adj[pd] = gbase[i] - ls;
                gbase[i] += tot[i];
#pragma unroll
                for (int w = 0; w < kWaves; ++w) {
                    waveCnt[w][pd] = ls;
                    ls += c[i][w];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kWideItems; ++j) {
            const uint32_t idx = cbase + wave * (64 * kWideItems) + j * 64 + lane;
            if (idx < end) {
                const uint32_t pos = waveCnt[wave][wide_pad(((k[j] >> shift) - base) & (R - 1u))] + rank[j];
                sKeys[pos] = k[j];
                sVals[pos] = v[j];
            }
        }
        __syncthreads();
        zero_counters();
        const uint32_t cn = min((uint32_t)kWideChunk, end - cbase);
        for (uint32_t p = tid; p < cn; p += kRadixBlock) {
            const uint32_t key = sKeys[p];
            const uint32_t dst = adj[wide_pad(((key >> shift) - base) & (R - 1u))] + p;
            keysOut[dst] = key;
            valsOut[dst] = sVals[p];
        }
        __syncthreads();
    }
}

static uint32_t wide_grid_for_capacity(uint32_t capacity) {
    uint32_t g = (capacity + kWideChunk - 1) / kWideChunk;  // (<= 1024 rows: radix_workspace_bytes)
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    return g;
}

static void wide_pass(uint32_t* kin, uint32_t* vin, uint32_t* kout, uint32_t* vout, const uint32_t* nPtr,
                      uint32_t grid, uint32_t shift, uint32_t base, int bits, uint32_t* hist, uint32_t* binTotals,
                      hipStream_t s, bool ballot, bool starts, uint32_t* tileStart, uint32_t numTiles,
                      uint32_t allTiles) {
    hist += kSuperWords;  // (radix_workspace_bytes: the narrow passes' super-group rows come first)
#define GSM_WIDE_DOWN(B, BAL, S)                                                                              \
    hipLaunchKernelGGL((k_wide_downsweep<B, BAL, S>), dim3(grid), dim3(kRadixBlock), 0, s, kin, vin, kout, vout, \
                       nPtr, shift, base, hist, binTotals, tileStart, numTiles, allTiles)
#define GSM_WIDE_PASS(B)                                                                                         \
    hipLaunchKernelGGL(k_wide_upsweep<B>, dim3(grid), dim3(kRadixBlock), 0, s, kin, nPtr, shift, base, hist);    \
    hipLaunchKernelGGL(k_wide_scan<B>, dim3((1u << B) / kWideScanDigits), dim3(256), 0, s, hist, grid, nPtr, binTotals); \
    if (ballot) {                                                                                                \
        if (starts) GSM_WIDE_DOWN(B, true, true);                                                                \
        else GSM_WIDE_DOWN(B, true, false);                                                                      \
    } else {                                                                                                     \
        if (starts) GSM_WIDE_DOWN(B, false, true);                                                               \
        else GSM_WIDE_DOWN(B, false, false);                                                                     \
    }
    switch (bits) {
        case 9: GSM_WIDE_PASS(9); break;
        case 10: GSM_WIDE_PASS(10); break;
        default: GSM_WIDE_PASS(11); break;
    }
#undef GSM_WIDE_PASS
#undef GSM_WIDE_DOWN
}

size_t sort_pass_hist_words(bool wide, int bits, uint32_t grid) {
    // narrow: digit-major counts hist[d][block] (k_radix_upsweep / k_radix_scan); wide: block-major rows
    // of 2^bits + kWideRowPad words (k_wide_upsweep); both behind the scanless super-group row sets
    const size_t rows = wide ? ((size_t)1 << bits) + kWideRowPad : ((size_t)1 << bits);
    return kSuperWords + rows * grid;
}

size_t radix_workspace_bytes(uint32_t capacity) {
    // the scanless super-group row sets (zero at allocation; see kSuperGroup), then the per-block digit
    // counts of the widest pass any sort of this capacity plans: 256 digits (narrow) or 2^kWideMaxBits
    const size_t narrow = sort_pass_hist_words(false, 8, radix_grid_for_capacity(capacity));
    const size_t wide = sort_pass_hist_words(true, (int)kWideMaxBits, wide_grid_for_capacity(capacity));
    return std::max(narrow, wide) * sizeof(uint32_t);
}

// the passes' footprints against the workspace (nothing is launched for a plan that does not fit)
static bool pass_fits(const SortSpace& ws, bool wide, int bits, uint32_t grid, size_t binWords) {
    if (!ws.hist || !ws.binTotals) return false;
    if (sort_pass_hist_words(wide, bits, grid) * sizeof(uint32_t) > ws.histBytes) return false;
    // narrow passes read <= 1024 blocks' rows (k_radix_scan's column in registers, the super rows)
    if (!wide && grid > kSuperRows * kSuperGroup) return false;
    return binWords <= ws.binWords;
}

uint32_t radix_grid_for_capacity(uint32_t capacity) {
    // <= 1024 blocks: k_radix_scan holds a digit's column in 4 registers per thread
    uint32_t g = (capacity + kRadixChunk - 1) / kRadixChunk;
    if (g > 1024) g = 1024;
    if (g < 1) g = 1;
    return g;
}

// one LSD pass; ts: a pass of radix_sort_tiles (its first writes the bucket starts, its last --
// starts = true -- the tile starts)
static void radix_pass(uint32_t* kin, uint32_t* vin, uint32_t* kout, uint32_t* vout, const uint32_t* nPtr,
                       uint32_t grid, uint32_t shift, int bits, uint32_t* hist, uint32_t* binTotals,
                       hipStream_t s, bool ballot, const TileStarts* ts = nullptr, bool starts = false,
                       int superSet = -1) {
    const TileStarts t = ts ? *ts : TileStarts{};
    // scanless (superSet 0 or 1): the row sets sit in front of the block counts
    uint32_t* super = superSet >= 0 ? hist + (size_t)superSet * kSuperSetWords : nullptr;
    uint32_t* superClear = superSet >= 0 ? hist + (size_t)(superSet ^ 1) * kSuperSetWords : nullptr;
    hist += kSuperWords;
    // 1 KiB of dynamic LDS on the downsweeps without tile starts: > 40 KiB a block, 3 blocks per CU like
    // the STARTS pass -- the first 4K tile pass at 4 blocks per CU measured 2.5 us slower (64.4-65.9
    // against 62.2-62.4 us; 1080p unchanged; r06, profiles/r06_sort_occupancy_ab.txt)
    const uint32_t ldsPad = starts ? 0u : 1024u;
#define GSM_RADIX_PASS(B, S)                                                                                \
    hipLaunchKernelGGL(k_radix_upsweep<B>, dim3(grid), dim3(kRadixBlock), 0, s, kin, nPtr, shift, hist, super, \
                       superClear);                                                                         \
    if (!super) hipLaunchKernelGGL(k_radix_scan, dim3(1u << B), dim3(256), 0, s, hist, grid, binTotals);  \
    if (ballot)                                                                                             \
        hipLaunchKernelGGL((k_radix_downsweep<B, true, S>), dim3(grid), dim3(kRadixBlock), ldsPad, s, kin, vin, kout, \
                           vout, nPtr, shift, hist, binTotals, t, super);                                   \
    else                                                                                                    \
        hipLaunchKernelGGL((k_radix_downsweep<B, false, S>), dim3(grid), dim3(kRadixBlock), ldsPad, s, kin, vin, kout, \
                           vout, nPtr, shift, hist, binTotals, t, super)
#define GSM_RADIX_BITS(S)                    \
    switch (bits) {                          \
        case 4: GSM_RADIX_PASS(4, S); break; \
        case 5: GSM_RADIX_PASS(5, S); break; \
        case 6: GSM_RADIX_PASS(6, S); break; \
        case 7: GSM_RADIX_PASS(7, S); break; \
        default: GSM_RADIX_PASS(8, S); break; \
    }
    if (starts) {
        GSM_RADIX_BITS(true)
    } else {
        GSM_RADIX_BITS(false)
    }
#undef GSM_RADIX_BITS
#undef GSM_RADIX_PASS
}

int radix_sort_pairs(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                     int firstDigit, int numDigits, const SortSpace& ws, hipStream_t s, bool ballot, bool scanlessOn) {
    const uint32_t grid = radix_grid_for_capacity(capacity);
    if (!pass_fits(ws, false, 8, grid, 256)) return kSortNoSpace;
    int cur = 0;
    const bool scanless = scanlessOn && numDigits % 2 == 0;
    for (int dgt = firstDigit; dgt < firstDigit + numDigits; ++dgt) {
        radix_pass(keys[cur], vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, grid, (uint32_t)dgt * 8u, 8, ws.hist,
                   ws.binTotals, s, ballot, nullptr, false, scanless ? (dgt - firstDigit) & 1 : -1);
        cur ^= 1;
    }
    return cur;
}

bool sort_bits_plan_fits(uint32_t capacity, uint32_t bits, bool wide, const SortSpace& ws) {
    const uint32_t grid = radix_grid_for_capacity(capacity), wgrid = wide_grid_for_capacity(capacity);
    const uint32_t narrowPasses = (bits + 7) / 8, widePasses = (bits + kWideMaxBits - 1) / kWideMaxBits;
    const bool useWide = wide && widePasses < narrowPasses;
    const uint32_t passes = useWide ? widePasses : narrowPasses;
    for (uint32_t p = 0, done = 0; p < passes; ++p) {
        uint32_t b = (bits - done + (passes - p) - 1) / (passes - p);
        b = useWide ? (b < 9 ? 9u : b) : (b < 4 ? 4u : b);
        if (!pass_fits(ws, useWide, (int)b, useWide ? wgrid : grid, (size_t)1 << b)) return false;
        done += b;
    }
    return true;
}

int radix_sort_bits(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity,
                    uint32_t shift, uint32_t bits, const SortSpace& ws, hipStream_t s,
                    bool ballot, bool wide, bool scanlessOn) {
    const uint32_t grid = radix_grid_for_capacity(capacity), wgrid = wide_grid_for_capacity(capacity);
    const uint32_t narrowPasses = (bits + 7) / 8;
    const uint32_t widePasses = (bits + kWideMaxBits - 1) / kWideMaxBits;
    // wide digits where they save a whole pass (32-bit keys: 3 passes of 11/11/10 bits instead of 4)
    const bool useWide = wide && widePasses < narrowPasses;
    const uint32_t passes = useWide ? widePasses : narrowPasses;
    const bool scanless = !useWide && scanlessOn && passes % 2 == 0;
    // near-equal digit widths; a digit wider than the bits left reads zero bits above the field
    auto width = [&](uint32_t p, uint32_t done) {
        const uint32_t b = (bits - done + (passes - p) - 1) / (passes - p);
        return useWide ? (b < 9 ? 9u : b) : (b < 4 ? 4u : b);
    };
    if (!sort_bits_plan_fits(capacity, bits, wide, ws)) return kSortNoSpace;  // the plan fits, or no launch
    int cur = 0;
    uint32_t done = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t b = width(p, done);
        if (useWide)
            wide_pass(keys[cur], vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, wgrid, shift + done, 0u, (int)b, ws.hist,
                      ws.binTotals, s, ballot, false, nullptr, 0u, 0u);
        else
            radix_pass(keys[cur], vals[cur], keys[cur ^ 1], vals[cur ^ 1], nPtr, grid, shift + done, (int)b, ws.hist,
                       ws.binTotals, s, ballot, nullptr, false, scanless ? (int)(p & 1u) : -1);
        done += b;
        cur ^= 1;
    }
    return cur;
}

// The frame sort's tile passes with the tile starts written by the last pass (TileStarts above).
// The keys' tile field holds tiles [tileBase, tileBase + numTiles) of allTiles.  With <= 2048 tiles
// in that range (a multi-GPU slab) and wide digits on, one wide pass sorts it, digits counted
// from tileBase; otherwise radix_sort_bits' narrow passes over the whole tile field (bits <= 16:
// one or two passes).  binTotals holds kSortTotalsWords words: the last pass's digit totals, the
// first pass's at +256, its bucket starts at +512 (narrow); the wide pass's 2048 totals.
int radix_sort_tiles(uint32_t* keys[2], uint32_t* vals[2], const uint32_t* nPtr, uint32_t capacity, uint32_t shift,
                     const SortSpace& ws, uint32_t* tileStart, uint32_t tileBase, uint32_t numTiles,
                     uint32_t allTiles, hipStream_t s, bool ballot, bool wide, bool scanlessOn) {
    const uint32_t grid = radix_grid_for_capacity(capacity);
    auto bitsFor = [](uint32_t tiles) {
        uint32_t b = 1;
        while (b < 16 && ((tiles - 1u) >> b)) b++;
        return b;
    };
    uint32_t bits = bitsFor(allTiles);
    const uint32_t localBits = bitsFor(numTiles);
    if (wide && bits > 8 && localBits <= kWideMaxBits) {
        const uint32_t wb = localBits < 9 ? 9 : localBits, wgrid = wide_grid_for_capacity(capacity);
        if (!pass_fits(ws, true, (int)wb, wgrid, (size_t)1 << wb)) return kSortNoSpace;
        wide_pass(keys[0], vals[0], keys[1], vals[1], nPtr, wgrid, shift, tileBase, (int)wb, ws.hist, ws.binTotals, s,
                  ballot, true, tileStart, numTiles, allTiles);
        return 1;
    }
    TileStarts ts{};
    ts.numTiles = allTiles;
    ts.tileStart = tileStart;
    if (bits <= 8) {  // one pass, one bucket
        const int b = (int)(bits < 4 ? 4 : bits);
        if (!pass_fits(ws, false, b, grid, 256)) return kSortNoSpace;
        radix_pass(keys[0], vals[0], keys[1], vals[1], nPtr, grid, shift, b, ws.hist, ws.binTotals, s, ballot, &ts, true);
        return 1;
    }
    // radix_sort_bits' digit widths (balanced: 6 + 8 / 8 + 6 at 4K and 5 + 7 / 7 + 5 at 1080p measured slower)
    const uint32_t lo = (bits + 1u) / 2u;
    const uint32_t hi = bits - lo < 4u ? 4u : bits - lo;  // (a digit wider than the bits left reads zeros)
    // totals of the last pass at 0, the first pass's at +256, its bucket starts at +512 (<= 256 each)
    if (!pass_fits(ws, false, (int)lo, grid, 768) || !pass_fits(ws, false, (int)hi, grid, 768)) return kSortNoSpace;
    TileStarts first{};
    first.bucketStartOut = ws.binTotals + 512;
    const bool scanless = scanlessOn;
    radix_pass(keys[0], vals[0], keys[1], vals[1], nPtr, grid, shift, (int)lo, ws.hist, ws.binTotals + 256, s, ballot,
               &first, false, scanless ? 0 : -1);
    ts.bucketStart = ws.binTotals + 512;
    ts.lowBits = lo;
    radix_pass(keys[1], vals[1], keys[0], vals[0], nPtr, grid, shift + lo, (int)hi, ws.hist, ws.binTotals, s, ballot,
               &ts, true, scanless ? 1 : -1);
    return 0;
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
    uint32_t inc = wave_scan_incl(tot);
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
template <bool BALLOT>
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
            pos[j] = wave_rank<8, BALLOT>(cnt, d, valid, lt);
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
template <bool BALLOT>
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
        const uint32_t r = wave_rank<8, BALLOT>(wcnt[wave], d, valid, lt);
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

// The blend's half-tile lists (skip flags in the value word, k_scatter): one row of 256 sorted
// entries (position row * 256 + tid) per call, in position order; wave ballots give the ranks, `tot`
// (LDS) the per-wave counts, base0/base1 the entries of earlier rows.
__device__ __forceinline__ void ts_half_row(uint32_t v, bool valid, uint32_t (*tot)[kTsThreads / 64], uint32_t& base0,
                                            uint32_t& base1, uint32_t* __restrict__ h0, uint32_t* __restrict__ h1) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const bool k0 = valid && !((v >> kHalfSkipShift) & 1u);
    const bool k1 = valid && !((v >> (kHalfSkipShift + 1)) & 1u);
    const uint64_t m0 = __ballot(k0), m1 = __ballot(k1);
    if (lane == 0) {
        tot[0][wave] = (uint32_t)__popcll(m0);
        tot[1][wave] = (uint32_t)__popcll(m1);
    }
    __syncthreads();
    uint32_t o0 = base0, o1 = base1, a0 = 0, a1 = 0;
#pragma unroll
    for (uint32_t w = 0; w < kTsThreads / 64; ++w) {
        if (w < wave) {
            o0 += tot[0][w];
            o1 += tot[1][w];
        }
        a0 += tot[0][w];
        a1 += tot[1][w];
    }
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (k0) h0[o0 + (uint32_t)__popcll(m0 & lt)] = v & kGidMask;
    if (k1) h1[o1 + (uint32_t)__popcll(m1 & lt)] = v & kGidMask;
    base0 += a0;
    base1 += a1;
    __syncthreads();  // tot is rewritten by the next row
}

// One workgroup per tile (a persistent variant that prefetched the next tile's run was slower:
// the sort is bound by LDS round trips and barriers, so resident workgroups matter more than
// memory latency).  FULL: also write the sorted run (keys and values) -- the reference's sorted
// arrays, read back by captured frames only; the blend walks the half-tile lists alone.
template <bool BALLOT, bool FULL>
__global__ __launch_bounds__(kTsThreads) void k_tile_sort(
    uint32_t* __restrict__ keysIn, uint32_t* __restrict__ valsIn, uint32_t* __restrict__ keysOut,
    uint32_t* __restrict__ valsOut, const uint32_t* __restrict__ tileStart, uint32_t tileBegin,
    uint32_t* __restrict__ half0, uint32_t* __restrict__ half1, uint32_t* __restrict__ halfCount,
    uint32_t tileCount) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[kTsCap];
    __shared__ __attribute__((aligned(16))) uint32_t vbuf[kTsCap];  // the run's values in input order
    __shared__ __attribute__((aligned(16))) uint32_t wcnt[4][256];
    __shared__ uint32_t part[4];
    __shared__ uint32_t tot[2][kTsThreads / 64];
    __shared__ uint32_t rowTot[2][kTsItems][kTsThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t t = tileBegin + blockIdx.x;
    const uint32_t start = tileStart[t];
    const uint32_t n = tileStart[t + 1] - start;
    if (n == 0) {  // uniform: the whole workgroup leaves
        if (tid == 0) halfCount[t] = halfCount[tileCount + t] = 0;
        return;
    }
    if (n > kTsCap) {  // rare: the same two passes streamed through global memory
        uint32_t base0 = 0, base1 = 0;
        ts_pass_global<BALLOT>(keysIn + start, valsIn + start, keysOut + start, valsOut + start, n, 0, wcnt, part, buf);
        ts_pass_global<BALLOT>(keysOut + start, valsOut + start, keysIn + start, valsIn + start, n, 8, wcnt, part, buf);
        for (uint32_t b = 0; b < n; b += kTsThreads) {
            const uint32_t i = b + tid;
            uint32_t v = 0;
            if (i < n) {
                v = valsIn[start + i];
                if constexpr (FULL) {
                    keysOut[start + i] = keysIn[start + i];
                    valsOut[start + i] = v;
                }
            }
            ts_half_row(v, i < n, tot, base0, base1, half0 + start, half1 + start);
        }
        if (tid == 0) {
            halfCount[t] = base0;
            halfCount[tileCount + t] = base1;
        }
        return;
    }
    const uint32_t* kin = keysIn + start;
    const uint32_t* vin = valsIn + start;
    const uint32_t E = (n + kTsThreads - 1) / kTsThreads;  // items per thread
    const uint32_t seg = wave * 64u * E;                    // this wave's segment of the run
    uint32_t x[kTsItems], pos[kTsItems];
    // all of the run's keys and values in flight at once (one memory latency per tile): unpredicated loads
    // at clamped indices for the first 2, 4 or 8 items (E is uniform), masked afterwards -- a load under
    // `i < n` whose value was used under it went out alone with its own wait (one round trip per item,
    // r06).  Word = depth << 16 | position in the run; the values wait in LDS for the sorted positions.
    auto load_run = [&](auto ne) {
        constexpr uint32_t NE = decltype(ne)::value;
#pragma unroll
        for (uint32_t j = 0; j < NE; ++j) {
            const uint32_t i = min(seg + j * 64u + lane, n - 1u);
            x[j] = kin[i];
            pos[j] = vin[i];
        }
#pragma unroll
        for (uint32_t j = NE; j < kTsItems; ++j) x[j] = pos[j] = 0u;
    };
    if (E <= 2u) load_run(std::integral_constant<uint32_t, 2>{});
    else if (E <= 4u) load_run(std::integral_constant<uint32_t, 4>{});
    else load_run(std::integral_constant<uint32_t, kTsItems>{});
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        const uint32_t i = seg + j * 64u + lane;
        const bool ok = j < E && i < n;
        x[j] = ok ? ((x[j] & 0xFFFFu) << 16) | i : 0u;
        pos[j] = ok ? pos[j] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        const uint32_t i = seg + j * 64u + lane;
        if (j < E && i < n) vbuf[i] = pos[j];
    }
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    ts_rank_pass<BALLOT>(x, pos, E, seg, n, 16, wcnt, part);  // low depth byte
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
    // high depth byte: the atomic ranks stay faster than ballot matches even though a tile's depths
    // share few high bytes (r02, config 3: 66.1 against 80.7 us with ballot ranks for this pass)
    ts_rank_pass<BALLOT>(x, pos, E, seg, n, 24, wcnt, part);
    // the sorted run staged in LDS by position, then read in position order (row j = positions
    // j * 256 + tid): coalesced key and value stores when FULL, and the half-tile lists compacted
    // with one ballot per row and half and a single barrier for all rows
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j)
        if (j < E && seg + j * 64u + lane < n) buf[pos[j]] = x[j];
    __syncthreads();
    uint32_t* kout = keysOut + start;
    uint32_t* vout = valsOut + start;
    const uint32_t tileBits = t << 16;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t v[kTsItems], r0[kTsItems], r1[kTsItems];  // value, rank among the row's kept entries
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        if (j >= E) break;
        const uint32_t p = j * kTsThreads + tid;
        v[j] = 0;
        if (p < n) {
            const uint32_t w = buf[p];
            v[j] = vbuf[w & 0xFFFFu];
            if constexpr (FULL) {
                kout[p] = tileBits | (w >> 16);
                vout[p] = v[j];
            }
        }
        const bool k0 = p < n && !((v[j] >> kHalfSkipShift) & 1u);
        const bool k1 = p < n && !((v[j] >> (kHalfSkipShift + 1)) & 1u);
        const uint64_t m0 = __ballot(k0), m1 = __ballot(k1);
        r0[j] = k0 ? (uint32_t)__popcll(m0 & lt) : 0xFFFFFFFFu;
        r1[j] = k1 ? (uint32_t)__popcll(m1 & lt) : 0xFFFFFFFFu;
        if (lane == 0) {
            rowTot[0][j][wave] = (uint32_t)__popcll(m0);
            rowTot[1][j][wave] = (uint32_t)__popcll(m1);
        }
    }
    __syncthreads();
    uint32_t base0 = 0, base1 = 0;
#pragma unroll
    for (uint32_t j = 0; j < kTsItems; ++j) {
        if (j >= E) break;
        uint32_t o0 = base0, o1 = base1;
#pragma unroll
        for (uint32_t w = 0; w < kTsThreads / 64; ++w) {
            const uint32_t c0 = rowTot[0][j][w], c1 = rowTot[1][j][w];
            if (w < wave) {
                o0 += c0;
                o1 += c1;
            }
            base0 += c0;
            base1 += c1;
        }
        if (r0[j] != 0xFFFFFFFFu) half0[start + o0 + r0[j]] = v[j] & kGidMask;
        if (r1[j] != 0xFFFFFFFFu) half1[start + o1 + r1[j]] = v[j] & kGidMask;
    }
    if (tid == 0) {
        halfCount[t] = base0;
        halfCount[tileCount + t] = base1;
    }
}

void tile_depth_sort(uint32_t* keysIn, uint32_t* valsIn, uint32_t* keysOut, uint32_t* valsOut,
                     const uint32_t* tileStart, uint32_t tileBegin, uint32_t numTiles, hipStream_t s,
                     bool ballot, uint32_t* half0, uint32_t* half1, uint32_t* halfCount, uint32_t tileCount,
                     bool full, int numCUs) {
    if (numTiles == 0) return;
    (void)numCUs;
#define GSM_TILE_SORT(B, F)                                                                                  \
    hipLaunchKernelGGL((k_tile_sort<B, F>), dim3(numTiles), dim3(kTsThreads), 0, s, keysIn, valsIn, keysOut, \
                       valsOut, tileStart, tileBegin, half0, half1, halfCount, tileCount)
    if (ballot) {
        if (full) GSM_TILE_SORT(true, true);
        else GSM_TILE_SORT(true, false);
    } else {
        if (full) GSM_TILE_SORT(false, true);
        else GSM_TILE_SORT(false, false);
    }
#undef GSM_TILE_SORT
}

// ---------------------------------------------------------------------------
// Create-time probe of lane-ordered same-address LDS atomics (see wave_rank).  Every wave of a
// 64 x 256 grid runs 64 rounds; each round draws a digit per lane from a hash with 1, 2, 8 or 64
// distinct values (every lane on one address, pairs, ...), takes one ds_add_rtn_u32 per lane on
// freshly zeroed counters, and compares the returned value with the lane's rank among the
// earlier lanes of the same digit (ballot match, which needs no ordering property).  Mismatches
// are counted with a vector atomic in global memory.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rank_probe(uint32_t* __restrict__ mismatches) {
    __shared__ uint32_t cnt[4][64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t bad = 0;
    for (uint32_t round = 0; round < 64; ++round) {
        cnt[wave][lane] = 0;
        wave_sync();
        uint32_t h = (blockIdx.x * 0x9E3779B1u) ^ (round * 0x85EBCA6Bu) ^ (wave * 0xC2B2AE35u) ^ (lane * 0x27D4EB2Fu);
        h ^= h >> 15;
        h *= 0x2C1B3C6Du;
        h ^= h >> 12;
        const uint32_t mask = (round & 3u) == 0 ? 0u : ((round & 3u) == 1 ? 1u : ((round & 3u) == 2 ? 7u : 63u));
        const uint32_t d = h & mask;
        const uint32_t got = atomicAdd(&cnt[wave][d], 1u);
        const uint64_t peers = match_digit<6>(d, true);
        if (got != (uint32_t)__popcll(peers & lt)) bad++;
        wave_sync();
    }
    if (bad) atomicAdd(mismatches, bad);
}

bool sort_lane_ordered_atomics(int device) {
    static std::mutex mu;
    static std::unordered_map<int, bool> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(device);
    if (it != cache.end()) return it->second;
    bool ok = false;
    uint32_t* d = nullptr;
    int prev = 0;
    hipGetDevice(&prev);
    // on a private non-blocking stream, synchronised alone: no other stream of the caller's process
    // waits for the probe (a renderer create or a first gsm_sort_pairs_u32 call never stalls the device)
    hipStream_t ps = nullptr;
    if (hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&ps, hipStreamNonBlocking) == hipSuccess &&
        hipMalloc(&d, 4) == hipSuccess) {
        uint32_t h = 1;
        if (hipMemsetAsync(d, 0, 4, ps) == hipSuccess) {
            hipLaunchKernelGGL(k_rank_probe, dim3(64), dim3(256), 0, ps, d);
            if (hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, ps) == hipSuccess && hipStreamSynchronize(ps) == hipSuccess)
                ok = h == 0;
        }
    }
    if (d) hipFree(d);
    if (ps) hipStreamDestroy(ps);
    (void)hipGetLastError();
    hipSetDevice(prev);
    cache[device] = ok;
    return ok;
}

Tuning tuning_from_env(int device) {
    Tuning t;
    const char* sv = getenv("GSM_SORT");
    t.fullRadix = sv && std::strcmp(sv, "radix4") == 0;
    const char* rv = getenv("GSM_SORT_RANK");
    t.ballotRank = (rv && std::strcmp(rv, "ballot") == 0) || !sort_lane_ordered_atomics(device);
    const char* bv = getenv("GSM_BLEND_SCHED");
    t.costOrder = !(bv && bv[0] == '0');
    const char* wv = getenv("GSM_BLEND_WAVES");
    const int w = wv ? atoi(wv) : 0;
    t.blendWaves = (w == 8 || w == 12 || w == 16) ? w : 0;
    const char* cv = getenv("GSM_BLEND_CLAIM");
    t.blendClaim = !cv ? 1 : std::strcmp(cv, "early") == 0 ? 0 : std::strcmp(cv, "auto") == 0 ? 2 : 1;
    const char* ws = getenv("GSM_SORT_WIDE");
    t.wideSort = !(ws && ws[0] == '0');
    const char* sc = getenv("GSM_SORT_SCAN");
    t.sortScanless = !(sc && std::strcmp(sc, "kernel") == 0);
    const char* bp = getenv("GSM_BLEND_PAIRS");
    t.blendPairs = !(bp && bp[0] == '0');
    const char* ps = getenv("GSM_BLEND_PAIR_SPLIT");
    if (ps) t.pairBucket = std::min(256, std::max(0, atoi(ps)));
    const char* fs = getenv("GSM_SCAN_FUSED");
    t.fusedScan = !(fs && fs[0] == '0');
    return t;
}

}  // namespace gsm
