// Probe (not part of the product): do stores from different workgroups into the same 64-B segment of
// UNCACHED device memory (hipDeviceMallocUncached) lose each other's bytes, where fine-grained and
// ordinary device memory keep them?  (uncached exchange memory rendered wrong
// virtual-rank slabs; the records of one slab are runs of 48-B records written by many workgroups,
// so a run boundary falls inside a segment that two workgroups write at about the same time.)
// Patterns, each over a 64 MiB buffer, every word checked after the kernel:
//   0  16-B words dealt round robin over the workgroups (neighbouring words: different CUs)
//   1  4-B words dealt round robin over the workgroups
//   2  runs of 3 x 16 B (one 48-B record per thread, consecutive threads' records adjacent) -- the
//      k_part_push layout, every run boundary inside a 64-B segment
//   3  the same records, each written by ONE workgroup as whole 64-B segments where possible (control)
//   hipcc --offload-arch=gfx950 -O3 -o uc_write_probe uc_write_probe.hip && ./uc_write_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x | 1u;
}
__global__ void k_write16_rr(uint4* p, unsigned words) {  // word w by block w % G
    const unsigned G = gridDim.x;
    for (unsigned k = threadIdx.x; ; k += blockDim.x) {
        const unsigned w = k * G + blockIdx.x;
        if (w >= words) break;
        const unsigned h = hash(w);
        p[w] = make_uint4(h, h + 1, h + 2, h + 3);
    }
}
__global__ void k_write4_rr(unsigned* p, unsigned words) {
    const unsigned G = gridDim.x;
    for (unsigned k = threadIdx.x; ; k += blockDim.x) {
        const unsigned w = k * G + blockIdx.x;
        if (w >= words) break;
        p[w] = hash(w);
    }
}
// record r (3 x 16 B) written by thread r: consecutive records of a block are adjacent, and the
// first / last records of neighbouring blocks share 64-B segments
__global__ void k_write_records(uint4* p, unsigned records) {
    const unsigned r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= records) return;
    for (unsigned j = 0; j < 3; ++j) {
        const unsigned w = 3 * r + j, h = hash(w);
        p[w] = make_uint4(h, h + 1, h + 2, h + 3);
    }
}
// the same words, consecutive threads of ONE block storing consecutive 16-B words (whole segments)
__global__ void k_write_records_block(uint4* p, unsigned records) {
    const unsigned base = blockIdx.x * blockDim.x * 3u, n = min(records * 3u - min(base, records * 3u), blockDim.x * 3u);
    for (unsigned j = threadIdx.x; j < n; j += blockDim.x) {
        const unsigned w = base + j, h = hash(w);
        p[w] = make_uint4(h, h + 1, h + 2, h + 3);
    }
}
__global__ void k_check16(const uint4* p, unsigned words, unsigned* bad) {
    unsigned c = 0;
    for (unsigned w = blockIdx.x * blockDim.x + threadIdx.x; w < words; w += gridDim.x * blockDim.x) {
        const unsigned h = hash(w);
        const uint4 v = p[w];
        c += (v.x != h) + (v.y != h + 1) + (v.z != h + 2) + (v.w != h + 3);
    }
    if (c) atomicAdd(bad, c);
}
__global__ void k_check4(const unsigned* p, unsigned words, unsigned* bad) {
    unsigned c = 0;
    for (unsigned w = blockIdx.x * blockDim.x + threadIdx.x; w < words; w += gridDim.x * blockDim.x) c += p[w] != hash(w);
    if (c) atomicAdd(bad, c);
}

int main() {
    const size_t bytes = 64ull << 20;
    unsigned* bad = nullptr;
    CK(hipMalloc(&bad, 4));
    const char* names[3] = {"uncached", "fine-grained", "device (hipMalloc)"};
    for (int kind = 0; kind < 3; ++kind) {
        for (int pat = 0; pat < 4; ++pat) {
            unsigned total = 0;
            for (int rep = 0; rep < 4; ++rep) {
                void* p = nullptr;
                if (kind == 2) CK(hipMalloc(&p, bytes));
                else CK(hipExtMallocWithFlags(&p, bytes, kind == 0 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
                CK(hipMemset(p, 0, bytes));
                CK(hipMemset(bad, 0, 4));
                const unsigned w16 = (unsigned)(bytes / 16), w4 = (unsigned)(bytes / 4), recs = w16 / 3;
                if (pat == 0) hipLaunchKernelGGL(k_write16_rr, dim3(2048), dim3(256), 0, 0, (uint4*)p, w16);
                if (pat == 1) hipLaunchKernelGGL(k_write4_rr, dim3(2048), dim3(256), 0, 0, (unsigned*)p, w4);
                if (pat == 2) hipLaunchKernelGGL(k_write_records, dim3((recs + 255) / 256), dim3(256), 0, 0, (uint4*)p, recs);
                if (pat == 3) hipLaunchKernelGGL(k_write_records_block, dim3((recs + 255) / 256), dim3(256), 0, 0, (uint4*)p, recs);
                CK(hipDeviceSynchronize());
                if (pat == 1) hipLaunchKernelGGL(k_check4, dim3(2048), dim3(256), 0, 0, (const unsigned*)p, w4, bad);
                else hipLaunchKernelGGL(k_check16, dim3(2048), dim3(256), 0, 0, (const uint4*)p, pat >= 2 ? recs * 3 : w16, bad);
                unsigned b = 0;
                CK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
                total += b;
                CK(hipFree(p));
            }
            std::printf("%-20s pattern %d: wrong 4-B words after the kernel, 4 reps of 64 MiB: %u\n", names[kind], pat, total);
        }
    }
    return 0;
}
