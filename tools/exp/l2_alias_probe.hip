// Probe (not part of the product): does memory that was written through a cached (L2 write-back)
// mapping, freed, and re-allocated as UNCACHED memory keep dirty L2 lines that are written back
// later, over data stored through the uncached mapping?  And does a system-scope release run on
// every XCD (buffer_wbl2 on each L2) right after the allocation prevent it?
//   hipcc --offload-arch=gfx950 -O3 -o l2_alias_probe l2_alias_probe.hip && ./l2_alias_probe
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

__global__ void k_fill(unsigned* p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void k_churn(unsigned* p, size_t n) {  // read-modify-write a large buffer: evicts the L2s
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = p[i] * 3u + 1u;
}
__global__ void k_count(const unsigned* p, size_t n, unsigned v, unsigned* bad) {
    unsigned c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += p[i] != v;
    if (c) atomicAdd(bad, c);
}
// every block: system-scope release + acquire on the L2 of the XCD it runs on (blocks are dealt
// round robin over the 8 XCDs, so 64 blocks reach every L2 several times)
__global__ void k_flush_l2() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
}

int main() {
    const size_t bytes = 64ull << 20, n = bytes / 4;
    unsigned *bad = nullptr, *churn = nullptr;
    CK(hipMalloc(&bad, 4));
    CK(hipMalloc(&churn, 512ull << 20));
    CK(hipMemset(churn, 0, 512ull << 20));
    for (int mode = 0; mode < 4; ++mode) {  // mode 1, 3: flush after the allocation; 2, 3: 8 rounds
        unsigned total = 0, reused = 0;
        const int rounds = mode >= 2 ? 8 : 4;
        for (int r = 0; r < rounds; ++r) {
            unsigned* a = nullptr;
            CK(hipMalloc(&a, bytes));
            hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, a, n, 0x11111111u);  // dirty lines in the L2s
            CK(hipDeviceSynchronize());
            CK(hipFree(a));
            unsigned* u = nullptr;
            CK(hipExtMallocWithFlags((void**)&u, bytes, hipDeviceMallocUncached));
            reused += (u == a);
            if (mode & 1) {
                hipLaunchKernelGGL(k_flush_l2, dim3(64), dim3(64), 0, 0);
                CK(hipDeviceSynchronize());
            }
            hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, u, n, 0x22222222u);
            hipLaunchKernelGGL(k_churn, dim3(4096), dim3(256), 0, 0, churn, (512ull << 20) / 4);
            CK(hipMemset(bad, 0, 4));
            hipLaunchKernelGGL(k_count, dim3(2048), dim3(256), 0, 0, u, n, 0x22222222u, bad);
            unsigned b = 0;
            CK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
            total += b;
            CK(hipFree(u));
        }
        std::printf("mode %d (%s): %d rounds, uncached allocation at the freed address %u times, "
                    "words clobbered after the uncached fill: %u\n", mode, (mode & 1) ? "L2 flush after alloc" : "no flush",
                    rounds, reused, total);
    }
    return 0;
}
