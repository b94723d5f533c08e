// Probe (not part of the product): uncached device memory (hipDeviceMallocUncached) allocated and
// freed in groups the way the multi-GPU exchange does it (one allocation per virtual rank, freed at
// the end of a case, sizes 1.9-6 MB): are words written by one kernel read back by the next kernel
// of the same stream?  (uncached exchange memory rendered wrong virtual-rank slabs.)
// Per allocation size: 8 rounds x 8 allocations, every 16-B word written by a grid-stride kernel,
// then checked by a second kernel (plain loads) and a third (system-coherent sc0 sc1 loads); the
// same for fine-grained memory as the control.
//   hipcc --offload-arch=gfx950 -O3 -o uc_alloc_probe uc_alloc_probe.hip && ./uc_alloc_probe
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
__global__ void k_fill(uint4* p, unsigned words, unsigned salt) {
    for (unsigned w = blockIdx.x * blockDim.x + threadIdx.x; w < words; w += gridDim.x * blockDim.x) {
        const unsigned h = hash(w ^ salt);
        p[w] = make_uint4(h, h + 1, h + 2, h + 3);
    }
}
template <bool SYS>
__global__ void k_check(const uint4* p, unsigned words, unsigned salt, unsigned* bad) {
    unsigned c = 0;
    for (unsigned w = blockIdx.x * blockDim.x + threadIdx.x; w < words; w += gridDim.x * blockDim.x) {
        const unsigned h = hash(w ^ salt);
        uint4 v;
        if (SYS) {
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(
                __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), 0, (int)(words * 16u), 0x00020000), (int)(w * 16u), 0, 17);
            v = make_uint4(r[0], r[1], r[2], r[3]);
        } else {
            v = p[w];
        }
        c += (v.x != h) + (v.y != h + 1) + (v.z != h + 2) + (v.w != h + 3);
    }
    if (c) atomicAdd(bad, c);
}

int main() {
    const size_t sizes[] = {1920000 + 4096, 2400000 + 4096, 2880000 + 4096, 4u << 20, (6u << 20) + 4096};
    unsigned* bad = nullptr;
    CK(hipMalloc(&bad, 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int kind = 0; kind < 2; ++kind) {
        for (size_t bytes : sizes) {
            unsigned badPlain = 0, badSys = 0;
            for (int round = 0; round < 8; ++round) {
                void* a[8];
                for (int i = 0; i < 8; ++i)
                    CK(hipExtMallocWithFlags(&a[i], bytes, kind == 0 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
                CK(hipMemsetAsync(bad, 0, 8, s));
                const unsigned words = (unsigned)(bytes / 16);
                for (int i = 0; i < 8; ++i)
                    hipLaunchKernelGGL(k_fill, dim3(512), dim3(256), 0, s, (uint4*)a[i], words, (unsigned)(round * 8 + i));
                for (int i = 0; i < 8; ++i) {
                    hipLaunchKernelGGL(k_check<false>, dim3(512), dim3(256), 0, s, (const uint4*)a[i], words,
                                       (unsigned)(round * 8 + i), bad);
                    hipLaunchKernelGGL(k_check<true>, dim3(512), dim3(256), 0, s, (const uint4*)a[i], words,
                                       (unsigned)(round * 8 + i), bad + 1);
                }
                unsigned b[2];
                CK(hipMemcpyAsync(b, bad, 8, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                badPlain += b[0];
                badSys += b[1];
                for (int i = 0; i < 8; ++i) CK(hipFree(a[i]));
            }
            std::printf("%-12s %8zu B x 8 allocations x 8 rounds: wrong 4-B words, plain loads %u, sc0 sc1 loads %u\n",
                        kind == 0 ? "uncached" : "fine-grained", bytes, badPlain, badSys);
        }
    }
    return 0;
}
