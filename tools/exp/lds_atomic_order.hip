// Probe (not part of the product): order in which the lanes of ONE ds_add_rtn_u32 wave
// instruction that hit the same LDS address receive their return values on gfx950.
// Reports whether the returned values increase with the lane id for every address.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_probe(const unsigned* digits, unsigned* rets, int bins) {
    __shared__ unsigned cnt[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned d = digits[gid] % bins;
    // one wave-wide instruction: all lanes of the wave issue this atomic together
    rets[gid] = atomicAdd(&cnt[d + (threadIdx.x >> 6) * 0], 1u);
}

int main() {
    const int waves = 4096, n = waves * 64;
    std::vector<unsigned> h(n);
    unsigned s = 12345;
    unsigned* dd; unsigned* rr;
    hipMalloc(&dd, n * 4); hipMalloc(&rr, n * 4);
    std::vector<unsigned> ret(n);
    for (int bins : {1, 2, 4, 16, 64, 256}) {
        for (int i = 0; i < n; ++i) { s = s * 1664525u + 1013904223u; h[i] = s >> 8; }
        hipMemcpy(dd, h.data(), n * 4, hipMemcpyHostToDevice);
        // one wave per block: the per-block counters start at 0 for each wave
        hipLaunchKernelGGL(k_probe, dim3(waves), dim3(64), 0, 0, dd, rr, bins);
        hipMemcpy(ret.data(), rr, n * 4, hipMemcpyDeviceToHost);
        long inorder = 0, pairs = 0, reverse = 0;
        for (int w = 0; w < waves; ++w)
            for (int a = 0; a < 64; ++a)
                for (int b = a + 1; b < 64; ++b) {
                    const int i = w * 64 + a, j = w * 64 + b;
                    if (h[i] % bins != h[j] % bins) continue;
                    pairs++;
                    if (ret[i] < ret[j]) inorder++; else reverse++;
                }
        printf("bins %3d: same-address lane pairs %ld, lower lane got lower value %ld, reverse %ld\n", bins, pairs, inorder, reverse);
    }
    return 0;
}
