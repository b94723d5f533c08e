// Probe (not part of the product): throughput of device-scope global atomicAdd (no return) on
// M distinct addresses, N atomics spread over the whole grid, as a function of M.  Decides whether
// histogram fusions that replace a kernel pass by global atomics can pay on MI355X.
//   hipcc --offload-arch=gfx950 -O3 -o atomic_rate atomic_rate.hip && ./atomic_rate
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_atomics(unsigned* __restrict__ hist, unsigned m, unsigned n, unsigned perThread) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned i = 0; i < perThread; ++i) {
        const unsigned e = t * perThread + i;
        if (e >= n) return;
        unsigned h = e * 0x9E3779B1u;
        h ^= h >> 15;
        atomicAdd(&hist[h % m], 1u);
    }
}

__global__ void k_stores(unsigned* __restrict__ hist, unsigned m, unsigned n, unsigned perThread) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned i = 0; i < perThread; ++i) {
        const unsigned e = t * perThread + i;
        if (e >= n) return;
        unsigned h = e * 0x9E3779B1u;
        h ^= h >> 15;
        hist[h % m] = e;
    }
}

int main() {
    unsigned* hist;
    hipMalloc(&hist, 64u << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const unsigned ms[] = {16384u, 102400u, 1u << 20, 8u << 20};
    const unsigned ns[] = {250000u, 2500000u, 13000000u};
    for (int kind = 0; kind < 2; ++kind)
        for (unsigned m : ms)
            for (unsigned n : ns) {
                const unsigned per = 4, threads = (n + per - 1) / per, grid = (threads + 255) / 256;
                float best = 1e30f;
                for (int r = 0; r < 3; ++r) {
                    hipMemset(hist, 0, (size_t)m * 4);
                    hipEventRecord(a);
                    if (kind == 0) hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(256), 0, 0, hist, m, n, per);
                    else hipLaunchKernelGGL(k_stores, dim3(grid), dim3(256), 0, 0, hist, m, n, per);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms_ = 0;
                    hipEventElapsedTime(&ms_, a, b);
                    if (ms_ < best) best = ms_;
                }
                printf("%-8s m=%9u n=%9u  %8.1f us  %7.1f G/s\n", kind == 0 ? "atomic" : "store", m, n, best * 1e3,
                       n / (best * 1e6));
            }
    return 0;
}
