// Probe (not part of the product): rocPRIM's device radix sort on the frame's key shape, to
// calibrate what an LSD sort of 2.63M (key, value) pairs can reach on gfx950.
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 2632483;
    const int endBit = argc > 2 ? atoi(argv[2]) : 28;
    std::vector<uint32_t> hk(n), hv(n);
    std::mt19937 rng(1);
    for (size_t i = 0; i < n; ++i) { hk[i] = rng() & ((1u << endBit) - 1u); hv[i] = (uint32_t)i; }
    uint32_t *k0, *k1, *v0, *v1;
    hipMalloc(&k0, n * 4); hipMalloc(&k1, n * 4); hipMalloc(&v0, n * 4); hipMalloc(&v1, n * 4);
    hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice);
    size_t tmp = 0;
    rocprim::radix_sort_pairs(nullptr, tmp, k0, k1, v0, v1, n, 0, endBit);
    void* t; hipMalloc(&t, tmp);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) rocprim::radix_sort_pairs(t, tmp, k0, k1, v0, v1, n, 0, endBit);
    const int reps = 50;
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) rocprim::radix_sort_pairs(t, tmp, k0, k1, v0, v1, n, 0, endBit);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    std::vector<uint32_t> out(n);
    hipMemcpy(out.data(), k1, n * 4, hipMemcpyDeviceToHost);
    bool ok = true;
    for (size_t i = 1; i < n; ++i) ok &= out[i - 1] <= out[i];
    printf("{\"n\": %zu, \"end_bit\": %d, \"us\": %.2f, \"gkeys_s\": %.2f, \"sorted\": %s}\n", n, endBit,
           ms / reps * 1000.0, n / (ms / reps * 1e-3) / 1e9, ok ? "true" : "false");
    return ok ? 0 : 1;
}
