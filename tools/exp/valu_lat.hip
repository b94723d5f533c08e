// Probe (not part of the product): dependent-issue latency of v_pk_mul_f16 / v_pk_add_f16 /
// v_pk_max_u16 / v_perm_b32 on gfx950: NC independent chains interleaved in program order (inline
// asm keeps the order), 1 wave per SIMD and 2 waves per SIMD.  Cycles per instruction from
// s_memtime (one wave) and from wall time.
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP1(i) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(a[i]) : "v"(m));
template <int NC>
__global__ void k_lat(unsigned* out, int iters, unsigned long long* cyc) {
    unsigned a[8];
    for (int k = 0; k < 8; ++k) a[k] = 0x3c003c00u + threadIdx.x + k;
    unsigned m = 0x3bff3c01u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 32 / NC; ++r) {
#pragma unroll
            for (int c = 0; c < NC; ++c) OP1(c)
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
    for (int k = 0; k < 8; ++k) s ^= a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, 1024 * 1024 * 4);
    hipMalloc(&cyc, 4096 * 8);
    const int iters = 8192;
    for (int wps = 1; wps <= 4; wps *= 2)
        for (int nc = 1; nc <= 8; nc *= 2) {
            dim3 grid(cus), block(256 * wps);
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                hipEvent_t a, b;
                hipEventCreate(&a);
                hipEventCreate(&b);
                hipEventRecord(a);
                if (nc == 1) hipLaunchKernelGGL(k_lat<1>, grid, block, 0, 0, out, iters, cyc);
                if (nc == 2) hipLaunchKernelGGL(k_lat<2>, grid, block, 0, 0, out, iters, cyc);
                if (nc == 4) hipLaunchKernelGGL(k_lat<4>, grid, block, 0, 0, out, iters, cyc);
                if (nc == 8) hipLaunchKernelGGL(k_lat<8>, grid, block, 0, 0, out, iters, cyc);
                hipEventRecord(b);
                hipEventSynchronize(b);
                hipEventElapsedTime(&ms, a, b);
            }
            unsigned long long c0;
            hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
            const double n = (double)iters * 32;
            printf("waves/SIMD %d chains %d: wave0 %.2f memtime-cyc/instr; SIMD wall %.2f ns/instr (%.2f cyc @2.4GHz per wave-instr per SIMD)\n",
                   wps, nc, c0 / n, ms * 1e6 / (n * wps), ms * 1e-3 * 2.4e9 / (n * wps));
        }
    return 0;
}
