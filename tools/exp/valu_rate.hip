// Probe (not part of the product): wave64 VALU issue rate on gfx950 for the instruction mix of
// the blend (v_pk_mul_f16 / v_pk_add_f16 chains, v_readlane, random ds_read_u16), at 1..8 waves
// per SIMD.  Prints cycles per wave-instruction per SIMD (clock from s_memtime deltas).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(1024) void k_rate(float* out, int iters, unsigned long long* cyc) {
    __shared__ unsigned short tbl[32768];
    for (int i = threadIdx.x; i < 32768; i += blockDim.x) tbl[i] = (unsigned short)(i * 7);
    __syncthreads();
    h2 a[8];
    for (int k = 0; k < 8; ++k) a[k] = h2{(_Float16)(threadIdx.x * 0.001f + k), (_Float16)(k * 0.5f)};
    const h2 m = {(_Float16)0.999f, (_Float16)1.001f};
    const h2 c = {(_Float16)0.01f, (_Float16)0.02f};
    unsigned idx = threadIdx.x * 2654435761u;
    unsigned acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {  // 16 independent pk ops per iteration (8 mul + 8 add)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = a[k] * m;
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = a[k] + c;
        } else if (MODE == 1) {  // dependent chain of 16 pk ops on one accumulator... x8 chains interleaved? no: 2 chains
#pragma unroll
            for (int k = 0; k < 8; ++k) { a[0] = a[0] * m; a[1] = a[1] + c; }
        } else if (MODE == 2) {  // 8 random ds_read_u16 + 8 pk ops
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                idx = idx * 1664525u + 1013904223u;
                acc += tbl[(idx >> 17) & 32767];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = a[k] * m;
        } else {  // 8 readlanes feeding pk ops
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                unsigned s = __builtin_amdgcn_readlane(__builtin_bit_cast(unsigned, a[k]), (it + k) & 63);
                a[k] = a[k] * __builtin_bit_cast(h2, s);
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = (float)acc;
    for (int k = 0; k < 8; ++k) s += (float)a[k].x + (float)a[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int cus = 256;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    cus = p.multiProcessorCount;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 1024 * 4096 * 4);
    hipMalloc(&cyc, 4096 * 8);
    const int iters = 4096;
    const char* names[4] = {"16 indep pk ops", "2 dep chains pk", "8 ds_read_u16 rnd + 8 pk", "8 readlane+8 pk"};
    const int instrs[4] = {16, 16, 16, 16};
    for (int mode = 0; mode < 4; ++mode)
        for (int wps = 1; wps <= 8; wps *= 2) {
            dim3 grid(cus), block(64 * 4 * wps);
            for (int rep = 0; rep < 2; ++rep) {
                hipEvent_t a, b;
                hipEventCreate(&a);
                hipEventCreate(&b);
                hipEventRecord(a);
                if (mode == 0) hipLaunchKernelGGL(k_rate<0>, grid, block, 0, 0, out, iters, cyc);
                if (mode == 1) hipLaunchKernelGGL(k_rate<1>, grid, block, 0, 0, out, iters, cyc);
                if (mode == 2) hipLaunchKernelGGL(k_rate<2>, grid, block, 0, 0, out, iters, cyc);
                if (mode == 3) hipLaunchKernelGGL(k_rate<3>, grid, block, 0, 0, out, iters, cyc);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                unsigned long long c0;
                hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
                if (rep == 1) {
                    // per SIMD: wps waves, each iters*instrs wave-instructions
                    double winstr = (double)wps * iters * instrs[mode];
                    printf("%-26s waves/SIMD %d: %.2f ms, memtime %.0f cyc -> %.2f memtime-cyc per wave-instr per SIMD; "
                           "at 2.4 GHz wall: %.2f cyc\n",
                           names[mode], wps, ms, (double)c0, c0 / winstr, ms * 1e-3 * 2.4e9 / winstr);
                }
            }
        }
    return 0;
}
