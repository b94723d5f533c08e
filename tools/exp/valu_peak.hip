// Probe (not part of the product): the VALU issue peak that prices the blend's roofline_valu.
//
// Every wave runs ITERS x 16 copies of ONE vector instruction on 8 independent accumulators
// (inline asm, so the count and the opcode are exact), with 1, 2, 4 and 8 waves per SIMD on every
// CU.  Reported per (instruction, waves/SIMD): chip-wide wave-instructions per ns (HIP events over
// the launch) and the implied cycles per instruction per SIMD at the clock measured in-kernel from
// s_memtime (shader clock) against s_memrealtime (100 MHz constant).
//   hipcc --offload-arch=gfx950 -O3 -o valu_peak valu_peak.hip && ./valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 2048;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void k_peak(unsigned* out, unsigned long long* clk) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    const unsigned m = 0x3C003C01u, c = 0x00010001u;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {(float)threadIdx.x, 1.f}, p1 = p0 + 1.f, p2 = p0 + 2.f, p3 = p0 + 3.f, p4 = p0 + 4.f, p5 = p0 + 5.f,
       p6 = p0 + 6.f, p7 = p0 + 7.f;
    const f2 pm = {0.999f, 1.001f}, pc = {0.5f, 0.25f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int rep = 0; rep < 2; ++rep) {
#define ACC(i)                                                                                                 \
    if (OP == 0) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(a##i) : "v"(m));                              \
    if (OP == 1) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a##i) : "v"(m));                              \
    if (OP == 2) asm volatile("v_pk_fma_f16 %0, %0, %1, %2" : "+v"(a##i) : "v"(m), "v"(c));                  \
    if (OP == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a##i) : "v"(m));                                 \
    if (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a##i) : "v"(m), "v"(c));                     \
    if (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(m));                                 \
    if (OP == 6) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a##i) : "v"(m));                              \
    if (OP == 7) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p##i) : "v"(pm));                             \
    if (OP == 8) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p##i) : "v"(pm), "v"(pc));               \
    if (OP == 9) asm volatile("v_add_f16 %0, %0, %1" : "+v"(a##i) : "v"(m));                                 \
    if (OP == 10) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(m), "v"(c));                   \
    if (OP == 11) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(m));  /* VCC never written */ \
    if (OP == 12) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a##i)); \
    if (OP == 13) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(a##i));                                          \
    if (OP == 14) asm volatile("v_exp_f32 %0, %0" : "+v"(a##i));                                              \
    if (OP == 15) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a##i) : "v"(m));                                \
    if (OP == 16) asm volatile("v_div_scale_f32 %0, vcc, %0, %1, %0" : "+v"(a##i) : "v"(m) : "vcc");         \
    if (OP == 17) asm volatile("v_div_fmas_f32 %0, %0, %1, %2" : "+v"(a##i) : "v"(m), "v"(c));               \
    if (OP == 18) asm volatile("v_div_fixup_f32 %0, %0, %1, %2" : "+v"(a##i) : "v"(m), "v"(c));              \
    if (OP == 19) asm volatile("v_rcp_f32 %0, %0" : "+v"(a##i));                                              \
    if (OP == 20) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a##i));                                             \
    if (OP == 21) asm volatile("v_fma_mix_f32 %0, %0, %1, %2 op_sel_hi:[0,1,0]" : "+v"(a##i) : "v"(m), "v"(c)); \
    if (OP == 22) asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(a##i));                                          \
    if (OP == 23) asm volatile("v_cndmask_b32 %0, %0, %1, s[0:1]" : "+v"(a##i) : "v"(m) : "s0", "s1");        \
    if (OP == 24) asm volatile("v_cmp_gt_f32 s[0:1], %0, %1" : : "v"(a##i), "v"(m) : "s0", "s1");             \
    if (OP == 25) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a##i) : "v"(m));                   \
    if (OP == 26) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(m) : "vcc"); \
    if (OP == 27) asm volatile("v_cmp_gt_f32_e64 s[" #i "*2+16:" #i "*2+17], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[" #i "*2+16:" #i "*2+17]" \
                               : "+v"(a##i) : "v"(m) : "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31"); \
    if (OP == 28) asm volatile("v_sub_f32 %0, %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(a##i) : "v"(m) : "s0", "s1"); \
    if (OP == 29) asm volatile("v_cmp_class_f32_e64 s[" #i "*2+16:" #i "*2+17], %0, %1" : : "v"(a##i), "v"(m) \
                               : "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31");
            REP8(ACC)
#undef ACC
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const f2 ps = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (unsigned)(ps.x + ps.y);
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int OP>
static void run(const char* name, int cus, unsigned* out, unsigned long long* clk, int perAcc = 1) {
    for (int wps = 1; wps <= 8; wps *= 2) {
        // waves per CU = 4 * wps, in workgroups of at most 1024 threads
        const int threads = 64 * 4 * wps;
        const int block = threads > 1024 ? 1024 : threads;
        const int perCU = threads / block;
        const dim3 grid(cus * perCU);
        float best = 1e30f;
        double ghz = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k_peak<OP>, grid, dim3(block), 0, 0, out, clk);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) {
                best = ms;
                unsigned long long h[2];
                hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
                ghz = (double)h[0] / ((double)h[1] * 10.0);  // s_memtime ticks per ns (memrealtime 100 MHz)
            }
            hipEventDestroy(a);
            hipEventDestroy(b);
        }
        const double waveInstr = (double)grid.x * (block / 64) * ITERS * 16.0 * perAcc;
        const double perNs = waveInstr / (best * 1e6);
        const double simds = cus * 4.0;
        // cycles per wave-instruction per SIMD at the in-kernel clock
        const double cyc = simds * ghz / perNs;
        printf("%-14s waves/SIMD=%d  %8.1f G wave-instr/s  clock %.2f GHz  %5.2f cycles/instr/SIMD\n", name, wps,
               perNs, ghz, cyc);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)cus * 2048 * 4);
    hipMalloc(&clk, (size_t)cus * 2 * 16);
    printf("%s, %d CUs\n", p.name, cus);
    run<0>("v_pk_mul_f16", cus, out, clk);
    run<1>("v_pk_add_f16", cus, out, clk);
    run<2>("v_pk_fma_f16", cus, out, clk);
    run<3>("v_mul_f32", cus, out, clk);
    run<4>("v_fma_f32", cus, out, clk);
    run<5>("v_add_u32", cus, out, clk);
    run<6>("v_pk_max_u16", cus, out, clk);
    run<7>("v_pk_mul_f32", cus, out, clk);
    run<8>("v_pk_fma_f32", cus, out, clk);
    run<9>("v_add_f16", cus, out, clk);
    run<10>("v_perm_b32", cus, out, clk);
    run<11>("v_cndmask_b32", cus, out, clk);
    run<12>("v_mov_b32_dpp", cus, out, clk);
    run<13>("v_cvt_f32_f16", cus, out, clk);
    run<14>("v_exp_f32", cus, out, clk);
    run<15>("v_max_u32", cus, out, clk);
    run<16>("v_div_scale_f32", cus, out, clk);
    run<17>("v_div_fmas_f32", cus, out, clk);
    run<18>("v_div_fixup_f32", cus, out, clk);
    run<19>("v_rcp_f32", cus, out, clk);
    run<20>("v_sqrt_f32", cus, out, clk);
    run<21>("v_fma_mix_f32", cus, out, clk);
    run<22>("v_cvt_f16_f32", cus, out, clk);
    run<23>("v_cndmask_b32_sgpr", cus, out, clk);
    run<24>("v_cmp_gt_f32", cus, out, clk);
    run<25>("v_cndmask_e64_vcc", cus, out, clk);
    run<26>("cmp_e32+cndmask_vcc", cus, out, clk, 2);
    run<27>("cmp_e64+cndmask_sN", cus, out, clk, 2);
    run<28>("sub+cndmask_s01", cus, out, clk, 2);
    run<29>("v_cmp_class_e64", cus, out, clk);
    return 0;
}
