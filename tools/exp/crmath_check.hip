// Probe (not part of the product; r06): cheaper correctly rounded fp32 square root and
// reciprocal sequences for k_project, checked bit for bit against the compiler's IEEE sequences
// (-fhip-fp32-correctly-rounded-divide-sqrt, the numeric contract of DESIGN.md 3) over EVERY 32-bit input.
//   sqrt_nb   v_sqrt_f32 + the two-neighbour residual test of the IEEE sequence, without its tiny-input
//             scaling and its special-class select (15 -> 9 VALU)
//   sqrt_rsq  v_rsq_f32, s = x r, one fma residual step s + (x - s s) r / 2 (5 VALU)
//   rcp_nr    v_rcp_f32 + one fma Newton step r + r (1 - b r) (3 VALU against 9 for 1.0f / b)
// Per sequence and input class (+normal, +subnormal, +-0, +inf, NaN, negative): inputs whose result bits
// differ from the IEEE sequence's, and the first few of them.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -o crmath_check crmath_check.hip && ./crmath_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

constexpr int kSeq = 3, kClass = 6;

__device__ __forceinline__ int cls(uint32_t u) {
    const uint32_t a = u & 0x7FFFFFFFu;
    if (a > 0x7F800000u) return 4;         // NaN
    if (u >> 31) return a == 0 ? 2 : 5;    // -0 / negative
    if (a == 0x7F800000u) return 3;        // +inf
    if (a == 0) return 2;                  // +0
    return a < 0x00800000u ? 1 : 0;        // subnormal / normal
}

__device__ __forceinline__ float sqrt_nb(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    float r = rd <= 0.0f ? sd : s;
    r = ru > 0.0f ? su : r;
    return r;
}
__device__ __forceinline__ float sqrt_rsq(float x) {
    const float r = __builtin_amdgcn_rsqf(x);
    const float s = x * r;
    const float e = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(e, 0.5f * r, s);
}
__device__ __forceinline__ float rcp_nr(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

__global__ void k_check(uint64_t base, unsigned long long* counts, uint32_t* first, uint32_t* lo, uint32_t* hi) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > 0xFFFFFFFFull) return;
    const uint32_t u = (uint32_t)i;
    const float x = __uint_as_float(u);
    const int c = cls(u);
    const uint32_t ref_s = __float_as_uint(__builtin_sqrtf(x));
    const uint32_t ref_r = __float_as_uint(1.0f / x);
    const uint32_t got[kSeq] = {__float_as_uint(sqrt_nb(x)), __float_as_uint(sqrt_rsq(x)), __float_as_uint(rcp_nr(x))};
    const uint32_t ref[kSeq] = {ref_s, ref_s, ref_r};
#pragma unroll
    for (int k = 0; k < kSeq; ++k) {
        if (got[k] != ref[k]) {
            const unsigned long long n = atomicAdd(&counts[k * kClass + c], 1ull);
            if (n < 4) first[(k * kClass + c) * 4 + n] = u;
            atomicMin(&lo[k * kClass + c], u);  // the range of the mismatching inputs (bit order)
            atomicMax(&hi[k * kClass + c], u);
        }
    }
}

int main() {
    unsigned long long* counts;
    uint32_t* first;
    hipMalloc(&counts, kSeq * kClass * 8);
    hipMalloc(&first, kSeq * kClass * 4 * 4);
    hipMemset(counts, 0, kSeq * kClass * 8);
    hipMemset(first, 0xFF, kSeq * kClass * 4 * 4);
    uint32_t *lo, *hi;
    hipMalloc(&lo, kSeq * kClass * 4);
    hipMalloc(&hi, kSeq * kClass * 4);
    hipMemset(lo, 0xFF, kSeq * kClass * 4);
    hipMemset(hi, 0, kSeq * kClass * 4);
    const uint64_t chunk = 1ull << 30;
    for (uint64_t b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(k_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, counts, first, lo, hi);
    unsigned long long h[kSeq * kClass];
    uint32_t f[kSeq * kClass * 4];
    hipMemcpy(h, counts, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    uint32_t hl[kSeq * kClass], hh[kSeq * kClass];
    hipMemcpy(hl, lo, sizeof(hl), hipMemcpyDeviceToHost);
    hipMemcpy(hh, hi, sizeof(hh), hipMemcpyDeviceToHost);
    const char* seq[kSeq] = {"sqrt_nb", "sqrt_rsq", "rcp_nr"};
    const char* cn[kClass] = {"+normal", "+subnormal", "+-0", "+inf", "NaN", "negative"};
    for (int k = 0; k < kSeq; ++k)
        for (int c = 0; c < kClass; ++c) {
            printf("%-9s %-11s mismatches %12llu", seq[k], cn[c], h[k * kClass + c]);
            if (h[k * kClass + c]) {
                float a, b;
                std::memcpy(&a, &hl[k * kClass + c], 4);
                std::memcpy(&b, &hh[k * kClass + c], 4);
                printf("  range [0x%08x (%g), 0x%08x (%g)]", hl[k * kClass + c], a, hh[k * kClass + c], b);
            }
            for (int j = 0; j < 4 && j < (int)h[k * kClass + c]; ++j) {
                float v;
                std::memcpy(&v, &f[(k * kClass + c) * 4 + j], 4);
                printf("  0x%08x (%g)", f[(k * kClass + c) * 4 + j], v);
            }
            printf("\n");
        }
    return 0;
}
