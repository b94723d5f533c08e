// Probe (not part of the product): calibrates rocprofv3's FETCH_SIZE on gfx950 for the access
// patterns of the blend (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./fetch_calib
// and divide each kernel's FETCH_SIZE (KiB) by the bytes it is known to move:
//   k_stream16   : 1 GiB read once, 16 B per lane, coalesced            -> guide: FETCH = bytes / 2
//   k_gather16   : 4M 16-B reads, one per distinct 128-B line of a 2 GiB buffer (no reuse, so every
//                  read misses L2 and the 256 MiB Infinity Cache)
//   k_gather4    : the same with 4-B reads
//   k_gather16x4 : 16-B reads, 4 per line at the 4 offsets of one 64-B half (2 lines per 128 B)
//   k_table      : 256 workgroups each copying the same 128 KiB table into LDS (the blend's prologue)
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_stream16(const uint4* __restrict__ src, size_t n, unsigned* out) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        acc.x ^= v.x;
        acc.y ^= v.y;
        acc.z ^= v.z;
        acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

// line i -> a pseudo-random distinct line of the buffer (multiplicative permutation mod 2^k)
__device__ __forceinline__ size_t perm_line(size_t i, size_t lines) { return (i * 2654435761ull) & (lines - 1); }

template <int BYTES, int PER_LINE>
__global__ void k_gather(const unsigned char* __restrict__ buf, size_t lines, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t line = perm_line(i / PER_LINE, lines);
        const size_t off = line * 128 + (i % PER_LINE) * 16;
        if (BYTES == 16) {
            const uint4 v = *(const uint4*)(buf + off);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else {
            acc ^= *(const unsigned*)(buf + off);
        }
    }
    if (acc == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(512) void k_table(const uint4* __restrict__ tbl, unsigned* out) {
    __shared__ uint4 lds[8192];  // 128 KiB
    for (int i = threadIdx.x; i < 8192; i += 512) lds[i] = tbl[i];
    __syncthreads();
    if (lds[threadIdx.x].x == 0x12345678u) out[0] = 1;
}

int main() {
    const size_t big = 2ull << 30;
    unsigned char* buf;
    unsigned* out;
    if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, big);
    const size_t lines = big / 128;  // 2^24
    const size_t n = 4u << 20;       // gathers / lines touched
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream16, dim3(2048), dim3(256), 0, 0, (const uint4*)buf, (size_t)(1ull << 30) / 16, out);
        hipLaunchKernelGGL((k_gather<16, 1>), dim3(2048), dim3(256), 0, 0, buf, lines, n, out);
        hipLaunchKernelGGL((k_gather<4, 1>), dim3(2048), dim3(256), 0, 0, buf, lines, n, out);
        hipLaunchKernelGGL((k_gather<16, 4>), dim3(2048), dim3(256), 0, 0, buf, lines, 4 * n, out);
        hipLaunchKernelGGL(k_table, dim3(256), dim3(512), 0, 0, (const uint4*)buf, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("known bytes: stream16 %zu, gather16 %zu lines x 16 B, gather4 %zu lines x 4 B, gather16x4 %zu "
           "lines x 64 B, table 256 x 131072 B (one 128 KiB table)\n",
           (size_t)1 << 30, n, n, n);
    return 0;
}
