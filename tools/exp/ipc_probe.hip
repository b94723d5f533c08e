// Probe (not part of the product): can two processes that share ONE GPU run the multi-GPU frame's
// transport -- an uncached allocation exported with hipIpcGetMemHandle and opened by the other
// process, plain stores of one process landing in the other's buffer, and device-side flag barriers
// (release fence + flag store into the peer's control words, a bounded spin on one's own) -- and
// what does one barrier round trip cost?
//   hipcc --offload-arch=gfx950 -O3 -o ipc_probe ipc_probe.hip
//   ./ipc_probe 0 DIR & ./ipc_probe 1 DIR; wait      (handles exchanged through files in DIR)
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "rank %d: %s failed: %s\n", rank, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr unsigned kWords = 1u << 20;  // data words per buffer
constexpr unsigned kCtl = 64;          // control words at the front: flag[src]

__global__ void k_fill(unsigned* __restrict__ peerData, unsigned tag, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        peerData[i] = tag ^ (i * 2654435761u);
}

// lane 0: release at system scope, store `epoch` into the peer's flag[me]; then spin (bounded) until
// my own flag[peer] reaches epoch.  status[0] = spins, status[1] = 1 on timeout.
__global__ void k_barrier(unsigned* peerCtl, unsigned* myCtl, int me, int peer, unsigned epoch,
                          unsigned* status, int arrive, int wait) {
    if (threadIdx.x != 0) return;
    if (arrive) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(peerCtl + me, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!wait || status[1]) return;  // after a timeout every later wait is skipped
    const unsigned long long t0 = wall_clock64();
    unsigned spins = 0;
    while (true) {
        const unsigned v = __hip_atomic_load(myCtl + peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int)(v - epoch) >= 0) break;
        if (wall_clock64() - t0 > 500000000ull) {  // 5 s at 100 MHz
            status[1] = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
        ++spins;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    status[0] = spins;
}

__global__ void k_check(const unsigned* __restrict__ data, unsigned tag, unsigned n, unsigned* bad) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        if (data[i] != (tag ^ (i * 2654435761u))) atomicAdd(bad, 1u);
}

int main(int argc, char** argv) {
    int rank = argc > 1 ? std::atoi(argv[1]) : 0;
    const std::string dir = argc > 2 ? argv[2] : "/tmp";
    const int peer = rank ^ 1;
    CK(hipSetDevice(0));
    unsigned* mine = nullptr;
    CK(hipExtMallocWithFlags((void**)&mine, (kCtl + kWords) * 4, hipDeviceMallocUncached));
    CK(hipMemset(mine, 0, (kCtl + kWords) * 4));
    unsigned* status = nullptr;
    CK(hipMalloc(&status, 16));
    CK(hipMemset(status, 0, 16));
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, mine));
    {
        const std::string tmp = dir + "/h" + std::to_string(rank) + ".tmp", fin = dir + "/h" + std::to_string(rank);
        FILE* f = std::fopen(tmp.c_str(), "wb");
        std::fwrite(&h, sizeof(h), 1, f);
        std::fclose(f);
        std::rename(tmp.c_str(), fin.c_str());
    }
    hipIpcMemHandle_t ph;
    {
        const std::string fin = dir + "/h" + std::to_string(peer);
        for (int i = 0; i < 600; ++i) {
            FILE* f = std::fopen(fin.c_str(), "rb");
            if (f) {
                size_t got = std::fread(&ph, sizeof(ph), 1, f);
                std::fclose(f);
                if (got == 1) break;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
        }
    }
    unsigned* theirs = nullptr;
    CK(hipIpcOpenMemHandle((void**)&theirs, ph, hipIpcMemLazyEnablePeerAccess));
    std::printf("rank %d: opened peer buffer %p (mine %p)\n", rank, (void*)theirs, (void*)mine);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // 1. data into the peer's buffer, then a barrier, then check what the peer wrote into mine
    const unsigned tagMine = 0x1000u + (unsigned)rank, tagPeer = 0x1000u + (unsigned)peer;
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, theirs + kCtl, tagMine, kWords);
    hipLaunchKernelGGL(k_barrier, dim3(1), dim3(64), 0, s, theirs, mine, rank, peer, 1u, status, 1, 1);
    hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, s, mine + kCtl, tagPeer, kWords, status + 2);
    CK(hipStreamSynchronize(s));
    unsigned st[4];
    CK(hipMemcpy(st, status, 16, hipMemcpyDeviceToHost));
    std::printf("rank %d: barrier spins %u timeout %u, mismatched words %u of %u\n", rank, st[0], st[1], st[2], kWords);
    // 2. barrier round trips: 2000 barriers back to back on the stream
    const int iters = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k_barrier, dim3(1), dim3(64), 0, s, theirs, mine, rank, peer, 2u + (unsigned)i, status, 1, 1);
    CK(hipStreamSynchronize(s));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    CK(hipMemcpy(st, status, 16, hipMemcpyDeviceToHost));
    std::printf("rank %d: %d barriers in %.0f us = %.2f us each, timeout %u\n", rank, iters, us, us / iters, st[1]);
    CK(hipIpcCloseMemHandle(theirs));
    CK(hipFree(mine));
    return st[1] != 0 || st[2] != 0;
}
