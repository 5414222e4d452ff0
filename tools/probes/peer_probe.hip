// Feasibility probes for an in-kernel multi-GPU hand-off (run on the GPU box):
//  mode "streams": two kernels on two streams of one process, each with G/2 one-per-CU workgroups, ping-pong an
//                  epoch flag through device memory with system-scope stores/loads for `iters` rounds: reports whether
//                  they ran concurrently (else the bounded spin gives up) and the round-trip time.
//  mode "ipc":     run as two processes (rank 0 and 1 on the same device): rank 0 exports a buffer with
//                  hipIpcGetMemHandle through a file, rank 1 opens it; the same ping-pong across processes.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <unistd.h>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                             \
        }                                                                        \
    } while (0)

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// side 0 writes mine[0] = 2k+1 after seeing theirs >= 2k; side 1 writes 2k+2 after seeing 2k+1. The payload
// (64 doubles) travels with the flag: written with system-scope stores before a system release, checked after.
__global__ void pingpong(unsigned* my_flag, const unsigned* peer_flag, double* peer_data, const double* my_data,
                         int side, int iters, unsigned* result) {
    if (blockIdx.x != 0) return;   // the other workgroups only occupy CUs
    const int lane = threadIdx.x;
    unsigned bad = 0, tmo = 0;
    for (int k = 0; k < iters && !tmo; ++k) {
        const unsigned want = side == 0 ? 2u * k : 2u * k + 1u;
        if (lane == 0) {
            unsigned spins = 0;
            while (ld_sys(peer_flag) < want) {
                if (++spins > (1u << 24)) { tmo = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        tmo = __shfl(tmo, 0);
        if (tmo) break;
        // check the payload the peer published with its last flag (value = its last flag value)
        if (k > 0 || side == 1) {
            const double v = __hip_atomic_load(my_data + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v != (double)want + lane) bad++;
        }
        const unsigned mine = want + 1;
        __hip_atomic_store(peer_data + lane, (double)mine + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st_sys(my_flag, mine);
    }
    if (lane == 0) {
        result[0] = tmo;
    }
    atomicAdd(result + 1, bad);
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "streams";
    const int iters = argc > 2 ? atoi(argv[2]) : 2000;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipFuncSetAttribute((const void*)pingpong, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    const int G = ncu / 2;
    if (mode == "streams") {
        unsigned *f0, *f1, *res;
        double *d0, *d1;
        CK(hipMalloc(&f0, 256));
        CK(hipMalloc(&f1, 256));
        CK(hipMalloc(&d0, 64 * 8));
        CK(hipMalloc(&d1, 64 * 8));
        CK(hipMalloc(&res, 64));
        CK(hipMemset(f0, 0, 256));
        CK(hipMemset(f1, 0, 256));
        CK(hipMemset(res, 0, 64));
        hipStream_t s0, s1;
        CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(pingpong, dim3(G), dim3(64), 96 * 1024, s0, f0, f1, d1, d0, 0, iters, res);
        hipLaunchKernelGGL(pingpong, dim3(G), dim3(64), 96 * 1024, s1, f1, f0, d0, d1, 1, iters, res + 4);
        CK(hipDeviceSynchronize());
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        unsigned h[8];
        CK(hipMemcpy(h, res, 32, hipMemcpyDeviceToHost));
        printf("{\"mode\": \"streams\", \"G_each\": %d, \"iters\": %d, \"timeout\": [%u, %u], \"bad\": [%u, %u], "
               "\"us_per_roundtrip\": %.3f}\n", G, iters, h[0], h[4], h[1], h[5], us / iters);
        return (h[0] || h[4] || h[1] || h[5]) ? 1 : 0;
    }
    // ipc: argv[3] = rank (0 / 1), argv[4] = handle file
    const int rank = atoi(argv[3]);
    const std::string hf = argv[4];
    // rank r owns flag[r] and data[r] in ONE buffer exported by rank 0; rank 1 allocates its own and exports too
    unsigned* flags;
    double* data;
    unsigned* res;
    CK(hipMalloc(&flags, 256));
    CK(hipMalloc(&data, 64 * 8));
    CK(hipMalloc(&res, 64));
    CK(hipMemset(flags, 0, 256));
    CK(hipMemset(res, 0, 64));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t hfl, hd;
    CK(hipIpcGetMemHandle(&hfl, flags));
    CK(hipIpcGetMemHandle(&hd, data));
    {
        std::ofstream o(hf + "." + std::to_string(rank) + ".tmp", std::ios::binary);
        o.write((const char*)&hfl, sizeof hfl);
        o.write((const char*)&hd, sizeof hd);
    }
    rename((hf + "." + std::to_string(rank) + ".tmp").c_str(), (hf + "." + std::to_string(rank)).c_str());
    const std::string pf = hf + "." + std::to_string(1 - rank);
    for (int t = 0; t < 3000 && access(pf.c_str(), F_OK) != 0; ++t) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    hipIpcMemHandle_t pfl, pd;
    {
        std::ifstream i(pf, std::ios::binary);
        i.read((char*)&pfl, sizeof pfl);
        i.read((char*)&pd, sizeof pd);
    }
    void *peer_flags, *peer_data;
    CK(hipIpcOpenMemHandle(&peer_flags, pfl, hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle(&peer_data, pd, hipIpcMemLazyEnablePeerAccess));
    // my flag lives in MY buffer (peer polls it remotely?) -- no: each side polls its OWN memory, the peer writes
    // there. So: my_flag (written by me) = the PEER's copy; peer_flag (polled by me) = my local buffer.
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(pingpong, dim3(G), dim3(64), 96 * 1024, 0, (unsigned*)peer_flags, flags, (double*)peer_data,
                       data, rank, iters, res);
    CK(hipDeviceSynchronize());
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    unsigned h[4];
    CK(hipMemcpy(h, res, 16, hipMemcpyDeviceToHost));
    printf("{\"mode\": \"ipc\", \"rank\": %d, \"G\": %d, \"iters\": %d, \"timeout\": %u, \"bad\": %u, \"us_total\": %.1f, "
           "\"us_per_roundtrip\": %.3f}\n", rank, G, iters, h[0], h[1], us, us / iters);
    CK(hipIpcCloseMemHandle(peer_flags));
    CK(hipIpcCloseMemHandle(peer_data));
    return (h[0] || h[1]) ? 1 : 0;
}
