// Shared helpers for the fem355 HIP kernels (gfx950 / CDNA4: wave64, 256 CUs in 8 XCDs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/fem355.h"

namespace fem {

constexpr unsigned PK_SITE_WINDOW = 4u;

// a gather window [lo, hi] (lo > hi: empty) must lie inside the nflags u-flags. One that does not is an invariant
// broken upstream (windows formed from the wrong pattern, or read before they were formed): the kernels then never
// index past the flag array AND end the launch with FEM_PCG_BAD_WINDOW, which fem_pcg_poll turns into an error
__device__ __forceinline__ bool pk_window_bad(int lo, int hi, int nflags) {
    return lo <= hi && (lo < 0 || hi >= nflags);
}
// the launch's final status after a give-up: a bad window, or a synchronisation timeout (the site word tells)
__device__ __forceinline__ int pk_fail_status(unsigned site) {
    return (site & 15u) == PK_SITE_WINDOW ? FEM_PCG_BAD_WINDOW : FEM_PCG_SYNC_TIMEOUT;
}

constexpr int WAVE = 64;
constexpr int NXCD = 8;

// ---------------------------------------------------------------- error plumbing (host)
void set_error(const char* fmt, ...);

#define FEM_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t _e = (call);                                                        \
        if (_e != hipSuccess) {                                                        \
            ::fem::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(_e)); \
            return FEM_EHIP;                                                           \
        }                                                                              \
    } while (0)

#define FEM_LAUNCHED()                                                                 \
    do {                                                                               \
        hipError_t _e = hipGetLastError();                                             \
        if (_e != hipSuccess) {                                                        \
            ::fem::set_error("%s:%d launch -> %s", __FILE__, __LINE__, hipGetErrorString(_e)); \
            return FEM_EHIP;                                                           \
        }                                                                              \
    } while (0)

inline hipStream_t S(fem_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// stream-ordered allocation from the library's private pool of the current device (runtime.hip): it keeps up to
// 256 MB of freed memory across synchronisations (with a threshold of 0 every synchronisation hands the memory back
// and the next allocation maps it again -- ~0.2 ms of host time per scratch allocation on the 10M pattern fill's
// critical path), and returns anything above that to the driver; the device's default pool is left untouched
hipError_t malloc_async(void** p, size_t bytes, hipStream_t st);
// free every kept per-stream scratch buffer and trim the private pools (fem_release_scratch)
int release_scratch();
// Stream-private scratch kept between calls (runtime.hip): `bytes` of device memory owned by stream st until a later
// call on the same stream asks for more (then reallocated, stream-ordered). For per-call scratch on the critical path:
// hipFreeAsync costs ~0.2 ms of host time here (measured on the 10M pattern fill, whose whole host call took 224 us
// with the spans' malloc / free against 17 us without), so such scratch is not freed per call.
hipError_t stream_scratch(void** p, size_t bytes, hipStream_t st);

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// grid for a grid-stride streaming kernel: enough blocks to fill 256 CUs a few times, multiple of 8 XCDs
inline int stream_grid(int64_t work_items, int block) {
    int64_t g = cdiv(work_items, block);
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    return (int)g;
}

// grid rounded to a multiple of the 8 XCDs (blockIdx % 8 selects the XCD), capped
inline int grid_multiple_of_xcd(int64_t blocks, int cap) {
    int64_t g = blocks;
    if (g > cap) g = cap;
    g = ((g + NXCD - 1) / NXCD) * NXCD;
    return (int)(g < NXCD ? NXCD : g);
}

// ---------------------------------------------------------------- device reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum over a 256-thread block; fixed tree -> deterministic. Result valid in every thread.
__device__ __forceinline__ double block_sum256(double v, double* lds4) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds4[w] = v;
    __syncthreads();
    double t = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    return t;
}
// the same over NT = 256 or 512 threads (lds: NT / 64 doubles; 512: the two 256-thread trees added)
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* lds) {
    static_assert(NT == 256 || NT == 512, "block_sum: 256 or 512 threads");
    if constexpr (NT == 256) {
        return block_sum256(v, lds);
    } else {
        v = wave_sum(v);
        const int w = threadIdx.x >> 6;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) lds[w] = v;
        __syncthreads();
        return ((lds[0] + lds[1]) + (lds[2] + lds[3])) + ((lds[4] + lds[5]) + (lds[6] + lds[7]));
    }
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// FEM_MM_ACQREL = 1 (A/B build): the grid hand-offs in C++ memory-model form -- the arrival counter
// updated with an agent-scope acq_rel atomic (the compiler's release writes back the XCD L2, its acquire invalidates
// the CU's L1) instead of the write-through form (sc1 partials drained by s_waitcnt vmcnt(0) before a relaxed atomic,
// sc1 loads after it: MI355X_MICROARCH.md "Valid forms", the default, measured cheaper)
#ifndef FEM_MM_ACQREL
#define FEM_MM_ACQREL 0
#endif
__device__ __forceinline__ void fem_drain_stores() {
#if !FEM_MM_ACQREL
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}
constexpr int FEM_ARRIVE_ORDER = FEM_MM_ACQREL ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED;

// Last-block-done ticket. Every block hands ONE 8-byte partial to the last-arriving block, in the write-through
// form of MI355X_MICROARCH.md §visibility ("Valid forms", first table row): the partial is stored `sc1`
// (relaxed agent-scope atomic store), the storing wave drains it with `s_waitcnt vmcnt(0)`, then one
// agent-scope atomic add on the counter signals; the last block reads every partial with `sc1` loads
// (sum_partials). No release fence: `buffer_wbl2` would write back every dirty line of the XCD's L2 (the
// q / r streams this kernel just wrote) in every block. The counter is re-armed by the last block.
__device__ __forceinline__ bool publish_partial(double partial, double* partials, unsigned* counter,
                                                int* lds_flag) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(&partials[blockIdx.x], partial, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fem_drain_stores();
        unsigned t = __hip_atomic_fetch_add(counter, 1u, FEM_ARRIVE_ORDER, __HIP_MEMORY_SCOPE_AGENT);
        int last = (t == gridDim.x - 1);
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    return *lds_flag != 0;
}

// Deterministic sum of n partials by one 256-thread block (fixed order), valid in every thread.
__device__ __forceinline__ double sum_partials(const double* partials, int n, double* lds4) {
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += 256)
        v += __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return block_sum256(v, lds4);
}

// Two-level (sharded) grid reduction. One counter takes ~12 ns per arrival (MI355X_MICROARCH.md row
// "fanin"), so 2048 arrivals on one word cost ~25 us. Blocks arrive on RED_SHARDS counters (blockIdx % shards,
// each on its own 128-byte line); the last arriver of a shard sums its shard's partials (fixed order) and
// arrives on the top counter; the last shard sums the shard sums (fixed order). Same `sc1` store / drain /
// atomic / `sc1` load hand-off as publish_partial. Deterministic: the summation order never depends on arrival.
// Layout of `counters`: (RED_SHARDS + 1) * 32 unsigned; `partials`: gridDim.x + RED_SHARDS doubles.
constexpr int RED_SHARDS = 32;


constexpr int RED_COUNTER_WORDS = (RED_SHARDS + 1) * 32;

template <int NT = 256>   // threads of the calling block (lds4: NT / 64 doubles)
__device__ __forceinline__ bool reduce_grid(double partial, double* partials, unsigned* counters, double* total,
                                            double* lds4, int* lds_flag) {
    const unsigned G = gridDim.x;
    const unsigned nsh = G < (unsigned)RED_SHARDS ? G : (unsigned)RED_SHARDS;
    const unsigned sh = blockIdx.x % RED_SHARDS;
    const unsigned in_shard = (G - sh + RED_SHARDS - 1) / RED_SHARDS;   // blocks b < G with b % shards == sh
    double* shard_sums = partials + G;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&partials[blockIdx.x], partial, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fem_drain_stores();
        unsigned t = __hip_atomic_fetch_add(&counters[sh * 32], 1u, FEM_ARRIVE_ORDER, __HIP_MEMORY_SCOPE_AGENT);
        int last = (t == in_shard - 1);
        if (last) __hip_atomic_store(&counters[sh * 32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    if (!*lds_flag) return false;
    double v = 0.0;
    for (unsigned i = threadIdx.x; i < in_shard; i += NT)
        v += __hip_atomic_load(&partials[sh + i * RED_SHARDS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = block_sum<NT>(v, lds4);
    if (threadIdx.x == 0) {
        __hip_atomic_store(&shard_sums[sh], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fem_drain_stores();
        unsigned* top = &counters[RED_SHARDS * 32];
        unsigned t = __hip_atomic_fetch_add(top, 1u, FEM_ARRIVE_ORDER, __HIP_MEMORY_SCOPE_AGENT);
        int last = (t == nsh - 1);
        if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    if (!*lds_flag) return false;
    double s = (threadIdx.x < nsh)
                   ? __hip_atomic_load(&shard_sums[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : 0.0;
    *total = block_sum<NT>(s, lds4);
    return true;
}

// value rc of entry E (= slice base + 64 k + lane) of a bs = 3 matrix in the plane-paired layout A (sell_pair3.hpp):
// the entry's 576-double chunk holds values (2t, 2t + 1) of lane l at 128 t + 2 l, value 8 at 512 + l
__device__ __forceinline__ int64_t sell_val_a(int64_t E, int rc) {
    const int64_t lane = E & 63;
    return (E - lane) * 9 + (rc < 8 ? 128 * (rc >> 1) + 2 * lane + (rc & 1) : 512 + lane);
}

// entry k of a SELL-64 slice of width w in the lane-paired layout (sell_pair.hpp), offset from the slice base, lane l
__device__ __forceinline__ int64_t pair_pos(int k, int w, int l) {
    const int np = w >> 1;
    return k < 2 * np ? (int64_t)(k >> 1) * 128 + 2 * l + (k & 1) : (int64_t)np * 128 + l;
}

}  // namespace fem
