// Lane-paired SELL-64 layout for bs = 1 with 16-bit column deltas: each lane reads two consecutive entries of its
// row with one 16-byte value load and one 4-byte column load (the plain layout issues an 8-byte and a 2-byte load
// per entry; tools/spmv_layout.py: 55.8 -> 47.8 us on the 10M Poisson matrix, warm).
// Slice s (width w, base p0 = slice_ptr[s]): entry k < 2*(w/2) of lane l at p0 + (k/2)*128 + 2*l + (k%2), the odd
// tail entry (w odd) at p0 + (w/2)*128 + l. Same footprint and slice_ptr as the plain layout.
#pragma once
#include "common.hpp"

namespace fem {

// plain -> paired layout (values and 16-bit deltas)
static __global__ void k_sell_pair(int64_t nslices, const int64_t* __restrict__ slice_ptr, const double* __restrict__ vin,
                            const int16_t* __restrict__ cin, double* __restrict__ vout, int16_t* __restrict__ cout) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        const int np = w >> 1;
        for (int k = 0; k < w; ++k) {
            const int64_t src = p0 + 64 * k + l;
            const int64_t dst = k < 2 * np ? p0 + (int64_t)(k >> 1) * 128 + 2 * l + (k & 1) : p0 + (int64_t)np * 128 + l;
            vout[dst] = vin[src];
            cout[dst] = cin[src];
        }
    }
}


// gathered x element: plain load (SC1 = 0), an agent-scope relaxed load (1: global_load sc1, the coherent form that
// may replace the consumer's acquire when every producer store was sc1, MI355X_MICROARCH.md, Valid forms), or a
// system-scope relaxed load (2: sc0 sc1, past this GPU's L2 -- rows another GPU wrote into this GPU's memory)
template <int SC1>
__device__ __forceinline__ double ldx(const double* p) {
    if constexpr (SC1 == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if constexpr (SC1 == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// SC1 = 3: per element, 2 (system scope) for columns outside [own_lo, own_hi) -- rows another GPU wrote into this
// GPU's memory, never cached here -- and 1 for the rest (this GPU's rows, L2-served)
template <int SC1>
__device__ __forceinline__ double ldx_col(const double* x, int col, int own_lo, int own_hi) {
    if constexpr (SC1 == 3) {
        if (col < own_lo || col >= own_hi) return ldx<2>(x + col);
        return ldx<1>(x + col);
    } else {
        return ldx<SC1>(x + col);
    }
}

// y_row (bs = 1) of one slice row in the paired layout; U pairs in flight
template <int U, int SC1 = 0>
__device__ __forceinline__ double sell_row_pair(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                                const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                const double* __restrict__ x, int own_lo = 0, int own_hi = 0) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int np = w >> 1;
    const int base = (int)(s * 64 + lane);
    const double2* v2 = reinterpret_cast<const double2*>(vals + p0) + lane;
    const int32_t* c2 = reinterpret_cast<const int32_t*>(cols + p0) + lane;
    double acc = 0.0;
    for (int j0 = 0; j0 < np; j0 += U) {
        int32_t cc[U];
        double2 vv[U];
        double x0[U], x1[U];
#pragma unroll
        for (int j = 0; j < U; ++j) cc[j] = (j0 + j < np) ? c2[64 * (j0 + j)] : 0;
#pragma unroll
        for (int j = 0; j < U; ++j) vv[j] = (j0 + j < np) ? v2[64 * (j0 + j)] : double2{0.0, 0.0};
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int lo = (int)(int16_t)(cc[j] & 0xffff), hi = (int)(int16_t)(cc[j] >> 16);
            x0[j] = (j0 + j < np) ? ldx_col<SC1>(x, base + lo, own_lo, own_hi) : 0.0;
            x1[j] = (j0 + j < np) ? ldx_col<SC1>(x, base + hi, own_lo, own_hi) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (j0 + j < np) {
                acc += vv[j].x * x0[j];
                acc += vv[j].y * x1[j];
            }
    }
    if (w & 1) {
        const int64_t t = p0 + (int64_t)np * 128 + lane;
        acc += vals[t] * ldx_col<SC1>(x, base + (int)cols[t], own_lo, own_hi);
    }
    return acc;
}

}  // namespace fem
