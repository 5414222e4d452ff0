// 16-byte value layouts of the bs = 3 SELL-64 matrix (elasticity). The plain layout stores the 9 values of a
// lane's block as 9 planes strided by 64, so a block costs 9 eight-byte loads + 1 column load + 3 gathers per lane
// (13 memory instructions for 74 bytes of matrix). Both layouts below keep slice_ptr, the footprint and the
// per-row summation order (entry k ascending, then r, then j) of the plain layout, so results are bit-identical.
//
// Plane-paired ("A"): entry k of slice s (base p0) occupies doubles [c, c + 576), c = 9*p0 + 576*k; lane l reads
//   values (2t, 2t+1), t = 0..3, as one double2 at c + 128 t + 2 l and value 8 at c + 512 + l; columns stay plain
//   (int16 delta at p0 + 64 k + l).                                         -> 1 + 5 + 3 = 9 instructions per block
// Entry-paired ("B"): entries 2j and 2j+1 of a lane (18 values, v = 9 a + e) occupy the chunk c = 9*p0 + 1152 j;
//   lane l reads values (2t, 2t+1), t = 0..8, as one double2 at c + 128 t + 2 l; the two column deltas are one
//   int32 at p0 + 128 j + 2 l (as the bs = 1 paired layout). Odd tail entry (w odd): plain planes at
//   c = 9*p0 + 1152*(w/2), value e at c + 64 e + l, column at p0 + 128*(w/2) + l.  -> 8 instructions per block
#pragma once
#include "common.hpp"

namespace fem {

typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename T, bool NT>
__device__ __forceinline__ T ld3(const T* p) {
    if constexpr (NT) {
        if constexpr (sizeof(T) == 16) {
            const f64x2 v = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p));
            return T{v.x, v.y};
        } else {
            return __builtin_nontemporal_load(p);
        }
    } else {
        return *p;
    }
}

// plain -> layout A (values only) / layout B (values and columns). One thread per (slice, lane).
static __global__ void k_sell3_to_a(int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                    const double* __restrict__ vin, double* __restrict__ vout) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        for (int k = 0; k < w; ++k) {
            const int64_t c = 9 * p0 + 576 * (int64_t)k;
            for (int e = 0; e < 8; ++e) vout[c + 128 * (e >> 1) + 2 * l + (e & 1)] = vin[c + 64 * e + l];
            vout[c + 512 + l] = vin[c + 512 + l];
        }
    }
}

// layout A -> plain (the solver layout's values back into the plain planes)
[[maybe_unused]] static __global__ void k_sell3_from_a(int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                                       const double* __restrict__ vin, double* __restrict__ vout) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        for (int k = 0; k < w; ++k) {
            const int64_t c = 9 * p0 + 576 * (int64_t)k;
            for (int e = 0; e < 8; ++e) vout[c + 64 * e + l] = vin[c + 128 * (e >> 1) + 2 * l + (e & 1)];
            vout[c + 512 + l] = vin[c + 512 + l];
        }
    }
}

[[maybe_unused]] static __global__ void k_sell3_to_b(int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                    const double* __restrict__ vin, const int16_t* __restrict__ cin,
                                    double* __restrict__ vout, int16_t* __restrict__ cout) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        const int np = w >> 1;
        for (int j = 0; j < np; ++j) {
            const int64_t c = 9 * p0 + 1152 * (int64_t)j;   // plain: entry 2j at c, entry 2j+1 at c + 576
            for (int v = 0; v < 18; ++v) {
                const int a = v / 9, e = v % 9;
                vout[c + 128 * (v >> 1) + 2 * l + (v & 1)] = vin[c + 576 * a + 64 * e + l];
            }
            cout[p0 + 128 * (int64_t)j + 2 * l] = cin[p0 + 64 * (2 * (int64_t)j) + l];
            cout[p0 + 128 * (int64_t)j + 2 * l + 1] = cin[p0 + 64 * (2 * (int64_t)j + 1) + l];
        }
        if (w & 1) {
            const int64_t c = 9 * p0 + 1152 * (int64_t)np;
            for (int e = 0; e < 9; ++e) vout[c + 64 * e + l] = vin[c + 64 * e + l];
            cout[p0 + 128 * (int64_t)np + l] = cin[p0 + 64 * (int64_t)(2 * np) + l];
        }
    }
}

// gather of the 3 components of block column cc (= 3 * node): three 8-byte loads (G = 0), or one 8-byte load and
// one 16-byte load at 8-byte alignment (G = 1)
typedef double f64x2u __attribute__((ext_vector_type(2), aligned(8)));
template <int G>
__device__ __forceinline__ void gather3(const double* __restrict__ x, int cc, double xv[3]) {
    if constexpr (G == 0) {
        xv[0] = x[cc];
        xv[1] = x[cc + 1];
        xv[2] = x[cc + 2];
    } else {
        xv[0] = x[cc];
        const f64x2u t = *reinterpret_cast<const f64x2u*>(x + cc + 1);
        xv[1] = t.x;
        xv[2] = t.y;
    }
}

__device__ __forceinline__ void blk3_fma(double out[3], const double* v, const double* xv) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < 3; ++j) out[r] += v[r * 3 + j] * xv[j];
}

// plain layout (reference for the lab); U blocks in flight
template <int U, bool NT>
__device__ __forceinline__ void sell3_row_plain(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                                const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                const double* __restrict__ x, double out[3]) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int base = (int)(s * 64 + lane);
    const int16_t* c = cols + p0 + lane;
    const double* vb = vals + 9 * p0 + lane;
    out[0] = out[1] = out[2] = 0.0;
    for (int k0 = 0; k0 < w; k0 += U) {
        int cc[U];
        double vv[U][9], xv[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) cc[u] = (k0 + u < w) ? 3 * (base + (int)ld3<int16_t, NT>(c + 64 * (k0 + u))) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < 9; ++e) vv[u][e] = (k0 + u < w) ? ld3<double, NT>(vb + 576 * (int64_t)(k0 + u) + 64 * e) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 3; ++j) xv[u][j] = (k0 + u < w) ? x[cc[u] + j] : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < w) blk3_fma(out, vv[u], xv[u]);
    }
}

// y (3 rows) of lane `lane` in slice s, layout A; U entries in flight
template <int U, bool NT, int G = 0>
__device__ __forceinline__ void sell3_row_a(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                            const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                            const double* __restrict__ x, double out[3]) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int base = (int)(s * 64 + lane);
    const int16_t* c = cols + p0 + lane;
    const double* vb = vals + 9 * p0;
    out[0] = out[1] = out[2] = 0.0;
    for (int k0 = 0; k0 < w; k0 += U) {
        int cc[U];
        double vv[U][9], xv[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) cc[u] = (k0 + u < w) ? 3 * (base + (int)ld3<int16_t, NT>(c + 64 * (k0 + u))) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double* ch = vb + 576 * (int64_t)(k0 + u);
            const double2* c2 = reinterpret_cast<const double2*>(ch) + lane;
            if (k0 + u < w) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const double2 d = ld3<double2, NT>(c2 + 64 * t);
                    vv[u][2 * t] = d.x;
                    vv[u][2 * t + 1] = d.y;
                }
                vv[u][8] = ld3<double, NT>(ch + 512 + lane);
            } else {
#pragma unroll
                for (int e = 0; e < 9; ++e) vv[u][e] = 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k0 + u < w) gather3<G>(x, cc[u], xv[u]);
            else xv[u][0] = xv[u][1] = xv[u][2] = 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < w) blk3_fma(out, vv[u], xv[u]);
    }
}

// layout B; U entry pairs in flight
template <int U, bool NT>
__device__ __forceinline__ void sell3_row_b(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                            const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                            const double* __restrict__ x, double out[3]) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int np = w >> 1;
    const int base = (int)(s * 64 + lane);
    const int32_t* c2 = reinterpret_cast<const int32_t*>(cols + p0) + lane;
    const double* vb = vals + 9 * p0;
    out[0] = out[1] = out[2] = 0.0;
    for (int j0 = 0; j0 < np; j0 += U) {
        int32_t cc[U];
        double vv[U][18], xv[U][6];
#pragma unroll
        for (int u = 0; u < U; ++u) cc[u] = (j0 + u < np) ? ld3<int32_t, NT>(c2 + 64 * (j0 + u)) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double2* ch = reinterpret_cast<const double2*>(vb + 1152 * (int64_t)(j0 + u)) + lane;
            if (j0 + u < np) {
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const double2 d = ld3<double2, NT>(ch + 64 * t);
                    vv[u][2 * t] = d.x;
                    vv[u][2 * t + 1] = d.y;
                }
            } else {
#pragma unroll
                for (int v = 0; v < 18; ++v) vv[u][v] = 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int lo = 3 * (base + (int)(int16_t)(cc[u] & 0xffff));
            const int hi = 3 * (base + (int)(int16_t)(cc[u] >> 16));
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                xv[u][j] = (j0 + u < np) ? x[lo + j] : 0.0;
                xv[u][3 + j] = (j0 + u < np) ? x[hi + j] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j0 + u < np) {
                blk3_fma(out, vv[u], xv[u]);
                blk3_fma(out, vv[u] + 9, xv[u] + 3);
            }
    }
    if (w & 1) {
        const double* ch = vb + 1152 * (int64_t)np + lane;
        const int cj = 3 * (base + (int)cols[p0 + 128 * (int64_t)np + lane]);
        double v[9], xv[3];
#pragma unroll
        for (int e = 0; e < 9; ++e) v[e] = ld3<double, NT>(ch + 64 * e);
#pragma unroll
        for (int j = 0; j < 3; ++j) xv[j] = x[cj + j];
        blk3_fma(out, v, xv);
    }
}

}  // namespace fem
