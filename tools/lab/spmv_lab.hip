// SpMV layout experiments (tools/spmv_layout.py): memory-instruction width probes and a lane-paired SELL-64
// layout in which each lane loads two consecutive entries of its row with one 16-byte value load and one 4-byte
// column load (the plain layout issues one 8-byte value and one 2-byte column load per entry).
//
// Paired layout of slice s (width w, base p0 = slice_ptr[s]): entry k < 2*(w/2) of lane l lives at
//   p0 + (k/2)*128 + 2*l + (k%2), the odd tail entry (w odd) at p0 + (w/2)*128 + l;
// same for the 16-bit column deltas. Footprint and slice_ptr are unchanged.
#include "sell_pair.hpp"
#include "sell_pair3.hpp"
#include "fem355_lab.h"

namespace fem {

// copy probes: W bytes per lane per instruction (8, 16, 32)
template <int W>
__global__ void __launch_bounds__(256) k_copy_w(const double* __restrict__ src, double* __restrict__ dst, int64_t n) {
    constexpr int D = W / 8;
    const int64_t nv = n / D;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
        if constexpr (D == 1) {
            dst[i] = src[i];
        } else if constexpr (D == 2) {
            reinterpret_cast<double2*>(dst)[i] = reinterpret_cast<const double2*>(src)[i];
        } else {
            const double2* s2 = reinterpret_cast<const double2*>(src) + 2 * i;
            double2 a = s2[0], b = s2[1];
            double2* d2 = reinterpret_cast<double2*>(dst) + 2 * i;
            d2[0] = a;
            d2[1] = b;
        }
    }
}

// read-only probe: sum of W-byte loads (no writes)
template <int W>
__global__ void __launch_bounds__(256) k_read_w(const double* __restrict__ src, int64_t n, double* __restrict__ out) {
    constexpr int D = W / 8;
    const int64_t nv = n / D;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
        if constexpr (D == 1) {
            acc += src[i];
        } else {
            const double2 v = reinterpret_cast<const double2*>(src)[i];
            acc += v.x + v.y;
        }
    }
    if (acc == 12345.678) out[0] = acc;   // keep the loads alive
}

template <int U>
__global__ void __launch_bounds__(256) k_spmv16_pair(int64_t nslices, int64_t nrows,
                                                     const int64_t* __restrict__ slice_ptr,
                                                     const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                     const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int xcd = blockIdx.x % NXCD;
    const int64_t lb = blockIdx.x / NXCD, nlb = gridDim.x / NXCD;
    const int64_t spx = (nslices + NXCD - 1) / NXCD;
    const int64_t end = min((int64_t)(xcd + 1) * spx, nslices);
    for (int64_t s = (int64_t)xcd * spx + lb * 4 + (threadIdx.x >> 6); s < end; s += nlb * 4) {
        const double acc = sell_row_pair<U>(s, lane, slice_ptr, cols, vals, x);
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = acc;
    }
}

// bs = 3 layout probes (sell_pair3.hpp): L = 0 plain, 1 plane-paired (A), 2 entry-paired (B)
template <int L, int U, bool NT>
__global__ void __launch_bounds__(256) k_spmv3_lab(int64_t nslices, int64_t nrows,
                                                   const int64_t* __restrict__ slice_ptr,
                                                   const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                   const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int xcd = blockIdx.x % NXCD;
    const int64_t lb = blockIdx.x / NXCD, nlb = gridDim.x / NXCD;
    const int64_t spx = (nslices + NXCD - 1) / NXCD;
    const int64_t end = min((int64_t)(xcd + 1) * spx, nslices);
    for (int64_t s = (int64_t)xcd * spx + lb * 4 + (threadIdx.x >> 6); s < end; s += nlb * 4) {
        double o[3];
        if constexpr (L == 0) sell3_row_plain<U, NT>(s, lane, slice_ptr, cols, vals, x, o);
        else if constexpr (L == 1) sell3_row_a<U, NT>(s, lane, slice_ptr, cols, vals, x, o);
        else if constexpr (L == 3) sell3_row_a<U, NT, 1>(s, lane, slice_ptr, cols, vals, x, o);
        else sell3_row_b<U, NT>(s, lane, slice_ptr, cols, vals, x, o);
        const int64_t row = s * 64 + lane;
        if (row < nrows) {
            y[3 * row] = o[0];
            y[3 * row + 1] = o[1];
            y[3 * row + 2] = o[2];
        }
    }
}

// persistent-geometry probe: one workgroup of T threads per CU (occupancy pinned by dynamic LDS), wave g owns the
// contiguous slice range [g S / W, (g+1) S / W) (XCD-contiguous logical order), U pairs in flight (paired layout)
template <int T, int U>
__global__ void __launch_bounds__(T) k_spmv_persist_lab(int64_t nslices, int64_t nrows,
                                                        const int64_t* __restrict__ slice_ptr,
                                                        const int16_t* __restrict__ cols,
                                                        const double* __restrict__ vals,
                                                        const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ double pad_lds[];
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;
    const int64_t W = (int64_t)G * (T / 64);
    const int64_t g = (int64_t)L * (T / 64) + (threadIdx.x >> 6);
    const int64_t s0 = g * nslices / W, s1 = (g + 1) * nslices / W;
    for (int64_t s = s0; s < s1; ++s) {
        const double acc = sell_row_pair<U>(s, lane, slice_ptr, cols, vals, x);
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = acc;
    }
    if (nrows < 0) pad_lds[threadIdx.x] = 0.0;
}

// the persistent-geometry probe on the production bs = 1 format: lane-paired values, slice-uniform deltas where
// k_sell_uniform found them (U = 2 pairs in flight, 1024 threads, as k_pcg_persist)
__global__ void __launch_bounds__(1024) k_spmv_persist_uni_lab(int64_t nslices, int64_t nrows,
                                                               const int64_t* __restrict__ slice_ptr,
                                                               const int16_t* __restrict__ cols,
                                                               const double* __restrict__ vals,
                                                               const int32_t* __restrict__ uoff,
                                                               const int16_t* __restrict__ ucol,
                                                               const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ double pad_lds[];
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;
    const int64_t W = (int64_t)G * 16;
    const int64_t g = (int64_t)L * 16 + (threadIdx.x >> 6);
    const int64_t s0 = g * nslices / W, s1 = (g + 1) * nslices / W;
    for (int64_t s = s0; s < s1; ++s) {
        const double acc = sell_row_pair<2>(s, lane, slice_ptr, cols, vals, x, 0, 0, uoff, ucol);
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = acc;
    }
    if (nrows < 0) pad_lds[threadIdx.x] = 0.0;
}

// symmetric-storage probe (bs = 1): only the upper triangle (col >= row) is stored, plain SELL-64 layout with a
// slice-uniform delta list per slice; the lower entries of a row are re-read from the upper storage of the rows
// they mirror: for lower delta d of slice s, lanes l >= d % 64 read slice s - d / 64 at base_a + l - d % 64, the
// others slice s - d / 64 - 1 at base_b + l - d % 64 + 64 (bases: slice offset + 64 k of delta +d there; -1: none).
// Same persistent geometry as above. x must be readable at [row - 32768, row + 32768) for every slice row.
__global__ void __launch_bounds__(1024) k_spmv_sym_lab(int64_t nslices, int64_t nrows, const int64_t* __restrict__ uptr,
                                                       const int32_t* __restrict__ ulist,
                                                       const int16_t* __restrict__ udel,
                                                       const int32_t* __restrict__ lptr,
                                                       const int32_t* __restrict__ ldel,
                                                       const int32_t* __restrict__ lbase,
                                                       const double* __restrict__ uvals, const double* __restrict__ x,
                                                       double* __restrict__ y) {
    extern __shared__ double pad_lds[];
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;
    const int64_t W = (int64_t)G * 16;
    const int64_t g = (int64_t)L * 16 + (threadIdx.x >> 6);
    const int64_t s0 = g * nslices / W, s1 = (g + 1) * nslices / W;
    for (int64_t s = s0; s < s1; ++s) {
        const int64_t p0 = uptr[s];
        const int w = (int)((uptr[s + 1] - p0) >> 6);
        const int16_t* ud = udel + ulist[s];
        const int base = (int)(s * 64 + lane);
        const double* uv = uvals + p0 + lane;
        double acc = 0.0;
        int k = 0;
        for (; k + 4 <= w; k += 4) {
            double v[4], xv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = uv[64 * (k + j)];
#pragma unroll
            for (int j = 0; j < 4; ++j) xv[j] = x[base + ud[k + j]];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += v[j] * xv[j];
        }
        for (; k < w; ++k) acc += uv[64 * k] * x[base + ud[k]];
        const int m0 = lptr[s], m1 = lptr[s + 1];
        int m = m0;
        for (; m + 2 <= m1; m += 2) {
            double v[2], xv[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int d = ldel[m + j];
                const int r = d & 63;
                const int ba = lbase[2 * (m + j)], bb = lbase[2 * (m + j) + 1];
                const int lp = lane - r;
                const int pos = lp >= 0 ? (ba >= 0 ? ba + lp : -1) : (bb >= 0 ? bb + lp + 64 : -1);
                v[j] = pos >= 0 ? uvals[pos] : 0.0;
                xv[j] = x[base - d];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) acc += v[j] * xv[j];
        }
        for (; m < m1; ++m) {
            const int d = ldel[m];
            const int r = d & 63;
            const int ba = lbase[2 * m], bb = lbase[2 * m + 1];
            const int lp = lane - r;
            const int pos = lp >= 0 ? (ba >= 0 ? ba + lp : -1) : (bb >= 0 ? bb + lp + 64 : -1);
            acc += (pos >= 0 ? uvals[pos] : 0.0) * x[base - d];
        }
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = acc;
    }
    if (nrows < 0) pad_lds[threadIdx.x] = 0.0;
}

// gather-volume probe: the uniform-slice SpMV with the odd entry of every pair taking the even entry's gathered x
// (MODE 1: WRONG result, 8 instead of 15 gathers per row on the Kuhn stencil) or with no gathers at all (MODE 2:
// x = 1) -- how much of the SpMV time the L2-served x gathers cost
template <int MODE>
__global__ void __launch_bounds__(1024) k_spmv_gather_lab(int64_t nslices, int64_t nrows,
                                                          const int64_t* __restrict__ slice_ptr,
                                                          const double* __restrict__ vals,
                                                          const int32_t* __restrict__ uoff,
                                                          const int16_t* __restrict__ ucol,
                                                          const double* __restrict__ x, double* __restrict__ y) {
    extern __shared__ double pad_lds[];
    const int lane = threadIdx.x & 63;
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;
    const int64_t W = (int64_t)G * 16;
    const int64_t g = (int64_t)L * 16 + (threadIdx.x >> 6);
    const int64_t s0 = g * nslices / W, s1 = (g + 1) * nslices / W;
    for (int64_t s = s0; s < s1; ++s) {
        const int uo = __builtin_amdgcn_readfirstlane(uoff[s]);
        if (uo < 0) continue;
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        const int np = w >> 1;
        const int base = (int)(s * 64 + lane);
        const double2* v2 = reinterpret_cast<const double2*>(vals + p0) + lane;
        const int32_t* c2 = reinterpret_cast<const int32_t*>(ucol + uo);
        double acc = 0.0;
        for (int j0 = 0; j0 < np; j0 += 2) {
            int32_t cc[2];
            double2 vv[2];
            double x0[2], x1[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) cc[j] = (j0 + j < np) ? c2[j0 + j] : 0;
#pragma unroll
            for (int j = 0; j < 2; ++j) vv[j] = (j0 + j < np) ? v2[64 * (j0 + j)] : double2{0.0, 0.0};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int lo = (int)(int16_t)(cc[j] & 0xffff);
                if constexpr (MODE == 2) {
                    x0[j] = 1.0 + lo;
                    x1[j] = 1.0;
                } else {
                    x0[j] = (j0 + j < np) ? x[base + lo] : 0.0;
                    x1[j] = x0[j];
                }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
                if (j0 + j < np) {
                    acc += vv[j].x * x0[j];
                    acc += vv[j].y * x1[j];
                }
        }
        if (w & 1) {
            const int64_t t = p0 + (int64_t)np * 128 + lane;
            acc += vals[t] * (MODE == 2 ? 1.0 : x[base + (int)ucol[uo + w - 1]]);
        }
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = acc;
    }
    if (nrows < 0) pad_lds[threadIdx.x] = 0.0;
}

}  // namespace fem

using namespace fem;

extern "C" {

int fem_lab_copy(int width, int read_only, const double* src, double* dst, int64_t n, int grid, fem_stream_t stream) {
    if (grid <= 0) grid = 2048;
    const hipStream_t st = S(stream);
    if (read_only) {
        if (width == 8) hipLaunchKernelGGL(k_read_w<8>, dim3(grid), dim3(256), 0, st, src, n, dst);
        else hipLaunchKernelGGL(k_read_w<16>, dim3(grid), dim3(256), 0, st, src, n, dst);
    } else if (width == 8) {
        hipLaunchKernelGGL(k_copy_w<8>, dim3(grid), dim3(256), 0, st, src, dst, n);
    } else if (width == 16) {
        hipLaunchKernelGGL(k_copy_w<16>, dim3(grid), dim3(256), 0, st, src, dst, n);
    } else {
        hipLaunchKernelGGL(k_copy_w<32>, dim3(grid), dim3(256), 0, st, src, dst, n);
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_sell_pair(int64_t nrows, const int64_t* slice_ptr, const double* vals, const int16_t* dcols,
                      double* vals_out, int16_t* dcols_out, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_sell_pair, dim3(stream_grid(ns * 64, 256)), dim3(256), 0, S(stream), ns, slice_ptr, vals,
                       dcols, vals_out, dcols_out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv16_pair(int u, int grid, int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols,
                        const double* vals, const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    if (grid <= 0) grid = grid_multiple_of_xcd(cdiv(ns, 4), 2048);
    grid = ((grid + NXCD - 1) / NXCD) * NXCD;
    const hipStream_t st = S(stream);
    if (u == 2) hipLaunchKernelGGL(k_spmv16_pair<2>, dim3(grid), dim3(256), 0, st, ns, nrows, slice_ptr, dcols, vals, x, y);
    else if (u == 8) hipLaunchKernelGGL(k_spmv16_pair<8>, dim3(grid), dim3(256), 0, st, ns, nrows, slice_ptr, dcols, vals, x, y);
    else hipLaunchKernelGGL(k_spmv16_pair<4>, dim3(grid), dim3(256), 0, st, ns, nrows, slice_ptr, dcols, vals, x, y);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv_persist(int threads, int u, int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                         const int16_t* dcols, const double* vals, const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    const hipStream_t st = S(stream);
#define LP(TT, UU)                                                                                              \
    hipLaunchKernelGGL((k_spmv_persist_lab<TT, UU>), dim3(grid), dim3(TT), (size_t)lds_bytes, st, ns, nrows, \
                       slice_ptr, dcols, vals, x, y)
    if (threads == 512) {
        if (u == 4) LP(512, 4); else LP(512, 8);
    } else if (threads == 1024) {
        if (u == 4) LP(1024, 4); else LP(1024, 8);
    } else {
        if (u == 4) LP(256, 4); else LP(256, 8);
    }
#undef LP
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_sell3_layout(int layout, int64_t nrows, const int64_t* slice_ptr, const double* vals,
                         const int16_t* dcols, double* vals_out, int16_t* dcols_out, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    const int g = stream_grid(ns * 64, 256);
    if (layout == 1) hipLaunchKernelGGL(k_sell3_to_a, dim3(g), dim3(256), 0, S(stream), ns, slice_ptr, vals, vals_out);
    else hipLaunchKernelGGL(k_sell3_to_b, dim3(g), dim3(256), 0, S(stream), ns, slice_ptr, vals, dcols, vals_out, dcols_out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv3(int layout, int u, int nt, int grid, int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols,
                  const double* vals, const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    if (grid <= 0) grid = grid_multiple_of_xcd(cdiv(ns, 4), 2048);
    grid = ((grid + NXCD - 1) / NXCD) * NXCD;
    const hipStream_t st = S(stream);
#define L3(LL, UU, NN) \
    hipLaunchKernelGGL((k_spmv3_lab<LL, UU, NN>), dim3(grid), dim3(256), 0, st, ns, nrows, slice_ptr, dcols, vals, x, y)
#define L3U(LL, NN)              \
    if (u == 2) L3(LL, 2, NN);   \
    else L3(LL, 1, NN);
#define L3N(LL)              \
    if (nt) { L3U(LL, true) } \
    else { L3U(LL, false) }
    if (layout == 0) { L3N(0) }
    else if (layout == 1) { L3N(1) }
    else if (layout == 3) { L3N(3) }
    else { L3N(2) }
#undef L3N
#undef L3U
#undef L3
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_sell_uniform(int64_t nrows, const int64_t* slice_ptr, const double* vals, const int16_t* dcols,
                         double* vals_out, int16_t* dcols_out, int16_t* ucol, int32_t* uoff, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_sell_uniform, dim3((unsigned)cdiv(ns, 4)), dim3(256), 0, S(stream), ns, nrows, slice_ptr, vals,
                       dcols, vals_out, dcols_out, ucol, uoff, 1);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv_persist_uni(int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                             const int16_t* pcols, const double* pvals, const int32_t* uoff, const int16_t* ucol,
                             const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_spmv_persist_uni_lab, dim3(grid), dim3(1024), (size_t)lds_bytes, S(stream), ns, nrows,
                       slice_ptr, pcols, pvals, uoff, ucol, x, y);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv_sym(int grid, int64_t lds_bytes, int64_t nrows, const int64_t* uptr, const int32_t* ulist,
                     const int16_t* udel, const int32_t* lptr, const int32_t* ldel, const int32_t* lbase,
                     const double* uvals, const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    hipLaunchKernelGGL(k_spmv_sym_lab, dim3(grid), dim3(1024), (size_t)lds_bytes, S(stream), ns, nrows, uptr, ulist,
                       udel, lptr, ldel, lbase, uvals, x, y);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_lab_spmv_gather(int mode, int grid, int64_t lds_bytes, int64_t nrows, const int64_t* slice_ptr,
                        const double* pvals, const int32_t* uoff, const int16_t* ucol, const double* x, double* y,
                        fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    if (mode == 2)
        hipLaunchKernelGGL(k_spmv_gather_lab<2>, dim3(grid), dim3(1024), (size_t)lds_bytes, S(stream), ns, nrows,
                           slice_ptr, pvals, uoff, ucol, x, y);
    else
        hipLaunchKernelGGL(k_spmv_gather_lab<1>, dim3(grid), dim3(1024), (size_t)lds_bytes, S(stream), ns, nrows,
                           slice_ptr, pvals, uoff, ucol, x, y);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // extern "C"
