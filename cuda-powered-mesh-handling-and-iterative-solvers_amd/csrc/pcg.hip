// SELL-64 SpMV and the device-resident (P)CG iteration (L2 + L3 of the hot path).
//
// Replaces the reference's per-iteration op chain (`solver/solver.py:182-224` / `:798-810`): EBE matvec via
// gather + bmm + index_add (`solver/element.py:429-464`), torch.sum dots and axpys. No host synchronisation
// inside the iteration: scalars, guards and the stop flag live in a device state word, kernels after a stop
// are no-ops, and the host polls once per chunk of iterations.
//
// Kernel schedules (same arithmetic, same results up to fp rounding order):
//   3-kernel  K1 spmv_dot : q = A p, p.q               -> alpha, guards            (default for bs = 3, dist)
//             K2 update   : r -= alpha q, z = w r, r.z -> stop test, beta
//             K3 pupdate  : x += alpha p ; p = z + beta p
//   fused     K1 spmv_dot : x += alpha' p' ; p = w r + beta p' computed on the fly for every gathered column
//                           (double-buffered p), q = A p, p.q
//             K2 update   (as above)                          -> 2 launches and 88 n bytes of vectors per iteration
//   deferred  d1 / d2 / d3: the 3-kernel work without grid atomics, each kernel re-summing the previous kernel's
//             per-block partials (default for bs = 1)
//   distributed single reduction: k_cg1_update / k_cg1_spmv (step evaluated in both), one exchange per iteration
// Grid reductions are deterministic two-level trees (common.hpp reduce_grid).
#include <rccl/rccl.h>
#include <stddef.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "sell_pair.hpp"
#include "sell_pair3.hpp"
#include "matfree.hpp"

namespace fem {

template <typename T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// Vector operands of the SpMV: a plain vector, or the fused p = w r + beta p_old evaluated per gathered dof.
struct VecPlain {
    const double* x;
    __device__ __forceinline__ double operator()(int64_t i) const { return x[i]; }
};
struct VecFusedP {
    const double* r;
    const double* w;
    const double* pold;
    double beta;
    __device__ __forceinline__ double operator()(int64_t i) const { return w[i] * r[i] + beta * pold[i]; }
};

// ---------------------------------------------------------------- SELL SpMV core
// One wave = one slice of 64 block rows; lane = row. Row entries are strided by 64, so every load of the
// wave (cols, each of the bs*bs value planes) is one contiguous 256/512-byte segment; on meshes numbered
// along lines the x gathers of neighbouring lanes are contiguous too. U entries per step: all U column loads,
// then U value loads, then U gathers are in flight together; the tail step is predicated.
// CI = int32_t: absolute block columns; CI = int16_t: 16-bit deltas col - row (half the index bytes)
#ifndef FEM_SPMV_UB
#define FEM_SPMV_UB 1
#endif
constexpr int SPMV_UB = FEM_SPMV_UB;   // bs > 1: blocks in flight per lane
#ifndef FEM_SPMV_NT3
#define FEM_SPMV_NT3 1
#endif
constexpr bool SPMV_NT3 = FEM_SPMV_NT3;   // bs > 1 in the PCG kernels: nontemporal matrix loads keep the p
                                          // gather window in L2 (10M elastic K1 420 -> 406 us, PMC 1.115x alg)

template <int BS, int U, bool NT, typename X, typename CI = int32_t>
__device__ __forceinline__ void sell_row(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                         const CI* __restrict__ cols, const double* __restrict__ vals,
                                         const X& x, double out[BS]) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const CI* c = cols + p0 + lane;
    const int base = (sizeof(CI) == 2) ? (int)(s * 64 + lane) : 0;
#pragma unroll
    for (int r = 0; r < BS; ++r) out[r] = 0.0;
    if (BS == 1) {
        const double* v = vals + p0 + lane;
        for (int k0 = 0; k0 < w; k0 += U) {
            int ci[U];
            double vi[U], xi[U];
#pragma unroll
            for (int j = 0; j < U; ++j) ci[j] = (k0 + j < w) ? base + (int)ld<CI, NT>(c + 64 * (k0 + j)) : 0;
#pragma unroll
            for (int j = 0; j < U; ++j) vi[j] = (k0 + j < w) ? ld<double, NT>(v + 64 * (k0 + j)) : 0.0;
#pragma unroll
            for (int j = 0; j < U; ++j) xi[j] = (k0 + j < w) ? x(ci[j]) : 0.0;
#pragma unroll
            for (int j = 0; j < U; ++j)
                if (k0 + j < w) out[0] += vi[j] * xi[j];
        }
    } else {
        // UB blocks in flight: UB column loads, UB*bs^2 plane loads, UB*bs gathers, then the FMAs in (k, r, j)
        // order — the same per-row order as one block at a time
        constexpr int UB = SPMV_UB;
        const double* v = vals + p0 * (BS * BS) + lane;
        for (int k0 = 0; k0 < w; k0 += UB) {
            int64_t cc[UB];
            double vv[UB][BS * BS], xv[UB][BS];
#pragma unroll
            for (int u = 0; u < UB; ++u)
                cc[u] = (k0 + u < w) ? (int64_t)(base + (int)ld<CI, NT>(c + 64 * (k0 + u))) * BS : 0;
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const double* vk = v + (int64_t)64 * BS * BS * (k0 + u);
#pragma unroll
                for (int e = 0; e < BS * BS; ++e) vv[u][e] = (k0 + u < w) ? ld<double, NT>(vk + 64 * e) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < UB; ++u)
#pragma unroll
                for (int j = 0; j < BS; ++j) xv[u][j] = (k0 + u < w) ? x(cc[u] + j) : 0.0;
#pragma unroll
            for (int u = 0; u < UB; ++u)
                if (k0 + u < w) {
#pragma unroll
                    for (int r = 0; r < BS; ++r)
#pragma unroll
                        for (int j = 0; j < BS; ++j) out[r] += vv[u][r * BS + j] * xv[u][j];
                }
        }
    }
}

// XCD-aware slice walk: XCD x (= blockIdx % 8 under the observed round-robin placement; speed only) owns the
// contiguous slice range [x*spx, (x+1)*spx), walked 4 slices (one per wave) per block step, so the x-gather
// window of an XCD stays in its own L2.
struct SliceWalk {
    int64_t s, end, step, first;
};

__device__ __forceinline__ SliceWalk slice_walk(int64_t nslices) {
    const int xcd = blockIdx.x % NXCD;
    const int64_t lb = blockIdx.x / NXCD, nlb = gridDim.x / NXCD;
    const int64_t spx = (nslices + NXCD - 1) / NXCD;
    const int64_t start = (int64_t)xcd * spx;
    const int64_t end = min(start + spx, nslices);
    return SliceWalk{start + lb * 4 + (threadIdx.x >> 6), end, nlb * 4, start};
}

constexpr int SPMV_U = 8;   // tools/spmv_tune.py: U=8 beats 4 and 16 on the 10M Poisson matrix (gfx950)
constexpr int SPMV_UP = 8;  // pairs in flight of the paired layout (tools/spmv_layout.py: 2, 4, 8 within 1 %)

// SpMV row of the 16-byte-value copy of the matrix: bs = 1 lane-paired layout (sell_pair.hpp), bs = 3 plane-paired
// layout A (sell_pair3.hpp: 4 sixteen-byte + 1 eight-byte value loads per block, nontemporal; tools/spmv3_layout.py:
// 10M elastic 369 -> 348 us stand-alone). Both keep the plain layout's per-row summation order.
#ifndef FEM_K1_U3
#define FEM_K1_U3 1   // bs = 3 blocks in flight per lane (layout A)
#endif
#ifndef FEM_K1_G3
#define FEM_K1_G3 0   // bs = 3 gathers: 0 = three 8-byte loads, 1 = 8 + 16 bytes
#endif
template <int BS>
__device__ __forceinline__ void sell_row_paired(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                                const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                const double* __restrict__ x, double out[BS]) {
    if constexpr (BS == 1) out[0] = sell_row_pair<SPMV_UP>(s, lane, slice_ptr, cols, vals, x);
    else sell3_row_a<FEM_K1_U3, SPMV_NT3, FEM_K1_G3>(s, lane, slice_ptr, cols, vals, x, out);
}

template <int BS, int U = SPMV_U, bool NT = false, typename CI = int32_t>
__global__ void __launch_bounds__(256) k_spmv(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                                              const CI* __restrict__ cols, const double* __restrict__ vals,
                                              const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    SliceWalk wk = slice_walk(nslices);
    const VecPlain xv{x};
    for (int64_t s = wk.s; s < wk.end; s += wk.step) {
        double o[BS];
        sell_row<BS, U, NT, VecPlain, CI>(s, lane, slice_ptr, cols, vals, xv, o);
        const int64_t row = s * 64 + lane;
        if (row < nrows) {
#pragma unroll
            for (int r = 0; r < BS; ++r) y[row * BS + r] = o[r];
        }
    }
}

// y = A x on the lane-paired layout (bs = 1; slice-uniform deltas where uoff says so): the solver layout's SpMV
template <int U>
__global__ void __launch_bounds__(256) k_spmv_pair(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                                                   const int16_t* __restrict__ pcols, const double* __restrict__ pvals,
                                                   const int32_t* __restrict__ uoff, const int16_t* __restrict__ ucol,
                                                   const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    SliceWalk wk = slice_walk(nslices);
    for (int64_t s = wk.s; s < wk.end; s += wk.step) {
        const double v = sell_row_pair<U>(s, lane, slice_ptr, pcols, pvals, x, 0, 0, uoff, ucol);
        const int64_t row = s * 64 + lane;
        if (row < nrows) y[row] = v;
    }
}

// y = A x on the plane-paired layout A (bs = 3, plain 16-bit columns): the bs = 3 solver layout's SpMV
__global__ void __launch_bounds__(256) k_spmv_a(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                                                const int16_t* __restrict__ cols, const double* __restrict__ pvals,
                                                const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    SliceWalk wk = slice_walk(nslices);
    for (int64_t s = wk.s; s < wk.end; s += wk.step) {
        double o[3];
        sell_row_paired<3>(s, lane, slice_ptr, cols, pvals, x, o);
        const int64_t row = s * 64 + lane;
        if (row < nrows) {
#pragma unroll
            for (int r = 0; r < 3; ++r) y[row * 3 + r] = o[r];
        }
    }
}

// ---------------------------------------------------------------- PCG device state
struct PcgState {
    double rz;        // r.z of the current iterate (rs_old)
    double pq;        // p.Ap of this iteration
    double alpha;     // alpha of this iteration (K1 -> K2)
    double alpha_x;   // alpha of the last completed update, for the deferred x update (K2 -> next K1 / finish)
    double beta;      // K2 -> next K1 / K3
    double rz_new;
    double tol, eps;
    int iter;         // completed iterations
    int status;       // FEM_PCG_*
    int halt;         // 1: solve ended, iteration kernels are no-ops
    int xupd;         // 3-kernel: K2 ran this iteration -> K3 applies x += alpha p
    int x_done;       // fused: 0 while an x update is pending (applied by the next K1 or by finish)
    int stop_iter;    // reported iteration of a guard stop (i+1 in the reference prints)
    int max_iter;
    int mode;
    int dist;         // 1: element-partitioned; reductions land in red[] and are all-reduced (RCCL) first
    double red[4];    // dist: rank-local partial sums p.q, r.z, r0.z0 (all-reduced in place)
    // deferred schedule: per-iteration state banked by the host's launch parity (see k_pcg_d*)
    struct Bank {
        double rz;        // r.z of the current iterate
        double beta;      // beta to form this iteration's p (unused: p is formed in d3)
        int iter;         // completed iterations
        int halt;
        int status;
        int stop_iter;
        int k2stop;       // set by d2 of this bank's iteration: FEM_PCG_BREAKDOWN / ALPHA_NAN
        int pad_;
        double alpha;     // written by d2 block 0 (read by d3)
        double pq;
        double rz_new;
    } bank[2];
    // persistent schedule: grid-barrier epochs completed so far. The sync words (group counters, top replicas,
    // u-flags) count monotonically across launches from this base, so a launch needs no memset of them first
    // (zeroed by fem_pcg_start, and by the host before the counters could wrap)
    unsigned pk_epoch;
    unsigned pk_pad_;
    // merged update (k_pcg_update2): launches completed since fem_pcg_start (the epoch its release word counts)
    unsigned u2_epoch;
    unsigned u2_pad_;
};

constexpr int PCG_BLOCK = 256;
constexpr int MAX_PARTIALS = 4096;   // >= grid + RED_SHARDS for every reduction kernel
enum { RED_K1 = 0, RED_K2 = 1, RED_INIT = 2, RED_N = 3 };

// alpha and the breakdown guards from p.Ap (`solver/solver.py:185-198` / `:800`)
__device__ __forceinline__ void finish_pq(PcgState* st, double pq) {
    st->pq = pq;
    if (st->mode != FEM_MODE_PCG) {
        if (fabs(pq) < st->eps || pq < 0.0) {                 // `solver/solver.py:187`
            st->status = FEM_PCG_BREAKDOWN;
            st->halt = 1;
            st->stop_iter = st->iter + 1;
        } else {
            const double a = st->rz / (pq + st->eps);          // `:194`
            st->alpha = a;
            if (isnan(a) || isinf(a)) {                        // `:196`
                st->status = FEM_PCG_ALPHA_NAN;
                st->halt = 1;
                st->stop_iter = st->iter + 1;
            }
        }
    } else {
        st->alpha = st->rz / pq;                              // `:800` (no guards)
    }
}

// stop test and beta from the new r.z (`solver/solver.py:208-222` / `:804-809`)
__device__ __forceinline__ void finish_rz(PcgState* st, double rz_new, double* hist, int64_t hist_len) {
    const bool cg = st->mode != FEM_MODE_PCG;
    const int it = st->iter;
    st->rz_new = rz_new;
    st->xupd = 1;
    st->x_done = 0;
    st->alpha_x = st->alpha;
    st->iter = it + 1;
    const double nrm = sqrt(rz_new);
    if (hist && it < hist_len) hist[it] = nrm;
    if (nrm < st->tol) {                                      // `:210` / `:805`
        st->status = FEM_PCG_CONVERGED;
        st->halt = 1;
        st->stop_iter = it + 1;
    } else {
        const double b = cg ? rz_new / (st->rz + st->eps) : rz_new / st->rz;   // `:213` / `:808`
        st->beta = b;
        if (cg && (isnan(b) || isinf(b))) {                   // `:214`
            st->status = FEM_PCG_BETA_NAN;
            st->halt = 1;
            st->stop_iter = it + 1;
        }
        st->rz = rz_new;
    }
}

struct RedBuf {
    double* partials;    // [RED_N][MAX_PARTIALS]
    unsigned* counters;  // [RED_N][RED_COUNTER_WORDS]
    __device__ __forceinline__ double* part(int k) const { return partials + k * MAX_PARTIALS; }
    __device__ __forceinline__ unsigned* cnt(int k) const { return counters + k * RED_COUNTER_WORDS; }
};

// K1. FUSED: p (in p_buf[iter & 1]) is formed on the fly from r, w and the previous p (p_buf[(iter+1) & 1]);
// this kernel also applies the deferred x += alpha_x p_prev to its own rows.
template <int BS, bool FUSED, bool DOT = true, typename CI = int32_t, bool PAIR = false>
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_spmv_dot(int64_t nslices, int64_t nrows,
                                                            const int64_t* __restrict__ slice_ptr,
                                                            const CI* __restrict__ cols,
                                                            const double* __restrict__ vals, double* __restrict__ p0,
                                                            double* __restrict__ p1, const double* __restrict__ r,
                                                            const double* __restrict__ w, double* __restrict__ x,
                                                            double* __restrict__ q, PcgState* __restrict__ st,
                                                            RedBuf red, int tune_rev) {
    __shared__ double lds4[4];
    __shared__ int flag;
    if (!FUSED && blockIdx.x == 0 && threadIdx.x == 0) st->xupd = 0;
    const int iter = st->iter;
    if (st->halt || iter >= st->max_iter) return;
    const int lane = threadIdx.x & 63;
    double dot = 0.0;
    SliceWalk wk = slice_walk(nslices);
    if (FUSED) {
        double* pnew = (iter & 1) ? p1 : p0;
        const double* pold = (iter & 1) ? p0 : p1;
        const double beta = st->beta, ax = st->alpha_x;
        const VecFusedP pv{r, w, pold, beta};
        for (int64_t s = wk.s; s < wk.end; s += wk.step) {
            double o[BS];
            sell_row<BS, SPMV_U, (BS > 1 && SPMV_NT3), decltype(pv), CI>(s, lane, slice_ptr, cols, vals, pv, o);
            const int64_t row = s * 64 + lane;
            if (row < nrows) {
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    const int64_t i = row * BS + c;
                    const double po = pold[i];
                    const double pn = w[i] * r[i] + beta * po;
                    x[i] += ax * po;
                    pnew[i] = pn;
                    q[i] = o[c];
                    dot += pn * o[c];
                }
            }
        }
    } else {
        const VecPlain pv{p0};
        // odd iterations sweep backwards (FEM_TUNE_REVERSE; parity from the device iteration count)
        const bool rev = tune_rev && (iter & 1);
        const int64_t mirror = wk.first + wk.end - 1;
        for (int64_t s0 = wk.s; s0 < wk.end; s0 += wk.step) {
            const int64_t s = rev ? mirror - s0 : s0;
            double o[BS];
            if constexpr (PAIR) sell_row_paired<BS>(s, lane, slice_ptr, cols, vals, p0, o);
            else sell_row<BS, SPMV_U, (BS > 1 && SPMV_NT3), decltype(pv), CI>(s, lane, slice_ptr, cols, vals, pv, o);
            const int64_t row = s * 64 + lane;
            if (row < nrows) {
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    q[row * BS + c] = o[c];
                    if (DOT) dot += p0[row * BS + c] * o[c];
                }
            }
        }
    }
    if (!DOT) return;
    // distributed: q is this rank's partial on interface rows; p.q_partial over ALL local rows summed over the
    // ranks is exactly p.q, so the rank sum rides in the halo all-reduce (k_halo_pack appends st->red[0])
    dot = block_sum256(dot, lds4);
    double pq;
    if (reduce_grid(dot, red.part(RED_K1), red.cnt(RED_K1), &pq, lds4, &flag) && threadIdx.x == 0) {
        if (st->dist) {
            st->red[0] = pq;
        } else {
            if (FUSED) st->x_done = 1;   // the pending x update was applied above by every block
            finish_pq(st, pq);
        }
    }
}

// K2: r <- r - alpha q (CG: masked), z = w r, partial r.z (CG: r.r since w is the 0/1 free mask)
// own (distributed only, else null): 1 on the rows (nodes) this rank owns, so shared dofs count once in r.z
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_update(int64_t n, double* __restrict__ r,
                                                          const double* __restrict__ q, const double* __restrict__ w,
                                                          PcgState* __restrict__ st, RedBuf red,
                                                          double* __restrict__ hist, int64_t hist_len,
                                                          const uint8_t* __restrict__ own, int bs) {
    __shared__ double lds4[4];
    __shared__ int flag;
    if (st->halt || st->iter >= st->max_iter) return;
    const double alpha = st->alpha;
    const bool cg = st->mode != FEM_MODE_PCG;
    double acc = 0.0;
    const int64_t n2 = n >> 1;
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double2* r2 = reinterpret_cast<double2*>(r);
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < n2; i += (int64_t)gridDim.x * PCG_BLOCK) {
        double2 rv = r2[i], qv = q2[i], wv = w2[i];
        rv.x = rv.x - alpha * qv.x;
        rv.y = rv.y - alpha * qv.y;
        if (cg) {
            if (wv.x == 0.0) rv.x = 0.0;
            if (wv.y == 0.0) rv.y = 0.0;
        }
        r2[i] = rv;
        if (own) {
            if (own[(2 * i) / bs]) acc += rv.x * (wv.x * rv.x);
            if (own[(2 * i + 1) / bs]) acc += rv.y * (wv.y * rv.y);
        } else {
            acc += rv.x * (wv.x * rv.x);
            acc += rv.y * (wv.y * rv.y);
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        int64_t i = n - 1;
        double rv = r[i] - alpha * q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        if (!own || own[i / bs]) acc += rv * (w[i] * rv);
    }
    acc = block_sum256(acc, lds4);
    double rz_new;
    if (reduce_grid(acc, red.part(RED_K2), red.cnt(RED_K2), &rz_new, lds4, &flag) && threadIdx.x == 0) {
        if (st->dist) st->red[1] = rz_new;   // all-reduced, then k_fin_rz
        else finish_rz(st, rz_new, hist, hist_len);
    }
}

// K3 (3-kernel schedule): x <- x + alpha p ; p <- w r + beta p (unless stopped in K2)
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_pupdate(int64_t n, double* __restrict__ x, double* __restrict__ p,
                                                           const double* __restrict__ r, const double* __restrict__ w,
                                                           const PcgState* __restrict__ st) {
    if (!st->xupd) return;
    const double alpha = st->alpha, beta = st->beta;
    const bool upd_p = !st->halt;
    const int64_t n2 = n >> 1;
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
    const double2* r2 = reinterpret_cast<const double2*>(r);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < n2; i += (int64_t)gridDim.x * PCG_BLOCK) {
        double2 pv = p2[i], xv = x2[i];
        xv.x += alpha * pv.x;
        xv.y += alpha * pv.y;
        x2[i] = xv;
        if (upd_p) {
            double2 rv = r2[i], wv = w2[i];
            pv.x = wv.x * rv.x + beta * pv.x;
            pv.y = wv.y * rv.y + beta * pv.y;
            p2[i] = pv;
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        int64_t i = n - 1;
        x[i] += alpha * p[i];
        if (upd_p) p[i] = w[i] * r[i] + beta * p[i];
    }
}

// K2 + K3 as ONE launch (3-kernel schedule, FEM_TUNE_UPD1): r <- r - alpha q, z = w r and the r.z partials; the
// last-arriving workgroup finishes r.z (stop test, beta: finish_rz) and releases the others through a write-through
// broadcast + an epoch word (MI355X_MICROARCH.md visibility table: sc1 stores drained before the releasing atomic,
// sc1 loads after the poll); then x <- x + alpha p and p <- z + beta p. Each thread keeps the z of its first U2_NPT
// elements in registers across the wait, so r and w are read once per iteration (8 vector streams instead of the
// two kernels' 10) and one launch boundary fewer. Every workgroup must be resident at once: the grid is sized from
// the occupancy query (u2_setup); the wait is bounded in time (FEM_PCG_SYNC_TIMEOUT, never a hang).
constexpr int U2_NPT = 8;                 // double2 elements per thread whose z stays in registers
enum { U2_REL = 0, U2_BC = 32, U2_WORDS = 96 };   // release word, broadcast (beta, halt)
constexpr unsigned U2_GIVEUP = 0xffffffffu;        // release-word value of a launch a waiter gave up on
constexpr uint64_t U2_WAIT_TICKS = 200000000ull;   // 2 s of s_memrealtime (100 MHz)
// sync-site code of a merged-update give-up (fem_pcg_sync_site; the persistent kernel's codes are 1-3)
constexpr int U2_SITE = 4;

// the give-up verdict (status, halt, site) with atomic stores: every writer of a given launch stores the same values
__device__ __forceinline__ void u2_give_up(PcgState* st, unsigned e) {
    __hip_atomic_store(&st->stop_iter, U2_SITE + 16 * (int)(e & 0x7ffffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->status, (int)FEM_PCG_SYNC_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->halt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The merged update's hand-off (every form of it): the block sums of r.z, the grid reduction, the last workgroup's
// finish_rz and release, the others' bounded wait and read of the broadcast (beta, halt). false: the launch gave up
// (no x / p update anywhere).
__device__ __forceinline__ bool u2_release(double acc, PcgState* __restrict__ st, RedBuf red, double* __restrict__ hist,
                                           int64_t hist_len, unsigned* __restrict__ sync, unsigned e, double* lds4,
                                           int* flag_p, double* bc_s, double& beta, bool& upd_p, bool& last) {
    int& flag = *flag_p;
    acc = block_sum256(acc, lds4);
    double rz_new;
    last = reduce_grid(acc, red.part(RED_K2), red.cnt(RED_K2), &rz_new, lds4, &flag);
    if (threadIdx.x == 0) {
        // The release word decides the launch ONCE, by compare-and-swap from the previous epoch (e - 1): the last
        // workgroup swaps in e (release), a waiter that gave up swaps in U2_GIVEUP. Whichever swap lands first
        // wins, so either every workgroup applies the x / p update or none does (then r holds r_{k+1} and x x_k,
        // the status is FEM_PCG_SYNC_TIMEOUT with the give-up site, and fem_pcg_solve re-solves from x0).
        double beta_ = 0.0, halt = 0.0;
        bool ok = true;
        if (last) {
            const int it0 = st->iter;
            finish_rz(st, rz_new, hist, hist_len);
            beta_ = st->beta;
            halt = st->halt ? 1.0 : 0.0;
            __hip_atomic_store(reinterpret_cast<double*>(sync + U2_BC), beta_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<double*>(sync + U2_BC) + 1, halt, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            // the broadcast's write-through stores drained before the release (the guide's sc1 hand-off form; the
            // asm's memory clobber also keeps the compiler from moving them past the swap); FEM_MM_ACQREL: a release
            // swap instead
            fem_drain_stores();
            unsigned expect = e - 1;
            if (!__hip_atomic_compare_exchange_strong(sync + U2_REL, &expect, e,
                                                      FEM_MM_ACQREL ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                // a waiter gave up first: undo the commit (the iteration did not complete) and keep its verdict
                st->iter = it0;
                u2_give_up(st, e);
                ok = false;
            }
        } else {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            unsigned v = 0;
            for (unsigned spins = 0;; ++spins) {
                v = __hip_atomic_load(sync + U2_REL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v != e - 1) break;   // released (e) or given up (U2_GIVEUP)
                if ((spins & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > U2_WAIT_TICKS) {
                    unsigned expect = e - 1;
                    if (__hip_atomic_compare_exchange_strong(sync + U2_REL, &expect, U2_GIVEUP, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        v = U2_GIVEUP;   // a workgroup that never became resident: stop instead of hanging
                    else
                        v = expect;      // the release landed first
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            // no load below may be moved above the poll by the compiler (the hardware issues it only after the
            // branch on the polled value); the broadcast is read with write-through (sc1) loads. FEM_MM_ACQREL: one
            // agent-scope acquire after the poll matched
#if FEM_MM_ACQREL
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#else
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
            if (v == e) {
                beta_ = __hip_atomic_load(reinterpret_cast<const double*>(sync + U2_BC), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
                halt = __hip_atomic_load(reinterpret_cast<const double*>(sync + U2_BC) + 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            } else {
                u2_give_up(st, e);
                ok = false;
            }
        }
        bc_s[0] = beta_;
        bc_s[1] = ok ? halt : -1.0;
    }
    __syncthreads();
    beta = bc_s[0];
    if (bc_s[1] < 0.0) return false;
    upd_p = bc_s[1] == 0.0;
    return true;
}

__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_update2(int64_t n, double* __restrict__ x, double* __restrict__ p,
                                                           double* __restrict__ r, const double* __restrict__ q,
                                                           const double* __restrict__ w, PcgState* __restrict__ st,
                                                           RedBuf red, double* __restrict__ hist, int64_t hist_len,
                                                           unsigned* __restrict__ sync, int hold) {
    __shared__ double lds4[4];
    __shared__ int flag;
    __shared__ double bc_s[2];
    if (st->halt || st->iter >= st->max_iter) return;
    if (hold && blockIdx.x == 0) {   // FEM_TUNE_U2_HOLD (tests): workgroup 0 arrives after every waiter gave up
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < U2_WAIT_TICKS + U2_WAIT_TICKS / 2) __builtin_amdgcn_s_sleep(127);
        }
        __syncthreads();
    }
    const unsigned e = st->u2_epoch + 1;
    const double alpha = st->alpha;
    const bool cg = st->mode != FEM_MODE_PCG;
    const int64_t n2 = n >> 1, stride = (int64_t)gridDim.x * PCG_BLOCK;
    const int64_t i0 = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x;
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double2* r2 = reinterpret_cast<double2*>(r);
    double2 z[U2_NPT];
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < U2_NPT; ++k) {
        const int64_t i = i0 + k * stride;
        z[k] = make_double2(0.0, 0.0);
        if (i < n2) {
            double2 rv = r2[i], qv = q2[i], wv = w2[i];
            rv.x = rv.x - alpha * qv.x;
            rv.y = rv.y - alpha * qv.y;
            if (cg) {
                if (wv.x == 0.0) rv.x = 0.0;
                if (wv.y == 0.0) rv.y = 0.0;
            }
            r2[i] = rv;
            z[k] = make_double2(wv.x * rv.x, wv.y * rv.y);
            acc += rv.x * z[k].x;
            acc += rv.y * z[k].y;
        }
    }
    for (int64_t i = i0 + U2_NPT * stride; i < n2; i += stride) {   // past the register capacity
        double2 rv = r2[i], qv = q2[i], wv = w2[i];
        rv.x = rv.x - alpha * qv.x;
        rv.y = rv.y - alpha * qv.y;
        if (cg) {
            if (wv.x == 0.0) rv.x = 0.0;
            if (wv.y == 0.0) rv.y = 0.0;
        }
        r2[i] = rv;
        acc += rv.x * (wv.x * rv.x);
        acc += rv.y * (wv.y * rv.y);
    }
    double ztail = 0.0;
    const bool tail = (n & 1) && blockIdx.x == 0 && threadIdx.x == 0;
    if (tail) {
        const int64_t i = n - 1;
        double rv = r[i] - alpha * q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        ztail = w[i] * rv;
        acc += rv * ztail;
    }
    double beta;
    bool upd_p, last;
    if (!u2_release(acc, st, red, hist, hist_len, sync, e, lds4, &flag, bc_s, beta, upd_p, last)) return;
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
#pragma unroll
    for (int k = 0; k < U2_NPT; ++k) {
        const int64_t i = i0 + k * stride;
        if (i < n2) {
            double2 pv = p2[i], xv = x2[i];
            xv.x += alpha * pv.x;
            xv.y += alpha * pv.y;
            x2[i] = xv;
            if (upd_p) {
                pv.x = z[k].x + beta * pv.x;
                pv.y = z[k].y + beta * pv.y;
                p2[i] = pv;
            }
        }
    }
    for (int64_t i = i0 + U2_NPT * stride; i < n2; i += stride) {
        double2 pv = p2[i], xv = x2[i];
        xv.x += alpha * pv.x;
        xv.y += alpha * pv.y;
        x2[i] = xv;
        if (upd_p) {
            const double2 rv = r2[i], wv = w2[i];
            pv.x = wv.x * rv.x + beta * pv.x;
            pv.y = wv.y * rv.y + beta * pv.y;
            p2[i] = pv;
        }
    }
    if (tail) {
        const int64_t i = n - 1;
        x[i] += alpha * p[i];
        if (upd_p) p[i] = ztail + beta * p[i];
    }
    if (last && threadIdx.x == 0) st->u2_epoch = e;   // every workgroup read the epoch before the release
}

// The merged update on the element-chunk operator: k_pcg_update2's thread layout (a double2 of dofs per thread-step,
// the z of the first U2_NPT in registers across the release, every vector stream read / written as 16-byte lanes),
// with q of each dof formed in place from the node-major slots -- q_d = the sum of node d / BS's slots, component
// d % BS, in ascending chunk order (k_mf_gather's sum, the same bits) -- so q is never stored. FROM_Q: q read from
// the array k_mf_gather wrote (the A/B form; the same bits again). The release protocol is k_pcg_update2's, and so is
// the order of every other operation: given equal q the update is bit-identical to k_pcg_update2's.
// (Round 5 ran one node per thread-step: three 8-byte accesses per vector 24 bytes apart across the lanes, 93 us for
// the 10M elastic cube's 380 MB.)
#ifndef FEM_MF_NTL
#define FEM_MF_NTL 0   // 1: the merged update reads the slots with non-temporal loads (read once)
#endif
// The first MF_QK slots of the node are loaded unconditionally (indices clamped to the node's last slot) and the ones
// past its count added as +0.0 -- the same bits (a sum started from +0.0 is never -0.0, and x + 0.0 == x otherwise),
// but the loads of all the thread's register-cached steps go out together instead of one dependent loop per dof
// (nodes have 2.06 slots on average on the 10M cube; more than MF_QK continue in a loop)
constexpr int MF_QK = 4;
#ifndef FEM_MF_QK_ON
#define FEM_MF_QK_ON 1   // 0: the plain loop (A/B)
#endif
template <int BS>
__device__ __forceinline__ double mf_q_dof(const MfOp& op, const double* __restrict__ slots, int64_t d) {
    const int64_t a = d / BS;
    const int c = (int)(d - a * BS);
    const int k0 = op.nptr[a], k1 = op.nptr[a + 1];
    double s = 0.0;
    if (FEM_MF_QK_ON && op.spos && k1 > k0) {   // node-major slots: the node's slots are k0 .. k1 - 1
        double v[MF_QK];
#pragma unroll
        for (int q = 0; q < MF_QK; ++q) {
            const int k = k0 + q < k1 ? k0 + q : k1 - 1;
#if FEM_MF_NTL
            v[q] = __builtin_nontemporal_load(&slots[(int64_t)k * BS + c]);
#else
            v[q] = slots[(int64_t)k * BS + c];
#endif
        }
#pragma unroll
        for (int q = 0; q < MF_QK; ++q) s += k0 + q < k1 ? v[q] : 0.0;
        for (int k = k0 + MF_QK; k < k1; ++k) s += slots[(int64_t)k * BS + c];
        return s;
    }
    for (int k = k0; k < k1; ++k) {
        const int64_t sl = op.spos ? k : op.nslot[k];
#if FEM_MF_NTL
        s += __builtin_nontemporal_load(&slots[sl * BS + c]);
#else
        s += slots[sl * BS + c];
#endif
    }
    return s;
}

// FEM_MF_QLDS = 1 (A/B): the slot values a wave's 128 dofs of one thread-step need -- one contiguous node-major range --
// staged into LDS by 16-byte lanes first (2-3 coalesced wave loads instead of 8 scattered 8-byte ones per dof pair),
// then summed from LDS in the same order (the same bits); ranges over MF_QCAP doubles take the direct loads.
// Measured slightly slower than the fixed-count direct loads (update 75.8-78.1 vs 73.4-75.9 us on the 10M elastic
// cube, profiles/r06l_mf_qlds_prof_ab.txt: the staging serialises a wave's thread-steps); off
#ifndef FEM_MF_QLDS
#define FEM_MF_QLDS 0
#endif
constexpr int MF_QCAP = 512;
template <int BS>
__device__ __forceinline__ bool mf_q_stage(const MfOp& op, const double* __restrict__ slots, double* qs, int64_t iw,
                                           int64_t i, int64_t n, int lane, double2& qv) {
    const int64_t d_lo = 2 * iw, d_hi = (2 * iw + 128 < n ? 2 * iw + 128 : n) - 1;
    const int64_t a_lo = d_lo / BS, a_hi = d_hi / BS;
    const int s_lo = op.nptr[a_lo], s_hi = op.nptr[a_hi + 1];
    const int64_t st0 = ((int64_t)BS * s_lo) & ~(int64_t)1;
    const int len = (int)((int64_t)BS * s_hi - st0);
    if (len > MF_QCAP) return false;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the previous step's LDS reads of this wave are done
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const double2* s2 = reinterpret_cast<const double2*>(slots + st0);
    for (int t = lane; 2 * t < len; t += 64) {
        if (2 * t + 1 < len) {
            const double2 v = s2[t];
            qs[2 * t] = v.x;
            qs[2 * t + 1] = v.y;
        } else {
            qs[2 * t] = slots[st0 + 2 * t];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double q[2] = {0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int64_t d = 2 * i + h;
        if (d < n) {
            const int64_t a = d / BS;
            const int c = (int)(d - a * BS);
            const int k0 = op.nptr[a], k1 = op.nptr[a + 1];
            double sum = 0.0;
            for (int k = k0; k < k1; ++k) sum += qs[(int64_t)BS * k + c - st0];
            q[h] = sum;
        }
    }
    qv = make_double2(q[0], q[1]);
    return true;
}

template <int BS, bool FROM_Q>
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_update2_mf(int64_t nn, double* __restrict__ x, double* __restrict__ p,
                                                              double* __restrict__ r, const double* __restrict__ q,
                                                              const double* __restrict__ w, PcgState* __restrict__ st,
                                                              RedBuf red, double* __restrict__ hist, int64_t hist_len,
                                                              unsigned* __restrict__ sync, int hold, MfOp op,
                                                              const double* __restrict__ slots) {
    __shared__ double lds4[4];
    __shared__ int flag;
    __shared__ double bc_s[2];
    if (st->halt || st->iter >= st->max_iter) return;
    if (hold && blockIdx.x == 0) {   // FEM_TUNE_U2_HOLD (tests)
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < U2_WAIT_TICKS + U2_WAIT_TICKS / 2) __builtin_amdgcn_s_sleep(127);
        }
        __syncthreads();
    }
    const unsigned e = st->u2_epoch + 1;
    const double alpha = st->alpha;
    const bool cg = st->mode != FEM_MODE_PCG;
    const int64_t n = nn * BS;
    const int64_t n2 = n >> 1, stride = (int64_t)gridDim.x * PCG_BLOCK;
    const int64_t i0 = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x;
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double2* r2 = reinterpret_cast<double2*>(r);
    constexpr bool QL = FEM_MF_QLDS && !FROM_Q;
    __shared__ double qst[QL ? PCG_BLOCK / 64 : 1][QL ? MF_QCAP : 1];
    const int lane = threadIdx.x & 63;
    double* qs = qst[QL ? (threadIdx.x >> 6) : 0];
    // q of the pair (2 i, 2 i + 1): staged when the node-major slots allow (every lane of the wave calls it: the wave's
    // first pair iw is uniform), else the direct fixed-count loads
    auto qpair = [&](int64_t i) -> double2 {
        if constexpr (FROM_Q) return q2[i];
        if constexpr (QL) {
            double2 qv;
            const int64_t iw = i - lane;
            if (op.spos && iw < n2 && mf_q_stage<BS>(op, slots, qs, iw, i, n, lane, qv)) return qv;
        }
        if (i >= n2) return make_double2(0.0, 0.0);
        return make_double2(mf_q_dof<BS>(op, slots, 2 * i), mf_q_dof<BS>(op, slots, 2 * i + 1));
    };
    double2 z[U2_NPT];
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < U2_NPT; ++k) {
        const int64_t i = i0 + k * stride;
        z[k] = make_double2(0.0, 0.0);
        const double2 qv = qpair(i);   // the whole wave (staging)
        if (i < n2) {
            double2 rv = r2[i], wv = w2[i];
            rv.x = rv.x - alpha * qv.x;
            rv.y = rv.y - alpha * qv.y;
            if (cg) {
                if (wv.x == 0.0) rv.x = 0.0;
                if (wv.y == 0.0) rv.y = 0.0;
            }
            r2[i] = rv;
            z[k] = make_double2(wv.x * rv.x, wv.y * rv.y);
            acc += rv.x * z[k].x;
            acc += rv.y * z[k].y;
        }
    }
    for (int64_t ib = i0 - lane + U2_NPT * stride; ib < n2; ib += stride) {   // past the register capacity (the
        const int64_t i = ib + lane;                                           // wave together: staging)
        const double2 qv = qpair(i);
        if (i >= n2) continue;
        double2 rv = r2[i], wv = w2[i];
        rv.x = rv.x - alpha * qv.x;
        rv.y = rv.y - alpha * qv.y;
        if (cg) {
            if (wv.x == 0.0) rv.x = 0.0;
            if (wv.y == 0.0) rv.y = 0.0;
        }
        r2[i] = rv;
        acc += rv.x * (wv.x * rv.x);
        acc += rv.y * (wv.y * rv.y);
    }
    double ztail = 0.0;
    const bool tail = (n & 1) && blockIdx.x == 0 && threadIdx.x == 0;
    if (tail) {
        const int64_t i = n - 1;
        double rv = r[i] - alpha * (FROM_Q ? q[i] : mf_q_dof<BS>(op, slots, i));
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        ztail = w[i] * rv;
        acc += rv * ztail;
    }
    double beta;
    bool upd_p, last;
    if (!u2_release(acc, st, red, hist, hist_len, sync, e, lds4, &flag, bc_s, beta, upd_p, last)) return;
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
#pragma unroll
    for (int k = 0; k < U2_NPT; ++k) {
        const int64_t i = i0 + k * stride;
        if (i < n2) {
            double2 pv = p2[i], xv = x2[i];
            xv.x += alpha * pv.x;
            xv.y += alpha * pv.y;
            x2[i] = xv;
            if (upd_p) {
                pv.x = z[k].x + beta * pv.x;
                pv.y = z[k].y + beta * pv.y;
                p2[i] = pv;
            }
        }
    }
    for (int64_t i = i0 + U2_NPT * stride; i < n2; i += stride) {
        double2 pv = p2[i], xv = x2[i];
        xv.x += alpha * pv.x;
        xv.y += alpha * pv.y;
        x2[i] = xv;
        if (upd_p) {
            const double2 rv = r2[i], wv = w2[i];
            pv.x = wv.x * rv.x + beta * pv.x;
            pv.y = wv.y * rv.y + beta * pv.y;
            p2[i] = pv;
        }
    }
    if (tail) {
        const int64_t i = n - 1;
        x[i] += alpha * p[i];
        if (upd_p) p[i] = ztail + beta * p[i];
    }
    if (last && threadIdx.x == 0) st->u2_epoch = e;
}

// ---------------------------------------------------------------- deferred schedule (3 kernels, no grid atomics)
// d1: q = A p and one p.q partial per block (plain store).  d2: every block re-sums d1's partials in fixed order
// (identical pq everywhere), alpha + guards, r update, one r.z partial per block.  d3: every block re-sums d2's
// partials -> stop test, beta, x/p update; block 0 writes the NEXT bank. Bank = host launch parity, so no kernel
// writes a state field its own blocks read.
template <int BS, typename CI = int32_t, bool PAIR = false>
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_d1(int64_t nslices, int64_t nrows,
                                                      const int64_t* __restrict__ slice_ptr,
                                                      const CI* __restrict__ cols, const double* __restrict__ vals,
                                                      const double* __restrict__ p, double* __restrict__ q,
                                                      const PcgState* __restrict__ st, int par, int rev,
                                                      double* __restrict__ partials) {
    __shared__ double lds4[4];
    const PcgState::Bank& bk = st->bank[par];
    if (bk.halt || bk.iter >= st->max_iter) return;
    const int lane = threadIdx.x & 63;
    double dot = 0.0;
    SliceWalk wk = slice_walk(nslices);
    const VecPlain pv{p};
    // rev: this XCD's slice range is swept end -> start, so the slices the previous sweep touched last (still in
    // the memory-side cache) are read first
    const int64_t mirror = rev ? wk.first + wk.end - 1 : -1;
    for (int64_t s0 = wk.s; s0 < wk.end; s0 += wk.step) {
        const int64_t s = rev ? mirror - s0 : s0;
        double o[BS];
        if constexpr (PAIR) sell_row_paired<BS>(s, lane, slice_ptr, cols, vals, p, o);
        else sell_row<BS, SPMV_U, (BS > 1 && SPMV_NT3), decltype(pv), CI>(s, lane, slice_ptr, cols, vals, pv, o);
        const int64_t row = s * 64 + lane;
        if (row < nrows) {
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                q[row * BS + c] = o[c];
                dot += p[row * BS + c] * o[c];
            }
        }
    }
    dot = block_sum256(dot, lds4);
    if (threadIdx.x == 0) partials[blockIdx.x] = dot;
}

constexpr int VPF = 4;   // double2 elements per thread loaded ahead of the partial re-sum in d2 / d3

__device__ __forceinline__ double sum_prev_partials(const double* __restrict__ part, int n, double* lds4) {
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += PCG_BLOCK) v += part[i];
    return block_sum256(v, lds4);
}

__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_d2(int64_t n, double* __restrict__ r, const double* __restrict__ q,
                                                      const double* __restrict__ w, PcgState* __restrict__ st, int par,
                                                      const double* __restrict__ part1, int n1,
                                                      double* __restrict__ part2) {
    __shared__ double lds4[4];
    PcgState::Bank& bk = st->bank[par];
    if (bk.halt || bk.iter >= st->max_iter) return;
    // this thread's first VPF elements are loaded before the partial re-sum, so its latency hides behind them
    const int64_t n2 = n >> 1;
    const int64_t i0 = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x, istep = (int64_t)gridDim.x * PCG_BLOCK;
    const double2* q2 = reinterpret_cast<const double2*>(q);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double2* r2 = reinterpret_cast<double2*>(r);
    double2 rp[VPF], qp[VPF], wp[VPF];
#pragma unroll
    for (int u = 0; u < VPF; ++u) {
        const int64_t i = i0 + u * istep;
        if (i < n2) {
            rp[u] = r2[i];
            qp[u] = q2[i];
            wp[u] = w2[i];
        }
    }
    const double pq = sum_prev_partials(part1, n1, lds4);
    const bool cg = st->mode != FEM_MODE_PCG;
    double alpha = 0.0;
    int stop = 0;
    if (cg) {
        if (fabs(pq) < st->eps || pq < 0.0) stop = FEM_PCG_BREAKDOWN;             // `solver/solver.py:187`
        else {
            alpha = bk.rz / (pq + st->eps);                                      // `:194`
            if (isnan(alpha) || isinf(alpha)) stop = FEM_PCG_ALPHA_NAN;          // `:196`
        }
    } else {
        alpha = bk.rz / pq;                                                      // `:800`
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        bk.pq = pq;
        bk.alpha = alpha;
        bk.k2stop = stop;
    }
    if (stop) return;
    double acc = 0.0;
    auto step = [&](int64_t i, double2 rv, const double2 qv, const double2 wv) {
        rv.x = rv.x - alpha * qv.x;
        rv.y = rv.y - alpha * qv.y;
        if (cg) {
            if (wv.x == 0.0) rv.x = 0.0;
            if (wv.y == 0.0) rv.y = 0.0;
        }
        r2[i] = rv;
        acc += rv.x * (wv.x * rv.x);
        acc += rv.y * (wv.y * rv.y);
    };
#pragma unroll
    for (int u = 0; u < VPF; ++u)
        if (i0 + u * istep < n2) step(i0 + u * istep, rp[u], qp[u], wp[u]);
    for (int64_t i = i0 + VPF * istep; i < n2; i += istep) step(i, r2[i], q2[i], w2[i]);
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        int64_t i = n - 1;
        double rv = r[i] - alpha * q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        acc += rv * (w[i] * rv);
    }
    acc = block_sum256(acc, lds4);
    if (threadIdx.x == 0) part2[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_d3(int64_t n, double* __restrict__ x, double* __restrict__ p,
                                                      const double* __restrict__ r, const double* __restrict__ w,
                                                      PcgState* __restrict__ st, int par,
                                                      const double* __restrict__ part2, int n2p,
                                                      double* __restrict__ hist, int64_t hist_len) {
    __shared__ double lds4[4];
    const PcgState::Bank bk = st->bank[par];
    PcgState::Bank& nx = st->bank[par ^ 1];
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (bk.halt || bk.iter >= st->max_iter) {
        if (lead) {
            nx = bk;
            nx.k2stop = 0;
        }
        return;
    }
    if (bk.k2stop) {   // guard stop in d2: the reference breaks before updating u (`solver/solver.py:187-198`)
        if (lead) {
            nx = bk;
            nx.halt = 1;
            nx.status = bk.k2stop;
            nx.stop_iter = bk.iter + 1;
            nx.k2stop = 0;
        }
        return;
    }
    const int64_t nh = n >> 1;
    const int64_t i0 = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x, istep = (int64_t)gridDim.x * PCG_BLOCK;
    double2* x2 = reinterpret_cast<double2*>(x);
    double2* p2 = reinterpret_cast<double2*>(p);
    const double2* r2 = reinterpret_cast<const double2*>(r);
    const double2* w2 = reinterpret_cast<const double2*>(w);
    double2 xp[VPF], pp[VPF], rp[VPF], wp[VPF];
#pragma unroll
    for (int u = 0; u < VPF; ++u) {   // loaded ahead of the partial re-sum (as in d2)
        const int64_t i = i0 + u * istep;
        if (i < nh) {
            xp[u] = x2[i];
            pp[u] = p2[i];
            rp[u] = r2[i];
            wp[u] = w2[i];
        }
    }
    const double rz_new = sum_prev_partials(part2, n2p, lds4);
    const bool cg = st->mode != FEM_MODE_PCG;
    const double nrm = sqrt(rz_new);
    const bool conv = nrm < st->tol;                                             // `:210` / `:805`
    double beta = 0.0;
    bool bnan = false;
    if (!conv) {
        beta = cg ? rz_new / (bk.rz + st->eps) : rz_new / bk.rz;                 // `:213` / `:808`
        bnan = cg && (isnan(beta) || isinf(beta));                               // `:214`
    }
    const bool upd_p = !conv && !bnan;
    const double alpha = bk.alpha;
    auto step = [&](int64_t i, double2 xv, double2 pv, const double2 rv, const double2 wv) {
        xv.x += alpha * pv.x;
        xv.y += alpha * pv.y;
        x2[i] = xv;
        if (upd_p) {
            pv.x = wv.x * rv.x + beta * pv.x;
            pv.y = wv.y * rv.y + beta * pv.y;
            p2[i] = pv;
        }
    };
#pragma unroll
    for (int u = 0; u < VPF; ++u)
        if (i0 + u * istep < nh) step(i0 + u * istep, xp[u], pp[u], rp[u], wp[u]);
    for (int64_t i = i0 + VPF * istep; i < nh; i += istep) step(i, x2[i], p2[i], r2[i], w2[i]);
    if ((n & 1) && lead) {
        int64_t i = n - 1;
        x[i] += alpha * p[i];
        if (upd_p) p[i] = w[i] * r[i] + beta * p[i];
    }
    if (lead) {
        nx = bk;
        nx.iter = bk.iter + 1;
        nx.rz_new = rz_new;
        nx.beta = beta;
        nx.k2stop = 0;
        if (hist && bk.iter < hist_len) hist[bk.iter] = nrm;
        if (conv || bnan) {
            nx.halt = 1;
            nx.status = conv ? FEM_PCG_CONVERGED : FEM_PCG_BETA_NAN;
            nx.stop_iter = bk.iter + 1;
        } else {
            nx.rz = rz_new;
        }
    }
}

// fused schedule, end of solve: apply the pending x += alpha_x p_last once
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_finish(int64_t n, double* __restrict__ x, const double* __restrict__ p0,
                                                          const double* __restrict__ p1, const PcgState* __restrict__ st) {
    if (st->x_done) return;
    // the last completed iteration (st->iter - 1) wrote its p into p_buf[(st->iter - 1) & 1]
    const double* p = ((st->iter - 1) & 1) ? p1 : p0;
    const double a = st->alpha_x;
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * PCG_BLOCK)
        x[i] += a * p[i];
}

__global__ void k_mark_x_done(PcgState* st) { st->x_done = 1; }

// start: (CG) x[fixed] = 0 beforehand; r = b - q (q = A x), (CG) r[fixed] = 0; rz = r.z;
// 3-kernel: p = z = w r.  fused: both p buffers = 0 and beta = alpha_x = 0, so the first K1 forms p = w r.
__global__ void __launch_bounds__(PCG_BLOCK) k_pcg_init(int64_t n, const double* __restrict__ b, double* __restrict__ r,
                                                        const double* __restrict__ q, const double* __restrict__ w,
                                                        double* __restrict__ p0, double* __restrict__ p1, int fused,
                                                        PcgState* __restrict__ st, RedBuf red,
                                                        const uint8_t* __restrict__ own, int bs) {
    __shared__ double lds4[4];
    __shared__ int flag;
    const bool cg = st->mode != FEM_MODE_PCG;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * PCG_BLOCK) {
        double rv = b[i] - q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        const double z = w[i] * rv;
        if (fused) {
            p0[i] = 0.0;
            p1[i] = 0.0;
        } else {
            p0[i] = z;
        }
        if (!own || own[i / bs]) acc += rv * z;
    }
    acc = block_sum256(acc, lds4);
    double rz;
    if (reduce_grid(acc, red.part(RED_INIT), red.cnt(RED_INIT), &rz, lds4, &flag) && threadIdx.x == 0) {
        if (st->dist) st->red[2] = rz;
        else st->rz = rz;
    }
}

// ---------------------------------------------------------------- distributed halo exchange + scalar finishing
// Interface dofs (nodes shared by several ranks' elements) carry rank-partial sums after the local SpMV. Every
// rank packs its partials into the compact global interface vector (zeros where it has no copy), RCCL sums it
// over the ranks, and every rank reads the full sums back: q is then identical on all copies of a node.
__device__ __forceinline__ bool halted(const PcgState* st) { return st && (st->halt || st->iter >= st->max_iter); }

// scalar != 0: also append st->red[0] (this rank's p.q partial) at buf[nI * bs]
__global__ void __launch_bounds__(256) k_halo_pack(const double* __restrict__ v, int bs, const int32_t* __restrict__ map,
                                                   int64_t nI, double* __restrict__ buf, const PcgState* __restrict__ st,
                                                   int scalar) {
    if (halted(st)) return;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nI * bs; t += (int64_t)gridDim.x * 256) {
        const int64_t j = t / bs;
        const int c = (int)(t - j * bs);
        const int32_t l = map[j];
        buf[t] = (l >= 0) ? v[(int64_t)l * bs + c] : 0.0;
    }
    if (scalar && blockIdx.x == 0 && threadIdx.x == 0) buf[nI * bs] = st->red[0];
}

// v[i] <- halo sum on interface rows; FIN: block 0 also finishes p.q (= buf[nI * bs]) into alpha / guards
template <bool FIN>
__global__ void __launch_bounds__(PCG_BLOCK) k_halo_unpack(int64_t nloc, int bs, const int32_t* __restrict__ pos,
                                                           const double* __restrict__ buf, double* __restrict__ v,
                                                           int64_t nI, PcgState* __restrict__ st) {
    if (halted(st)) return;
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < nloc * bs; i += (int64_t)gridDim.x * PCG_BLOCK) {
        const int64_t node = i / bs;
        const int32_t j = pos[node];
        if (j >= 0) v[i] = buf[(int64_t)j * bs + (i - node * bs)];
    }
    if (FIN && blockIdx.x == 0 && threadIdx.x == 0) finish_pq(st, buf[nI * bs]);
}

__global__ void k_fin_rz(PcgState* st, double* hist, int64_t hist_len) {
    if (halted(st)) return;
    finish_rz(st, st->red[1], hist, hist_len);
}

__global__ void k_set_rz(PcgState* st) { st->rz = st->red[2]; }

// deferred schedule start: bank 0 holds the initial iterate's r.z
__global__ void k_bank_init(PcgState* st) {
    st->bank[0].rz = st->rz;
    st->bank[0].rz_new = st->rz;
}

// ---------------------------------------------------------------- single-reduction distributed iteration
// Chronopoulos–Gear form of the same preconditioned CG (the "single reduction" CG): with u = z = w r and
// v = A u carried alongside r, an iteration's two dot products g = r.z (owned rows) and d = u.v (all local rows;
// rank partials of an operator sum, like p.q above) are formed back to back and ride in ONE all-reduce together
// with the interface rows of v:
//     beta = g / g_prev,  p.Ap = d - beta g / alpha_prev,  alpha = g / p.Ap
//     p = u + beta p,  s = v + beta s (= A p),  x += alpha p,  r -= alpha s,  u = w r,  v = A u
// One collective and three kernels per iteration instead of two collectives and six kernels. Same stop test
// (sqrt(r.z) < tol, `solver/solver.py:210` / `:805`) and guards (`:187-198`, `:214`); the rounding differs from
// the two-reduction form, which the N>1 contract allows (1e-10 on u, +-2 iterations).
// The all-reduce is out of place: `send` keeps zeros at the interface nodes this rank has no copy of.
//   step (every block of the next two kernels, cg1_eval): stop test on g of the last update, beta, p.Ap, alpha,
//                             guards; committed (iter += 1, ...) by the last block of k_cg1_spmv
//   k_cg1_update (grid)     : p, s, x, r, u; g partial of the new iterate -> st->red[1]
//   k_cg1_spmv   (grid)     : v = A u (local), d partial; interface rows of v and [g, d] -> send
// neighbour exchange (fem_pcg_set_p2p) seen by the single-reduction kernels; P = 0: all-reduce path. Message
// slots are symmetric (the slot for peer r holds the same nodes in the same order in psend and precv), so one table
// serves both directions: csrc[J P + r] = offset of node J's component 0 in rank r's slot (-1: this rank, -2: r does
// not touch J), ssrc[r] = offset of rank r's [g, d] (-1: this rank).
struct P2PArgs {
    int P;
    const int32_t* csrc;
    const int32_t* ssrc;
    double* psend;
    const double* precv;
};

// rank-ordered sum of the [g, d] pairs (p2p) or the all-reduced pair
__device__ __forceinline__ double cg1_scalar(const double* recv, const double* send, int64_t off, int k,
                                             const P2PArgs& x) {
    if (!x.P) return recv[off + k];
    double acc = 0.0;
    for (int r = 0; r < x.P; ++r) {
        const int src = x.ssrc[r];
        acc += (src < 0) ? send[off + k] : x.precv[src + k];
    }
    return acc;
}

// the single-reduction step as a value: every block of k_cg1_update and k_cg1_spmv evaluates it from the unchanged
// state and the exchanged [g, d] (identical result everywhere), the last block of k_cg1_spmv commits it
struct Cg1Step {
    int go;          // 1: update + SpMV run this iteration
    int stop;        // 1: a stop decision to commit (status / halt / stop_iter below)
    int status, stop_iter;
    int it;
    double g, d, alpha, beta, pq;
    int has_pq;
};

__device__ __forceinline__ Cg1Step cg1_eval(const PcgState* st, double g, double d) {
    Cg1Step k{};
    k.it = st->iter;
    k.g = g;
    k.d = d;
    k.status = st->status;
    k.stop_iter = st->stop_iter;
    if (st->halt) return k;
    const bool cg = st->mode != FEM_MODE_PCG;
    const int it = k.it;
    double beta = 0.0;
    if (it > 0) {
        if (sqrt(g) < st->tol) {
            k.stop = 1;
            k.status = FEM_PCG_CONVERGED;
            k.stop_iter = it;
            return k;
        }
        beta = cg ? g / (st->rz + st->eps) : g / st->rz;
        if (cg && (isnan(beta) || isinf(beta))) {
            k.stop = 1;
            k.status = FEM_PCG_BETA_NAN;
            k.stop_iter = it;
            return k;
        }
    }
    if (it >= st->max_iter) {   // poll reports FEM_PCG_MAXITER
        k.stop = 1;
        return k;
    }
    const double pq = (it == 0) ? d : d - beta * g / st->alpha;
    k.pq = pq;
    k.has_pq = 1;
    double alpha;
    if (cg) {
        if (fabs(pq) < st->eps || pq < 0.0) {
            k.stop = 1;
            k.status = FEM_PCG_BREAKDOWN;
            k.stop_iter = it + 1;
            return k;
        }
        alpha = g / (pq + st->eps);
        if (isnan(alpha) || isinf(alpha)) {
            k.stop = 1;
            k.status = FEM_PCG_ALPHA_NAN;
            k.stop_iter = it + 1;
            return k;
        }
    } else {
        alpha = g / pq;
    }
    k.alpha = alpha;
    k.beta = beta;
    k.go = 1;
    return k;
}

// the step's state writes (one thread)
__device__ __forceinline__ void cg1_commit(PcgState* st, const Cg1Step& k, double* hist, int64_t hist_len) {
    st->xupd = k.go;
    if (!k.go && !k.stop) return;   // halted before this pass
    if (k.it > 0) {
        st->rz_new = k.g;
        if (hist && k.it - 1 < hist_len) hist[k.it - 1] = sqrt(k.g);
    }
    if (k.has_pq) st->pq = k.pq;
    if (k.stop) {
        st->status = k.status;
        st->stop_iter = k.stop_iter;
        st->halt = 1;
        return;
    }
    st->rz = k.g;
    st->alpha = k.alpha;
    st->beta = k.beta;
    st->iter = k.it + 1;
}

// The gather-free distributed element-chunk iteration: d = u.v reduced in the chunk walk (MF_DOT), an interface-only
// pack kernel (k_cg1_mf_iface), and v of every dof formed from the slots inside k_cg1_update<true> (the fixed-count
// loads of mf_q_dof): no v vector written or read. It saves the gather pass's v stream and pays a second grid
// reduction and one more launch, so it wins on large partitions only (world-1 RCCL lines, round 6: 1.73M nodes 285.5
// vs 302.7 us per iteration, 216k nodes -- the N = 8 rank share of the 10M cube -- 55.2 vs 53.8 us): chosen per
// context at fem_pcg_set_operator_mf when the partition has at least MF_NOGATHER_MIN_NODES nodes (the linear fit of
// the two points crosses at ~330k). FEM_MF_DIST_NOGATHER = 0 / 1 (build) or FEM355_MF_NOGATHER=0 / 1 (run) force
// either form. Both pack the same exchange message, so ranks may differ in the form they run.
#ifndef FEM_MF_DIST_NOGATHER
#define FEM_MF_DIST_NOGATHER -1
#endif
constexpr int64_t MF_NOGATHER_MIN_NODES = 400000;
// Every vector read and written as 16-byte lanes (a double2 of dofs per thread-step; round 5: one 8-byte dof per
// thread), the per-dof arithmetic unchanged. MF: v from the element-chunk operator's slots (never stored)
template <bool MF = false>
__global__ void __launch_bounds__(PCG_BLOCK) k_cg1_update(int64_t n, int bs, double* __restrict__ x,
                                                          double* __restrict__ r, double* __restrict__ p,
                                                          double* __restrict__ sv, double* __restrict__ u,
                                                          const double* __restrict__ v, const double* __restrict__ w,
                                                          const double* __restrict__ recv,
                                                          const int32_t* __restrict__ ipos,
                                                          const uint8_t* __restrict__ own, PcgState* __restrict__ st,
                                                          RedBuf red, P2PArgs xp, const double* __restrict__ send,
                                                          int64_t off, MfOp op = MfOp{},
                                                          const double* __restrict__ slots = nullptr) {
    __shared__ double lds4[4];
    __shared__ int flag;
    const Cg1Step k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
    if (!k.go) return;
    const double alpha = k.alpha, beta = k.beta;
    const bool cg = st->mode != FEM_MODE_PCG;
    double acc = 0.0;
    // one dof: v (exchanged where the node is shared), then p, s, x, r, u; returns r.u when the node is owned
    auto dof = [&](int64_t i, double vi, double ui, double pi0, double si0, double xi, double ri0, double wi, double& po,
                   double& so, double& xo, double& ro, double& uo) -> double {
        const int64_t node = i / bs;
        const int32_t j = ipos ? ipos[node] : -1;
        if (j >= 0) {
            const int c = (int)(i - node * bs);
            if (xp.P) {   // rank-ordered sum of the partials (own partial = the local row itself)
                double a = 0.0;
                for (int q = 0; q < xp.P; ++q) {
                    const int src = xp.csrc[(int64_t)j * xp.P + q];
                    if (src == -1) a += vi;
                    else if (src >= 0) a += xp.precv[src + c];
                }
                vi = a;
            } else {
                vi = recv[(int64_t)j * bs + c];
            }
        }
        po = ui + beta * pi0;
        so = vi + beta * si0;
        xo = xi + alpha * po;
        double rv = ri0 - alpha * so;
        if (cg && wi == 0.0) rv = 0.0;
        ro = rv;
        uo = wi * rv;
        return (!own || own[node]) ? rv * uo : 0.0;
    };
    const int64_t n2 = n >> 1;
    auto vpair = [&](int64_t i2) -> double2 {
        if constexpr (MF)
            return bs == 3 ? make_double2(mf_q_dof<3>(op, slots, 2 * i2), mf_q_dof<3>(op, slots, 2 * i2 + 1))
                           : make_double2(mf_q_dof<1>(op, slots, 2 * i2), mf_q_dof<1>(op, slots, 2 * i2 + 1));
        return reinterpret_cast<const double2*>(v)[i2];
    };
    for (int64_t i2 = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i2 < n2; i2 += (int64_t)gridDim.x * PCG_BLOCK) {
        const double2 v2 = vpair(i2), u2 = reinterpret_cast<const double2*>(u)[i2];
        const double2 p2 = reinterpret_cast<const double2*>(p)[i2], s2 = reinterpret_cast<const double2*>(sv)[i2];
        const double2 x2 = reinterpret_cast<const double2*>(x)[i2], r2 = reinterpret_cast<const double2*>(r)[i2];
        const double2 w2 = reinterpret_cast<const double2*>(w)[i2];
        double2 po, so, xo, ro, uo;
        acc += dof(2 * i2, v2.x, u2.x, p2.x, s2.x, x2.x, r2.x, w2.x, po.x, so.x, xo.x, ro.x, uo.x);
        acc += dof(2 * i2 + 1, v2.y, u2.y, p2.y, s2.y, x2.y, r2.y, w2.y, po.y, so.y, xo.y, ro.y, uo.y);
        reinterpret_cast<double2*>(p)[i2] = po;
        reinterpret_cast<double2*>(sv)[i2] = so;
        reinterpret_cast<double2*>(x)[i2] = xo;
        reinterpret_cast<double2*>(r)[i2] = ro;
        reinterpret_cast<double2*>(u)[i2] = uo;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // the odd dof
        const int64_t i = n - 1;
        double po, so, xo, ro, uo;
        double vt;
        if constexpr (MF) vt = bs == 3 ? mf_q_dof<3>(op, slots, i) : mf_q_dof<1>(op, slots, i);
        else vt = v[i];
        acc += dof(i, vt, u[i], p[i], sv[i], x[i], r[i], w[i], po, so, xo, ro, uo);
        p[i] = po;
        sv[i] = so;
        x[i] = xo;
        r[i] = ro;
        u[i] = uo;
    }
    acc = block_sum256(acc, lds4);
    double g;
    if (reduce_grid(acc, red.part(RED_K2), red.cnt(RED_K2), &g, lds4, &flag) && threadIdx.x == 0) st->red[1] = g;
}

// r0 = b - A x0 (A x0 halo-summed in q; CG: masked), u0 = w r0, p = s = 0; g0 partial -> st->red[1]
__global__ void __launch_bounds__(PCG_BLOCK) k_cg1_init(int64_t n, int bs, const double* __restrict__ b,
                                                        double* __restrict__ r, const double* __restrict__ q,
                                                        const double* __restrict__ w, double* __restrict__ p,
                                                        double* __restrict__ sv, double* __restrict__ u,
                                                        const uint8_t* __restrict__ own, PcgState* __restrict__ st,
                                                        RedBuf red) {
    __shared__ double lds4[4];
    __shared__ int flag;
    const bool cg = st->mode != FEM_MODE_PCG;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * PCG_BLOCK) {
        double rv = b[i] - q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        const double z = w[i] * rv;
        u[i] = z;
        p[i] = 0.0;
        sv[i] = 0.0;
        if (!own || own[i / bs]) acc += rv * z;
    }
    acc = block_sum256(acc, lds4);
    double g;
    if (reduce_grid(acc, red.part(RED_INIT), red.cnt(RED_INIT), &g, lds4, &flag) && threadIdx.x == 0) {
        st->red[1] = g;
        st->rz = g;
    }
}

template <int BS, typename CI, bool PAIR>
__global__ void __launch_bounds__(PCG_BLOCK) k_cg1_spmv(int64_t nslices, int64_t nrows,
                                                        const int64_t* __restrict__ slice_ptr,
                                                        const CI* __restrict__ cols, const double* __restrict__ vals,
                                                        const double* __restrict__ u, double* __restrict__ v,
                                                        const int32_t* __restrict__ ipos, double* __restrict__ send,
                                                        int64_t off, PcgState* __restrict__ st, RedBuf red,
                                                        int always, int tune_rev, P2PArgs xp,
                                                        const double* __restrict__ recv, double* hist,
                                                        int64_t hist_len) {
    __shared__ double lds4[4];
    __shared__ int flag;
    Cg1Step k{};
    if (!always) {   // the step of this pass (read before the last block commits it)
        k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
        if (!k.go) {
            if (blockIdx.x == 0 && threadIdx.x == 0) cg1_commit(st, k, hist, hist_len);
            return;
        }
    }
    const int lane = threadIdx.x & 63;
    double dot = 0.0;
    const SliceWalk wk = slice_walk(nslices);
    const VecPlain uv{u};
    // sweep direction alternating with the iteration parity (FEM_TUNE_REVERSE, as k_pcg_spmv_dot): the iteration
    // count after this pass's step
    const bool rev = tune_rev && ((always ? st->iter : k.it + 1) & 1);
    const int64_t mirror = wk.first + wk.end - 1;
    for (int64_t s0 = wk.s; s0 < wk.end; s0 += wk.step) {
        const int64_t s = rev ? mirror - s0 : s0;
        double o[BS];
        if constexpr (PAIR) sell_row_paired<BS>(s, lane, slice_ptr, cols, vals, u, o);
        else sell_row<BS, SPMV_U, (BS > 1 && SPMV_NT3), decltype(uv), CI>(s, lane, slice_ptr, cols, vals, uv, o);
        const int64_t row = s * 64 + lane;
        if (row < nrows) {
            const int32_t j = ipos ? ipos[row] : -1;
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                v[row * BS + c] = o[c];
                dot += u[row * BS + c] * o[c];
                if (j >= 0) {
                    if (xp.P) {   // straight into every peer's message slot for this node
                        for (int r = 0; r < xp.P; ++r) {
                            const int dst = xp.csrc[(int64_t)j * xp.P + r];
                            if (dst >= 0) xp.psend[dst + c] = o[c];
                        }
                    } else {
                        send[(int64_t)j * BS + c] = o[c];
                    }
                }
            }
        }
    }
    dot = block_sum256(dot, lds4);
    double d;
    if (reduce_grid(dot, red.part(RED_K1), red.cnt(RED_K1), &d, lds4, &flag) && threadIdx.x == 0) {
        if (!always) cg1_commit(st, k, hist, hist_len);   // every block has read the state by now
        st->red[0] = d;
        send[off] = st->red[1];
        send[off + 1] = d;
        for (int r = 0; r < xp.P; ++r) {
            const int dst = xp.ssrc[r];
            if (dst >= 0) {
                xp.psend[dst] = st->red[1];
                xp.psend[dst + 1] = d;
            }
        }
    }
}


// ---------------------------------------------------------------- distributed single-reduction iteration, fused
// One launch per iteration between two exchanges (N > 1): step, update of the own rows, u hand-off to the
// neighbouring workgroups by flags (no grid barrier: only the workgroups whose rows the SpMV reaches), SpMV of the
// same rows, pack, and ONE two-value grid reduction (g, d) whose last block commits the step and writes [g, d].
// Replaces k_cg1_update + k_cg1_spmv (two launches and two reduction tails). Every workgroup must be resident
// (the host sizes the grid from the occupancy query); a flag wait that exceeds the spin limit ends the solve with
// FEM_PCG_SYNC_TIMEOUT. Hand-off: u stores sc1 + drain + workgroup barrier + relaxed flag; consumer: relaxed poll,
// one agent acquire, plain gathers (MI355X_MICROARCH.md "Valid forms").
constexpr int C1F_BLOCK = 256;
constexpr unsigned C1F_SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ bool reduce_grid_pair(double a, double b, double* pa, double* pb, unsigned* counters,
                                                 double* ta, double* tb, double* lds4, int* lds_flag) {
    const unsigned G = gridDim.x;
    const unsigned nsh = G < (unsigned)RED_SHARDS ? G : (unsigned)RED_SHARDS;
    const unsigned sh = blockIdx.x % RED_SHARDS;
    const unsigned in_shard = (G - sh + RED_SHARDS - 1) / RED_SHARDS;
    double* sa = pa + G;
    double* sb = pb + G;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&pa[blockIdx.x], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&pb[blockIdx.x], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(&counters[sh * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == in_shard - 1);
        if (last) __hip_atomic_store(&counters[sh * 32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    if (!*lds_flag) return false;
    double va = 0.0, vb = 0.0;
    for (unsigned i = threadIdx.x; i < in_shard; i += C1F_BLOCK) {
        va += __hip_atomic_load(&pa[sh + i * RED_SHARDS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vb += __hip_atomic_load(&pb[sh + i * RED_SHARDS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    va = block_sum256(va, lds4);
    vb = block_sum256(vb, lds4);
    if (threadIdx.x == 0) {
        __hip_atomic_store(&sa[sh], va, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sb[sh], vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned* top = &counters[RED_SHARDS * 32];
        const unsigned t = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = (t == nsh - 1);
        if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = last;
    }
    __syncthreads();
    if (!*lds_flag) return false;
    const double s1 = (threadIdx.x < nsh) ? __hip_atomic_load(&sa[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    const double s2 = (threadIdx.x < nsh) ? __hip_atomic_load(&sb[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    *ta = block_sum256(s1, lds4);
    *tb = block_sum256(s2, lds4);
    return true;
}

struct Cg1FArgs {
    int64_t nslices, nrows;
    const int64_t* slice_ptr;
    const void* cols;
    const double* vals;
    double *x, *r, *p, *sv, *u, *v;
    const double* w;
    const int32_t* ipos;
    const uint8_t* own;
    double* send;
    const double* recv;
    int64_t off;
    PcgState* st;
    RedBuf red;
    P2PArgs xp;
    double* hist;
    int64_t hist_len;
    const int32_t* win;   // [2 G]: first / last logical workgroup of each workgroup's gather window
    unsigned* flags;      // [G lines] u-flags (epochs = iteration numbers), then the give-up word; zeroed at start
    int tune_rev;
};

template <int BS, typename CI, bool PAIR>
__global__ void __launch_bounds__(C1F_BLOCK) k_cg1_fused(Cg1FArgs a) {
    __shared__ double lds4[4];
    __shared__ int flag;
    __shared__ int ok_lds;
    PcgState* st = a.st;
    const Cg1Step k = cg1_eval(st, cg1_scalar(a.recv, a.send, a.off, 0, a.xp), cg1_scalar(a.recv, a.send, a.off, 1, a.xp));
    if (!k.go) {
        if (blockIdx.x == 0 && threadIdx.x == 0) cg1_commit(st, k, a.hist, a.hist_len);
        return;
    }
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;   // XCD-contiguous logical order
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t sA = (int64_t)L * a.nslices / G, sB = (int64_t)(L + 1) * a.nslices / G;
    const bool cg = st->mode != FEM_MODE_PCG;
    const double alpha = k.alpha, beta = k.beta;
    const unsigned e = (unsigned)k.it + 1;
    unsigned* tmo = a.flags + (size_t)G * 32;
    // ---- update of the own rows (as k_cg1_update), u stored sc1 for the hand-off
    double gp = 0.0;
    for (int64_t sl = sA + wv; sl < sB; sl += C1F_BLOCK / 64) {
        const int64_t node = sl * 64 + lane;
        if (node >= a.nrows) continue;
        const int32_t j = a.ipos ? a.ipos[node] : -1;
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            const int64_t i = node * BS + c;
            double vi = a.v[i];
            if (j >= 0) {
                if (a.xp.P) {
                    double acc = 0.0;
                    for (int r = 0; r < a.xp.P; ++r) {
                        const int src = a.xp.csrc[(int64_t)j * a.xp.P + r];
                        if (src == -1) acc += vi;
                        else if (src >= 0) acc += a.xp.precv[src + c];
                    }
                    vi = acc;
                } else {
                    vi = a.recv[(int64_t)j * BS + c];
                }
            }
            const double pi = a.u[i] + beta * a.p[i];
            const double si = vi + beta * a.sv[i];
            a.p[i] = pi;
            a.sv[i] = si;
            a.x[i] += alpha * pi;
            double ri = a.r[i] - alpha * si;
            const double wi = a.w[i];
            if (cg && wi == 0.0) ri = 0.0;
            a.r[i] = ri;
            const double ui = wi * ri;
            __hip_atomic_store(a.u + i, ui, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!a.own || a.own[node]) gp += ri * ui;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its u stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.flags + (size_t)L * 32, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- wait for the u of the gather window
    if (wv == 0) {
        // never outside the flag array; a window outside it ends the solve with FEM_PCG_BAD_WINDOW (reported, not run)
        const int wraw0 = a.win[L], wraw1 = a.win[G + L];
        const int wlo = max(wraw0, 0), whi = min(wraw1, G - 1);
        bool ok = true;
        if (pk_window_bad(wraw0, wraw1, G)) {
            if (lane == 0) __hip_atomic_store(tmo, PK_SITE_WINDOW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
        }
        for (int b0 = wlo; b0 <= whi && ok; b0 += 64) {
            const int jw = b0 + lane;
            bool done = jw > whi;
            for (unsigned spins = 0; !__all(done); ++spins) {
                if (!done) done = __hip_atomic_load(a.flags + (size_t)jw * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= e;
                if ((spins & 63) == 63 && __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = false;
                    break;
                }
                if (spins >= C1F_SPIN_LIMIT) {
                    __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (lane == 0) {
            ok_lds = ok;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!ok_lds) {   // a neighbour never arrived (or a bad window): end the solve (the reduction is abandoned)
        if (threadIdx.x == 0) {
            st->status = pk_fail_status(__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            st->halt = 1;
        }
        return;
    }
    // ---- v = A u over the own slices, interface rows packed, d partial
    const CI* cols = reinterpret_cast<const CI*>(a.cols);
    const VecPlain uv{a.u};
    const bool rev = a.tune_rev && ((k.it + 1) & 1);
    double dot = 0.0;
    for (int64_t t = sA + wv; t < sB; t += C1F_BLOCK / 64) {
        const int64_t sl = rev ? sA + sB - 1 - t : t;
        double o[BS];
        if constexpr (PAIR) sell_row_paired<BS>(sl, lane, a.slice_ptr, cols, a.vals, a.u, o);
        else sell_row<BS, SPMV_U, (BS > 1 && SPMV_NT3), decltype(uv), CI>(sl, lane, a.slice_ptr, cols, a.vals, uv, o);
        const int64_t row = sl * 64 + lane;
        if (row < a.nrows) {
            const int32_t j = a.ipos ? a.ipos[row] : -1;
#pragma unroll
            for (int c = 0; c < BS; ++c) {
                a.v[row * BS + c] = o[c];
                dot += a.u[row * BS + c] * o[c];
                if (j >= 0) {
                    if (a.xp.P) {
                        for (int r = 0; r < a.xp.P; ++r) {
                            const int dst = a.xp.csrc[(int64_t)j * a.xp.P + r];
                            if (dst >= 0) a.xp.psend[dst + c] = o[c];
                        }
                    } else {
                        a.send[(int64_t)j * BS + c] = o[c];
                    }
                }
            }
        }
    }
    gp = block_sum256(gp, lds4);
    dot = block_sum256(dot, lds4);
    double gt, dt;
    if (reduce_grid_pair(gp, dot, a.red.part(RED_K2), a.red.part(RED_K1), a.red.cnt(RED_K1), &gt, &dt, lds4, &flag) &&
        threadIdx.x == 0) {
        cg1_commit(st, k, a.hist, a.hist_len);   // every block has evaluated the step by now
        st->red[1] = gt;
        st->red[0] = dt;
        a.send[a.off] = gt;
        a.send[a.off + 1] = dt;
        for (int r = 0; r < a.xp.P; ++r) {
            const int dst = a.xp.ssrc[r];
            if (dst >= 0) {
                a.xp.psend[dst] = gt;
                a.xp.psend[dst + 1] = dt;
            }
        }
    }
}

// gather window per logical workgroup of a G-workgroup slice split (generic column type)
template <typename CI>
__global__ void k_c1f_window(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                             const CI* __restrict__ cols, int G, int* __restrict__ lo, int* __restrict__ hi) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t sl = t >> 6;
        const int l = (int)(t & 63);
        const int64_t row = sl * 64 + l;
        const int64_t p0 = slice_ptr[sl];
        const int w = (int)((slice_ptr[sl + 1] - p0) >> 6);
        int64_t cmin = row < nrows ? row : nrows - 1, cmax = cmin;
        for (int kk = 0; kk < w; ++kk) {
            int64_t c = (int64_t)cols[p0 + 64 * kk + l];
            if constexpr (sizeof(CI) == 2) c += row;
            cmin = c < cmin ? c : cmin;
            cmax = c > cmax ? c : cmax;
        }
        if (cmax >= nrows) cmax = nrows - 1;
        if (cmin < 0) cmin = 0;
        auto owner = [&](int64_t r) { return (int)((((r >> 6) + 1) * G - 1) / nslices); };
        const int me = owner(row < nrows ? row : nrows - 1);
        int olo = owner(cmin), ohi = owner(cmax);
        for (int off = 32; off > 0; off >>= 1) {
            const int a2 = __shfl_xor(olo, off), b2 = __shfl_xor(ohi, off);
            olo = a2 < olo ? a2 : olo;
            ohi = b2 > ohi ? b2 : ohi;
        }
        if (l == 0) {
            atomicMin(lo + me, olo);
            atomicMax(hi + me, ohi);
        }
    }
}

}  // namespace fem
#include "pcg_persist.hpp"
#include "pcg_persist3.hpp"
#include "pcg_persist_gv.hpp"
namespace fem {

// ---------------------------------------------------------------- constraint projections (CG_CONSTRAINED)
// `enforce_constraints` (`solver/solver.py:478-510`: RBE2 then SPC) and `new_enforce_constraints` (`:665-700`:
// SPC, RBE2, then RBE3 sets in order) on the displacement after every update; the r-zeroing of SPC dofs and RBE2
// slaves is the 0/1 mask w of the CG. One 256-thread block, phases separated by barriers so that each step sees the
// previous one, RBE2 as gather-then-scatter (the reference's vectorised assignment), RBE3 groups sequential with a
// fixed-order block sum. `always` = 1 at start (the reference enforces once before the loop).
struct Constraints {
    int64_t R, S, G;
    const int64_t* rbe2_slave;   // [R] dofs
    const int64_t* rbe2_master;  // [R]
    double* tmp;                 // [R]
    const int64_t* spc_dof;      // [S]
    const double* spc_val;       // [S]
    const int64_t* r3_ptr;       // [G+1] entry ranges of the groups (set-major, dof ascending)
    const int64_t* r3_master;    // [G] master dof of the group
    const double* r3_wsum;       // [G] weight sum of the group's set
    const int64_t* r3_slave;     // [E] slave dofs
    const double* r3_w;          // [E]
    int order;                   // 0: RBE2, SPC (constrained_cg) ; 1: SPC, RBE2, RBE3 (new_constrained_cg)
};

// r (nullable): also zero the residual at SPC dofs and RBE2 slaves (the standalone enforce_* entry point; inside
// the CG that masking is the weight vector w)
// parts: bit 0 = the SPC / RBE2 copies, bit 1 = the RBE3 means (large SPC / RBE2 sets run as grid kernels)
__global__ void __launch_bounds__(256) k_constraints(double* __restrict__ x, double* __restrict__ r, Constraints c,
                                                     const PcgState* st, int always, int parts) {
    __shared__ double lds4[4];
    if (!always && !st->xupd) return;
    if (!(parts & 1)) c.R = c.S = 0;
    if (!(parts & 2)) c.G = 0;
    const int t0 = threadIdx.x;
    auto rbe2 = [&]() {
        for (int64_t t = t0; t < c.R; t += 256) c.tmp[t] = x[c.rbe2_master[t]];
        __syncthreads();
        for (int64_t t = t0; t < c.R; t += 256) {
            x[c.rbe2_slave[t]] = c.tmp[t];
            if (r) r[c.rbe2_slave[t]] = 0.0;
        }
        __syncthreads();
    };
    auto spc = [&]() {
        for (int64_t t = t0; t < c.S; t += 256) {
            x[c.spc_dof[t]] = c.spc_val[t];
            if (r) r[c.spc_dof[t]] = 0.0;
        }
        __syncthreads();
    };
    if (c.order == 0) {
        rbe2();
        spc();
    } else {
        spc();
        rbe2();
        for (int64_t g = 0; g < c.G; ++g) {
            double v = 0.0;
            for (int64_t e = c.r3_ptr[g] + t0; e < c.r3_ptr[g + 1]; e += 256) v += c.r3_w[e] * x[c.r3_slave[e]];
            v = block_sum256(v, lds4);
            if (t0 == 0) x[c.r3_master[g]] = v / (c.r3_wsum[g] + 1e-30);   // `:697-698`
            __syncthreads();
        }
    }
}

// grid-wide variants of the two copy phases for large sets (one launch each keeps gather-before-scatter and the
// reference's phase order)
enum { CON_GATHER = 0, CON_SCATTER = 1, CON_SPC = 2 };
template <int PH>
__global__ void __launch_bounds__(256) k_con_phase(double* __restrict__ x, double* __restrict__ r, Constraints c,
                                                   const PcgState* st, int always) {
    if (!always && !st->xupd) return;
    const int64_t m = PH == CON_SPC ? c.S : c.R;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < m; t += (int64_t)gridDim.x * 256) {
        if (PH == CON_GATHER) {
            c.tmp[t] = x[c.rbe2_master[t]];
        } else if (PH == CON_SCATTER) {
            x[c.rbe2_slave[t]] = c.tmp[t];
            if (r) r[c.rbe2_slave[t]] = 0.0;
        } else {
            x[c.spc_dof[t]] = c.spc_val[t];
            if (r) r[c.spc_dof[t]] = 0.0;
        }
    }
}

// set-up validation of caller index arrays (a bad index would otherwise be an out-of-bounds store)
__global__ void k_check_range(const int64_t* __restrict__ v, int64_t m, int64_t lo, int64_t hi, int* __restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        if (v[i] < lo || v[i] >= hi) atomicOr(bad, 1);
}

__global__ void k_check_ptr(const int64_t* __restrict__ ptr, int64_t g, int* __restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g; i += (int64_t)gridDim.x * blockDim.x)
        if (ptr[i + 1] < ptr[i] || (i == 0 && ptr[0] != 0)) atomicOr(bad, 1);
}

// HBM ceiling probe: dst = src, 16 B per lane, grid-stride (the measured "STREAM copy" roof of SURVEY §8(d))
__global__ void __launch_bounds__(256) k_stream_copy(const double2* __restrict__ src, double2* __restrict__ dst,
                                                     int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

// read-only sweep: 16-byte loads summed; the store happens only for an impossible sum (keeps the loads alive)
__global__ void __launch_bounds__(256) k_stream_read(const double2* __restrict__ src, int64_t n2, double* __restrict__ out) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const double2 v = src[i];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

__global__ void k_zero_fixed(int64_t n, double* __restrict__ x, const double* __restrict__ w) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (w[i] == 0.0) x[i] = 0.0;
}

}  // namespace fem

using namespace fem;

// ---------------------------------------------------------------- host-side context
struct fem_pcg {
    int64_t nrows, nslices, n;
    int bs;
    const int64_t* slice_ptr;
    const int32_t* cols;
    const double* vals;
    const double* b;
    double* x;
    const double* w;
    double* hist;
    int64_t hist_len;
    int mode;
    double tol, eps;
    hipStream_t stream;
    int fused;          // schedule 1: p formed inside the SpMV
    int deferred;       // schedule 2: partial sums finished by the next kernel (banked state)
    int64_t launched;   // iterations enqueued since start (the deferred schedule's bank parity)
    int64_t sell_ent;   // SELL entries (slice_ptr[nslices]) when the caller gave it (fem_pcg_set_entries), else -1
    const int16_t* cols16;  // optional 16-bit column deltas (fem_sell_delta16): used instead of cols when set
    int has_con;            // CG_CONSTRAINED projections set (fem_pcg_set_constraints)
    int tune;               // FEM_TUNE_* flags (fem_pcg_set_tuning)
    int paired;             // the SpMV reads pvals / pcols16 (lane-paired copy, refreshed by fem_pcg_start)
    double* pvals;
    int16_t* pcols16;
    int32_t* puoff;         // FEM_TUNE_PK_UNI (bs = 1): per-slice offset into pucol, -1 = per-lane deltas
    int16_t* pucol;
    int pext;               // pvals / pcols16 / puoff / pucol belong to the caller (fem_pcg_set_layout): never freed
    const int32_t* pwin_ext;   // the caller's gather windows for a pwin_G-workgroup grid (nullable)
    int pwin_G;
    Constraints con;
    // owned device memory
    double* r;
    double* p0;
    double* p1;
    double* q;
    RedBuf red;
    PcgState* st;
    PcgState* st_host;  // pinned
    int grid_spmv, grid_vec;
    hipGraphExec_t graph;
    int graph_k;
    int max_iter;       // device-side iteration cap armed by fem_pcg_start
    // distributed (element-partitioned) mode: dist = 1; exchanges by RCCL on `comm`, or (comm == NULL) by the
    // caller between fem_pcg_dist_phase calls (single-process multi-partition validation)
    int dist;
    ncclComm_t comm;
    int64_t nI;         // global interface nodes
    const int32_t* imap;  // [nI] local row of interface node j on this rank, -1 if absent
    const int32_t* ipos;  // [nrows] interface index of a local row, -1 for interior rows
    const uint8_t* own;   // [nrows] 1 where this rank owns the node (lowest rank touching it)
    double* hbuf;         // [nI * bs] compact interface vector
    // single-reduction variant (k_cg1_*): s = A p, u = w r, and the out-of-place exchange [v interface | g | d]
    int cg1;
    double* cg1_s;
    double* cg1_u;
    double* cg1_send;
    double* cg1_recv;
    // neighbour exchange (fem_pcg_set_p2p): the single-reduction all-reduce replaced by grouped send/recv with every
    // other rank ([g, d | shared interface rows] per peer) and a fixed-rank-order sum into cg1_recv
    int p2p;
    int p2p_nranks;
    std::vector<int> peer_rank;
    std::vector<int64_t> peer_off, peer_cnt;   // doubles, into psend / precv
    int64_t p2p_total;
    const int32_t* p2p_csrc;   // [nI][nranks] slot offset of node J's component 0 for rank r, -1 own, -2 absent
    const int32_t* p2p_ssrc;   // [nranks] precv offset of rank r's [g, d], -1 own
    double* psend;
    double* precv;
    // fused distributed iteration (FEM_TUNE_C1F): one launch per iteration, u hand-off by flags
    int c1f;
    int c1f_grid;
    int c1f_win_ok;
    int32_t* c1f_win;      // [2 G]
    unsigned* c1f_flags;   // (G + 1) lines
    // persistent schedule (3): requested by fem_pcg_set_schedule, active after fem_pcg_start when supported
    int persist_req;
    int persist_fit_only;   // schedule 4 (auto) on bs = 3: no overflow build (the 3-kernel schedule instead)
    int persist;
    int pk_grid;          // workgroups (one per CU, multiple of 8)
    int pk_win_ok;        // gather windows computed for this matrix
    int32_t* pk_win;      // [2 G]: first workgroups, then last workgroups of the gather windows
    double* pk_part;      // [2][2][G]
    unsigned* pk_sync;    // (18 + G) lines, zeroed before every launch
    int pk_ovf;           // overflow build (more than PK_MAXS slices per wave)
    double* pk_v;         // [n] v of the overflow rows
    int pk_coop;          // launch through hipLaunchCooperativeKernel (fem_pcg_solve; FEM_TUNE_PK_COOP elsewhere)
    int pk_gv;            // pipelined persistent iteration (FEM_TUNE_PK_GV, pcg_persist_gv.hpp)
    double* gv_buf;       // its vectors: u, w, q, z, m[0], m[1] ([6 n])
    int64_t gv_cap;       // doubles gv_buf holds
    int gv_init_pending;  // the next launch forms w0 = A u0, m0 and gamma0 / delta0
    int64_t pk_epochs;    // upper bound of the barrier epochs enqueued since the sync words were last zeroed
    hipEvent_t pev[2];    // fem_pcg_profile's events of the persistent launch (created once per context)
    // distributed persistent schedule (fem_pcg_set_rows): rows partitioned over ranks, one persistent launch per
    // rank, u hand-offs and rank sums through the ranks' comm blocks (pcg_persist.hpp DIST build)
    int pd;
    int pd_rank, pd_nranks, pd_grid_req;
    int64_t pd_split[PK_MAX_RANKS + 1];   // global slice bounds of the ranks
    char* pd_block;                       // this rank's comm block (hipMalloc: exportable through IPC)
    int64_t pd_block_bytes, pd_off_flag, pd_off_red, pd_off_rflag;
    int64_t pd_off_m1;    // FEM_TUNE_PK_GV: the second m region of the comm block (m[0] is the u region at 0)
    char* pd_peer[PK_MAX_RANKS];          // comm blocks of all ranks (own included), set by fem_pcg_set_peers
    int pd_peers_ok;
    int32_t* pd_pub;                      // [G][nranks][2] rows of each local workgroup gathered by each rank
    int pd_init_pending;                  // the next launch runs the distributed init (r0, u0, r0.u0)
    unsigned long long* pd_prof;          // fem_pcg_set_prof: launches run the phase-clock build into this buffer
    // merged update (FEM_TUNE_UPD1, 3-kernel schedule): K2 + K3 as one launch of u2_grid resident workgroups
    int upd1;
    int u2_grid;
    unsigned* u2_sync;                    // [U2_WORDS]: release epoch, broadcast (beta, halt), give-up
    // element-chunk operator (fem_pcg_set_operator_mf): K1 = k_pcg_mf_dot + k_mf_gather instead of a SELL SpMV
    fem_mf* mf;
    double* mf_sl;  // this context's slot buffer [nslots * bs] (no other context or stream writes it)
    int64_t mf_sl_cap;   // doubles mf_sl holds (a later operator with more slots reallocates it)
    int mf_nogather;     // distributed element-chunk iteration: the gather-free form (FEM_MF_DIST_NOGATHER)
    int mf_qfuse;   // the merged update reads q from the slots (no gather launch); set per launch of K1 + update2
};

#define FEM_NCCL(call)                                                                         \
    do {                                                                                       \
        ncclResult_t _r = (call);                                                              \
        if (_r != ncclSuccess) {                                                               \
            ::fem::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, ncclGetErrorString(_r)); \
            return FEM_ERCCL;                                                                  \
        }                                                                                      \
    } while (0)

// columns of the paired matrix copy: bs = 1 pairs its columns, bs = 3 (layout A) keeps cols16
static const int16_t* pcols(const fem_pcg* s) { return s->bs == 1 ? s->pcols16 : s->cols16; }

static double* st_red(fem_pcg* s, int k) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(s->st) + offsetof(PcgState, red)) + k;
}

// K1 on the element-chunk operator (matfree.hpp): the chunks' slot values of q = A p and the p.q partials (sum over
// every chunk's local nodes of p . slot = p . A p), then alpha as k_pcg_spmv_dot; the slots are summed into q by
// k_mf_gather. Workgroups walk chunks XCD-contiguously (chunk ranges per XCD, consecutive chunks at once).
template <int BS>
__global__ void __launch_bounds__(MF_BLOCK) k_pcg_mf_dot(MfOp op, const double* __restrict__ p,
                                                         double* __restrict__ slots, PcgState* __restrict__ st,
                                                         RedBuf red) {
    __shared__ MfKernelLds<BS, MF_DOT> L;
    __shared__ double lds4[MF_BLOCK / 64];
    __shared__ int flag;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->xupd = 0;
    if (st->halt || st->iter >= st->max_iter) return;
    double dot = mf_walk_any<BS, MF_DOT>(op, p, slots, L);
    dot = block_sum<MF_BLOCK>(dot, lds4);
    double pq;
    if (reduce_grid<MF_BLOCK>(dot, red.part(RED_K1), red.cnt(RED_K1), &pq, lds4, &flag) && threadIdx.x == 0)
        finish_pq(st, pq);
}

// Distributed single-reduction iteration on the element-chunk operator (BASELINE configs[3] as north_star puts it:
// element partitions, the rank's own elements formed in every application, the halo-DOF partials exchanged inside the
// iteration). Replaces k_cg1_spmv's SpMV by two launches: the rank's chunks into its slots (v = A_r u, never a matrix),
// then the slot gather -- v per local node in ascending chunk order, d = u.v over all local rows (the rank partials of
// an operator sum, as k_cg1_spmv's), the interface rows packed for the exchange, the step committed by the last block.
// k_cg1_update then reads v like the assembled path's q.
template <int BS>
__global__ void __launch_bounds__(MF_BLOCK) k_cg1_mf_slots(MfOp op, const double* __restrict__ u,
                                                           double* __restrict__ slots, const PcgState* __restrict__ st,
                                                           int always, P2PArgs xp, const double* __restrict__ recv,
                                                           const double* __restrict__ send, int64_t off) {
    __shared__ MfKernelLds<BS, MF_APPLY> L;
    if (!always) {   // the step of this pass, from the unchanged state (committed by k_cg1_mf_gather)
        const Cg1Step k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
        if (!k.go) return;
    }
    (void)mf_walk_any<BS, MF_APPLY>(op, u, slots, L);
}

// FEM_MF_DIST_NOGATHER: the walk also reduces d = u.v (sum over the slots of u_node . slot) -> st->red[0]
template <int BS>
__global__ void __launch_bounds__(MF_BLOCK) k_cg1_mf_slots_dot(MfOp op, const double* __restrict__ u,
                                                               double* __restrict__ slots, PcgState* __restrict__ st,
                                                               int always, P2PArgs xp, const double* __restrict__ recv,
                                                               const double* __restrict__ send, int64_t off,
                                                               RedBuf red) {
    __shared__ MfKernelLds<BS, MF_DOT> L;
    __shared__ double lds4[MF_BLOCK / 64];
    __shared__ int flag;
    if (!always) {   // the step of this pass, from the unchanged state (committed by k_cg1_mf_iface)
        const Cg1Step k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
        if (!k.go) return;
    }
    double dot = mf_walk_any<BS, MF_DOT>(op, u, slots, L);
    dot = block_sum<MF_BLOCK>(dot, lds4);
    double d;
    if (reduce_grid<MF_BLOCK>(dot, red.part(RED_K1), red.cnt(RED_K1), &d, lds4, &flag) && threadIdx.x == 0)
        st->red[0] = d;
}

// FEM_MF_DIST_NOGATHER: the interface rows only -- their slot sums packed for the exchange -- and [g, d]; the last
// block commits the step
template <int BS>
__global__ void __launch_bounds__(PCG_BLOCK) k_cg1_mf_iface(MfOp op, const double* __restrict__ slots,
                                                            const int32_t* __restrict__ imap, int64_t nI,
                                                            double* __restrict__ send, int64_t off,
                                                            PcgState* __restrict__ st, RedBuf red, int always,
                                                            P2PArgs xp, const double* __restrict__ recv, double* hist,
                                                            int64_t hist_len) {
    __shared__ double lds4[4];
    __shared__ int flag;
    Cg1Step k{};
    if (!always) {
        k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
        if (!k.go) {
            if (blockIdx.x == 0 && threadIdx.x == 0) cg1_commit(st, k, hist, hist_len);
            return;
        }
    }
    for (int64_t j = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; j < nI; j += (int64_t)gridDim.x * PCG_BLOCK) {
        const int32_t a = imap[j];
        if (a < 0) continue;   // an interface node of other ranks only (send keeps its zeros)
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            const double o = mf_q_dof<BS>(op, slots, (int64_t)a * BS + c);
            if (xp.P) {   // straight into every peer's message slot for this node
                for (int q = 0; q < xp.P; ++q) {
                    const int dst = xp.csrc[j * xp.P + q];
                    if (dst >= 0) xp.psend[dst + c] = o;
                }
            } else {
                send[j * BS + c] = o;
            }
        }
    }
    double unused;   // the grid reduction as a completion count: its last block packs [g, d] and commits
    if (reduce_grid(0.0, red.part(RED_INIT), red.cnt(RED_INIT), &unused, lds4, &flag) && threadIdx.x == 0) {
        if (!always) cg1_commit(st, k, hist, hist_len);   // every block of the three kernels has read the state
        const double d = st->red[0];
        send[off] = st->red[1];
        send[off + 1] = d;
        for (int q = 0; q < xp.P; ++q) {
            const int dst = xp.ssrc[q];
            if (dst >= 0) {
                xp.psend[dst] = st->red[1];
                xp.psend[dst + 1] = d;
            }
        }
    }
}

template <int BS>
__global__ void __launch_bounds__(PCG_BLOCK) k_cg1_mf_gather(MfOp op, const double* __restrict__ slots,
                                                             const double* __restrict__ u, double* __restrict__ v,
                                                             const int32_t* __restrict__ ipos, double* __restrict__ send,
                                                             int64_t off, PcgState* __restrict__ st, RedBuf red,
                                                             int always, P2PArgs xp, const double* __restrict__ recv,
                                                             double* hist, int64_t hist_len) {
    __shared__ double lds4[4];
    __shared__ int flag;
    Cg1Step k{};
    if (!always) {
        k = cg1_eval(st, cg1_scalar(recv, send, off, 0, xp), cg1_scalar(recv, send, off, 1, xp));
        if (!k.go) {
            if (blockIdx.x == 0 && threadIdx.x == 0) cg1_commit(st, k, hist, hist_len);
            return;
        }
    }
    double dot = 0.0;
    for (int64_t a = (int64_t)blockIdx.x * PCG_BLOCK + threadIdx.x; a < op.nnodes;
         a += (int64_t)gridDim.x * PCG_BLOCK) {
        double o[BS];
#pragma unroll
        for (int c = 0; c < BS; ++c) o[c] = 0.0;
        const int k0 = op.nptr[a], k1 = op.nptr[a + 1];
        if (FEM_MF_QK_ON && op.spos && k1 > k0) {   // the update's fixed-count loads (mf_q_dof): the same bits
            double v[MF_QK][BS];
#pragma unroll
            for (int q = 0; q < MF_QK; ++q) {
                const int k = k0 + q < k1 ? k0 + q : k1 - 1;
#pragma unroll
                for (int c = 0; c < BS; ++c) v[q][c] = slots[(int64_t)k * BS + c];
            }
#pragma unroll
            for (int q = 0; q < MF_QK; ++q)
#pragma unroll
                for (int c = 0; c < BS; ++c) o[c] += k0 + q < k1 ? v[q][c] : 0.0;
            for (int kk = k0 + MF_QK; kk < k1; ++kk)
#pragma unroll
                for (int c = 0; c < BS; ++c) o[c] += slots[(int64_t)kk * BS + c];
        } else {
            for (int kk = k0; kk < k1; ++kk) {
                const int64_t sl = op.spos ? kk : op.nslot[kk];
#pragma unroll
                for (int c = 0; c < BS; ++c) o[c] += slots[sl * BS + c];
            }
        }
        const int32_t j = ipos ? ipos[a] : -1;
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            v[a * BS + c] = o[c];
            dot += u[a * BS + c] * o[c];
            if (j >= 0) {
                if (xp.P) {   // straight into every peer's message slot for this node
                    for (int r = 0; r < xp.P; ++r) {
                        const int dst = xp.csrc[(int64_t)j * xp.P + r];
                        if (dst >= 0) xp.psend[dst + c] = o[c];
                    }
                } else {
                    send[(int64_t)j * BS + c] = o[c];
                }
            }
        }
    }
    dot = block_sum256(dot, lds4);
    double d;
    if (reduce_grid(dot, red.part(RED_K1), red.cnt(RED_K1), &d, lds4, &flag) && threadIdx.x == 0) {
        if (!always) cg1_commit(st, k, hist, hist_len);   // every block of the three kernels has read the state
        st->red[0] = d;
        send[off] = st->red[1];
        send[off + 1] = d;
        for (int r = 0; r < xp.P; ++r) {
            const int dst = xp.ssrc[r];
            if (dst >= 0) {
                xp.psend[dst] = st->red[1];
                xp.psend[dst + 1] = d;
            }
        }
    }
}

static int launch_mf_dot(fem_pcg* s) {
    const MfOp op = mf_op(s->mf);
    double* sl = s->mf_sl;
    const int G = mf_resident_grid(s->bs == 3 ? (const void*)k_pcg_mf_dot<3> : (const void*)k_pcg_mf_dot<1>, MF_BLOCK,
                                   op.nchunks);
    if (s->bs == 3) hipLaunchKernelGGL(k_pcg_mf_dot<3>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->p0, sl, s->st, s->red);
    else hipLaunchKernelGGL(k_pcg_mf_dot<1>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->p0, sl, s->st, s->red);
    FEM_LAUNCHED();
    s->mf_qfuse = s->upd1 && !(s->tune & FEM_TUNE_MF_GATHER);
    if (op.nnodes > 0 && !s->mf_qfuse) {
        if (s->bs == 3) hipLaunchKernelGGL(k_mf_gather<3>, dim3(stream_grid(op.nnodes, 256)), dim3(256), 0, s->stream, op, sl, s->q);
        else hipLaunchKernelGGL(k_mf_gather<1>, dim3(stream_grid(op.nnodes, 256)), dim3(256), 0, s->stream, op, sl, s->q);
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

static int launch_spmv_dot(fem_pcg* s) {
    if (s->mf) return launch_mf_dot(s);
    if (s->cols16) {
#define FEM_K1D(B, F, D)                                                                                           \
    hipLaunchKernelGGL((k_pcg_spmv_dot<B, F, D, int16_t>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream,     \
                       s->nslices, s->nrows, s->slice_ptr, s->cols16, s->vals, s->p0, s->p1, s->r, s->w, s->x, s->q, \
                       s->st, s->red, s->tune & FEM_TUNE_REVERSE)
        if (s->paired && !s->fused) {   // 16-byte-value copy of the matrix (sell_pair.hpp / sell_pair3.hpp)
            if (s->bs == 1)
                hipLaunchKernelGGL((k_pcg_spmv_dot<1, false, true, int16_t, true>), dim3(s->grid_spmv), dim3(PCG_BLOCK),
                                   0, s->stream, s->nslices, s->nrows, s->slice_ptr, pcols(s), s->pvals, s->p0, s->p1,
                                   s->r, s->w, s->x, s->q, s->st, s->red, s->tune & FEM_TUNE_REVERSE);
            else
                hipLaunchKernelGGL((k_pcg_spmv_dot<3, false, true, int16_t, true>), dim3(s->grid_spmv), dim3(PCG_BLOCK),
                                   0, s->stream, s->nslices, s->nrows, s->slice_ptr, pcols(s), s->pvals, s->p0, s->p1,
                                   s->r, s->w, s->x, s->q, s->st, s->red, s->tune & FEM_TUNE_REVERSE);
        } else if (s->dist) {
            if (s->bs == 1) FEM_K1D(1, false, true);
            else FEM_K1D(3, false, true);
        } else if (s->bs == 1) {
            if (s->fused) FEM_K1D(1, true, true);
            else FEM_K1D(1, false, true);
        } else {
            if (s->fused) FEM_K1D(3, true, true);
            else FEM_K1D(3, false, true);
        }
#undef FEM_K1D
        FEM_LAUNCHED();
        return FEM_OK;
    }
#define FEM_K1(B, F, D)                                                                                            \
    hipLaunchKernelGGL((k_pcg_spmv_dot<B, F, D>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices,   \
                       s->nrows, s->slice_ptr, s->cols, s->vals, s->p0, s->p1, s->r, s->w, s->x, s->q, s->st, s->red,  \
                       s->tune & FEM_TUNE_REVERSE)
    if (s->dist) {
        if (s->bs == 1) FEM_K1(1, false, true);
        else FEM_K1(3, false, true);
    } else if (s->bs == 1) {
        if (s->fused) FEM_K1(1, true, true);
        else FEM_K1(1, false, true);
    } else {
        if (s->fused) FEM_K1(3, true, true);
        else FEM_K1(3, false, true);
    }
#undef FEM_K1
    FEM_LAUNCHED();
    return FEM_OK;
}

static int launch_update(fem_pcg* s) {
    hipLaunchKernelGGL(k_pcg_update, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->r, s->q, s->w, s->st,
                       s->red, s->hist, s->hist_len, s->dist ? s->own : nullptr, s->bs);
    FEM_LAUNCHED();
    return FEM_OK;
}

static int launch_pupdate(fem_pcg* s);

// ---------------------------------------------------------------- distributed iteration, phase by phase
// iteration : [0] K1 (local A p, p.q partial over all local rows) + pack q and p.q | sum hbuf (nI*bs + 1)
//             [1] unpack q, alpha + guards from the summed p.q | [2] K2 (r, r.z over owned rows) | sum red[1]
//             [3] beta/stop (k_fin_rz) + K3                       -> two collectives per iteration
// start     : [10] (CG: x[fixed]=0) A x + pack | sum hbuf | [11] unpack + r0, r0.z0 | sum red[2] | [12] rz
static int halo_pack(fem_pcg* s, const double* v, bool guarded, bool scalar) {
    hipLaunchKernelGGL(k_halo_pack, dim3(stream_grid(s->nI * s->bs + 1, 256)), dim3(256), 0, s->stream, v, s->bs,
                       s->imap, s->nI, s->hbuf, guarded ? (const PcgState*)s->st : nullptr, scalar ? 1 : 0);
    FEM_LAUNCHED();
    return FEM_OK;
}

// single-reduction pieces (k_cg1_*); the group path (comm == NULL) copies send -> recv so the caller's in-place
// group sum sees this rank's buffer, the RCCL path all-reduces send -> recv out of place
static int64_t cg1_len(const fem_pcg* s) { return s->nI * s->bs + 2; }

static P2PArgs p2p_args(const fem_pcg* s) {
    P2PArgs x{};
    if (s->p2p) {
        x.P = s->p2p_nranks;
        x.csrc = s->p2p_csrc;
        x.ssrc = s->p2p_ssrc;
        x.psend = s->psend;
        x.precv = s->precv;
    }
    return x;
}

static int cg1_spmv(fem_pcg* s, int always) {
    const int64_t off = s->nI * s->bs;
    const int32_t* ipos = s->nI > 0 ? s->ipos : nullptr;
    if (s->mf && s->mf_nogather) {   // chunks into the slots + d, then the interface pack only
        const MfOp op = mf_op(s->mf);
        const P2PArgs xp = p2p_args(s);
        if (op.nchunks > 0) {
            const void* fn = s->bs == 3 ? (const void*)k_cg1_mf_slots_dot<3> : (const void*)k_cg1_mf_slots_dot<1>;
            const int G = mf_resident_grid(fn, MF_BLOCK, op.nchunks);
            if (s->bs == 3)
                hipLaunchKernelGGL(k_cg1_mf_slots_dot<3>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->cg1_u,
                                   s->mf_sl, s->st, always, xp, s->cg1_recv, s->cg1_send, off, s->red);
            else
                hipLaunchKernelGGL(k_cg1_mf_slots_dot<1>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->cg1_u,
                                   s->mf_sl, s->st, always, xp, s->cg1_recv, s->cg1_send, off, s->red);
            FEM_LAUNCHED();
        } else {   // no element on this rank: d = 0
            FEM_HIP(hipMemsetAsync(st_red(s, 0), 0, sizeof(double), s->stream));
        }
        const int Gi = grid_multiple_of_xcd(cdiv(s->nI > 0 ? s->nI : 1, PCG_BLOCK), 1024);
        const int32_t* imap = s->nI > 0 ? s->imap : nullptr;
        if (s->bs == 3)
            hipLaunchKernelGGL(k_cg1_mf_iface<3>, dim3(Gi), dim3(PCG_BLOCK), 0, s->stream, op, s->mf_sl, imap, s->nI,
                               s->cg1_send, off, s->st, s->red, always, xp, s->cg1_recv, s->hist, s->hist_len);
        else
            hipLaunchKernelGGL(k_cg1_mf_iface<1>, dim3(Gi), dim3(PCG_BLOCK), 0, s->stream, op, s->mf_sl, imap, s->nI,
                               s->cg1_send, off, s->st, s->red, always, xp, s->cg1_recv, s->hist, s->hist_len);
        FEM_LAUNCHED();
        if (!s->comm && s->p2p) return FEM_OK;
        if (!s->comm)
            FEM_HIP(hipMemcpyAsync(s->cg1_recv, s->cg1_send, sizeof(double) * (size_t)cg1_len(s),
                                   hipMemcpyDeviceToDevice, s->stream));
        return FEM_OK;
    }
    if (s->mf) {   // element-chunk operator: the rank's chunks into the context's slots, then the slot gather
        const MfOp op = mf_op(s->mf);
        const P2PArgs xp = p2p_args(s);
        if (op.nchunks > 0) {
            const void* fn = s->bs == 3 ? (const void*)k_cg1_mf_slots<3> : (const void*)k_cg1_mf_slots<1>;
            const int G = mf_resident_grid(fn, MF_BLOCK, op.nchunks);
            if (s->bs == 3)
                hipLaunchKernelGGL(k_cg1_mf_slots<3>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->cg1_u, s->mf_sl,
                                   s->st, always, xp, s->cg1_recv, s->cg1_send, off);
            else
                hipLaunchKernelGGL(k_cg1_mf_slots<1>, dim3(G), dim3(MF_BLOCK), 0, s->stream, op, s->cg1_u, s->mf_sl,
                                   s->st, always, xp, s->cg1_recv, s->cg1_send, off);
            FEM_LAUNCHED();
        }
        const int Gg = grid_multiple_of_xcd(cdiv(s->nrows, PCG_BLOCK), 1024);
        if (s->bs == 3)
            hipLaunchKernelGGL(k_cg1_mf_gather<3>, dim3(Gg), dim3(PCG_BLOCK), 0, s->stream, op, s->mf_sl, s->cg1_u,
                               s->q, ipos, s->cg1_send, off, s->st, s->red, always, xp, s->cg1_recv, s->hist,
                               s->hist_len);
        else
            hipLaunchKernelGGL(k_cg1_mf_gather<1>, dim3(Gg), dim3(PCG_BLOCK), 0, s->stream, op, s->mf_sl, s->cg1_u,
                               s->q, ipos, s->cg1_send, off, s->st, s->red, always, xp, s->cg1_recv, s->hist,
                               s->hist_len);
        FEM_LAUNCHED();
        if (!s->comm && s->p2p) return FEM_OK;
        if (!s->comm)
            FEM_HIP(hipMemcpyAsync(s->cg1_recv, s->cg1_send, sizeof(double) * (size_t)cg1_len(s),
                                   hipMemcpyDeviceToDevice, s->stream));
        return FEM_OK;
    }
#define FEM_CG1(B, CI, PR, C, V)                                                                                   \
    hipLaunchKernelGGL((k_cg1_spmv<B, CI, PR>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices,     \
                       s->nrows, s->slice_ptr, C, V, s->cg1_u, s->q, ipos, s->cg1_send, off, s->st, s->red, always, \
                       s->tune & FEM_TUNE_REVERSE, p2p_args(s), s->cg1_recv, s->hist, s->hist_len)
    if (s->paired && s->bs == 1) FEM_CG1(1, int16_t, true, pcols(s), s->pvals);
    else if (s->paired) FEM_CG1(3, int16_t, true, pcols(s), s->pvals);
    else if (s->cols16 && s->bs == 1) FEM_CG1(1, int16_t, false, s->cols16, s->vals);
    else if (s->cols16) FEM_CG1(3, int16_t, false, s->cols16, s->vals);
    else if (s->bs == 1) FEM_CG1(1, int32_t, false, s->cols, s->vals);
    else FEM_CG1(3, int32_t, false, s->cols, s->vals);
#undef FEM_CG1
    FEM_LAUNCHED();
    if (!s->comm && s->p2p) return FEM_OK;   // group path: the caller moves psend -> peers' precv
    if (!s->comm)
        FEM_HIP(hipMemcpyAsync(s->cg1_recv, s->cg1_send, sizeof(double) * (size_t)cg1_len(s), hipMemcpyDeviceToDevice,
                               s->stream));
    return FEM_OK;
}

static int cg1_step_update(fem_pcg* s) {
    if (s->mf && s->mf_nogather)
        hipLaunchKernelGGL(k_cg1_update<true>, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->bs, s->x,
                           s->r, s->p0, s->cg1_s, s->cg1_u, s->q, s->w, s->cg1_recv, s->nI > 0 ? s->ipos : nullptr,
                           s->own, s->st, s->red, p2p_args(s), s->cg1_send, s->nI * s->bs, mf_op(s->mf), s->mf_sl);
    else
        hipLaunchKernelGGL(k_cg1_update<false>, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->bs, s->x,
                           s->r, s->p0, s->cg1_s, s->cg1_u, s->q, s->w, s->cg1_recv, s->nI > 0 ? s->ipos : nullptr,
                           s->own, s->st, s->red, p2p_args(s), s->cg1_send, s->nI * s->bs);
    FEM_LAUNCHED();
    return FEM_OK;
}

// fused iteration setup (at fem_pcg_start of a single-reduction distributed context with FEM_TUNE_C1F): the grid
// (resident by the occupancy query), the gather windows of this matrix, zeroed flags
static const void* c1f_fn(const fem_pcg* s) {
    if (s->paired && s->bs == 1) return (const void*)k_cg1_fused<1, int16_t, true>;
    if (s->paired) return (const void*)k_cg1_fused<3, int16_t, true>;
    if (s->cols16 && s->bs == 1) return (const void*)k_cg1_fused<1, int16_t, false>;
    if (s->cols16) return (const void*)k_cg1_fused<3, int16_t, false>;
    if (s->bs == 1) return (const void*)k_cg1_fused<1, int32_t, false>;
    return (const void*)k_cg1_fused<3, int32_t, false>;
}

// Context buffers of bs = 1 solves (vectors, reduction words, the paired matrix copy, persistent-kernel words) are
// recycled through a process-wide cache keyed by (device, exact size) instead of hipFree'd: tearing down a 10M
// context cost 1.4 ms (4 % of a 682-iteration solve) with hipFree and with the stream-ordered pool alike, and
// repeated solves on one matrix ask for the same sizes. At most PCG_CACHE_KEEP bytes are kept (oldest freed first).
// RCCL buffers and bs = 3 contexts keep plain hipMalloc: with recycled buffers the 10M elastic SpMV ran 311 -> 367 us
// (whatever the match order; cause not found), for 1 ms less teardown.
#ifndef FEM_PCG_POOL
#define FEM_PCG_POOL 1
#endif
// cap of the cache (FEM355_PCG_CACHE_MB, default 1024 MB: a 10M-row bs = 1 context with its paired matrix copy is
// ~330 MB); fem_pcg_release_cache() hands everything back to the driver (the Python layer calls it at exit and
// before retrying a failed allocation)
static size_t pcg_cache_keep() {
    static const size_t keep = [] {
        const char* e = getenv("FEM355_PCG_CACHE_MB");
        const long long mb = e ? atoll(e) : 1024;
        return (size_t)(mb < 0 ? 0 : mb) << 20;
    }();
    return keep;
}

namespace {
struct DevBuf {
    void* p;
    size_t bytes;
    int dev;
};
std::mutex dev_cache_mu;
std::vector<DevBuf> dev_cache;   // free buffers, oldest first
std::vector<DevBuf> dev_live;    // handed out by pool_alloc
size_t dev_cache_bytes = 0;
}  // namespace

static hipError_t pool_alloc(void** p, size_t bytes, hipStream_t, bool cached) {
    if (!FEM_PCG_POOL || !cached) return hipMalloc(p, bytes);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(dev_cache_mu);
    // oldest first: a context created after another one's teardown gets the same buffers in the same roles
    for (size_t i = 0; i < dev_cache.size(); ++i) {
        if (dev_cache[i].bytes == bytes && dev_cache[i].dev == dev) {
            *p = dev_cache[i].p;
            dev_cache_bytes -= bytes;
            dev_live.push_back(dev_cache[i]);
            dev_cache.erase(dev_cache.begin() + (ptrdiff_t)i);
            return hipSuccess;
        }
    }
    e = hipMalloc(p, bytes);
    if (e == hipSuccess) dev_live.push_back({*p, bytes, dev});
    return e;
}

// the caller's stream must not use p any more: the buffer can be handed to another context at once
static void pool_free(void* p, hipStream_t st) {
    if (!p) return;
    if (!FEM_PCG_POOL) {
        (void)hipFree(p);
        return;
    }
    (void)hipStreamSynchronize(st);
    std::lock_guard<std::mutex> g(dev_cache_mu);
    for (size_t i = 0; i < dev_live.size(); ++i) {
        if (dev_live[i].p != p) continue;
        dev_cache.push_back(dev_live[i]);
        dev_cache_bytes += dev_live[i].bytes;
        dev_live.erase(dev_live.begin() + (ptrdiff_t)i);
        while (dev_cache_bytes > pcg_cache_keep() && !dev_cache.empty()) {
            (void)hipFree(dev_cache.front().p);
            dev_cache_bytes -= dev_cache.front().bytes;
            dev_cache.erase(dev_cache.begin());
        }
        return;
    }
    (void)hipFree(p);
}

static size_t pool_release_all() {
    std::lock_guard<std::mutex> g(dev_cache_mu);
    size_t freed = 0;
    for (const DevBuf& b : dev_cache) {
        (void)hipFree(b.p);
        freed += b.bytes;
    }
    dev_cache.clear();
    dev_cache_bytes = 0;
    return freed;
}

// Pinned host status words are recycled too: hipHostFree synchronises the device and unpins (1.4 ms per context).
static std::mutex host_mu;
static std::vector<void*> host_free_list;

static hipError_t host_state_alloc(void** p, size_t bytes) {
    {
        std::lock_guard<std::mutex> g(host_mu);
        if (!host_free_list.empty()) {
            *p = host_free_list.back();
            host_free_list.pop_back();
            return hipSuccess;
        }
    }
    return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

static void host_state_free(void* p, hipStream_t st) {
    if (!p) return;
    (void)hipStreamSynchronize(st);   // no copy of this context may still target the buffer
    std::lock_guard<std::mutex> g(host_mu);
    host_free_list.push_back(p);
}

static int c1f_setup(fem_pcg* s) {
    s->c1f = 0;
    if (!(s->tune & FEM_TUNE_C1F) || !s->dist || !s->cg1 || s->nslices == 0 || s->mf) return FEM_OK;
    int dev = 0, ncu = 0, nb = 0;
    FEM_HIP(hipGetDevice(&dev));
    FEM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, c1f_fn(s), C1F_BLOCK, 0));
    if (nb < 1 || ncu < NXCD) return FEM_OK;
    const int per = nb < 2 ? nb : 2;   // 8 waves per CU (4 per CU: 10M 103 -> 93 us, 1.2M tets 21.6 -> 25.1 us)
    int G = (ncu / NXCD) * NXCD * per;
    while (G > NXCD && (int64_t)G > s->nslices) G -= NXCD;   // at least one slice per workgroup
    if (G != s->c1f_grid) {
        if (s->c1f_win) (void)hipFree(s->c1f_win);
        if (s->c1f_flags) (void)hipFree(s->c1f_flags);
        s->c1f_win = nullptr;
        s->c1f_flags = nullptr;
        FEM_HIP(hipMalloc(&s->c1f_win, sizeof(int32_t) * 2 * G));
        FEM_HIP(hipMalloc(&s->c1f_flags, sizeof(unsigned) * 32 * (size_t)(G + 1)));
        s->c1f_grid = G;
        s->c1f_win_ok = 0;
    }
    if (!s->c1f_win_ok) {
        std::vector<int32_t> lohi(2 * (size_t)G);
        for (int i = 0; i < G; ++i) {
            lohi[i] = G;
            lohi[G + i] = -1;
        }
        FEM_HIP(hipMemcpyAsync(s->c1f_win, lohi.data(), sizeof(int32_t) * 2 * G, hipMemcpyHostToDevice, s->stream));
        if (s->cols16)
            hipLaunchKernelGGL(k_c1f_window<int16_t>, dim3(stream_grid(s->nslices * 64, 256)), dim3(256), 0, s->stream,
                               s->nslices, s->nrows, s->slice_ptr, s->cols16, G, s->c1f_win, s->c1f_win + G);
        else
            hipLaunchKernelGGL(k_c1f_window<int32_t>, dim3(stream_grid(s->nslices * 64, 256)), dim3(256), 0, s->stream,
                               s->nslices, s->nrows, s->slice_ptr, s->cols, G, s->c1f_win, s->c1f_win + G);
        FEM_LAUNCHED();
        FEM_HIP(hipStreamSynchronize(s->stream));   // lohi must outlive the copy
        s->c1f_win_ok = 1;
    }
    FEM_HIP(hipMemsetAsync(s->c1f_flags, 0, sizeof(unsigned) * 32 * (size_t)(G + 1), s->stream));
    s->c1f = 1;
    return FEM_OK;
}

// merged update (k_pcg_update2) for the single-GPU 3-kernel schedule: grid = every workgroup resident at once
// (occupancy query, cached per device; the value is idempotent, so a racing first query only repeats the work)
static int u2_setup(fem_pcg* s) {
    s->upd1 = 0;
    if (!(s->tune & FEM_TUNE_UPD1) || s->dist || s->fused || s->deferred || s->persist || s->has_con || s->n < 2)
        return FEM_OK;
    // per instantiation launched (the element-chunk operator's forms sum the slots in the update and hold more
    // registers): every workgroup of the launch must be resident at once
    static std::atomic<int> occ[3][64];
    const int var = s->mf ? (s->bs == 3 ? 2 : 1) : 0;
    int dev = 0;
    FEM_HIP(hipGetDevice(&dev));
    int per_cu = occ[var][dev & 63].load();
    if (per_cu == 0) {
        int ncu = 0, nb = 0;
        FEM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        // the element-chunk forms: the smaller residency of the two (slot sums / q read) per block size
        int nb2 = 0;
        const void* fn = var == 0 ? (const void*)k_pcg_update2 : var == 1 ? (const void*)k_pcg_update2_mf<1, false>
                                                                       : (const void*)k_pcg_update2_mf<3, false>;
        const void* fn2 = var == 0 ? fn : var == 1 ? (const void*)k_pcg_update2_mf<1, true>
                                                   : (const void*)k_pcg_update2_mf<3, true>;
        FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb2, fn2, PCG_BLOCK, 0));
        FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, PCG_BLOCK, 0));
        nb = nb2 < nb ? nb2 : nb;
        per_cu = (nb < 1 || ncu < NXCD) ? -1 : ((ncu / NXCD) * NXCD) * (nb < 8 ? nb : 8);
        occ[var][dev & 63].store(per_cu);
    }
    if (per_cu < 0) return FEM_OK;   // no resident grid: the two-kernel update stays
    int64_t want = cdiv(s->n / 2 + 1, PCG_BLOCK);
    want = cdiv(want, NXCD) * NXCD;
    if (s->tune & FEM_TUNE_U2_SMALL) want = NXCD;   // tests: past the register-cached elements at small n
    s->u2_grid = (int)(want < per_cu ? want : per_cu);
    if (!s->u2_sync) {
        hipError_t e = pool_alloc((void**)&s->u2_sync, sizeof(unsigned) * U2_WORDS, s->stream, s->bs == 1);
        if (e != hipSuccess) {
            set_error("u2_setup: %s", hipGetErrorString(e));
            return FEM_EHIP;
        }
    }
    FEM_HIP(hipMemsetAsync(s->u2_sync, 0, sizeof(unsigned) * U2_WORDS, s->stream));
    s->upd1 = 1;
    return FEM_OK;
}

static int launch_update2(fem_pcg* s) {
    const int hold = (s->tune & FEM_TUNE_U2_HOLD) ? 1 : 0;
    if (s->mf) {   // node form; q from the operator's slots inside the update unless a gather launch wrote it
        const MfOp op = mf_op(s->mf);
        const double* sl = s->mf_sl;
        const int64_t nn = s->nrows;
#define FEM_U2MF(B, FQ)                                                                                               \
    hipLaunchKernelGGL((k_pcg_update2_mf<B, FQ>), dim3(s->u2_grid), dim3(PCG_BLOCK), 0, s->stream, nn, s->x, s->p0,    \
                       s->r, s->q, s->w, s->st, s->red, s->hist, s->hist_len, s->u2_sync, hold, op, sl)
        if (s->bs == 3) {
            if (s->mf_qfuse) FEM_U2MF(3, false);
            else FEM_U2MF(3, true);
        } else {
            if (s->mf_qfuse) FEM_U2MF(1, false);
            else FEM_U2MF(1, true);
        }
#undef FEM_U2MF
        FEM_LAUNCHED();
        return FEM_OK;
    }
    hipLaunchKernelGGL(k_pcg_update2, dim3(s->u2_grid), dim3(PCG_BLOCK), 0, s->stream, s->n, s->x, s->p0, s->r, s->q,
                       s->w, s->st, s->red, s->hist, s->hist_len, s->u2_sync, hold);
    FEM_LAUNCHED();
    return FEM_OK;
}

static int c1f_launch(fem_pcg* s) {
    Cg1FArgs a{};
    a.nslices = s->nslices;
    a.nrows = s->nrows;
    a.slice_ptr = s->slice_ptr;
    if (s->paired) {
        a.cols = pcols(s);
        a.vals = s->pvals;
    } else if (s->cols16) {
        a.cols = s->cols16;
        a.vals = s->vals;
    } else {
        a.cols = s->cols;
        a.vals = s->vals;
    }
    a.x = s->x;
    a.r = s->r;
    a.p = s->p0;
    a.sv = s->cg1_s;
    a.u = s->cg1_u;
    a.v = s->q;
    a.w = s->w;
    a.ipos = s->nI > 0 ? s->ipos : nullptr;
    a.own = s->own;
    a.send = s->cg1_send;
    a.recv = s->cg1_recv;
    a.off = s->nI * s->bs;
    a.st = s->st;
    a.red = s->red;
    a.xp = p2p_args(s);
    a.hist = s->hist;
    a.hist_len = s->hist_len;
    a.win = s->c1f_win;
    a.flags = s->c1f_flags;
    a.tune_rev = (s->tune & FEM_TUNE_REVERSE) ? 1 : 0;
    void* args[] = {&a};
    FEM_HIP(hipLaunchKernel(c1f_fn(s), dim3(s->c1f_grid), dim3(C1F_BLOCK), args, 0, s->stream));
    FEM_LAUNCHED();
    if (!s->comm && !s->p2p)   // group path: the caller sums recv in place
        FEM_HIP(hipMemcpyAsync(s->cg1_recv, s->cg1_send, sizeof(double) * (size_t)cg1_len(s), hipMemcpyDeviceToDevice,
                               s->stream));
    return FEM_OK;
}

static int dist_phase(fem_pcg* s, int phase) {
    int rc = FEM_OK;
    if (s->mf && !s->cg1 && phase < 10) {
        set_error("dist_phase: the element-chunk operator runs the single-reduction distributed iteration (variant 1)");
        return FEM_EARG;
    }
    switch (phase) {
        case 0:
            if ((rc = launch_spmv_dot(s))) return rc;
            return halo_pack(s, s->q, true, true);
        case 1:
            hipLaunchKernelGGL(k_halo_unpack<true>, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->nrows, s->bs,
                               s->ipos, s->hbuf, s->q, s->nI, s->st);
            FEM_LAUNCHED();
            return FEM_OK;
        case 2:
            return launch_update(s);
        case 3:
            hipLaunchKernelGGL(k_fin_rz, dim3(1), dim3(1), 0, s->stream, s->st, s->hist, s->hist_len);
            FEM_LAUNCHED();
            return launch_pupdate(s);
        case 10:
            if (s->mode == FEM_MODE_CG_STABLE) {
                hipLaunchKernelGGL(k_zero_fixed, dim3(stream_grid(s->n, 256)), dim3(256), 0, s->stream, s->n, s->x,
                                   s->w);
                FEM_LAUNCHED();
            }
            if (s->mf) {
                if ((rc = mf_apply(s->mf, s->x, s->q, s->mf_sl, s->stream))) return rc;
            } else if ((rc = (s->cols16 ? fem_spmv16(s->nrows, s->bs, s->slice_ptr, s->cols16, s->vals, s->x, s->q,
                                                     s->stream)
                                        : fem_spmv(s->nrows, s->bs, s->slice_ptr, s->cols, s->vals, s->x, s->q,
                                                   s->stream)))) {
                return rc;
            }
            return halo_pack(s, s->q, false, false);
        case 11:
            hipLaunchKernelGGL(k_halo_unpack<false>, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->nrows, s->bs,
                               s->ipos, s->hbuf, s->q, s->nI, (PcgState*)nullptr);
            FEM_LAUNCHED();
            hipLaunchKernelGGL(k_pcg_init, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->b, s->r, s->q,
                               s->w, s->p0, s->p1, 0, s->st, s->red, s->own, s->bs);
            FEM_LAUNCHED();
            return FEM_OK;
        case 12:
            hipLaunchKernelGGL(k_set_rz, dim3(1), dim3(1), 0, s->stream, s->st);
            FEM_LAUNCHED();
            return FEM_OK;
        case 4:   // single-reduction iteration: step + update + v = A u and pack | sum [v interface | g | d]
            if (!s->cg1) break;
            if (s->c1f) return c1f_launch(s);
            if ((rc = cg1_step_update(s))) return rc;
            return cg1_spmv(s, 0);
        case 20:  // single-reduction start (after 10): unpack A x0, r0, u0, g0; v0 = A u0 and pack | sum
            if (!s->cg1) break;
            hipLaunchKernelGGL(k_halo_unpack<false>, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->nrows, s->bs,
                               s->ipos, s->hbuf, s->q, s->nI, (PcgState*)nullptr);
            FEM_LAUNCHED();
            hipLaunchKernelGGL(k_cg1_init, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->bs, s->b, s->r,
                               s->q, s->w, s->p0, s->cg1_s, s->cg1_u, s->own, s->st, s->red);
            FEM_LAUNCHED();
            return cg1_spmv(s, 1);
        default:
            break;
    }
    set_error("dist_phase: unknown phase %d%s", phase, s->cg1 ? " (single-reduction: 10, 20, then 4)" : "");
    return FEM_EARG;
}

// device buffer summed over the ranks after `phase`
static void dist_buffer(fem_pcg* s, int phase, double** ptr, int64_t* n) {
    *ptr = nullptr;
    *n = 0;
    if (phase == 0) {
        *ptr = s->hbuf;
        *n = s->nI * s->bs + 1;     // interface rows of q + this rank's p.q partial
    } else if (phase == 10) {
        *ptr = s->hbuf;
        *n = s->nI * s->bs;
    } else if (phase == 2) {
        *ptr = st_red(s, 1);
        *n = 1;
    } else if (phase == 11) {
        *ptr = st_red(s, 2);
        *n = 1;
    } else if (s->cg1 && !s->p2p && (phase == 4 || phase == 20)) {
        *ptr = s->cg1_recv;       // group path: summed in place (cg1_spmv copied send -> recv)
        *n = cg1_len(s);
    }
}

static int dist_exchange(fem_pcg* s, int phase) {
    if (s->cg1 && s->p2p && (phase == 4 || phase == 20)) {
        if (!s->comm) {
            set_error("distributed PCG without a communicator: drive it with fem_pcg_dist_phase");
            return FEM_EARG;
        }
        if (!s->peer_rank.empty()) {
            FEM_NCCL(ncclGroupStart());
            for (size_t i = 0; i < s->peer_rank.size(); ++i) {
                FEM_NCCL(ncclSend(s->psend + s->peer_off[i], (size_t)s->peer_cnt[i], ncclFloat64, s->peer_rank[i],
                                  s->comm, s->stream));
                FEM_NCCL(ncclRecv(s->precv + s->peer_off[i], (size_t)s->peer_cnt[i], ncclFloat64, s->peer_rank[i],
                                  s->comm, s->stream));
            }
            FEM_NCCL(ncclGroupEnd());
        }
        return FEM_OK;   // the next step / update kernels sum the messages in rank order
    }
    double* p;
    int64_t n;
    dist_buffer(s, phase, &p, &n);
    if (n <= 0) return FEM_OK;
    if (!s->comm) {
        set_error("distributed PCG without a communicator: drive it with fem_pcg_dist_phase");
        return FEM_EARG;
    }
    if (s->cg1 && (phase == 4 || phase == 20))
        FEM_NCCL(ncclAllReduce(s->cg1_send, s->cg1_recv, (size_t)n, ncclFloat64, ncclSum, s->comm, s->stream));
    else
        FEM_NCCL(ncclAllReduce(p, p, (size_t)n, ncclFloat64, ncclSum, s->comm, s->stream));
    return FEM_OK;
}

// the parts of one distributed iteration after the local SpMV (for fem_pcg_profile's kernel buckets)
static int launch_exchange_dot(fem_pcg* s) {
    if (!s->dist) return FEM_OK;
    int rc;
    if ((rc = halo_pack(s, s->q, true, true))) return rc;
    if ((rc = dist_exchange(s, 0))) return rc;
    return dist_phase(s, 1);
}

// projections on x: one block for small sets, else gather / scatter / SPC grid phases (+ one block for RBE3)
static const int64_t CON_SMALL = 8192;
static int launch_constraints(hipStream_t stream, double* x, double* r, const Constraints& c, const PcgState* st,
                              int always) {
    if (c.R + c.S <= CON_SMALL) {
        hipLaunchKernelGGL(k_constraints, dim3(1), dim3(256), 0, stream, x, r, c, st, always, 3);
        FEM_LAUNCHED();
        return FEM_OK;
    }
    auto phase = [&](int ph) {
        const int64_t m = ph == CON_SPC ? c.S : c.R;
        if (m == 0) return;
        const dim3 g(stream_grid(m, 256));
        if (ph == CON_GATHER) hipLaunchKernelGGL(k_con_phase<CON_GATHER>, g, dim3(256), 0, stream, x, r, c, st, always);
        if (ph == CON_SCATTER) hipLaunchKernelGGL(k_con_phase<CON_SCATTER>, g, dim3(256), 0, stream, x, r, c, st, always);
        if (ph == CON_SPC) hipLaunchKernelGGL(k_con_phase<CON_SPC>, g, dim3(256), 0, stream, x, r, c, st, always);
    };
    if (c.order == 0) {
        phase(CON_GATHER);
        phase(CON_SCATTER);
        phase(CON_SPC);
    } else {
        phase(CON_SPC);
        phase(CON_GATHER);
        phase(CON_SCATTER);
        if (c.G) hipLaunchKernelGGL(k_constraints, dim3(1), dim3(256), 0, stream, x, r, c, st, always, 2);
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

static int launch_pupdate(fem_pcg* s) {
    if (s->fused) return FEM_OK;
    hipLaunchKernelGGL(k_pcg_pupdate, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->x, s->p0, s->r, s->w,
                       s->st);
    FEM_LAUNCHED();
    if (s->has_con) return launch_constraints(s->stream, s->x, nullptr, s->con, s->st, 0);
    return FEM_OK;
}

// K2, and in the distributed mode the r.z all-reduce and the stop test / beta that follow it
static int launch_update_finish(fem_pcg* s) {
    int rc;
    if ((rc = launch_update(s))) return rc;
    if (!s->dist) return FEM_OK;
    if ((rc = dist_exchange(s, 2))) return rc;
    hipLaunchKernelGGL(k_fin_rz, dim3(1), dim3(1), 0, s->stream, s->st, s->hist, s->hist_len);
    FEM_LAUNCHED();
    return FEM_OK;
}

static int launch_deferred(fem_pcg* s, int which) {
    const int par = (int)(s->launched & 1);
    const int rev = (s->tune & FEM_TUNE_REVERSE) ? par : 0;
    if (which == 0) {
        if (s->paired && s->bs == 1) {
            hipLaunchKernelGGL((k_pcg_d1<1, int16_t, true>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream,
                               s->nslices, s->nrows, s->slice_ptr, pcols(s), s->pvals, s->p0, s->q, s->st, par, rev,
                               s->red.partials);
        } else if (s->paired) {
            hipLaunchKernelGGL((k_pcg_d1<3, int16_t, true>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream,
                               s->nslices, s->nrows, s->slice_ptr, pcols(s), s->pvals, s->p0, s->q, s->st, par, rev,
                               s->red.partials);
        } else if (s->cols16) {
            if (s->bs == 1)
                hipLaunchKernelGGL((k_pcg_d1<1, int16_t>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices,
                                   s->nrows, s->slice_ptr, s->cols16, s->vals, s->p0, s->q, s->st, par, rev, s->red.partials);
            else
                hipLaunchKernelGGL((k_pcg_d1<3, int16_t>), dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices,
                                   s->nrows, s->slice_ptr, s->cols16, s->vals, s->p0, s->q, s->st, par, rev, s->red.partials);
        } else if (s->bs == 1)
            hipLaunchKernelGGL(k_pcg_d1<1>, dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices, s->nrows,
                               s->slice_ptr, s->cols, s->vals, s->p0, s->q, s->st, par, rev, s->red.partials);
        else
            hipLaunchKernelGGL(k_pcg_d1<3>, dim3(s->grid_spmv), dim3(PCG_BLOCK), 0, s->stream, s->nslices, s->nrows,
                               s->slice_ptr, s->cols, s->vals, s->p0, s->q, s->st, par, rev, s->red.partials);
    } else if (which == 1) {
        hipLaunchKernelGGL(k_pcg_d2, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->r, s->q, s->w, s->st,
                           par, s->red.partials, s->grid_spmv, s->red.partials + MAX_PARTIALS);
    } else {
        hipLaunchKernelGGL(k_pcg_d3, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->x, s->p0, s->r, s->w,
                           s->st, par, s->red.partials + MAX_PARTIALS, s->grid_vec, s->hist, s->hist_len);
        s->launched++;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

static int launch_persist(fem_pcg* s, int k, unsigned long long* prof = nullptr);

static int launch_iterations(fem_pcg* s, int k) {
    if (s->dist && !s->comm) {
        set_error("distributed PCG without a communicator: drive it with fem_pcg_dist_phase");
        return FEM_EARG;
    }
    if (s->persist) return launch_persist(s, k);
    if (s->deferred && !s->dist) {
        for (int i = 0; i < k; ++i) {
            int rc;
            if ((rc = launch_deferred(s, 0)) || (rc = launch_deferred(s, 1)) || (rc = launch_deferred(s, 2))) return rc;
        }
        return FEM_OK;
    }
    if (s->dist && s->cg1) {
        for (int i = 0; i < k; ++i) {
            int rc;
            if ((rc = dist_phase(s, 4)) || (rc = dist_exchange(s, 4))) return rc;
            s->launched++;
        }
        return FEM_OK;
    }
    for (int i = 0; i < k; ++i) {
        int rc;
        if ((rc = launch_spmv_dot(s))) return rc;
        if (s->upd1) {
            if ((rc = launch_update2(s))) return rc;
        } else {
            if ((rc = launch_exchange_dot(s))) return rc;
            if ((rc = launch_update_finish(s))) return rc;
            if ((rc = launch_pupdate(s))) return rc;
        }
        s->launched++;
    }
    return FEM_OK;
}

extern "C" {

int fem_spmv(int64_t nrows, int bs, const int64_t* slice_ptr, const int32_t* cols, const double* vals, const double* x,
             double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    const int grid = grid_multiple_of_xcd(cdiv(ns, 4), 2048);
    if (bs == 1)
        hipLaunchKernelGGL(k_spmv<1>, dim3(grid), dim3(256), 0, S(stream), ns, nrows, slice_ptr, cols, vals, x, y);
    else if (bs == 3)
        hipLaunchKernelGGL(k_spmv<3>, dim3(grid), dim3(256), 0, S(stream), ns, nrows, slice_ptr, cols, vals, x, y);
    else {
        set_error("fem_spmv: block size %d unsupported", bs);
        return FEM_EARG;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_spmv16(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* dcols, const double* vals,
               const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns == 0) return FEM_OK;
    const int grid = grid_multiple_of_xcd(cdiv(ns, 4), 2048);
    if (bs == 1)
        hipLaunchKernelGGL((k_spmv<1, SPMV_U, false, int16_t>), dim3(grid), dim3(256), 0, S(stream), ns, nrows,
                           slice_ptr, dcols, vals, x, y);
    else if (bs == 3)
        hipLaunchKernelGGL((k_spmv<3, SPMV_U, false, int16_t>), dim3(grid), dim3(256), 0, S(stream), ns, nrows,
                           slice_ptr, dcols, vals, x, y);
    else {
        set_error("fem_spmv16: block size %d unsupported", bs);
        return FEM_EARG;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

// validate the caller's constraint arrays against [0, n) on `stream` (one sync) and fill c (tmp not allocated)
static int make_constraints(const char* fn, int64_t n, hipStream_t stream, int order, int64_t R,
                            const int64_t* rbe2_slave, const int64_t* rbe2_master, int64_t S, const int64_t* spc_dof,
                            const double* spc_val, int64_t G, const int64_t* r3_ptr, const int64_t* r3_master,
                            const double* r3_wsum, const int64_t* r3_slave, const double* r3_w, Constraints* c) {
    if (R < 0 || S < 0 || G < 0 || (R && (!rbe2_slave || !rbe2_master)) || (S && (!spc_dof || !spc_val)) ||
        (G && (!r3_ptr || !r3_master || !r3_wsum)) || (order != 0 && order != 1) || (order == 0 && G)) {
        set_error("%s: bad sizes / pointers / order", fn);
        return FEM_EARG;
    }
    int* bad = nullptr;
    FEM_HIP(::fem::malloc_async((void**)&bad, sizeof(int) * 2, stream));
    FEM_HIP(hipMemsetAsync(bad, 0, sizeof(int) * 2, stream));
    auto chk = [&](const int64_t* v, int64_t m) {
        if (m > 0)
            hipLaunchKernelGGL(k_check_range, dim3(stream_grid(m, 256)), dim3(256), 0, stream, v, m, (int64_t)0, n, bad);
    };
    chk(rbe2_slave, R);
    chk(rbe2_master, R);
    chk(spc_dof, S);
    chk(r3_master, G);
    int64_t E = 0;
    if (G) {
        hipLaunchKernelGGL(k_check_ptr, dim3(stream_grid(G, 256)), dim3(256), 0, stream, r3_ptr, G, bad + 1);
        FEM_HIP(hipMemcpyAsync(&E, r3_ptr + G, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    }
    int hbad[2] = {0, 0};
    FEM_HIP(hipMemcpyAsync(hbad, bad, sizeof(hbad), hipMemcpyDeviceToHost, stream));
    FEM_HIP(hipStreamSynchronize(stream));
    if (!hbad[1] && E > 0) {
        if (!r3_slave || !r3_w) hbad[1] = 1;
        else {
            chk(r3_slave, E);
            FEM_HIP(hipMemcpyAsync(hbad, bad, sizeof(int), hipMemcpyDeviceToHost, stream));
            FEM_HIP(hipStreamSynchronize(stream));
        }
    }
    FEM_HIP(hipFreeAsync(bad, stream));
    if (hbad[0] || hbad[1]) {
        set_error("%s: %s", fn, hbad[0] ? "a constraint dof is outside [0, n)" : "RBE3 group pointer is not a CSR offset array");
        return FEM_EARG;
    }
    *c = Constraints{};
    c->R = R;
    c->S = S;
    c->G = G;
    c->rbe2_slave = rbe2_slave;
    c->rbe2_master = rbe2_master;
    c->spc_dof = spc_dof;
    c->spc_val = spc_val;
    c->r3_ptr = r3_ptr;
    c->r3_master = r3_master;
    c->r3_wsum = r3_wsum;
    c->r3_slave = r3_slave;
    c->r3_w = r3_w;
    c->order = order;
    return FEM_OK;
}

int fem_pcg_set_constraints(fem_pcg* s, int order, int64_t R, const int64_t* rbe2_slave, const int64_t* rbe2_master,
                            int64_t S, const int64_t* spc_dof, const double* spc_val, int64_t G, const int64_t* r3_ptr,
                            const int64_t* r3_master, const double* r3_wsum, const int64_t* r3_slave,
                            const double* r3_w) {
    if (s->mode != FEM_MODE_CG_CONSTRAINED || s->dist || s->fused || s->deferred || s->graph || s->mf) {
        set_error("fem_pcg_set_constraints: needs a CG_CONSTRAINED, single-GPU, 3-kernel context without a graph "
                  "over an assembled matrix");
        return FEM_EARG;
    }
    Constraints c;
    const int rc = make_constraints("fem_pcg_set_constraints", s->n, s->stream, order, R, rbe2_slave, rbe2_master, S,
                                    spc_dof, spc_val, G, r3_ptr, r3_master, r3_wsum, r3_slave, r3_w, &c);
    if (rc != FEM_OK) return rc;
    if (s->con.tmp) (void)hipFree(s->con.tmp);
    s->con.tmp = nullptr;
    if (R > 0) FEM_HIP(hipMalloc(&c.tmp, sizeof(double) * (size_t)R));
    s->con = c;
    s->has_con = 1;
    return FEM_OK;
}

int fem_enforce_constraints(double* x, double* r, int64_t n, int order, int64_t R, const int64_t* rbe2_slave,
                            const int64_t* rbe2_master, int64_t S, const int64_t* spc_dof, const double* spc_val,
                            int64_t G, const int64_t* r3_ptr, const int64_t* r3_master, const double* r3_wsum,
                            const int64_t* r3_slave, const double* r3_w, fem_stream_t stream) {
    if (!x || n < 0) {
        set_error("fem_enforce_constraints: null x / negative n");
        return FEM_EARG;
    }
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    Constraints c;
    const int rc = make_constraints("fem_enforce_constraints", n, st, order, R, rbe2_slave, rbe2_master, S, spc_dof,
                                    spc_val, G, r3_ptr, r3_master, r3_wsum, r3_slave, r3_w, &c);
    if (rc != FEM_OK) return rc;
    if (R > 0) FEM_HIP(::fem::malloc_async((void**)&c.tmp, sizeof(double) * (size_t)R, st));
    const int lrc = launch_constraints(st, x, r, c, nullptr, 1);
    if (lrc != FEM_OK) return lrc;
    if (c.tmp) FEM_HIP(hipFreeAsync(c.tmp, st));
    return FEM_OK;
}

int fem_pcg_set_tuning(fem_pcg* s, int flags) {
    if (s->graph) {
        set_error("fem_pcg_set_tuning: drop the captured graph first");
        return FEM_EARG;
    }
    s->tune = flags;
    return FEM_OK;
}

int fem_pcg_set_cols16(fem_pcg* s, const int16_t* dcols) {
    if (s->graph) {
        set_error("fem_pcg_set_cols16: drop the captured graph first");
        return FEM_EARG;
    }
    s->cols16 = dcols;
    if (!dcols) s->paired = 0;
    return FEM_OK;
}

int fem_stream_copy(const double* src, double* dst, int64_t n, int grid, fem_stream_t stream) {
    if (grid <= 0) grid = 2048;
    hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, S(stream), (const double2*)src, (double2*)dst, n / 2);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_stream_read(const double* src, double* out, int64_t n, int grid, fem_stream_t stream) {
    if (grid <= 0) grid = 4096;
    hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, S(stream), (const double2*)src, n / 2, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_create(int64_t nrows, int bs, const int64_t* slice_ptr, const int32_t* cols, const double* vals,
                   const double* b, double* x, const double* w, int mode, double tol, double eps, double* hist,
                   int64_t hist_len, fem_stream_t stream, fem_pcg** out) {
    if (bs != 1 && bs != 3) {
        set_error("fem_pcg_create: block size %d unsupported", bs);
        return FEM_EARG;
    }
    if (mode != FEM_MODE_CG_STABLE && mode != FEM_MODE_PCG && mode != FEM_MODE_CG_CONSTRAINED) {
        set_error("fem_pcg_create: unknown mode %d", mode);
        return FEM_EARG;
    }
    if (((uintptr_t)b | (uintptr_t)x | (uintptr_t)w) & 15) {
        set_error("fem_pcg_create: vectors must be 16-byte aligned");
        return FEM_EARG;
    }
    fem_pcg* s = new fem_pcg();
    s->tune = FEM_TUNE_REVERSE | FEM_TUNE_PAIR | FEM_TUNE_PK_SC1 | FEM_TUNE_PK_PACK | FEM_TUNE_PK_UNI | FEM_TUNE_UPD1;
    s->nrows = nrows;
    s->bs = bs;
    s->nslices = cdiv(nrows, 64);
    s->n = nrows * bs;
    s->sell_ent = -1;
    s->slice_ptr = slice_ptr;
    s->cols = cols;
    s->vals = vals;
    s->b = b;
    s->x = x;
    s->w = w;
    s->hist = hist;
    s->hist_len = hist ? hist_len : 0;
    s->mode = mode;
    s->tol = tol;
    s->eps = eps;
    s->stream = S(stream);
    s->fused = 0;   // measured: 3-kernel 0.103 ms/it vs fused 0.121 on 10M Poisson (profiles/)
    s->graph = nullptr;
    s->graph_k = 0;
    s->max_iter = 0x7fffffff;
    s->grid_spmv = grid_multiple_of_xcd(cdiv(s->nslices, 4), 2048);
    s->grid_vec = grid_multiple_of_xcd(cdiv(s->n / 2 + 1, PCG_BLOCK), 1024);
    size_t vec = sizeof(double) * (size_t)(s->n + 2);
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = pool_alloc((void**)&s->r, vec, s->stream, s->bs == 1);
    if (e == hipSuccess) e = pool_alloc((void**)&s->p0, vec, s->stream, s->bs == 1);
    if (e == hipSuccess) e = pool_alloc((void**)&s->p1, vec, s->stream, s->bs == 1);
    if (e == hipSuccess) e = pool_alloc((void**)&s->q, vec, s->stream, s->bs == 1);
    if (e == hipSuccess)
        e = pool_alloc((void**)&s->red.partials, sizeof(double) * RED_N * MAX_PARTIALS, s->stream, s->bs == 1);
    if (e == hipSuccess)
        e = pool_alloc((void**)&s->red.counters, sizeof(unsigned) * RED_N * RED_COUNTER_WORDS, s->stream, s->bs == 1);
    if (e == hipSuccess) e = hipMemsetAsync(s->red.counters, 0, sizeof(unsigned) * RED_N * RED_COUNTER_WORDS, s->stream);
    if (e == hipSuccess) e = pool_alloc((void**)&s->st, sizeof(PcgState), s->stream, s->bs == 1);
    if (e == hipSuccess) e = host_state_alloc((void**)&s->st_host, sizeof(PcgState));
    if (e != hipSuccess) {
        set_error("fem_pcg_create: allocation failed: %s", hipGetErrorString(e));
        fem_pcg_destroy(s);
        return FEM_EHIP;
    }
    *out = s;
    return FEM_OK;
}

int fem_pcg_set_operator_mf(fem_pcg* s, fem_mf* m) {
    if (!s || !m || mf_bs(m) != s->bs || mf_nodes(m) != s->nrows) {
        set_error("fem_pcg_set_operator_mf: the operator's block size / node count do not match the context");
        return FEM_EARG;
    }
    if (s->pd || s->has_con || s->graph || s->mode == FEM_MODE_CG_CONSTRAINED) {
        set_error("fem_pcg_set_operator_mf: contexts without constraints (CG_STABLE / PCG mode), the row-partitioned "
                  "schedule or a captured graph only");
        return FEM_EARG;
    }
    if (s->dist && !s->cg1) {
        set_error("fem_pcg_set_operator_mf: a distributed context runs the element-chunk operator in the "
                  "single-reduction variant only (fem_pcg_set_dist_variant(s, 1))");
        return FEM_EARG;
    }
    // the context's own slots (concurrent solves / applications never share them), sized for THIS operator: a second
    // operator over the same nodes with more elements (more slots) gets a larger buffer, never the old one
    const int64_t need = (int64_t)mf_bs(m) * (int64_t)mf_nslots(m);
    if (need > s->mf_sl_cap) {
        if (s->mf_sl) FEM_HIP(hipFree(s->mf_sl));
        s->mf_sl = nullptr;
        s->mf_sl_cap = 0;
        FEM_HIP(hipMalloc(&s->mf_sl, sizeof(double) * (size_t)need));
        s->mf_sl_cap = need;
    }
    s->mf = m;
    {
        const char* e = getenv("FEM355_MF_NOGATHER");
        s->mf_nogather = e ? (atoi(e) != 0)
                           : FEM_MF_DIST_NOGATHER >= 0 ? FEM_MF_DIST_NOGATHER
                                                       : (int)(mf_nodes(m) >= MF_NOGATHER_MIN_NODES);
    }
    s->fused = s->deferred = s->persist_req = s->persist_fit_only = s->persist = 0;
    s->cols16 = nullptr;
    s->pext = 0;
    return FEM_OK;
}

int fem_pcg_set_entries(fem_pcg* s, int64_t entries) {
    if (entries < 0) {
        set_error("fem_pcg_set_entries: negative entry count %lld", (long long)entries);
        return FEM_EARG;
    }
    s->sell_ent = entries;
    return FEM_OK;
}

int fem_pcg_set_schedule(fem_pcg* s, int sched) {
    if (s->graph) {
        set_error("fem_pcg_set_schedule: drop the captured graph first (fem_pcg_use_graph(s, 0))");
        return FEM_EARG;
    }
    if (sched < 0 || sched > 4) {
        set_error("fem_pcg_set_schedule: unknown schedule %d", sched);
        return FEM_EARG;
    }
    // 4 = auto: the persistent schedule when it applies -- for bs = 3 only while every wave's slices fit on chip (the
    // overflow build streams most of the 10M-tet elastic state and measured 633 vs 436 us per iteration), else the
    // 3-kernel schedule; for bs = 1 schedule 3 (its overflow build beats the deferred fallback)
    if (s->mf) {   // the element-chunk operator runs the 3-kernel schedule only (4 = auto selects it)
        if (sched != 0 && sched != 4) {
            set_error("fem_pcg_set_schedule: the element-chunk operator runs the 3-kernel schedule");
            return FEM_EARG;
        }
        s->fused = s->deferred = s->persist_req = s->persist_fit_only = s->persist = 0;
        return FEM_OK;
    }
    const bool auto3 = sched == 4 && s->bs == 3;
    if (sched == 4) sched = (s->dist || s->mode == FEM_MODE_CG_CONSTRAINED) ? 0 : 3;
    if (sched != 0 && s->dist) {
        set_error("fem_pcg_set_schedule: the distributed path runs the 3-kernel schedule");
        return FEM_EARG;
    }
    if (sched != 0 && s->mode == FEM_MODE_CG_CONSTRAINED) {
        set_error("fem_pcg_set_schedule: the constrained CG runs the 3-kernel schedule (projection after K3)");
        return FEM_EARG;
    }
    s->fused = sched == 1;
    s->deferred = (sched == 2 || sched == 3) && !auto3;   // 3 falls back to the deferred schedule when unsupported
    s->persist_req = sched == 3;
    s->persist_fit_only = auto3 ? 1 : 0;
    s->persist = 0;
    return FEM_OK;
}

int fem_pcg_persist_profile(fem_pcg* s, int k, unsigned long long* host_out, int* grid) {
    if (!s->persist || s->pk_ovf || k <= 0) {
        set_error("fem_pcg_persist_profile: the context does not run the (register-resident) persistent schedule");
        return FEM_EARG;
    }
    const size_t nb = sizeof(unsigned long long) * (size_t)s->pk_grid * (PK_NPROF + PK_WAVES);
    unsigned long long* d = nullptr;
    FEM_HIP(hipMalloc(&d, nb));
    FEM_HIP(hipMemsetAsync(d, 0, nb, s->stream));
    int rc = launch_persist(s, k, d);
    if (!rc) {
        const hipError_t e1 = hipMemcpyAsync(host_out, d, nb, hipMemcpyDeviceToHost, s->stream);
        const hipError_t e2 = hipStreamSynchronize(s->stream);
        if (e1 != hipSuccess || e2 != hipSuccess) {
            set_error("fem_pcg_persist_profile: %s", hipGetErrorString(e1 != hipSuccess ? e1 : e2));
            rc = FEM_EHIP;
        }
    }
    (void)hipFree(d);
    if (grid) *grid = s->pk_grid;
    return rc;
}

int fem_pcg_get_schedule(fem_pcg* s) {
    if (s->persist) return 3;
    if (s->fused) return 1;
    return s->deferred ? 2 : 0;
}

__global__ void k_sell_sl_pattern(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                                  const int16_t* __restrict__ cin, int16_t* __restrict__ pout,
                                  int16_t* __restrict__ ucol, int32_t* __restrict__ uoff, int G, int* __restrict__ win,
                                  int2* __restrict__ span);

int fem_sell_sl_pattern(int64_t nrows, const int64_t* slice_ptr, const int16_t* dcols, int G, int16_t* pcols,
                        int16_t* ucol, int32_t* uoff, int32_t* win, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns <= 0) return FEM_OK;
    hipStream_t st = S(stream);
    int2* span = nullptr;   // per-slice owner spans, reduced into the windows (sl_pattern_slice, k_win_from_spans)
    if (G > 0) FEM_HIP(::fem::stream_scratch((void**)&span, sizeof(int2) * (size_t)ns, st));
    hipLaunchKernelGGL(k_sell_sl_pattern, dim3((unsigned)cdiv(ns, 4)), dim3(256), 0, st, ns, nrows, slice_ptr,
                       dcols, pcols, ucol, uoff, G > 0 ? G : 0, win, span);
    FEM_LAUNCHED();
    if (G > 0) {
        hipLaunchKernelGGL(k_win_from_spans, dim3((unsigned)cdiv((int64_t)G * 64, 256)), dim3(256), 0, st, G, ns,
                           (const int2*)span, win);
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

int fem_sell_sl_unpair(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* dcols, const int32_t* uoff,
                       const int16_t* ucol, const int32_t* rowptr, const double* svals, double* vals,
                       fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns <= 0) return FEM_OK;
    if (bs == 3) {
        hipLaunchKernelGGL(k_sell3_from_a, dim3(stream_grid(ns * 64, 256)), dim3(256), 0, S(stream), ns, slice_ptr,
                           svals, vals);
        FEM_LAUNCHED();
        return FEM_OK;
    }
    hipLaunchKernelGGL(k_sell_sl_unpair, dim3(stream_grid(ns * 64, 256)), dim3(256), 0, S(stream), ns, slice_ptr, dcols,
                       uoff, ucol, rowptr, nrows, svals, vals);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_spmv_sl(int64_t nrows, int bs, const int64_t* slice_ptr, const int16_t* pcols, const double* svals,
                const int32_t* uoff, const int16_t* ucol, const double* x, double* y, fem_stream_t stream) {
    const int64_t ns = cdiv(nrows, 64);
    if (ns <= 0) return FEM_OK;
    // slice_walk needs a multiple of 8 workgroups (one XCD range each)
    if (bs == 3) {   // pcols: the plain 16-bit deltas (layout A pairs values only)
        hipLaunchKernelGGL(k_spmv_a, dim3(grid_multiple_of_xcd(cdiv(ns, 4), 2048)), dim3(256), 0, S(stream), ns, nrows,
                           slice_ptr, pcols, svals, x, y);
        FEM_LAUNCHED();
        return FEM_OK;
    }
    hipLaunchKernelGGL(k_spmv_pair<SPMV_UP>, dim3(grid_multiple_of_xcd(cdiv(ns, 4), 2048)), dim3(256), 0, S(stream), ns, nrows,
                       slice_ptr, pcols, svals, uoff, ucol, x, y);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_set_layout(fem_pcg* s, const double* svals, const int16_t* pcols, const int32_t* uoff,
                       const int16_t* ucol, const int32_t* win, int G) {
    if ((s->bs != 1 && s->bs != 3) || !s->cols16 || s->dist || s->pd || (s->bs == 1 && !pcols)) {
        set_error("fem_pcg_set_layout: single-GPU contexts with 16-bit columns only (fem_pcg_set_cols16 first); "
                  "bs = 1 needs the paired columns");
        return FEM_EARG;
    }
    if (!s->pext) {   // buffers of an earlier refresh go back to the pool
        pool_free(s->pvals, s->stream);
        pool_free(s->pcols16, s->stream);
        pool_free(s->puoff, s->stream);
        pool_free(s->pucol, s->stream);
    }
    s->pext = 1;
    s->pvals = const_cast<double*>(svals);
    s->pcols16 = s->bs == 1 ? const_cast<int16_t*>(pcols) : nullptr;   // bs = 3: layout A reads cols16
    s->puoff = s->bs == 1 ? const_cast<int32_t*>(uoff) : nullptr;
    s->pucol = s->bs == 1 ? const_cast<int16_t*>(ucol) : nullptr;
    s->pwin_ext = win;
    s->pwin_G = win ? G : 0;
    s->pk_win_ok = 0;
    return FEM_OK;
}

int fem_pcg_uniform_slices(fem_pcg* s, int64_t s_begin, int64_t s_end, int64_t* uniform, int64_t* nslices,
                           int64_t* index_bytes) {
    if (s_end < 0 || s_end > s->nslices) s_end = s->nslices;
    if (s_begin < 0) s_begin = 0;
    if (s_begin > s_end) s_begin = s_end;
    *uniform = 0;
    *nslices = s_end - s_begin;
    *index_bytes = 0;
    if (s->nslices == 0) return FEM_OK;
    std::vector<int64_t> sp((size_t)s->nslices + 1);
    std::vector<int32_t> h((size_t)s->nslices, -1);
    FEM_HIP(hipMemcpyAsync(sp.data(), s->slice_ptr, sizeof(int64_t) * sp.size(), hipMemcpyDeviceToHost, s->stream));
    const bool uni = s->paired && s->puoff && (s->tune & FEM_TUNE_PK_UNI) && s->bs == 1;
    if (uni) FEM_HIP(hipMemcpyAsync(h.data(), s->puoff, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    const int64_t idx = s->cols16 ? 2 : 4;
    int64_t c = 0, ib = 0;
    for (int64_t i = s_begin; i < s_end; ++i) {
        const int64_t wdt = (sp[i + 1] - sp[i]) / 64;
        if (h[i] >= 0) {
            ++c;
            ib += 2 * ((wdt + 1) & ~int64_t(1));
        } else {
            ib += idx * 64 * wdt;
        }
    }
    *uniform = c;
    *index_bytes = ib;
    return FEM_OK;
}

static size_t pk_sync_words(int G) { return (size_t)(18 + G) * PK_LINE; }

// distributed builds: 4 register slots per wave when the rank's slices fit (every rank of a 10M-tet system at
// N >= 2: fewer loop-carried registers, no spills), else 7
constexpr int PK_MAXS_DIST = 4;
static const void* persist_fn_dist(bool prof, int maxs) {
    if (!prof && maxs <= 1) return (const void*)k_pcg_persist<1, false, true, false, true>;   // 8 pairs in flight
    if (!prof && maxs == 2) return (const void*)k_pcg_persist<2, false, true, false, true>;   // 4 pairs in flight
    if (maxs <= PK_MAXS_DIST)
        return prof ? (const void*)k_pcg_persist<PK_MAXS_DIST, true, true, false, true>
                    : (const void*)k_pcg_persist<PK_MAXS_DIST, false, true, false, true>;
    return prof ? (const void*)k_pcg_persist<PK_MAXS, true, true, false, true>
                : (const void*)k_pcg_persist<PK_MAXS, false, true, false, true>;
}
static int dist_maxs(const fem_pcg* s) {
    const int64_t nloc = s->pd_split[s->pd_rank + 1] - s->pd_split[s->pd_rank];
    const int64_t maxL = (nloc + s->pk_grid - 1) / s->pk_grid;
    return (int)((maxL + PK_WAVES - 1) / PK_WAVES);
}

// small: slices per wave of the packed assignment (1, 2, 3-4 select the one-, two-, four-slot build with 8, 4, 4 lane
// pairs in flight; 0 the 7-slot build with 2)
static const void* persist_fn(bool prof, bool gsc1, bool ovf = false, int small = 0) {
    if (small >= 1 && small <= 4 && !prof && !ovf && gsc1)
        return small == 1 ? (const void*)k_pcg_persist<1, false, true>
             : small == 2 ? (const void*)k_pcg_persist<2, false, true>
                          : (const void*)k_pcg_persist<4, false, true>;
    if (ovf) return gsc1 ? (const void*)k_pcg_persist<PK_MAXS, false, true, true>
                         : (const void*)k_pcg_persist<PK_MAXS, false, false, true>;
    if (prof) return gsc1 ? (const void*)k_pcg_persist<PK_MAXS, true, true> : (const void*)k_pcg_persist<PK_MAXS, true, false>;
    return gsc1 ? (const void*)k_pcg_persist<PK_MAXS, false, true> : (const void*)k_pcg_persist<PK_MAXS, false, false>;
}

// bs = 3 (pcg_persist3.hpp): P3_MAXS slices per wave on chip, the overflow build past that (single GPU), the DIST
// build when the rank's slices fit
static const void* persist3_fn(bool ovf, bool dist) {
    if (dist) return (const void*)k_pcg_persist3<P3_MAXS, false, true>;
    return ovf ? (const void*)k_pcg_persist3<P3_MAXS, true> : (const void*)k_pcg_persist3<P3_MAXS, false>;
}
static size_t persist_lds(const fem_pcg* s) { return s->bs == 3 ? P3_LDS : PK_LDS; }
static int persist_maxs(const fem_pcg* s) { return s->bs == 3 ? P3_MAXS : PK_MAXS; }

// schedule 3 prerequisites: bs = 1 (lane-paired copy) or bs = 3 (plane-paired copy), 16-bit columns, single GPU, no
// projections, capacity (every wave <= MAXS slices, else the overflow build), one resident PK_T-thread workgroup per CU
static int persist_setup_dist(fem_pcg* s);

static int persist_setup(fem_pcg* s) {
    s->persist = 0;
    if (s->pd) return persist_setup_dist(s);
    if (!s->persist_req) return FEM_OK;
    if ((s->bs != 1 && s->bs != 3) || !s->paired || s->dist || s->mode == FEM_MODE_CG_CONSTRAINED || s->nslices == 0)
        return FEM_OK;
    int dev = 0, ncu = 0;
    FEM_HIP(hipGetDevice(&dev));
    FEM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int G = (ncu / NXCD) * NXCD;
    if (G < NXCD) return FEM_OK;
    // past MAXS slices per wave: the overflow build (packed assignment only; overflow rows streamed from HBM)
    const bool ovf = s->nslices > (int64_t)G * PK_WAVES * persist_maxs(s);
    if (ovf && (!(s->tune & FEM_TUNE_PK_PACK) || s->persist_fit_only)) return FEM_OK;
    // residency of every build, queried once per device and block size (host calls of ~tens of us per solve)
    // (the entry is published only after every build's attribute call succeeded, under a lock: a setup that fails
    // midway, or a second thread, must not find "resident" before the LDS attribute of every build is set)
    static std::mutex occ_mu;
    static int occ_cache[2][64] = {};   // 0 unknown, 1 resident, 2 not
    int occ;
    {
        std::lock_guard<std::mutex> lk(occ_mu);
        int& slot = occ_cache[s->bs == 3][dev & 63];
        if (slot == 0) {
            int res = 1;
            for (int v = 0; v < (s->bs == 3 ? 2 : 9) && res == 1; ++v) {
                const void* f = s->bs == 3 ? persist3_fn(v == 1, false)
                              : v >= 6 ? persist_fn(false, true, false, v == 8 ? 4 : v - 5)
                                       : persist_fn((v & 1) && v < 4, v & 2, v >= 4);
                FEM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_lds(s)));
                int nb = 0;
                FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, PK_T, persist_lds(s)));
                if (nb < 1) res = 2;
            }
            slot = res;
        }
        occ = slot;
    }
    if (occ != 1) return FEM_OK;
    if (s->pk_grid != G) {
        pool_free(s->pk_win, s->stream);
        pool_free(s->pk_part, s->stream);
        pool_free(s->pk_sync, s->stream);
        s->pk_win = nullptr;
        s->pk_part = nullptr;
        s->pk_sync = nullptr;
        FEM_HIP(pool_alloc((void**)&s->pk_win, sizeof(int32_t) * 2 * G, s->stream, s->bs == 1));
        FEM_HIP(pool_alloc((void**)&s->pk_part, sizeof(double) * 4 * G, s->stream, s->bs == 1));
        FEM_HIP(pool_alloc((void**)&s->pk_sync, sizeof(unsigned) * pk_sync_words(G), s->stream, s->bs == 1));
        s->pk_grid = G;
        s->pk_win_ok = 0;
    }
    if (!s->pk_win_ok && s->pwin_ext && s->pwin_G == G) {   // formed with the solver-layout pattern
        FEM_HIP(hipMemcpyAsync(s->pk_win, s->pwin_ext, sizeof(int32_t) * 2 * G, hipMemcpyDeviceToDevice, s->stream));
        s->pk_win_ok = 1;
    }
    if (!s->pk_win_ok) {   // [lo | hi] per logical workgroup, from the matrix columns (no host round trip)
        hipLaunchKernelGGL(k_pk_window_init, dim3(cdiv(G, 256)), dim3(256), 0, s->stream, G, G, s->pk_win);
        FEM_LAUNCHED();
        hipLaunchKernelGGL(k_pk_window, dim3(stream_grid(s->nslices * 64, 256)), dim3(256), 0, s->stream, s->nslices,
                           s->nrows, s->slice_ptr, s->cols16, G, s->pk_win, s->pk_win + G);
        FEM_LAUNCHED();
        s->pk_win_ok = 1;
    }
    if (ovf && !s->pk_v) FEM_HIP(pool_alloc((void**)&s->pk_v, sizeof(double) * (size_t)s->n, s->stream, s->bs == 1));
    s->pk_ovf = ovf ? 1 : 0;
    s->persist = 1;
    s->pk_gv = 0;
    if ((s->tune & FEM_TUNE_PK_GV) && (s->tune & FEM_TUNE_PK_SC1) && s->bs == 1 && !ovf && s->mode == FEM_MODE_PCG) {
        const int64_t maxL = (s->nslices + G - 1) / G;
        const int pack = (int)((maxL + PK_WAVES - 1) / PK_WAVES);
        if (pack <= GV_MAXS) {
            static std::mutex gv_mu;
            static int gv_ok[64] = {};   // per device: 0 unknown, 1 resident, 2 not
            std::lock_guard<std::mutex> lk(gv_mu);
            int& slot = gv_ok[dev & 63];
            if (slot == 0) {
                int res = 1;
                for (int v = 0; v < 2 && res == 1; ++v) {
                    const void* f = v ? (const void*)k_pcg_persist_gv<2> : (const void*)k_pcg_persist_gv<1>;
                    FEM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GV_LDS));
                    int nb = 0;
                    FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, PK_T, GV_LDS));
                    if (nb < 1) res = 2;
                }
                slot = res;
            }
            s->pk_gv = slot == 1;
        }
    }
    return FEM_OK;
}

// schedule 3 over a row-partitioned multi-rank system (fem_pcg_set_rows / fem_pcg_set_peers already ran): the
// prerequisites of the single-GPU schedule, this rank's slices within the register capacity (no overflow build),
// one resident workgroup per CU for the chosen grid
static int persist_setup_dist(fem_pcg* s) {
    if ((s->bs != 1 && s->bs != 3) || !s->paired || s->dist || s->mode == FEM_MODE_CG_CONSTRAINED) {
        set_error("distributed persistent PCG: needs bs = 1 or 3, 16-bit columns with the paired copy, no element "
                  "partition, no constraints");
        return FEM_EARG;
    }
    if (!s->pd_peers_ok) {
        set_error("distributed persistent PCG: fem_pcg_set_peers first");
        return FEM_EARG;
    }
    const int G = s->pk_grid;
    const int64_t nloc = s->pd_split[s->pd_rank + 1] - s->pd_split[s->pd_rank];
    if ((nloc + G - 1) / G > (int64_t)PK_WAVES * persist_maxs(s)) {
        set_error("distributed persistent PCG: %lld slices on this rank exceed the register capacity of %d workgroups",
                  (long long)nloc, G);
        return FEM_EARG;
    }
    for (int v = 0; v < (s->bs == 3 ? 1 : 2); ++v) {
        const void* f = s->bs == 3 ? persist3_fn(false, true) : persist_fn_dist(v == 1, dist_maxs(s));
        FEM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_lds(s)));
        int nb = 0;
        FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, PK_T, persist_lds(s)));
        if (nb < 1) {
            set_error("distributed persistent PCG: kernel does not fit one workgroup per CU");
            return FEM_EARG;
        }
    }
    s->pk_ovf = 0;
    s->persist = 1;
    s->pk_gv = 0;
    if (s->pd_off_m1 > 0 && s->mode == FEM_MODE_PCG && dist_maxs(s) <= GV_MAXS) {   // pipelined DIST build
        int res = 1;
        for (int v = 0; v < 2 && res == 1; ++v) {
            const void* f = v ? (const void*)k_pcg_persist_gv<2, true> : (const void*)k_pcg_persist_gv<1, true>;
            FEM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GV_LDS));
            int nb = 0;
            FEM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, PK_T, GV_LDS));
            if (nb < 1) res = 2;
        }
        s->pk_gv = res == 1;
    }
    return FEM_OK;
}

// one persistent launch of k iterations (schedule 3); prof (device, [G][PK_NPROF]) selects the instrumented build
static int persist_reset_sync(fem_pcg* s) {
    FEM_HIP(hipMemsetAsync(s->pk_sync, 0, sizeof(unsigned) * pk_sync_words(s->pk_grid), s->stream));
    FEM_HIP(hipMemsetAsync(&s->st->pk_epoch, 0, sizeof(unsigned), s->stream));
    s->pk_epochs = 0;
    return FEM_OK;
}

static int launch_persist(fem_pcg* s, int k, unsigned long long* prof) {
    const int G = s->pk_grid;
    // the sync words count epochs across launches (no memset per launch); zero them long before the group counters
    // (epoch * G / 8) could wrap 32 bits
    if (s->pk_epochs + k + 1 > (int64_t(1) << 24)) {
        if (s->pd) {   // the other ranks write into this rank's words: only fem_pcg_start (+ a host barrier) resets
            set_error("distributed persistent PCG: 2^24 iterations since fem_pcg_start; restart the solve");
            return FEM_EARG;
        }
        const int rc = persist_reset_sync(s);
        if (rc) return rc;
    }
    s->pk_epochs += k + 1;
    PkArgs a;
    a.nslices = s->nslices;
    a.nrows = s->nrows;
    a.slice_ptr = s->slice_ptr;
    a.cols = s->pcols16;
    a.vals = s->pvals;
    const bool uni = (s->tune & FEM_TUNE_PK_UNI) && s->puoff;
    a.uoff = uni ? s->puoff : nullptr;
    a.ucol = uni ? s->pucol : nullptr;
    a.x = s->x;
    a.r = s->r;
    a.p = s->p0;
    a.s = s->p1;
    a.u = s->q;
    a.w = s->w;
    a.win = s->pk_win;
    a.part = s->pk_part;
    a.sync = s->pk_sync;
    a.st = s->st;
    a.hist = s->hist;
    a.hist_len = s->hist_len;
    a.kmax = k;
    a.rev = (s->tune & FEM_TUNE_REVERSE) ? 1 : 0;
    a.prof = prof;
    a.v = s->pk_ovf ? s->pk_v : nullptr;
    {   // packed slice assignment: m = ceil(max slices of a workgroup / waves) per wave
        const int64_t maxL = (s->nslices + G - 1) / G;
        a.pack = (s->tune & FEM_TUNE_PK_PACK) ? (int)((maxL + PK_WAVES - 1) / PK_WAVES) : 0;
    }
    a.sbase = 0;
    a.rank = 0;
    a.nranks = 1;
    for (int q = 0; q < PK_MAX_RANKS; ++q) a.peer[q] = nullptr;
    a.off_flag = a.off_red = a.off_rflag = 0;
    a.pub = nullptr;
    a.b = s->b;
    a.init = 0;
    if (s->pd) {   // distributed: this rank's slices, comm blocks, the init on the first launch after start
        const int64_t S0 = s->pd_split[s->pd_rank], S1 = s->pd_split[s->pd_rank + 1];
        a.nslices = S1 - S0;
        a.sbase = S0;
        a.rank = s->pd_rank;
        a.nranks = s->pd_nranks;
        for (int q = 0; q < s->pd_nranks; ++q) a.peer[q] = s->pd_peer[q];
        a.off_flag = s->pd_off_flag;
        a.off_red = s->pd_off_red;
        a.off_rflag = s->pd_off_rflag;
        a.pub = s->pd_pub;
        a.u = reinterpret_cast<double*>(s->pd_block);
        a.init = s->pd_init_pending;
        s->pd_init_pending = 0;
        const int64_t maxL = (a.nslices + G - 1) / G;
        a.pack = (int)((maxL + PK_WAVES - 1) / PK_WAVES);
    }
    if (s->pk_gv && s->bs == 1) {   // pipelined (pcg_persist_gv.hpp): packed slices, <= GV_MAXS per wave
        if (prof) {
            set_error("persistent PCG: no instrumented (PROF) build of the pipelined iteration");
            return FEM_EARG;
        }
        if (!s->pd) {
            const int64_t maxL = (s->nslices + G - 1) / G;
            a.pack = (int)((maxL + PK_WAVES - 1) / PK_WAVES);
        }   // (distributed: this rank's packing, set above)
        const int64_t n = s->n;
        GvArgs g;
        g.u = s->gv_buf;
        g.w = s->gv_buf + n;
        g.q = s->gv_buf + 2 * n;
        g.z = s->gv_buf + 3 * n;
        if (s->pd) {   // the gathered m in the comm blocks: m[0] the u region, m[1] after it
            g.m[0] = reinterpret_cast<double*>(s->pd_block);
            g.m[1] = reinterpret_cast<double*>(s->pd_block + s->pd_off_m1);
            g.moff[0] = 0;
            g.moff[1] = s->pd_off_m1;
            g.init = 0;   // (a.init)
        } else {
            g.m[0] = s->gv_buf + 4 * n;
            g.m[1] = s->gv_buf + 5 * n;
            g.moff[0] = g.moff[1] = 0;
            g.init = s->gv_init_pending;
            s->gv_init_pending = 0;
        }
        s->pk_epochs += 2;   // the init barriers
        void* gargs[] = {&a, &g};
        const void* gfn = s->pd ? (a.pack <= 1 ? (const void*)k_pcg_persist_gv<1, true> : (const void*)k_pcg_persist_gv<2, true>)
                                : (a.pack <= 1 ? (const void*)k_pcg_persist_gv<1> : (const void*)k_pcg_persist_gv<2>);
        if (s->pk_coop || (s->tune & FEM_TUNE_PK_COOP))
            FEM_HIP(hipLaunchCooperativeKernel(gfn, dim3(G), dim3(PK_T), gargs, GV_LDS, s->stream));
        else
            FEM_HIP(hipLaunchKernel(gfn, dim3(G), dim3(PK_T), gargs, GV_LDS, s->stream));
        FEM_LAUNCHED();
        s->launched += k;
        return FEM_OK;
    }
    void* args[] = {&a};
    if (s->pd && !prof && s->pd_prof) a.prof = prof = s->pd_prof;
    if (s->bs == 3) {   // plane-paired values, per-lane 16-bit node deltas; no instrumented build
        if (prof && !s->pd) {
            set_error("persistent PCG: no instrumented (PROF) build for bs = 3");
            return FEM_EARG;
        }
        a.cols = s->cols16;
        a.uoff = nullptr;
        a.ucol = nullptr;
        a.prof = nullptr;
        if (!s->pd) {   // k_pcg_persist3 always takes the packed assignment
            const int64_t maxL = (s->nslices + G - 1) / G;
            a.pack = (int)((maxL + PK_WAVES - 1) / PK_WAVES);
        }
    }
    const void* fn = s->bs == 3 ? persist3_fn(s->pk_ovf != 0, s->pd != 0)
                   : s->pd ? persist_fn_dist(prof != nullptr, a.pack)
                           : persist_fn(prof != nullptr && !s->pk_ovf, (s->tune & FEM_TUNE_PK_SC1) != 0, s->pk_ovf != 0,
                                        (a.pack <= 4 && !(s->tune & FEM_TUNE_PK_WIDE)) ? a.pack : 0);
    // the grid spins on inter-workgroup flags, so all G workgroups must be resident together: one per CU is
    // what the occupancy query promised, and a cooperative launch makes the runtime guarantee it (or fail) even
    // when other streams / processes hold CUs. A plain launch (the bench's fixed-iteration runs) relies on the
    // occupancy check; should residency still fail, every spin is bounded and the launch ends with
    // FEM_PCG_SYNC_TIMEOUT (fem_pcg_solve then re-solves on the deferred schedule).
    if (s->pk_coop || (s->tune & FEM_TUNE_PK_COOP))
        FEM_HIP(hipLaunchCooperativeKernel(fn, dim3(G), dim3(PK_T), args, persist_lds(s), s->stream));
    else
        FEM_HIP(hipLaunchKernel(fn, dim3(G), dim3(PK_T), args, persist_lds(s), s->stream));
    FEM_LAUNCHED();
    s->launched += k;
    return FEM_OK;
}

int fem_pcg_pipelined(fem_pcg* s, int* on) {
    *on = (s && s->persist && s->pk_gv) ? 1 : 0;
    return FEM_OK;
}

int fem_pcg_persist_build(fem_pcg* s, int* slots, int* overflow, int* pack) {
    *slots = 0;
    *overflow = 0;
    *pack = 0;
    if (!s->persist || s->pk_grid <= 0) return FEM_OK;
    const int G = s->pk_grid;
    int64_t ns = s->nslices;
    if (s->pd) ns = s->pd_split[s->pd_rank + 1] - s->pd_split[s->pd_rank];
    const int64_t maxL = (ns + G - 1) / G;
    const int pk = (int)((maxL + PK_WAVES - 1) / PK_WAVES);
    *overflow = s->pk_ovf;
    *pack = (s->bs == 3 || s->pd || (s->tune & FEM_TUNE_PK_PACK)) ? pk : 0;
    // the same selection as launch_persist (persist_fn / persist_fn_dist / persist3_fn, non-instrumented)
    if (s->bs == 3) {
        *slots = P3_MAXS;
    } else if (s->pd) {
        *slots = pk <= 1 ? 1 : pk == 2 ? 2 : pk <= PK_MAXS_DIST ? PK_MAXS_DIST : PK_MAXS;
    } else {
        const int small = (*pack <= 4 && !(s->tune & FEM_TUNE_PK_WIDE)) ? *pack : 0;
        *slots = (small >= 1 && small <= 4 && !s->pk_ovf && (s->tune & FEM_TUNE_PK_SC1))
                     ? (small == 1 ? 1 : small == 2 ? 2 : 4) : PK_MAXS;
    }
    return FEM_OK;
}

// The solver layout of a bs = 1 pattern (FEM_TUNE_PK_UNI + lane pairing decided from the pattern alone, once per
// pattern): the qualification of k_sell_uniform on the plain 16-bit deltas (padding entries are delta 0 by
// construction and get value 0 from the assembly), uoff / ucol of the uniform slices, and the lane-paired per-lane
// deltas pout (a uniform slice's list deltas at every lane, like k_sell_uniform's copy). The value kernels then write
// the paired layout directly (fem_assemble_tet4_sl), so a solve needs no conversion pass.
// With G > 0 the same pass also forms the persistent schedule's gather windows for a G-workgroup grid (k_pk_window's
// work: the union of the slice's deltas, one atomic pair per slice), so the solve's start needs neither pass.
__global__ void __launch_bounds__(256) k_sell_sl_pattern(int64_t nslices, int64_t nrows,
                                                         const int64_t* __restrict__ slice_ptr,
                                                         const int16_t* __restrict__ cin, int16_t* __restrict__ pout,
                                                         int16_t* __restrict__ ucol, int32_t* __restrict__ uoff, int G,
                                                         int* __restrict__ win, int2* __restrict__ span) {
    __shared__ int cand_all[4][SU_MAXW];
    const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;   // one wave per slice
    if (s >= nslices) return;   // wave-uniform
    const int l = threadIdx.x & 63;
    const int64_t p0 = slice_ptr[s];
    sl_pattern_slice(s, l, nslices, nrows, slice_ptr, [&](int k) { return (int)cin[p0 + 64 * k + l]; }, pout, ucol,
                     uoff, G, win, cand_all[(threadIdx.x >> 6) & 3], span);
}

// host view of the state: the deferred schedule keeps it in the bank of the current launch parity
static PcgState state_view(const fem_pcg* s) {
    PcgState h = *s->st_host;
    if (s->deferred && !s->dist && !s->persist) {
        const PcgState::Bank& b = h.bank[s->launched & 1];
        h.iter = b.iter;
        h.status = b.status;
        h.halt = b.halt;
        h.stop_iter = b.stop_iter;
        h.rz = b.rz;
        h.rz_new = b.rz_new;
        h.pq = b.pq;
        h.alpha = b.alpha;
        h.beta = b.beta;
    }
    return h;
}

// (re)build the 16-byte-value matrix copy used by the SpMV when FEM_TUNE_PAIR is set: bs = 1 lane-paired values and
// columns (sell_pair.hpp), bs = 3 plane-paired values (sell_pair3.hpp layout A; columns stay cols16)
static int refresh_pairing(fem_pcg* s) {
    const bool want = (s->bs == 1 || s->bs == 3) && s->cols16 && (s->tune & FEM_TUNE_PAIR) && !s->fused;
    s->paired = 0;
    if (s->pext) {   // the matrix was assembled in the solver layout: nothing to convert
        if (!want) {
            set_error("PCG: a solver-layout matrix needs the paired schedules (FEM_TUNE_PAIR, 16-bit columns, not fused)");
            return FEM_EARG;
        }
        s->paired = 1;
        return FEM_OK;
    }
    if (!want || s->nslices == 0) return FEM_OK;
    int64_t ent = s->sell_ent;
    if (ent < 0) {   // not given by the caller: one device-to-host read (a host sync)
        FEM_HIP(hipMemcpyAsync(&ent, s->slice_ptr + s->nslices, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream));
        FEM_HIP(hipStreamSynchronize(s->stream));
    }
    if (s->bs == 3) {
        if (!s->pvals) FEM_HIP(pool_alloc((void**)&s->pvals, sizeof(double) * 9 * (size_t)ent, s->stream, s->bs == 1));
        s->pcols16 = nullptr;
        hipLaunchKernelGGL(k_sell3_to_a, dim3(stream_grid(s->nslices * 64, 256)), dim3(256), 0, s->stream, s->nslices,
                           s->slice_ptr, s->vals, s->pvals);
        FEM_LAUNCHED();
        s->paired = 1;
        return FEM_OK;
    }
    if (!s->pvals) {
        FEM_HIP(pool_alloc((void**)&s->pvals, sizeof(double) * (size_t)ent, s->stream, s->bs == 1));
        FEM_HIP(pool_alloc((void**)&s->pcols16, sizeof(int16_t) * (size_t)ent, s->stream, s->bs == 1));
    }
    s->paired = 1;
    // slice-uniform deltas (sell_pair.hpp): read by the persistent schedule; the paired copy of the uniform slices
    // stays valid for every other reader. One pass writes both (the other slices get k_sell_pair's copy)
    if ((s->tune & FEM_TUNE_PK_UNI) && 2 * (ent / 64) + 2 < (int64_t)INT32_MAX) {
        if (!s->puoff) {
            FEM_HIP(pool_alloc((void**)&s->puoff, sizeof(int32_t) * (size_t)s->nslices, s->stream, true));
            FEM_HIP(pool_alloc((void**)&s->pucol, sizeof(int16_t) * (size_t)(2 * (ent / 64) + 2), s->stream, true));
        }
        hipLaunchKernelGGL(k_sell_uniform, dim3((unsigned)cdiv(s->nslices, 4)), dim3(256), 0, s->stream, s->nslices,
                           s->nrows, s->slice_ptr, s->vals, s->cols16, s->pvals, s->pcols16, s->pucol, s->puoff, 1);
        FEM_LAUNCHED();
        return FEM_OK;
    }
    hipLaunchKernelGGL(k_sell_pair, dim3(stream_grid(s->nslices * 64, 256)), dim3(256), 0, s->stream, s->nslices,
                       s->slice_ptr, s->vals, s->cols16, s->pvals, s->pcols16);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_start(fem_pcg* s) {
    if (s->mf && s->dist && !s->cg1) {   // fem_pcg_set_dist resets the variant to 0: refuse at setup, not at phase 0
        set_error("fem_pcg_start: a distributed element-chunk context needs the single-reduction variant "
                  "(fem_pcg_set_dist_variant(s, 1))");
        return FEM_EARG;
    }
    {
        int prc = refresh_pairing(s);
        if (!prc) prc = persist_setup(s);
        if (!prc) prc = c1f_setup(s);
        if (!prc) prc = u2_setup(s);
        if (prc) return prc;
    }
    PcgState h{};
    h.tol = s->tol;
    h.eps = s->eps;
    h.mode = s->mode;
    h.max_iter = s->max_iter;
    h.x_done = 1;
    h.dist = s->dist;
    *s->st_host = h;
    FEM_HIP(hipMemcpyAsync(s->st, s->st_host, sizeof(PcgState), hipMemcpyHostToDevice, s->stream));
    int rc;
    if (s->dist) {
        if (!s->comm) return FEM_OK;   // phase-driven by the caller from phase 10 on
        if (s->cg1) {
            if ((rc = dist_phase(s, 10)) || (rc = dist_exchange(s, 10)) || (rc = dist_phase(s, 20)) ||
                (rc = dist_exchange(s, 20)))
                return rc;
            return FEM_OK;
        }
        if ((rc = dist_phase(s, 10)) || (rc = dist_exchange(s, 10)) || (rc = dist_phase(s, 11)) ||
            (rc = dist_exchange(s, 11)) || (rc = dist_phase(s, 12)))
            return rc;
        return FEM_OK;
    }
    if (s->mode == FEM_MODE_CG_STABLE) {
        hipLaunchKernelGGL(k_zero_fixed, dim3(stream_grid(s->n, 256)), dim3(256), 0, s->stream, s->n, s->x, s->w);
        FEM_LAUNCHED();
    }
    if (s->pd) {   // distributed persistent: the first launch forms r0, u0 and r0.u0 itself (k_pcg_persist DIST init)
        if (!s->persist) {
            set_error("distributed persistent PCG: setup failed");
            return FEM_EARG;
        }
        FEM_HIP(hipMemsetAsync(s->pk_sync, 0, sizeof(unsigned) * pk_sync_words(s->pk_grid), s->stream));
        // the whole comm block, u included: no row of an earlier solve (or a non-finite one) survives into this one
        FEM_HIP(hipMemsetAsync(s->pd_block, 0, (size_t)s->pd_block_bytes, s->stream));
        FEM_HIP(hipMemsetAsync(&s->st->pk_epoch, 0, sizeof(unsigned), s->stream));
        s->pk_epochs = 0;
        s->pd_init_pending = 1;
        s->launched = 0;
        if (s->pk_gv) {   // pipelined: its vectors u, w, q, z (global length); m lives in the comm block
            const int64_t need = 6 * s->n;
            if (need > s->gv_cap) {
                pool_free(s->gv_buf, s->stream);
                s->gv_buf = nullptr;
                s->gv_cap = 0;
                FEM_HIP(pool_alloc((void**)&s->gv_buf, sizeof(double) * (size_t)need, s->stream, true));
                s->gv_cap = need;
            }
            FEM_HIP(hipMemsetAsync(s->gv_buf, 0, sizeof(double) * (size_t)need, s->stream));
        }
        return FEM_OK;   // every rank must finish its start before any rank launches (a host barrier)
    }
    if (s->mf) {   // element-chunk operator: r0 = b - A x0 from the element formula
        if ((rc = mf_apply(s->mf, s->x, s->q, s->mf_sl, s->stream))) return rc;
    } else if (s->pext) {   // solver layout: r0 = b - A x0 from the paired values
        if (s->bs == 1)
            hipLaunchKernelGGL(k_spmv_pair<SPMV_UP>, dim3(s->grid_spmv), dim3(256), 0, s->stream, s->nslices, s->nrows,
                               s->slice_ptr, s->pcols16, s->pvals, s->puoff, s->pucol, s->x, s->q);
        else
            hipLaunchKernelGGL(k_spmv_a, dim3(s->grid_spmv), dim3(256), 0, s->stream, s->nslices, s->nrows,
                               s->slice_ptr, s->cols16, s->pvals, s->x, s->q);
        FEM_LAUNCHED();
    } else if ((rc = (s->cols16 ? fem_spmv16(s->nrows, s->bs, s->slice_ptr, s->cols16, s->vals, s->x, s->q, s->stream)
                                 : fem_spmv(s->nrows, s->bs, s->slice_ptr, s->cols, s->vals, s->x, s->q, s->stream))))
        return rc;
    if (s->persist) {   // single-reduction start: r0 = b - A x0, u0 = w r0 (in q), p = s = 0, g0 -> red[1]
        const int zrc = persist_reset_sync(s);   // after the state upload: zeroes st->pk_epoch too
        if (zrc) return zrc;
        if (s->pk_gv) {   // pipelined: its vectors (q = z = 0; u, w, m formed by the first launch)
            const int64_t need = 6 * s->n;
            if (need > s->gv_cap) {
                pool_free(s->gv_buf, s->stream);
                s->gv_buf = nullptr;
                s->gv_cap = 0;
                FEM_HIP(pool_alloc((void**)&s->gv_buf, sizeof(double) * (size_t)need, s->stream, true));
                s->gv_cap = need;
            }
            FEM_HIP(hipMemsetAsync(s->gv_buf, 0, sizeof(double) * (size_t)need, s->stream));
            s->gv_init_pending = 1;
        }
        hipLaunchKernelGGL(k_cg1_init, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->bs, s->b, s->r,
                           s->q, s->w, s->p0, s->p1, s->q, (const uint8_t*)nullptr, s->st, s->red);
        FEM_LAUNCHED();
        s->launched = 0;
        return FEM_OK;
    }
    hipLaunchKernelGGL(k_pcg_init, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->b, s->r, s->q, s->w, s->p0,
                       s->p1, s->fused, s->st, s->red, (const uint8_t*)nullptr, s->bs);
    FEM_LAUNCHED();
    if (s->has_con) {   // the reference enforces once after r0 = F - K u0 (`solver/solver.py:548-553`)
        const int rc = launch_constraints(s->stream, s->x, nullptr, s->con, s->st, 1);
        if (rc != FEM_OK) return rc;
    }
    s->launched = 0;
    if (s->deferred) {
        hipLaunchKernelGGL(k_bank_init, dim3(1), dim3(1), 0, s->stream, s->st);
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

int fem_pcg_dist_phase(fem_pcg* s, int phase) {
    if (!s->dist) {
        set_error("fem_pcg_dist_phase: context is not in distributed mode");
        return FEM_EARG;
    }
    return dist_phase(s, phase);
}

int fem_pcg_dist_buffer(fem_pcg* s, int phase, double** ptr, int64_t* n) {
    dist_buffer(s, phase, ptr, n);
    return FEM_OK;
}

// ---------------------------------------------------------------- RCCL bootstrap + distributed setup
int fem_comm_unique_id(char* out128) {
    ncclUniqueId id;
    FEM_NCCL(ncclGetUniqueId(&id));
    memcpy(out128, id.internal, sizeof(id.internal));
    return FEM_OK;
}

int fem_comm_init(int nranks, int rank, const char* id128, void** comm) {
    ncclUniqueId id;
    memcpy(id.internal, id128, sizeof(id.internal));
    ncclComm_t c;
    FEM_NCCL(ncclCommInitRank(&c, nranks, id, rank));
    *comm = c;
    return FEM_OK;
}

int fem_comm_destroy(void* comm) {
    if (comm) FEM_NCCL(ncclCommDestroy((ncclComm_t)comm));
    return FEM_OK;
}

int fem_allreduce_sum(void* comm, double* buf, int64_t n, fem_stream_t stream) {
    FEM_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclFloat64, ncclSum, (ncclComm_t)comm, S(stream)));
    return FEM_OK;
}

int fem_halo_pack(const double* v, int bs, const int32_t* imap, int64_t nI, double* buf, fem_stream_t stream) {
    if (nI <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_halo_pack, dim3(stream_grid(nI * bs, 256)), dim3(256), 0, S(stream), v, bs, imap, nI, buf,
                       (const PcgState*)nullptr, 0);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_halo_unpack(double* v, int bs, const int32_t* ipos, int64_t nrows, const double* buf, fem_stream_t stream) {
    hipLaunchKernelGGL(k_halo_unpack<false>, dim3(stream_grid(nrows * bs, PCG_BLOCK)), dim3(PCG_BLOCK), 0, S(stream),
                       nrows, bs, ipos, buf, v, (int64_t)0, (PcgState*)nullptr);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_halo_sum(void* comm, double* v, int bs, const int32_t* imap, int64_t nI, const int32_t* ipos, int64_t nrows,
                 double* buf, fem_stream_t stream) {
    int rc;
    if ((rc = fem_halo_pack(v, bs, imap, nI, buf, stream))) return rc;
    if (nI > 0) FEM_NCCL(ncclAllReduce(buf, buf, (size_t)(nI * bs), ncclFloat64, ncclSum, (ncclComm_t)comm, S(stream)));
    return fem_halo_unpack(v, bs, ipos, nrows, buf, stream);
}

int fem_pcg_set_dist(fem_pcg* s, int enable, void* comm, int64_t nI, const int32_t* imap, const int32_t* ipos,
                     const uint8_t* own) {
    if (enable && (s->graph || s->fused)) {
        set_error("fem_pcg_set_dist: the distributed path runs the 3-kernel schedule without a captured graph");
        return FEM_EARG;
    }
    if (s->hbuf) (void)hipFree(s->hbuf);
    s->hbuf = nullptr;
    for (double** b : {&s->cg1_s, &s->cg1_u, &s->cg1_send, &s->cg1_recv}) {   // sized by nI: set the variant after
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    s->cg1 = 0;
    s->p2p = 0;
    s->dist = enable ? 1 : 0;
    s->comm = enable ? (ncclComm_t)comm : nullptr;
    s->nI = nI;
    s->imap = imap;
    s->ipos = ipos;
    s->own = own;
    if (enable) FEM_HIP(hipMalloc(&s->hbuf, sizeof(double) * (size_t)(nI * s->bs + 1)));
    return FEM_OK;
}

int fem_pcg_set_dist_variant(fem_pcg* s, int variant) {
    if (!s->dist || s->graph || (variant != 0 && variant != 1)) {
        set_error("fem_pcg_set_dist_variant: needs a distributed context without a captured graph, variant 0 or 1");
        return FEM_EARG;
    }
    if (s->mf && variant == 0) {
        set_error("fem_pcg_set_dist_variant: the element-chunk operator runs the single-reduction variant (1) only");
        return FEM_EARG;
    }
    for (double** b : {&s->cg1_s, &s->cg1_u, &s->cg1_send, &s->cg1_recv}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    s->cg1 = variant;
    s->p2p = 0;   // maps refer to the single-reduction buffers: set them again after the variant
    if (variant == 1) {
        FEM_HIP(hipMalloc(&s->cg1_s, sizeof(double) * (size_t)s->n));
        FEM_HIP(hipMalloc(&s->cg1_u, sizeof(double) * (size_t)s->n));
        FEM_HIP(hipMalloc(&s->cg1_send, sizeof(double) * (size_t)cg1_len(s)));
        FEM_HIP(hipMalloc(&s->cg1_recv, sizeof(double) * (size_t)cg1_len(s)));
        FEM_HIP(hipMemset(s->cg1_send, 0, sizeof(double) * (size_t)cg1_len(s)));   // non-local interface nodes
        FEM_HIP(hipMemset(s->cg1_recv, 0, sizeof(double) * (size_t)cg1_len(s)));
    }
    return FEM_OK;
}

int fem_pcg_set_p2p(fem_pcg* s, int nranks, int npeer, const int* peer_rank, const int64_t* peer_cnt,
                    const int32_t* csrc, const int32_t* ssrc) {
    if (!s->dist || !s->cg1 || s->graph || nranks < 1 || npeer < 0 || npeer >= nranks) {
        set_error("fem_pcg_set_p2p: needs a single-reduction distributed context without a captured graph");
        return FEM_EARG;
    }
    if (s->psend) (void)hipFree(s->psend);
    if (s->precv) (void)hipFree(s->precv);
    s->psend = s->precv = nullptr;
    s->peer_rank.assign(peer_rank, peer_rank + npeer);
    s->peer_cnt.assign(peer_cnt, peer_cnt + npeer);
    s->peer_off.resize(npeer);
    int64_t tot = 0;
    for (int i = 0; i < npeer; ++i) {
        if (peer_cnt[i] < 2) {
            set_error("fem_pcg_set_p2p: every message carries the [g, d] pair (count >= 2)");
            return FEM_EARG;
        }
        s->peer_off[i] = tot;
        tot += peer_cnt[i];
    }
    s->p2p_total = tot;
    s->p2p_nranks = nranks;
    s->p2p_csrc = csrc;
    s->p2p_ssrc = ssrc;
    if (tot > 0) {
        FEM_HIP(hipMalloc(&s->psend, sizeof(double) * (size_t)tot));
        FEM_HIP(hipMalloc(&s->precv, sizeof(double) * (size_t)tot));
    }
    s->p2p = 1;
    return FEM_OK;
}

int fem_p2p_deliver(fem_pcg* const* ctx, int P, fem_stream_t stream) {
    for (int a = 0; a < P; ++a) {
        const fem_pcg* A = ctx[a];
        if (!A->p2p || A->p2p_nranks != P) {
            set_error("fem_p2p_deliver: context %d has no neighbour exchange over %d ranks", a, P);
            return FEM_EARG;
        }
        for (size_t i = 0; i < A->peer_rank.size(); ++i) {
            const int b = A->peer_rank[i];
            const fem_pcg* B = ctx[b];
            size_t j = 0;
            while (j < B->peer_rank.size() && B->peer_rank[j] != a) ++j;
            if (j == B->peer_rank.size() || B->peer_cnt[j] != A->peer_cnt[i]) {
                set_error("fem_p2p_deliver: ranks %d and %d disagree on their message", a, b);
                return FEM_EARG;
            }
            FEM_HIP(hipMemcpyAsync(B->precv + B->peer_off[j], A->psend + A->peer_off[i],
                                   sizeof(double) * (size_t)A->peer_cnt[i], hipMemcpyDeviceToDevice, S(stream)));
        }
    }
    return FEM_OK;
}

int fem_pcg_p2p_buffers(fem_pcg* s, double** psend, double** precv, int64_t* total) {
    *psend = s->psend;
    *precv = s->precv;
    *total = s->p2p_total;
    return FEM_OK;
}

// single-process validation of the distributed iteration: sum P ranks' exchange buffers (rank order) and
// write the sum back to every one of them (what ncclAllReduce does across processes)
__global__ void k_group_sum(double* const* bufs, int P, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int r = 0; r < P; ++r) s += bufs[r][i];
        for (int r = 0; r < P; ++r) bufs[r][i] = s;
    }
}

int fem_group_allreduce(double* const* dev_ptr_array, int P, int64_t n, fem_stream_t stream) {
    if (n <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_group_sum, dim3(stream_grid(n, 256)), dim3(256), 0, S(stream), dev_ptr_array, P, n);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_iterate(fem_pcg* s, int k) {
    if (k <= 0) return FEM_OK;
    // the deferred schedule's graph was captured from bank parity 0 over an even number of iterations
    const bool parity_ok = !s->deferred || ((s->launched & 1) == 0 && (s->graph_k & 1) == 0);
    if (s->graph && s->graph_k > 0 && k % s->graph_k == 0 && parity_ok && !s->persist) {
        for (int i = 0; i < k / s->graph_k; ++i) FEM_HIP(hipGraphLaunch(s->graph, s->stream));
        s->launched += k;
        return FEM_OK;
    }
    return launch_iterations(s, k);
}

int fem_pcg_finish(fem_pcg* s) {
    if (!s->fused) return FEM_OK;
    hipLaunchKernelGGL(k_pcg_finish, dim3(s->grid_vec), dim3(PCG_BLOCK), 0, s->stream, s->n, s->x, s->p0, s->p1, s->st);
    FEM_LAUNCHED();
    hipLaunchKernelGGL(k_mark_x_done, dim3(1), dim3(1), 0, s->stream, s->st);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_use_graph(fem_pcg* s, int k) {
    if (s->graph) {
        (void)hipGraphExecDestroy(s->graph);
        s->graph = nullptr;
        s->graph_k = 0;
    }
    if (k <= 0 || s->persist) return FEM_OK;   // the persistent schedule is one launch per chunk already
    hipGraph_t g;
    const int64_t saved = s->launched;
    s->launched = 0;
    FEM_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
    int rc = launch_iterations(s, k);
    hipError_t e = hipStreamEndCapture(s->stream, &g);
    s->launched = saved;
    if (rc) return rc;
    if (e != hipSuccess) {
        set_error("fem_pcg_use_graph: capture failed: %s", hipGetErrorString(e));
        return FEM_EHIP;
    }
    e = hipGraphInstantiate(&s->graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        set_error("fem_pcg_use_graph: instantiate failed: %s", hipGetErrorString(e));
        s->graph = nullptr;
        return FEM_EHIP;
    }
    s->graph_k = k;
    return FEM_OK;
}

static int fem_pcg_poll_raw(fem_pcg* s, int* iters, int* status, double* rz);
int fem_pcg_poll(fem_pcg* s, int* iters, int* status, double* rz) { return fem_pcg_poll_raw(s, iters, status, rz); }

int fem_pcg_release_cache(void) { return (int)(pool_release_all() >> 20); }

static int fem_pcg_poll_raw(fem_pcg* s, int* iters, int* status, double* rz) {
    FEM_HIP(hipMemcpyAsync(s->st_host, s->st, sizeof(PcgState), hipMemcpyDeviceToHost, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    const PcgState h = state_view(s);
    int stt = h.status;
    // single reduction: the stop test of the last update runs in the next step, which also sets halt
    if (stt == FEM_PCG_RUNNING && h.iter >= h.max_iter && (!(s->dist && s->cg1) || h.halt)) stt = FEM_PCG_MAXITER;
    // a guard stop reports the reference's printed iteration (i+1); a synchronisation give-up reports the last
    // committed iteration (its stop_iter holds the give-up site code: fem_pcg_sync_site)
    if (iters) *iters = (stt == FEM_PCG_BREAKDOWN || stt == FEM_PCG_ALPHA_NAN) ? h.stop_iter : h.iter;
    if (status) *status = stt;
    if (rz) *rz = (h.iter > 0) ? h.rz_new : h.rz;
    if (stt == FEM_PCG_BAD_WINDOW) {
        set_error("PCG: a workgroup's gather window lay outside the u-flag array (internal invariant broken; the "
                  "launch ended without running, iterate not meaningful)");
        return FEM_ESTATE;
    }
    return FEM_OK;
}

int fem_pcg_debug_window(fem_pcg* s, int L, int lo, int hi) {
    int32_t* win = s->persist ? s->pk_win : s->c1f_win;
    const int G = s->persist ? s->pk_grid : s->c1f_grid;
    if (!win || G <= 0 || L < 0 || L >= G) {
        set_error("fem_pcg_debug_window: no gather windows in this context (or L outside [0, %d))", G);
        return FEM_EARG;
    }
    FEM_HIP(hipMemcpyAsync(win + L, &lo, sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
    FEM_HIP(hipMemcpyAsync(win + G + L, &hi, sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    return FEM_OK;
}

int fem_pcg_sync_site(fem_pcg* s, int* site) {
    FEM_HIP(hipMemcpyAsync(s->st_host, s->st, sizeof(PcgState), hipMemcpyDeviceToHost, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    const PcgState h = state_view(s);
    *site = h.status == FEM_PCG_SYNC_TIMEOUT ? h.stop_iter : 0;
    return FEM_OK;
}

int fem_pcg_scalars(fem_pcg* s, double* out6) {
    FEM_HIP(hipMemcpyAsync(s->st_host, s->st, sizeof(PcgState), hipMemcpyDeviceToHost, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    const PcgState h = state_view(s);
    out6[0] = h.rz;
    out6[1] = h.pq;
    out6[2] = h.alpha;
    out6[3] = h.beta;
    out6[4] = h.rz_new;
    out6[5] = (double)h.iter;
    return FEM_OK;
}

// one solve attempt from the x currently in s->x
static int pcg_solve_once(fem_pcg* s, int max_iter, int chunk, int* it, int* stt, double* rz) {
    s->max_iter = max_iter;
    int rc = fem_pcg_start(s);
    s->max_iter = 0x7fffffff;
    if (rc) return rc;
    if (chunk <= 0) chunk = 32;
    // the persistent kernel stops itself on convergence: one launch and one poll per 8192 iterations (~0.4 s at
    // 10M tets; bounded launches keep a non-converging solve interruptible between them)
    if (s->persist) chunk = max_iter < 8192 ? max_iter : 8192;
    int done = 0;
    *it = 0;
    *stt = FEM_PCG_RUNNING;
    while (done < max_iter) {
        int k = chunk < max_iter - done ? chunk : max_iter - done;
        if ((rc = fem_pcg_iterate(s, k))) return rc;
        done += k;
        if ((rc = fem_pcg_poll_raw(s, it, stt, rz))) return rc;
        if (*stt != FEM_PCG_RUNNING) break;
        if (chunk < 256 && !s->persist) chunk *= 2;   // poll less often once the solve is clearly long
    }
    return FEM_OK;
}

int fem_pcg_solve(fem_pcg* s, int max_iter, int chunk, int* iters, int* status, double* rz) {
    // the persistent schedule: cooperative launches, and a copy of x0 so that a launch whose grid synchronisation
    // gave up (FEM_PCG_SYNC_TIMEOUT: the workgroups were not all resident) is re-solved on the deferred schedule
    // from the same start instead of returning a meaningless iterate
    double* x0 = nullptr;
    if (s->pd) {   // ranks must pass a host barrier between their starts and their first launches
        set_error("fem_pcg_solve: a distributed persistent context is driven by start / iterate / poll per rank");
        return FEM_EARG;
    }
    const bool may_persist = s->persist_req && (s->bs == 1 || s->bs == 3) && !s->dist &&
                             s->mode != FEM_MODE_CG_CONSTRAINED;
    // the merged update (k_pcg_update2) waits on every workgroup of its grid as well: same recovery
    const bool may_upd = (s->tune & FEM_TUNE_UPD1) && !s->dist && s->mode != FEM_MODE_CG_CONSTRAINED;
    if (may_persist || may_upd) {
        FEM_HIP(pool_alloc((void**)&x0, sizeof(double) * (size_t)(s->n + 2), s->stream, true));
        FEM_HIP(hipMemcpyAsync(x0, s->x, sizeof(double) * (size_t)s->n, hipMemcpyDeviceToDevice, s->stream));
    }
    // FEM355_PK_COOP=0 turns the cooperative launch off (rocprofv3 7.2 segfaults in its exit handler after a
    // process made one: profiling runs of bench.py set it; the bench's timed launches are plain either way)
    static const int coop = [] {
        const char* e = getenv("FEM355_PK_COOP");
        return e ? atoi(e) : 1;
    }();
    s->pk_coop = coop;
    int it = 0, stt = FEM_PCG_RUNNING;
    int rc = pcg_solve_once(s, max_iter, chunk, &it, &stt, rz);
    s->pk_coop = 0;
    if (!rc && stt == FEM_PCG_SYNC_TIMEOUT && x0) {
        rc = hipMemcpyAsync(s->x, x0, sizeof(double) * (size_t)s->n, hipMemcpyDeviceToDevice, s->stream) == hipSuccess
                 ? FEM_OK : FEM_EHIP;
        const int req0 = s->persist_req, tune0 = s->tune;
        s->persist_req = 0;   // fem_pcg_start now sets up the deferred schedule (set_schedule(3) implied deferred)
        s->tune &= ~FEM_TUNE_UPD1;   // and the two-kernel update
        if (!rc) rc = pcg_solve_once(s, max_iter, chunk, &it, &stt, rz);
        s->persist_req = req0;
        s->tune = tune0;
    }
    pool_free(x0, s->stream);
    if (rc) return rc;
    if ((rc = fem_pcg_finish(s))) return rc;
    if ((rc = fem_pcg_poll(s, &it, &stt, rz))) return rc;
    if (iters) *iters = it;
    if (status) *status = stt;
    return FEM_OK;
}

int fem_pcg_profile(fem_pcg* s, int k, int every, double* ms, int* n) {
    // k iterations enqueued on the solver stream; iterations i % every == 0 are bracketed by hip events
    // around each of their kernels (on the stream the kernels run on), the others launch bare.
    if (every < 1) every = 1;
    double acc[3] = {0, 0, 0};
    int rc = FEM_OK;
    if (s->persist) {   // bucket 0: persistent launches of `every` iterations (per-iteration time = ms / n); the
                        // two events live with the context (no event creation next to a timed launch)
        if (!s->pev[0]) {
            FEM_HIP(hipEventCreate(&s->pev[0]));
            FEM_HIP(hipEventCreate(&s->pev[1]));
        }
        for (int i = 0; i < k && !rc; i += every) {
            const int kk = every < k - i ? every : k - i;
            FEM_HIP(hipEventRecord(s->pev[0], s->stream));
            rc = launch_persist(s, kk);
            FEM_HIP(hipEventRecord(s->pev[1], s->stream));
            FEM_HIP(hipEventSynchronize(s->pev[1]));   // launches of `every` < k are timed one by one
            float t = 0.f;
            FEM_HIP(hipEventElapsedTime(&t, s->pev[0], s->pev[1]));
            acc[0] += t;
        }
        if (ms) ms[0] = acc[0], ms[1] = 0.0, ms[2] = 0.0;
        if (n) n[0] = k, n[1] = 0, n[2] = 0;
        return rc;
    }
    const int ns = (k + every - 1) / every;
    std::vector<hipEvent_t> evs((size_t)ns * 4);
    for (auto& e : evs) FEM_HIP(hipEventCreate(&e));
    int si = 0;
    for (int i = 0; i < k && !rc; ++i) {
        if (i % every) {
            rc = launch_iterations(s, 1);
            continue;
        }
        if (s->dist && s->cg1) {   // buckets: [0] v = A u + pack, [1] all-reduce, [2] step + update
            (void)hipEventRecord(evs[4 * si + 3], s->stream);
            rc = cg1_step_update(s);
            (void)hipEventRecord(evs[4 * si + 0], s->stream);
            if (!rc) rc = cg1_spmv(s, 0);
            (void)hipEventRecord(evs[4 * si + 1], s->stream);
            if (!rc) rc = dist_exchange(s, 4);
            (void)hipEventRecord(evs[4 * si + 2], s->stream);
            s->launched++;
            ++si;
            continue;
        }
        const bool dfr = s->deferred && !s->dist;
        if (s->upd1) {   // buckets: [0] SpMV, [1] merged update, [2] empty
            (void)hipEventRecord(evs[4 * si + 0], s->stream);
            rc = launch_spmv_dot(s);
            (void)hipEventRecord(evs[4 * si + 1], s->stream);
            if (!rc) rc = launch_update2(s);
            (void)hipEventRecord(evs[4 * si + 2], s->stream);
            (void)hipEventRecord(evs[4 * si + 3], s->stream);
            s->launched++;
            ++si;
            continue;
        }
        (void)hipEventRecord(evs[4 * si + 0], s->stream);
        rc = dfr ? launch_deferred(s, 0) : launch_spmv_dot(s);
        (void)hipEventRecord(evs[4 * si + 1], s->stream);
        if (!rc && !dfr) rc = launch_exchange_dot(s);
        if (!rc) rc = dfr ? launch_deferred(s, 1) : launch_update_finish(s);
        (void)hipEventRecord(evs[4 * si + 2], s->stream);
        if (!rc) rc = dfr ? launch_deferred(s, 2) : launch_pupdate(s);
        (void)hipEventRecord(evs[4 * si + 3], s->stream);
        ++si;
    }
    FEM_HIP(hipStreamSynchronize(s->stream));
    for (int i = 0; i < si; ++i) {
        float t;
        for (int j = 0; j < 3; ++j) {
            // single-reduction: events 3 -> 0 bracket step + update (bucket 2)
            const bool c1 = s->dist && s->cg1;
            (void)hipEventElapsedTime(&t, evs[4 * i + (c1 && j == 2 ? 3 : j)], evs[4 * i + (c1 && j == 2 ? 0 : j + 1)]);
            acc[j] += t;
        }
    }
    for (auto& e : evs) (void)hipEventDestroy(e);
    for (int j = 0; j < 3; ++j) {
        if (ms) ms[j] = acc[j];
        if (n) n[j] = si;
    }
    return rc;
}

// ------------------------------------------------------------------ distributed persistent schedule
int fem_pcg_set_rows(fem_pcg* s, int nranks, int rank, const int64_t* slice_split, int grid) {
    if (nranks < 1 || nranks > PK_MAX_RANKS || rank < 0 || rank >= nranks || !slice_split) {
        set_error("fem_pcg_set_rows: nranks %d (1..%d), rank %d", nranks, PK_MAX_RANKS, rank);
        return FEM_EARG;
    }
    if ((s->bs != 1 && s->bs != 3) || s->dist || s->mode == FEM_MODE_CG_CONSTRAINED || s->pd) {
        set_error("fem_pcg_set_rows: bs = 1 or 3, not element-partitioned, not constrained, once per context");
        return FEM_EARG;
    }
    if (slice_split[0] != 0 || slice_split[nranks] != s->nslices) {
        set_error("fem_pcg_set_rows: the split must cover slices [0, %lld)", (long long)s->nslices);
        return FEM_EARG;
    }
    for (int q = 0; q < nranks; ++q)
        if (slice_split[q + 1] <= slice_split[q]) {
            set_error("fem_pcg_set_rows: rank %d owns no slice", q);
            return FEM_EARG;
        }
    int dev = 0, ncu = 0;
    FEM_HIP(hipGetDevice(&dev));
    FEM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int G = grid > 0 ? grid : (ncu / NXCD) * NXCD;
    if (G < NXCD || G % NXCD || G > ncu) {
        set_error("fem_pcg_set_rows: grid %d must be a multiple of %d within %d CUs", G, NXCD, ncu);
        return FEM_EARG;
    }
    s->pd_rank = rank;
    s->pd_nranks = nranks;
    for (int q = 0; q <= nranks; ++q) s->pd_split[q] = slice_split[q];
    // comm block: u (global length) [| m[1] (FEM_TUNE_PK_GV, bs = 1)] | u-flags of all nranks * G workgroups | rank
    // sums | rank epoch lines
    const int64_t line = sizeof(unsigned) * PK_LINE;
    const int64_t vreg = (int64_t)cdiv(sizeof(double) * (s->n + 2), 256) * 256;
    s->pd_off_m1 = ((s->tune & FEM_TUNE_PK_GV) && s->bs == 1) ? vreg : 0;
    s->pd_off_flag = vreg + s->pd_off_m1;
    s->pd_off_red = s->pd_off_flag + (int64_t)nranks * G * line;
    s->pd_off_rflag = s->pd_off_red + 256;
    s->pd_block_bytes = s->pd_off_rflag + PK_MAX_RANKS * NXCD * line;   // [rank][XCD group] epoch lines
    if (s->tune & FEM_TUNE_DIST_FINE)   // fine-grained device memory: coherent for the other GPUs' accesses
        FEM_HIP(hipExtMallocWithFlags((void**)&s->pd_block, (size_t)s->pd_block_bytes, hipDeviceMallocFinegrained));
    else
        FEM_HIP(hipMalloc((void**)&s->pd_block, (size_t)s->pd_block_bytes));
    FEM_HIP(hipMemsetAsync(s->pd_block, 0, (size_t)s->pd_block_bytes, s->stream));
    // the single-GPU persistent buffers for this grid, and the gather windows in global workgroup ids
    pool_free(s->pk_win, s->stream);
    pool_free(s->pk_part, s->stream);
    pool_free(s->pk_sync, s->stream);
    FEM_HIP(pool_alloc((void**)&s->pk_win, sizeof(int32_t) * (2 * G + 2), s->stream, true));
    FEM_HIP(pool_alloc((void**)&s->pk_part, sizeof(double) * 4 * G, s->stream, true));
    FEM_HIP(pool_alloc((void**)&s->pk_sync, sizeof(unsigned) * pk_sync_words(G), s->stream, true));
    s->pk_grid = G;
    std::vector<int32_t> lohi(2 * (size_t)G + 2);
    for (int i = 0; i < G; ++i) {
        lohi[i] = nranks * G;
        lohi[G + i] = -1;
    }
    lohi[2 * G] = 0x7fffffff;
    lohi[2 * G + 1] = -1;
    FEM_HIP(hipMemcpyAsync(s->pk_win, lohi.data(), sizeof(int32_t) * lohi.size(), hipMemcpyHostToDevice, s->stream));
    PkSplit sp{};
    for (int q = 0; q <= nranks; ++q) sp.b[q] = slice_split[q];
    const int64_t nloc = slice_split[rank + 1] - slice_split[rank];
    hipLaunchKernelGGL(k_pk_window_dist, dim3(stream_grid(nloc * 64, 256)), dim3(256), 0, s->stream, slice_split[rank],
                       nloc, s->nrows, s->slice_ptr, s->cols, G, sp, nranks, s->pk_win, s->pk_win + G,
                       s->pk_win + 2 * G);
    FEM_LAUNCHED();
    FEM_HIP(hipStreamSynchronize(s->stream));   // lohi must outlive the copy
    s->pk_win_ok = 1;
    s->pd = 1;
    s->pd_peers_ok = 0;
    s->persist_req = 1;
    s->deferred = 1;
    s->fused = 0;
    return FEM_OK;
}

int fem_pcg_comm_block(fem_pcg* s, void** base, int64_t* bytes) {
    if (!s->pd) {
        set_error("fem_pcg_comm_block: fem_pcg_set_rows first");
        return FEM_EARG;
    }
    if (base) *base = s->pd_block;
    if (bytes) *bytes = s->pd_block_bytes;
    return FEM_OK;
}

int fem_pcg_col_window(fem_pcg* s, int64_t* lo, int64_t* hi) {
    if (!s->pd) {
        set_error("fem_pcg_col_window: fem_pcg_set_rows first");
        return FEM_EARG;
    }
    int32_t w[2];
    FEM_HIP(hipMemcpyAsync(w, s->pk_win + 2 * s->pk_grid, sizeof w, hipMemcpyDeviceToHost, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    *lo = w[0];
    *hi = w[1];
    return FEM_OK;
}

int fem_pcg_set_peers(fem_pcg* s, void* const* bases, const int64_t* need_lo, const int64_t* need_hi) {
    if (!s->pd) {
        set_error("fem_pcg_set_peers: fem_pcg_set_rows first");
        return FEM_EARG;
    }
    const int N = s->pd_nranks, G = s->pk_grid, r = s->pd_rank;
    for (int q = 0; q < N; ++q) {
        s->pd_peer[q] = q == r ? s->pd_block : (char*)bases[q];
        if (!s->pd_peer[q]) {
            set_error("fem_pcg_set_peers: no comm block for rank %d", q);
            return FEM_EARG;
        }
    }
    // for each local workgroup and rank q: {-1, -1} when q never waits on it, else the rows [lo, hi) of it that q
    // gathers (possibly none). q waits on the contiguous range of global workgroups between the owners of its
    // column window's ends -- a workgroup in that range without rows (fewer slices than workgroups) still raises
    // its flag there
    const int64_t S0 = s->pd_split[r], nloc = s->pd_split[r + 1] - S0;
    auto owner = [&](int64_t row) {   // global logical workgroup owning a row (k_pk_window_dist's owner)
        const int64_t sl = row >> 6;
        int q = 0;
        while (q + 1 < N && s->pd_split[q + 1] <= sl) ++q;
        const int64_t S = s->pd_split[q + 1] - s->pd_split[q], tl = sl - s->pd_split[q];
        const int64_t L = ((tl + 1) * G - 1) / S;
        return (int64_t)q * G + (L < G ? L : G - 1);
    };
    std::vector<int32_t> pub((size_t)G * N * 2, -1);
    // FEM_TUNE_DIST_DROP (fault injection, tests only): this rank publishes nothing, so the ranks that gather its
    // rows give up on their u-flags and the launch ends with FEM_PCG_SYNC_TIMEOUT on every rank
    for (int q = 0; q < N && !(s->tune & FEM_TUNE_DIST_DROP); ++q) {
        if (q == r || need_hi[q] < need_lo[q]) continue;
        const int64_t glo = owner(need_lo[q]), ghi = owner(need_hi[q]);
        for (int L = 0; L < G; ++L) {
            const int64_t Lg = (int64_t)r * G + L;
            if (Lg < glo || Lg > ghi) continue;
            const int64_t rlo = (S0 + (int64_t)L * nloc / G) * 64;
            const int64_t rhi = std::min<int64_t>((S0 + (int64_t)(L + 1) * nloc / G) * 64, s->nrows);
            const int64_t lo = std::max<int64_t>(rlo, need_lo[q]), hi = std::min<int64_t>(rhi, need_hi[q] + 1);
            pub[((size_t)L * N + q) * 2] = (int32_t)std::max<int64_t>(lo, 0);
            pub[((size_t)L * N + q) * 2 + 1] = (int32_t)std::max<int64_t>(hi, std::max<int64_t>(lo, 0));
        }
    }
    if (!s->pd_pub) FEM_HIP(hipMalloc((void**)&s->pd_pub, sizeof(int32_t) * pub.size()));
    FEM_HIP(hipMemcpyAsync(s->pd_pub, pub.data(), sizeof(int32_t) * pub.size(), hipMemcpyHostToDevice, s->stream));
    FEM_HIP(hipStreamSynchronize(s->stream));
    s->pd_peers_ok = 1;
    return FEM_OK;
}

int fem_pcg_dist_debug(fem_pcg* s, int which, int32_t* host_out, int64_t n) {
    if (!s->pd) {
        set_error("fem_pcg_dist_debug: not a distributed persistent context");
        return FEM_EARG;
    }
    const int G = s->pk_grid, N = s->pd_nranks;
    if (which == 0) {   // gather windows [G] lo, [G] hi (global workgroups), then the column window
        FEM_HIP(hipMemcpyAsync(host_out, s->pk_win, sizeof(int32_t) * std::min<int64_t>(n, 2 * G + 2),
                               hipMemcpyDeviceToHost, s->stream));
    } else if (which == 1) {   // the u-flag of every global workgroup in this rank's comm block
        for (int64_t i = 0; i < std::min<int64_t>(n, (int64_t)N * G); ++i)
            FEM_HIP(hipMemcpyAsync(host_out + i, s->pd_block + s->pd_off_flag + i * sizeof(unsigned) * PK_LINE,
                                   sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    } else if (which == 2) {   // pub [G][N][2]
        FEM_HIP(hipMemcpyAsync(host_out, s->pd_pub, sizeof(int32_t) * std::min<int64_t>(n, (int64_t)G * N * 2),
                               hipMemcpyDeviceToHost, s->stream));
    } else if (which == 3) {   // the rank epoch lines [rank][XCD group]
        for (int64_t i = 0; i < std::min<int64_t>(n, (int64_t)N * NXCD); ++i)
            FEM_HIP(hipMemcpyAsync(host_out + i, s->pd_block + s->pd_off_rflag + i * sizeof(unsigned) * PK_LINE,
                                   sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    } else if (which == 4) {   // local sync words: group counters, top replicas, give-up word
        for (int64_t i = 0; i < std::min<int64_t>(n, 18); ++i)
            FEM_HIP(hipMemcpyAsync(host_out + i, s->pk_sync + i * PK_LINE, sizeof(int32_t), hipMemcpyDeviceToHost,
                                   s->stream));
    }
    FEM_HIP(hipStreamSynchronize(s->stream));
    return FEM_OK;
}

int fem_stream_create_cu(int part, int nparts, void** stream) {
    int dev = 0, ncu = 0;
    FEM_HIP(hipGetDevice(&dev));
    FEM_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (nparts < 1 || part < 0 || part >= nparts) {
        set_error("fem_stream_create_cu: part %d of %d", part, nparts);
        return FEM_EARG;
    }
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int cu = 0; cu < ncu; ++cu)
        if (cu % nparts == part) mask[(size_t)cu / 32] |= 1u << (cu % 32);
    hipStream_t st = nullptr;
    FEM_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    *stream = st;
    return FEM_OK;
}

int fem_stream_destroy(void* stream) {
    FEM_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
    return FEM_OK;
}

int fem_pcg_set_prof(fem_pcg* s, unsigned long long* dev_buf) {
    if (!s->pd) {
        set_error("fem_pcg_set_prof: distributed persistent contexts only (single GPU: fem_pcg_persist_profile)");
        return FEM_EARG;
    }
    s->pd_prof = dev_buf;
    return FEM_OK;
}

int fem_ipc_handle(void* ptr, char* out64) {
    hipIpcMemHandle_t h;
    FEM_HIP(hipIpcGetMemHandle(&h, ptr));
    static_assert(sizeof(h) <= 64, "IPC handle size");
    memset(out64, 0, 64);
    memcpy(out64, &h, sizeof h);
    return FEM_OK;
}

int fem_ipc_open(const char* h64, void** ptr) {
    hipIpcMemHandle_t h;
    memcpy(&h, h64, sizeof h);
    FEM_HIP(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    return FEM_OK;
}

int fem_ipc_close(void* ptr) {
    FEM_HIP(hipIpcCloseMemHandle(ptr));
    return FEM_OK;
}

void fem_pcg_destroy(fem_pcg* s) {
    if (!s) return;
    if (s->pev[0]) (void)hipEventDestroy(s->pev[0]);
    if (s->pd_block) (void)hipFree(s->pd_block);
    if (s->pd_pub) (void)hipFree(s->pd_pub);
    if (s->pev[1]) (void)hipEventDestroy(s->pev[1]);
    if (s->graph) (void)hipGraphExecDestroy(s->graph);
    pool_free(s->r, s->stream);
    pool_free(s->p0, s->stream);
    pool_free(s->p1, s->stream);
    pool_free(s->q, s->stream);
    pool_free(s->red.partials, s->stream);
    pool_free(s->red.counters, s->stream);
    if (s->hbuf) (void)hipFree(s->hbuf);
    if (s->cg1_s) (void)hipFree(s->cg1_s);
    if (s->cg1_u) (void)hipFree(s->cg1_u);
    if (s->cg1_send) (void)hipFree(s->cg1_send);
    if (s->cg1_recv) (void)hipFree(s->cg1_recv);
    if (s->psend) (void)hipFree(s->psend);
    if (s->precv) (void)hipFree(s->precv);
    if (s->c1f_win) (void)hipFree(s->c1f_win);
    if (s->c1f_flags) (void)hipFree(s->c1f_flags);
    if (s->con.tmp) (void)hipFree(s->con.tmp);
    if (s->mf_sl) (void)hipFree(s->mf_sl);
    if (s->pext) {   // the caller's solver-layout arrays
        s->pvals = nullptr;
        s->pcols16 = nullptr;
        s->puoff = nullptr;
        s->pucol = nullptr;
    }
    pool_free(s->pvals, s->stream);
    pool_free(s->pcols16, s->stream);
    pool_free(s->puoff, s->stream);
    pool_free(s->pucol, s->stream);
    pool_free(s->pk_win, s->stream);
    pool_free(s->pk_part, s->stream);
    pool_free(s->pk_sync, s->stream);
    pool_free(s->pk_v, s->stream);
    pool_free(s->gv_buf, s->stream);
    pool_free(s->u2_sync, s->stream);
    pool_free(s->st, s->stream);
    host_state_free(s->st_host, s->stream);
    delete s;
}

}  // extern "C"
