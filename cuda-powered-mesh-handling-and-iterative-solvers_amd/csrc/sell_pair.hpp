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

// Slice-uniform column deltas (FEM_TUNE_PK_UNI). When the 64 rows of a slice take their columns at the same
// offsets from the row (every row's deltas a subset of one sorted list of `w` deltas -- FEM meshes numbered along a
// structured sweep, e.g. every slice of the Kuhn cubes), the slice stores that list ONCE: ucol[uoff[s] + k] = delta of
// entry k for every lane, and rows lacking an offset hold a zero value there (the lane-paired value layout is kept,
// entries in list order). The SpMV then reads the deltas with wave-uniform loads: 10 -> 8 bytes per entry on the
// matrix stream. Real entries keep their order within the row (ascending column), so every row sum adds the same
// products in the same order, with +-0 terms interleaved. Other slices: uoff[s] = -1, per-lane deltas as before.
// k_sell_uniform writes the paired values / deltas of the uniform slices (pcols16 stays a valid per-lane copy: kernels
// that ignore uoff read the same entries) and, with pair_rest, the plain lane-paired copy (k_sell_pair) of every other
// slice -- one pass over the matrix instead of k_sell_pair followed by a rewrite of nearly every slice. A slice qualifies when: it is full (no rows
// past nrows), width <= SU_MAXW, the row of greatest length has exactly w entries (no extra padding), every other
// row's real deltas are a subsequence of that row's, every padded column row + delta lies in [0, nrows), and the
// trailing SELL padding entries of every row are (delta 0, value 0).
constexpr int SU_MAXW = 64;

constexpr int PK_T = 1024;               // threads per workgroup of the persistent schedule (16 waves, 4 per SIMD)
constexpr int PK_WAVES = PK_T / 64;

// gather window per logical workgroup: the first and last workgroup owning a column of its rows. A slice-uniform
// slice (sell_pair.hpp) makes every lane gather at the whole slice's delta list, i.e. also at offsets its own row
// lacks (value 0 there). So the window of a slice is taken over the UNION of its rows' deltas applied to every row
// of the slice: [s*64 + min delta, s*64 + 63 + max delta]. Every column any lane reads is then inside a window the
// workgroup waits on -- no read of an unsynchronised u, whose value (0 * Inf = NaN) would otherwise matter.
__device__ __forceinline__ void pk_slice_span(int64_t s, int64_t nrows, int dmin, int dmax, int64_t* cmin, int64_t* cmax) {
    for (int off = 32; off > 0; off >>= 1) {
        const int a2 = __shfl_xor(dmin, off), b2 = __shfl_xor(dmax, off);
        dmin = a2 < dmin ? a2 : dmin;
        dmax = b2 > dmax ? b2 : dmax;
    }
    int64_t lo = s * 64 + dmin, hi = s * 64 + 63 + dmax;
    if (hi >= nrows) hi = nrows - 1;
    if (lo < 0) lo = 0;
    if (lo > hi) lo = hi;
    *cmin = lo;
    *cmax = hi;
}

// a slice's lane-paired 16-bit deltas (pair_pos) written as one 32-bit store per pair (entries 2 k2, 2 k2 + 1 of lane
// l are adjacent halves), then the unpaired last entry of an odd width: full 256-byte rows per store instruction
#ifndef FEM_SL_SKIP
#define FEM_SL_SKIP 0
#endif
template <class Delta>
__device__ __forceinline__ void sl_store_pairs(int16_t* __restrict__ out, int w, int l, const Delta& delta) {
#if FEM_SL_SKIP & 2
    return;
#endif
    const int np = w >> 1;
    int32_t* o32 = reinterpret_cast<int32_t*>(out);   // out = pout + slice start: 128-byte aligned
    for (int k2 = 0; k2 < np; ++k2)
        o32[k2 * 64 + l] = (int32_t)((uint32_t)(uint16_t)delta(2 * k2) | ((uint32_t)(uint16_t)delta(2 * k2 + 1) << 16));
    if (w & 1) out[(int64_t)np * 128 + l] = (int16_t)delta(w - 1);
}

// The solver layout of one slice s of a bs = 1 pattern, by the wave whose lane l is row s * 64 + l (k_sell_sl_pattern,
// and k_sell_fill_graph right after it wrote the slice's deltas): see k_sell_sl_pattern (pcg.hip). cand: SU_MAXW ints of
// the wave's LDS. delta(k): this lane's plain 16-bit delta of entry k of the slice (each lane reads only its own row's
// entries before the shuffles) -- from memory (k_sell_sl_pattern) or from the rows the fill pass holds in LDS.
// span != null: the slice's owner-workgroup span (owner(cmin), owner(cmax)) is stored in span[s] and the windows are
// formed from all spans by k_win_from_spans, instead of two atomics per slice on `win` (the G windows share a few
// cache lines: 54,000 atomics on 16 lines serialise in the L2 -- 72 us of the 10M fill pass).
template <class Delta>
__device__ __forceinline__ void sl_pattern_slice(int64_t s, int l, int64_t nslices, int64_t nrows,
                                                 const int64_t* __restrict__ slice_ptr, const Delta& delta,
                                                 int16_t* __restrict__ pout, int16_t* __restrict__ ucol,
                                                 int32_t* __restrict__ uoff, int G, int* __restrict__ win, int* cand,
                                                 int2* __restrict__ span = nullptr) {
#if FEM_SL_SKIP & 4   // timing builds only (wrong layout): the fill pass without the solver layout
    return;
#endif
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int64_t row = s * 64 + l;
#if FEM_SL_SKIP & 1
    G = 0;
#endif
    if (G > 0) {   // gather window (k_pk_window): the delta union of the slice over its owner workgroup
        int dmin = 0, dmax = 0;
        if (row < nrows)
            for (int k = 0; k < w; ++k) {
                const int d = delta(k);
                dmin = d < dmin ? d : dmin;
                dmax = d > dmax ? d : dmax;
            }
        int64_t cmin, cmax;
        pk_slice_span(s, nrows, dmin, dmax, &cmin, &cmax);
        const int64_t WV = (int64_t)G * PK_WAVES;
        auto owner = [&](int64_t r) { return (int)((((r >> 6) + 1) * WV - 1) / nslices / PK_WAVES); };
        if (l == 0) {
            if (span) {
                span[s] = make_int2(owner(cmin), owner(cmax));
            } else {
                const int me = owner(row);
                atomicMin(win + me, owner(cmin));
                atomicMax(win + G + me, owner(cmax));
            }
        }
    }
    bool ok = (s + 1) * 64 <= nrows && w > 0 && w <= SU_MAXW;
    int len = 0;
    if (ok) {
        int prev = -(1 << 30);
        for (int k = 0; k < w; ++k) {
            const int d = delta(k);
            if (len == k && d > prev) {
                ++len;
                prev = d;
            } else if (d != 0) {
                ok = false;
            }
        }
    }
    ok = __all(ok);
    const unsigned long long full = __ballot(ok && len == w);
    if (ok && full) {
        const int c = __builtin_ctzll(full);
        for (int k = 0; k < w; ++k) {
            const int d = __shfl(delta(k), c, 64);
            if (l == 0) cand[k] = d;
            const int64_t col = row + d;
            if (col < 0 || col >= nrows) ok = false;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int i = 0;
        for (int k = 0; k < len && ok; ++k) {
            const int d = delta(k);
            while (i < w && cand[i] < d) ++i;
            if (i == w || cand[i] != d) ok = false;
            ++i;
        }
    } else {
        ok = false;
    }
    ok = __all(ok);
    if (!ok) {
        if (l == 0) uoff[s] = -1;
        sl_store_pairs(pout + p0, w, l, delta);
        return;
    }
    const int32_t uo = (int32_t)(2 * (p0 >> 6));   // even: the deltas are read as int32 pairs
    sl_store_pairs(pout + p0, w, l, [&](int k) { return cand[k]; });
    for (int k = l; k < w; k += 64) ucol[uo + k] = (int16_t)cand[k];
    if (l == 0) uoff[s] = uo;
}
// the gather windows from the per-slice owner spans (sl_pattern_slice with span): a wave per owner workgroup me, its
// slices {s : owner(s) = me} (owner is monotone in s) found by binary search, min / max over their spans; an owner
// without slices gets the empty window (G, -1) of k_pk_window_init
__attribute__((unused)) static __global__ void __launch_bounds__(256) k_win_from_spans(int G, int64_t nslices,
                                                                                       const int2* __restrict__ span,
                                                                                       int* __restrict__ win) {
    const int me = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int l = threadIdx.x & 63;
    if (me >= G) return;   // wave-uniform
    const int64_t WV = (int64_t)G * PK_WAVES;
    auto owner_s = [&](int64_t s) { return (int)(((s + 1) * WV - 1) / nslices / PK_WAVES); };
    auto first = [&](int o) {   // first slice whose owner is >= o
        int64_t lo = 0, hi = nslices;
        while (lo < hi) {
            const int64_t m = (lo + hi) >> 1;
            if (owner_s(m) < o) lo = m + 1;
            else hi = m;
        }
        return lo;
    };
    const int64_t s0 = first(me), s1 = first(me + 1);
    int lo = G, hi = -1;
    for (int64_t s = s0 + l; s < s1; s += 64) {
        const int2 v = span[s];
        lo = v.x < lo ? v.x : lo;
        hi = v.y > hi ? v.y : hi;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const int a = __shfl_xor(lo, off), b = __shfl_xor(hi, off);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if (l == 0) {
        win[me] = lo;
        win[G + me] = hi;
    }
}

__attribute__((unused)) static __global__ void __launch_bounds__(256) k_sell_uniform(int64_t nslices, int64_t nrows,
                                                             const int64_t* __restrict__ slice_ptr,
                                                             const double* __restrict__ vin,
                                                             const int16_t* __restrict__ cin, double* __restrict__ vout,
                                                             int16_t* __restrict__ cout, int16_t* __restrict__ ucol,
                                                             int32_t* __restrict__ uoff, int pair_rest) {
    __shared__ int cand_all[4][SU_MAXW];
    const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;   // one wave per slice
    const int l = threadIdx.x & 63;
    int* cand = cand_all[(threadIdx.x >> 6) & 3];
    if (s >= nslices) return;   // wave-uniform
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int64_t row = s * 64 + l;
    bool ok = (s + 1) * 64 <= nrows && w > 0 && w <= SU_MAXW;
    // real entries of this row: the strictly increasing prefix of its deltas; the rest must be (0, 0.0) padding
    int len = 0;
    if (ok) {
        int prev = -(1 << 30);
        for (int k = 0; k < w; ++k) {
            const int d = cin[p0 + 64 * k + l];
            if (len == k && d > prev) {
                ++len;
                prev = d;
            } else if (d != 0 || vin[p0 + 64 * k + l] != 0.0) {
                ok = false;
            }
        }
    }
    ok = __all(ok);
    const unsigned long long full = __ballot(ok && len == w);
    if (ok && full) {
        const int c = __builtin_ctzll(full);   // the lowest full-length row supplies the delta list
        for (int k = 0; k < w; ++k) {
            const int d = __shfl((int)cin[p0 + 64 * k + l], c, 64);
            if (l == 0) cand[k] = d;
            const int64_t col = row + d;
            if (col < 0 || col >= nrows) ok = false;
        }
        // cand (written by lane 0) visible to the whole wave
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int i = 0;
        for (int k = 0; k < len && ok; ++k) {   // subsequence check
            const int d = cin[p0 + 64 * k + l];
            while (i < w && cand[i] < d) ++i;
            if (i == w || cand[i] != d) ok = false;
            ++i;
        }
    } else {
        ok = false;
    }
    ok = __all(ok);
    const int32_t uo = (int32_t)(2 * (p0 >> 6));   // even: the deltas are read as int32 pairs
    const int np = w >> 1;
    if (!ok) {
        if (l == 0) uoff[s] = -1;
        if (pair_rest) {   // k_sell_pair's copy of this slice
            for (int k = 0; k < w; ++k) {
                const int64_t src = p0 + 64 * k + l;
                const int64_t dst = k < 2 * np ? p0 + (int64_t)(k >> 1) * 128 + 2 * l + (k & 1) : p0 + (int64_t)np * 128 + l;
                vout[dst] = vin[src];
                cout[dst] = cin[src];
            }
        }
        return;
    }
    int kr = 0;   // next real entry of this row
    for (int k = 0; k < w; ++k) {
        const int d = cand[k];
        double v = 0.0;
        if (kr < len && (int)cin[p0 + 64 * kr + l] == d) {
            v = vin[p0 + 64 * kr + l];
            ++kr;
        }
        const int64_t dst = k < 2 * np ? p0 + (int64_t)(k >> 1) * 128 + 2 * l + (k & 1) : p0 + (int64_t)np * 128 + l;
        vout[dst] = v;
        cout[dst] = (int16_t)d;
    }
    for (int k = l; k < w; k += 64) ucol[uo + k] = (int16_t)cand[k];
    if (l == 0) uoff[s] = uo;
}

// plain SELL values of a solver-layout (paired, slice-uniform) bs = 1 matrix: lane l walks its row's plain deltas and
// the slice's list (uniform) or maps plain entry k to its paired position (other slices); padding entries zero
__attribute__((unused)) static __global__ void __launch_bounds__(256) k_sell_sl_unpair(int64_t nslices,
                                                               const int64_t* __restrict__ slice_ptr,
                                                               const int16_t* __restrict__ cin,
                                                               const int32_t* __restrict__ uoff,
                                                               const int16_t* __restrict__ ucol,
                                                               const int32_t* __restrict__ rowptr, int64_t nrows,
                                                               const double* __restrict__ vin,
                                                               double* __restrict__ vout) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        const int64_t row = s * 64 + l;
        const int len = row < nrows ? rowptr[row + 1] - rowptr[row] : 0;
        const int uo = uoff[s];
        int u = 0;
        for (int k = 0; k < w; ++k) {
            double v = 0.0;
            if (k < len) {
                int pos = k;
                if (uo >= 0) {   // the list position of this entry's delta (rows' deltas are subsequences of it)
                    const int d = cin[p0 + 64 * k + l];
                    while (u < w && (int)ucol[uo + u] < d) ++u;
                    pos = u++;
                }
                v = vin[p0 + pair_pos(pos, w, l)];
            }
            vout[p0 + 64 * k + l] = v;
        }
    }
}

// y_row (bs = 1) of one slice row in the paired layout; U pairs in flight. UNI: the slice's deltas from the
// wave-uniform list ucl (k_sell_uniform), else per lane from cols.
template <int U, int SC1, bool UNI>
__device__ __forceinline__ double sell_row_pair_body(int64_t p0, int w, int base, int lane,
                                                     const int16_t* __restrict__ cols, const int16_t* __restrict__ ucl,
                                                     const double* __restrict__ vals, const double* __restrict__ x,
                                                     int own_lo, int own_hi) {
    const int np = w >> 1;
    const double2* v2 = reinterpret_cast<const double2*>(vals + p0) + lane;
    const int32_t* c2 = UNI ? reinterpret_cast<const int32_t*>(ucl) : reinterpret_cast<const int32_t*>(cols + p0) + lane;
    double acc = 0.0;
    for (int j0 = 0; j0 < np; j0 += U) {
        int32_t cc[U];
        double2 vv[U];
        double x0[U], x1[U];
#pragma unroll
        for (int j = 0; j < U; ++j) cc[j] = (j0 + j < np) ? c2[UNI ? (j0 + j) : 64 * (j0 + j)] : 0;
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
        const int d = UNI ? (int)ucl[w - 1] : (int)cols[t];
        acc += vals[t] * ldx_col<SC1>(x, base + d, own_lo, own_hi);
    }
    return acc;
}

// uoff / ucol (nullable): the slice-uniform deltas of k_sell_uniform
template <int U, int SC1 = 0>
__device__ __forceinline__ double sell_row_pair(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                                const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                                const double* __restrict__ x, int own_lo = 0, int own_hi = 0,
                                                const int32_t* __restrict__ uoff = nullptr,
                                                const int16_t* __restrict__ ucol = nullptr) {
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int base = (int)(s * 64 + lane);
    if (uoff) {
        const int uo = __builtin_amdgcn_readfirstlane(uoff[s]);
        if (uo >= 0) return sell_row_pair_body<U, SC1, true>(p0, w, base, lane, cols, ucol + uo, vals, x, own_lo, own_hi);
    }
    return sell_row_pair_body<U, SC1, false>(p0, w, base, lane, cols, nullptr, vals, x, own_lo, own_hi);
}

}  // namespace fem
