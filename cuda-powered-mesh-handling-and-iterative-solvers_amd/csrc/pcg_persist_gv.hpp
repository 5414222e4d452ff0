// Pipelined persistent Jacobi-PCG (FEM_TUNE_PK_GV; bs = 1, single GPU, systems whose slices fit 1-2 per wave: the
// 1M-tet configs[1] cube, the N = 8 rank share of the 10M one).
//
// The persistent kernel of pcg_persist.hpp runs the single-reduction (Chronopoulos-Gear) iteration: SpMV, then a
// grid barrier that every workgroup waits on before it can form the step -- at these sizes the barrier and the
// u hand-off are most of the iteration (9.4 us at 1M, of which the SpMV phase is ~4 us). This kernel runs the
// Ghysels-Vanroose pipelined form of the same Jacobi-PCG (the recurrences of "Hiding global synchronization latency
// in the preconditioned Conjugate Gradient algorithm", Alg. 4, with M^-1 = diag(w)):
//
//   init  : r0 = b - A x0, u0 = w r0 (k_cg1_init), w0 = A u0, m0 = w w0; gamma0 = r0.u0, delta0 = w0.u0
//   iter i: (gamma_i, delta_i reduced over the grid) || n_i = A m_i          <- the reduction hides behind the SpMV
//           beta = gamma_i / gamma_{i-1}, alpha = gamma_i / (delta_i - beta gamma_i / alpha_{i-1})  (i = 0: beta = 0)
//           z = n + beta z, q = m + beta q, s = w + beta s, p = u + beta p
//           x += alpha p, r -= alpha s, u -= alpha q, w -= alpha z, m = w (.) w
//           gamma_{i+1} = r.u and delta_{i+1} = w.u partials posted, the barrier arrival of iteration i + 1
//
// The arrival on the grid barrier is posted BEFORE the SpMV and waited for after it, so the barrier's fan-in / fan-out
// runs while the matrix streams. The recurrences for u = M^-1 r and w = A u replace two products by updates, so the
// iterates leave the single-reduction ones at rounding level and drift further as the solve proceeds (the method's
// known attainable-accuracy limit); tests/test_gpu_pipelined.py states the tolerances this build meets.
//
// Layout and hand-offs as k_pcg_persist (one 1024-thread workgroup per CU, packed slices, XCD-grouped barrier
// counters, u-flags in the sync words, sc1 gathers): m is the gathered vector, double-buffered by iteration parity
// (m_{i+1} is written while other workgroups may still gather m_i: a workgroup passes barrier i + 1 only after every
// workgroup arrived, i.e. finished its SpMV of iteration i). State per row on chip: r, u, w, p, s, q, z, m in
// registers, x and the Jacobi weight in LDS; r, p, s, x and the GV vectors u, w, q, z in HBM between launches.
#pragma once
#include "pcg_persist.hpp"

namespace fem {

#ifndef FEM_GV_PROBE
#define FEM_GV_PROBE 0   // timing builds only (wrong results): 1 no barrier wait in the loop, 2 no m-flag wait
#endif

struct GvArgs {
    double* u;     // M^-1 r by recurrence
    double* w;     // A u by recurrence
    double* q;     // M^-1 s
    double* z;     // A q
    double* m[2];  // gathered m = w (.) w, by iteration parity
    int init;      // first launch after fem_pcg_start: form w0 = A u0 and m0, reduce gamma0 / delta0 (single GPU;
                   // DIST: PkArgs::init, which also forms r0 = b - A x0)
    int64_t moff[2];   // DIST: byte offsets of m[0] / m[1] in every rank's comm block (m[i] = own block + moff[i])
};

#ifndef FEM_GV_U1
#define FEM_GV_U1 8   // one-slot build: lane pairs in flight per slice
#endif
#ifndef FEM_GV_SYNCWAVE
#define FEM_GV_SYNCWAVE 0   // measured neutral (profiles/r06za_gv_syncwave_ab.txt): off
#endif
#ifndef FEM_GV_EARLY
#define FEM_GV_EARLY 1   // post gamma / delta and arrive before the x update and the m hand-off
#endif
constexpr bool GV_EARLY = FEM_GV_EARLY;
constexpr int GV_MAXS = 2;   // slices per wave (packed assignment)
// LDS: head (wave sums of gamma [0, 16), the ok word, the barrier sums [18, 20), wave sums of delta [20, 36)), then x
// and the Jacobi weights of the workgroup's rows
constexpr size_t GV_LDS_HEAD = 512;
#ifndef FEM_GV_BIGLDS
#define FEM_GV_BIGLDS 0   // A/B: the single-reduction LDS size; measured no different (profiles/r06zb_gv_biglds_ab.txt)
#endif
constexpr size_t GV_LDS = FEM_GV_BIGLDS ? PK_LDS : GV_LDS_HEAD + sizeof(double) * 2 * GV_MAXS * PK_WAVES * 64;

// arrival of this workgroup on the grid barrier of epoch e (thread 0; the caller drained the partial stores):
// pk_barrier's counters -- the arrival that completes a group adds to the 8 replicas of the top counter
__device__ __forceinline__ void gv_arrive(unsigned* sy, int grp, unsigned nper, unsigned e) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(sy + PK_GRP + grp * PK_LINE, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
#if FEM_GV_PROBE   // (timing builds: workgroups run epochs apart, so whichever add completes a group's count bumps)
    if ((old + 1) % nper == 0)
#else
    if (old == e * nper - 1)
#endif
        for (int r = 0; r < NXCD; ++r)
            __hip_atomic_fetch_add(sy + PK_GEN + r * PK_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait for every arrival of epoch e, then wave 0 sums the G partials of gamma (pg) and delta (pd) in fixed order
// (identical scalars in every workgroup) -> out[0], out[1]; a workgroup barrier hands them to the other waves
__device__ __forceinline__ bool gv_wait(unsigned* sy, int grp, unsigned e, int* lds_ok, const double* pg,
                                        const double* pd, int G, double* out) {
    if (threadIdx.x < 64) {
        int okv = 0;
        if (threadIdx.x == 0) okv = pk_wait_ge(sy + PK_GEN + grp * PK_LINE, e * NXCD, sy + PK_TMO) ? 1 : 0;
        okv = __builtin_amdgcn_readfirstlane(okv);
        if (okv) {
            const int lane = threadIdx.x & 63;
            double vg = 0.0, vd = 0.0;
#pragma unroll 4
            for (int i = lane; i < G; i += 64) {
                vg += __hip_atomic_load(pg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                vd += __hip_atomic_load(pd + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const double g = wave_sum(vg), d = wave_sum(vd);
            if (threadIdx.x == 0) {
                out[0] = g;
                out[1] = d;
            }
        }
        if (threadIdx.x == 0) *lds_ok = okv;
    }
    __syncthreads();
    return *lds_ok != 0;
}

// the two partial sums of this workgroup (waves in order), valid in thread 0; ends on a workgroup barrier after
// every wave drained its stores (the m rows of the update)
__device__ __forceinline__ void gv_block_sums(double a, double b, double* lds16, double* sa, double* sb, bool drain) {
    a = wave_sum(a);
    b = wave_sum(b);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        lds16[w] = a;
        lds16[PK_WAVES + 4 + w] = b;   // (after the ok word and the barrier sums of the head)
    }
    if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tb = 0.0;
#pragma unroll
        for (int i = 0; i < PK_WAVES; ++i) {
            ta += lds16[i];
            tb += lds16[PK_WAVES + 4 + i];
        }
        *sa = ta;
        *sb = tb;
    }
}

// DIST (rows partitioned over ranks, pcg_persist.hpp's comm blocks): the arrival half of pk_barrier_dist, called by
// wave 0 of every workgroup after thread 0 posted its partials. The arrival that completes the rank's count makes
// its wave sum the G partials (gamma in pg, delta in pd; fixed order) and announce them to every rank -- system
// stores into bank e & 1 of each rank's comm block, a system release, then epoch e on this rank's 8 replica lines
// there (one per XCD group).
__device__ __forceinline__ void gv_arrive_dist(const PkArgs& a, unsigned* sy, int grp, unsigned nper, unsigned e,
                                               const double* pg, const double* pd, int G) {
    const int lane = threadIdx.x & 63;
    int last = 0;
    if (lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(sy + PK_GRP + grp * PK_LINE, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old == e * nper - 1) {
            const unsigned old2 = __hip_atomic_fetch_add(sy + PK_GEN, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = old2 == e * NXCD - 1;
        }
    }
    last = __builtin_amdgcn_readfirstlane(last);
    if (last) {
        double vg = 0.0, vd = 0.0;
#pragma unroll 4
        for (int i = lane; i < G; i += 64) {
            vg += __hip_atomic_load(pg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            vd += __hip_atomic_load(pd + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const double g = wave_sum(vg), d = wave_sum(vd);
        const int bank = (int)(e & 1u);
        if (lane < a.nranks) {
            double* red = reinterpret_cast<double*>(a.peer[lane] + a.off_red) + (bank * PK_MAX_RANKS + a.rank) * 2;
            __hip_atomic_store(red, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(red + 1, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane < a.nranks * NXCD)
            __hip_atomic_store(reinterpret_cast<unsigned*>(a.peer[lane / NXCD] + a.off_rflag) +
                                   (a.rank * NXCD + lane % NXCD) * PK_LINE,
                               e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// DIST: the waiting half -- epoch e from every rank on this XCD group's replica lines, then the ranks' (gamma,
// delta) summed in rank order (identical bits on every rank) -> out[0], out[1]
__device__ __forceinline__ bool gv_wait_dist(const PkArgs& a, unsigned* sy, int grp, unsigned e, int* lds_ok,
                                             double* out) {
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        unsigned* tmo = sy + PK_TMO;
        const unsigned* rf = reinterpret_cast<const unsigned*>(a.peer[a.rank] + a.off_rflag);
        int okv = 1;
        bool done = lane >= a.nranks;
        const uint64_t t0 = pk_now();
        for (unsigned spins = 0; !__all(done); ++spins) {
            if (!done)
                done = __hip_atomic_load(rf + (lane * NXCD + grp) * PK_LINE, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) >= e;
            if ((spins & 63) == 63 && pk_ld(tmo)) {
                okv = 0;
                break;
            }
            if ((spins & 63) == 63 && pk_expired(t0, PK_RANK_WAIT_TICKS)) {
                pk_st(tmo, 3u + 16u * e);
                okv = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (okv) {
            const double* red = reinterpret_cast<const double*>(a.peer[a.rank] + a.off_red) +
                                (int)(e & 1u) * PK_MAX_RANKS * 2;
            double g = 0.0, d = 0.0;
            for (int q = 0; q < a.nranks; ++q) {   // rank order: the same sum on every rank
                g += __hip_atomic_load(red + 2 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                d += __hip_atomic_load(red + 2 * q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (lane == 0) {
                out[0] = g;
                out[1] = d;
            }
        }
        if (lane == 0) *lds_ok = okv;
    }
    __syncthreads();
    return *lds_ok != 0;
}

// DIST: row `row` of m (the region at byte offset moff of the comm blocks) also lands in the comm block of every
// rank in pubmask whose gathered range holds it (pk_publish_row for the m regions)
__device__ __forceinline__ void gv_publish_row(const PkArgs& a, int L, unsigned pubmask, unsigned row, double v,
                                               int64_t moff) {
    for (int q = 0; q < a.nranks; ++q) {
        if (!(pubmask & (1u << q))) continue;
        const int32_t* pr = a.pub + (L * a.nranks + q) * 2;
        if ((int)row >= pr[0] && (int)row < pr[1])
            __hip_atomic_store(reinterpret_cast<double*>(a.peer[q] + moff) + row, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int MAXS, bool DIST = false>
__global__ void __launch_bounds__(PK_T) k_pcg_persist_gv(PkArgs a, GvArgs gv) {
    static_assert(MAXS >= 1 && MAXS <= GV_MAXS, "slots per wave");
    // lane pairs in flight per slice (pk_u: 8 for one slot, 4 for two)
    constexpr int GU = MAXS == 1 ? FEM_GV_U1 : pk_u<MAXS, false>();
    static_assert(GV_LDS_HEAD >= sizeof(double) * (2 * PK_WAVES + 4), "LDS head: two sets of wave sums");
    extern __shared__ __attribute__((aligned(16))) double pk_lds_raw[];
    double* lds16 = pk_lds_raw;
    int& lds_ok = *reinterpret_cast<int*>(pk_lds_raw + PK_WAVES);
    double* lds_dg = pk_lds_raw + PK_WAVES + 2;
    double* pk_lds = pk_lds_raw + GV_LDS_HEAD / sizeof(double);
    const int G = gridDim.x;
    const unsigned nper = (unsigned)(G / NXCD);
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;   // XCD-contiguous logical order
    const int grp = L / (int)nper;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // packed assignment: a.pack (<= MAXS, host) slices per wave in order
    const int sL0 = (int)((int64_t)L * a.nslices / G);
    const int nL = (int)((int64_t)(L + 1) * a.nslices / G) - sL0;
    // FEM_GV_SYNCWAVE: when the workgroup's slices leave a wave free, wave 0 takes none -- it is the wave that polls
    // the grid barrier, which it then does while the other waves run the SpMV (the sums are read under it too)
    const int wsl = (FEM_GV_SYNCWAVE && nL <= (PK_WAVES - 1) * a.pack) ? wv - 1 : wv;
    const int lo = wsl < 0 ? nL : (wsl * a.pack < nL ? wsl * a.pack : nL);
    const int s0 = sL0 + lo + (DIST ? (int)a.sbase : 0);   // DIST: this rank's slices start at global slice sbase
    const int nreg = nL - lo < a.pack ? nL - lo : a.pack;
    const int nrows = (int)a.nrows;
    const unsigned rb = (unsigned)s0 * 64u + (unsigned)lane;
    double* xl = pk_lds + wv * MAXS * 64 + lane;
    double* wl = pk_lds + PK_WAVES * MAXS * 64 + wv * MAXS * 64 + lane;
    unsigned* sy = a.sync;
    PcgState* st = a.st;
    // m-flags: the sync words (single GPU), or the comm block's lines of all ranks' workgroups (DIST)
    unsigned* uf = DIST ? reinterpret_cast<unsigned*>(a.peer[a.rank] + a.off_flag) : sy + PK_UFLAG;
    const int Lg = DIST ? a.rank * G + L : L;
    const int olo = DIST ? (int)(a.sbase * 64) : 0;   // this rank's rows [olo, ohi)
    const int ohi = DIST ? (int)((a.sbase + a.nslices) * 64 < a.nrows ? (a.sbase + a.nslices) * 64 : a.nrows) : 0;
    unsigned pubmask = 0;   // DIST: ranks that gather rows of this workgroup
    bool ghost = false;     // DIST: this workgroup gathers rows of other ranks
    if constexpr (DIST) {
        for (int q = 0; q < a.nranks; ++q)
            if (q != a.rank && a.pub[(L * a.nranks + q) * 2] >= 0) pubmask |= 1u << q;
        ghost = a.win[L] < a.rank * G || a.win[G + L] >= (a.rank + 1) * G;
    }
#define GV_ON(j) ((j) < nreg && lane < nrows - (s0 + (j)) * 64)

    const double tol = st->tol;
    const int max_iter = st->max_iter;
    int it = st->iter, halt = st->halt, status = st->status, stop_iter = st->stop_iter;
    double gam_old = st->rz, alpha_prev = st->alpha, beta = st->beta, pq = st->pq, rz_new = st->rz_new;
    double gam = st->red[1], del = st->red[2];   // of the current iterate (reduced at the last launch's end)
    unsigned ep = st->pk_epoch;                   // last barrier / flag epoch used

    double rr[MAXS], uu[MAXS], ww[MAXS], pp[MAXS], ss[MAXS], qq[MAXS], zz[MAXS], mm[MAXS], nn[MAXS];
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
        const unsigned row = rb + 64u * j;
        const bool on = GV_ON(j);
        rr[j] = on ? a.r[row] : 0.0;
        pp[j] = on ? a.p[row] : 0.0;
        ss[j] = on ? a.s[row] : 0.0;
        xl[j * 64] = on ? a.x[row] : 0.0;
        const double wj = on ? a.w[row] : 0.0;
        wl[j * 64] = wj;
        uu[j] = on ? gv.u[row] : 0.0;
        ww[j] = on ? gv.w[row] : 0.0;
        qq[j] = on ? gv.q[row] : 0.0;
        zz[j] = on ? gv.z[row] : 0.0;
        mm[j] = wj * ww[j];   // how every m was formed: bit-identical, no load
        nn[j] = 0.0;
    }
    const int nflags = (DIST ? a.nranks : 1) * G;
    const int wraw0 = a.win[L], wraw1 = a.win[G + L];
    const int wlo = max(wraw0, 0), whi = min(wraw1, nflags - 1);
    bool fail = false;
    if (pk_window_bad(wraw0, wraw1, nflags)) {
        if (threadIdx.x == 0) pk_st(sy + PK_TMO, PK_SITE_WINDOW);
        fail = true;
    }
    const bool st_loaded = !halt;
    if (threadIdx.x == 0) lds_ok = 1;   // (read only after a workgroup barrier)
    const int64_t* slp = pk_launder(a.slice_ptr);
    const int16_t* cop = pk_launder(a.cols);
    const double* vap = pk_launder(a.vals);
    const int32_t* uop = a.uoff ? pk_launder(a.uoff) : nullptr;
    const int16_t* ucp = a.uoff ? pk_launder(a.ucol) : nullptr;
    static_assert(!DIST || GV_EARLY, "the distributed build posts its arrival in the update");
    // n[j] = (A v)[rows of slot j]: a workgroup whose gather window reaches other ranks reads their rows past this
    // GPU's L2 (mode 3, as k_pcg_persist's DIST build)
    auto spmv = [&](const double* v, double* out) {
        if (DIST && ghost) {
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) out[j] = sell_row_pair<GU, 3>(s0 + j, lane, slp, cop, vap, v, olo, ohi, uop, ucp);
                asm volatile("" ::: "memory");
            }
        } else {
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) out[j] = sell_row_pair<GU, 1>(s0 + j, lane, slp, cop, vap, v, olo, ohi, uop, ucp);
                asm volatile("" ::: "memory");
            }
        }
    };
    // a row of the gathered vector: this GPU's copy, and (DIST) the comm blocks of the ranks that gather it
    auto put_row = [&](double* dst, int64_t moff, unsigned row, double v) {
        __hip_atomic_store(dst + row, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (DIST) {
            if (pubmask) gv_publish_row(a, L, pubmask, row, v, moff);
        }
    };
    // thread 0, after every wave drained its row stores: the flag of epoch e here and (DIST) where rows were published
    auto raise_flag = [&](unsigned e) {
        pk_st(uf + Lg * PK_LINE, e);
        if constexpr (DIST) {
            if (pubmask) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                pk_publish_flag(a, Lg, pubmask, e);
            }
        }
    };
    // thread 0 posts this workgroup's (gamma, delta) partials of epoch e; the arrival (wave 0 for DIST)
    auto post_arrive = [&](unsigned e, double gs, double ds) {
        double* pb = a.part + (size_t)(e & 1u) * 2 * G;
        if (threadIdx.x == 0) {
            __hip_atomic_store(pb + L, gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(pb + G + L, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (DIST) {
            if (threadIdx.x < 64) gv_arrive_dist(a, sy, grp, nper, e, pb, pb + G, G);
        } else {
            if (threadIdx.x == 0) gv_arrive(sy, grp, nper, e);
        }
    };
    auto wait_sums = [&](unsigned e) -> bool {
        if constexpr (DIST) {
            return gv_wait_dist(a, sy, grp, e, &lds_ok, lds_dg);
        } else {
            double* pb = a.part + (size_t)(e & 1u) * 2 * G;
            return gv_wait(sy, grp, e, &lds_ok, pb, pb + G, G, lds_dg);
        }
    };
    // wave 0 waits for the flags of the gather window to reach e (bounded; a give-up fails the launch)
    auto wait_window = [&](unsigned e) -> bool {
        if (wv == 0 && !(FEM_GV_PROBE & 2)) {   // (probe 2, timing only: no m-flag wait)
            bool ok = true;
            for (int b0 = wlo; b0 <= whi && ok; b0 += 64) {
                const int jw = b0 + lane;
                bool done = jw > whi;
                const uint64_t t0 = pk_now();
                for (unsigned spins = 0; !__all(done); ++spins) {
                    if (!done)
                        done = (DIST ? __hip_atomic_load(uf + jw * PK_LINE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                     : pk_ld(uf + jw * PK_LINE)) >= e;
                    if ((spins & 63) == 63 && pk_ld(sy + PK_TMO)) {
                        ok = false;
                        break;
                    }
                    if ((spins & 63) == 63 && pk_expired(t0, PK_WAIT_TICKS)) {
                        pk_st(sy + PK_TMO, 2u + 16u * e);
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (lane == 0) {
                lds_ok = ok;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        return lds_ok != 0;
    };

    // ---- DIST first launch (the distributed counterpart of k_cg1_init + the single-GPU init below):
    //   phase A: r0 = b - A x0 over the own rows (x0 global-length, the same on every rank), u0 = w r0 published in
    //            the m[1] regions (epoch E1), a full barrier (gamma0 = r0.u0)
    //   phase B: w0 = A u0 (u0 gathered from the m[1] regions), m0 = w w0 published in the m[0] regions (epoch E2),
    //            gamma0 / delta0 = w0.u0 reduced by a full barrier
    // (update 0 writes m1 into m[1] only after the E2 barrier, i.e. after every rank's phase-B SpMV read u0 there)
    if constexpr (DIST) {
        if (a.init && !halt && !fail) {
            const double* xvp = pk_launder(a.x);
            double* mreg1 = gv.m[1];
            double gp = 0.0;
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) {
                    const double q = sell_row_pair<GU, 0>(s0 + j, lane, slp, cop, vap, xvp, 0, 0, uop, ucp);
                    const unsigned row = rb + 64u * j;
                    const bool on = GV_ON(j);
                    const double rv = on ? a.b[row] - q : 0.0;
                    const double wj = wl[j * 64];
                    rr[j] = rv;
                    uu[j] = wj * rv;
                    pp[j] = ss[j] = qq[j] = zz[j] = 0.0;
                    if (on) put_row(mreg1, gv.moff[1], row, uu[j]);
                    gp += rr[j] * uu[j];
                }
                asm volatile("" ::: "memory");
            }
            double gs = 0.0, ds = 0.0;
            gv_block_sums(gp, 0.0, lds16, &gs, &ds, true);   // (every wave drained its u0 rows)
            const unsigned e1 = ep + 1;
            if (threadIdx.x == 0) raise_flag(e1);
            post_arrive(e1, gs, 0.0);
            if (!wait_sums(e1)) fail = true;
            ep = e1;
            if (!fail && wait_window(e1)) {
                spmv(mreg1, nn);
                double gp2 = 0.0, dp2 = 0.0;
#pragma unroll
                for (int j = 0; j < MAXS; ++j) {
                    if (j < nreg) {
                        const unsigned row = rb + 64u * j;
                        const bool on = GV_ON(j);
                        ww[j] = on ? nn[j] : 0.0;
                        mm[j] = wl[j * 64] * ww[j];
                        if (on) put_row(gv.m[0], gv.moff[0], row, mm[j]);
                        gp2 += rr[j] * uu[j];
                        dp2 += ww[j] * uu[j];
                    }
                }
                gv_block_sums(gp2, dp2, lds16, &gs, &ds, true);
                const unsigned e2 = ep + 1;
                if (threadIdx.x == 0) raise_flag(e2);
                post_arrive(e2, gs, ds);
                if (!wait_sums(e2)) {
                    fail = true;
                } else {
                    gam = lds_dg[0];
                    del = lds_dg[1];
                    gam_old = gam;
                }
                ep = e2;
            } else {
                fail = true;
            }
        }
    }

    // ---- first launch: w0 = A u0 (u0 = w r0 in a.u, written by k_cg1_init before this launch), m0, gamma0, delta0
    if (!DIST && gv.init && !halt && !fail) {
        const double* u0 = pk_launder(a.u);
        double gp = 0.0, dp = 0.0;
#pragma unroll
        for (int j = 0; j < MAXS; ++j) {
            if (j < nreg) {
                const double v = sell_row_pair<GU, 1>(s0 + j, lane, slp, cop, vap, u0, 0, 0, uop, ucp);
                const unsigned row = rb + 64u * j;
                const bool on = GV_ON(j);
                const double wj = wl[j * 64];
                uu[j] = wj * rr[j];   // k_cg1_init's u0, bit for bit
                ww[j] = on ? v : 0.0;
                mm[j] = wj * ww[j];
                pp[j] = ss[j] = qq[j] = zz[j] = 0.0;
                if (on) __hip_atomic_store(gv.m[0] + row, mm[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gp += rr[j] * uu[j];
                dp += ww[j] * uu[j];
            }
            asm volatile("" ::: "memory");
        }
        double gs = 0.0, ds = 0.0;
        gv_block_sums(gp, dp, lds16, &gs, &ds, true);
        const unsigned e = ep + 1;
        double* pb = a.part + (size_t)(e & 1u) * 2 * G;
        if (threadIdx.x == 0) {
            __hip_atomic_store(pb + L, gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(pb + G + L, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pk_st(uf + L * PK_LINE, e);   // m0 of this workgroup's rows
            gv_arrive(sy, grp, nper, e);
        }
        if (!wait_sums(e)) {
            fail = true;
        } else {
            gam = lds_dg[0];
            del = lds_dg[1];
            gam_old = gam;
        }
        ep = e;
    }

    int k = 0;
    if (!halt && !fail) {
        for (k = 0; k < a.kmax; ++k) {
            // ---- the arrival of this iteration (its partials were posted by the last update), then the m window
            if (!GV_EARLY && k > 0 && threadIdx.x == 0) gv_arrive(sy, grp, nper, ep);
            if (!wait_window(ep)) {
                fail = true;
                break;
            }
            // ---- n = A m (m of this iteration's parity), while the barrier completes
            spmv(pk_launder((it & 1) ? gv.m[1] : gv.m[0]), nn);   // (no dynamic kernarg index)
            // ---- gamma, delta of this iterate
            if (k > 0 && !(FEM_GV_PROBE & 1)) {   // (probe 1, timing only: no wait, stale scalars)
                if (!wait_sums(ep)) {
                    fail = true;
                    break;
                }
                gam = lds_dg[0];
                del = lds_dg[1];
            }
            // ---- step (the single-reduction step's tests: stop on sqrt(r.u) < tol, `solver/solver.py:805`)
            double bnew = 0.0;
            bool stop = false;
            if (it > 0) {
                rz_new = gam;
                const double nrm = sqrt(gam);
                if (L == 0 && threadIdx.x == 0 && a.hist && it - 1 < a.hist_len) a.hist[it - 1] = nrm;
                if (nrm < tol) {
                    status = FEM_PCG_CONVERGED;
                    stop_iter = it;
                    stop = true;
                } else {
                    bnew = gam / gam_old;
                }
            }
            if (!stop && it >= max_iter) stop = true;
            double al = 0.0;
            if (!stop) {
                pq = (it == 0) ? del : del - bnew * gam / alpha_prev;
                al = gam / pq;
            }
            if (stop) {
                halt = 1;
                break;
            }
            gam_old = gam;
            alpha_prev = al;
            beta = bnew;
            // ---- update the own rows, post m of the next iteration and its gamma / delta partials
            double gp = 0.0, dp = 0.0;
            double* mst = pk_launder((it & 1) ? gv.m[0] : gv.m[1]);   // m of iteration it + 1
            unsigned rbi = rb;
            asm volatile("" : "+v"(rbi));
            const unsigned e = ep + 1;
            if constexpr (GV_EARLY) {
                // the vectors gamma / delta need first, their partials posted and the arrival on barrier e made at
                // once; x and the hand-off of m follow (the arrival no longer waits for the m stores to drain)
#pragma unroll
                for (int j = 0; j < MAXS; ++j) {
                    if (j < nreg) {
                        zz[j] = nn[j] + bnew * zz[j];
                        qq[j] = mm[j] + bnew * qq[j];
                        ss[j] = ww[j] + bnew * ss[j];
                        pp[j] = uu[j] + bnew * pp[j];
                        rr[j] = rr[j] - al * ss[j];
                        uu[j] = uu[j] - al * qq[j];
                        ww[j] = ww[j] - al * zz[j];
                        gp += rr[j] * uu[j];
                        dp += ww[j] * uu[j];
                    }
                }
                double gs = 0.0, ds = 0.0;
                gv_block_sums(gp, dp, lds16, &gs, &ds, false);
                post_arrive(e, gs, ds);
                const int64_t moff = (it & 1) ? gv.moff[0] : gv.moff[1];
#pragma unroll
                for (int j = 0; j < MAXS; ++j) {
                    if (j < nreg) {
                        xl[j * 64] += al * pp[j];
                        mm[j] = wl[j * 64] * ww[j];
                        if (GV_ON(j)) put_row(mst, moff, rbi + 64u * j, mm[j]);
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its m stores
                __syncthreads();
                if (threadIdx.x == 0) raise_flag(e);
            } else {
#pragma unroll
                for (int j = 0; j < MAXS; ++j) {
                    if (j < nreg) {
                        zz[j] = nn[j] + bnew * zz[j];
                        qq[j] = mm[j] + bnew * qq[j];
                        ss[j] = ww[j] + bnew * ss[j];
                        pp[j] = uu[j] + bnew * pp[j];
                        xl[j * 64] += al * pp[j];
                        rr[j] = rr[j] - al * ss[j];
                        uu[j] = uu[j] - al * qq[j];
                        ww[j] = ww[j] - al * zz[j];
                        mm[j] = wl[j * 64] * ww[j];
                        if (GV_ON(j))
                            __hip_atomic_store(mst + (rbi + 64u * j), mm[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        gp += rr[j] * uu[j];
                        dp += ww[j] * uu[j];
                    }
                }
                double gs = 0.0, ds = 0.0;
                gv_block_sums(gp, dp, lds16, &gs, &ds, true);   // (every wave drained its m stores)
                if (threadIdx.x == 0) {
                    double* pb = a.part + (size_t)(e & 1u) * 2 * G;
                    __hip_atomic_store(pb + L, gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pb + G + L, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    pk_st(uf + L * PK_LINE, e);
                }
            }
            it += 1;
            ep = e;
        }
    }
    // ---- chunk end without a stop: reduce the posted gamma / delta (the next launch starts from them); stop test
    if (!fail && !halt && k == a.kmax && a.kmax > 0) {
        if (!GV_EARLY && threadIdx.x == 0) gv_arrive(sy, grp, nper, ep);   // (GV_EARLY: arrived in the update)
        if (!wait_sums(ep)) {
            fail = true;
        } else {
            gam = lds_dg[0];
            del = lds_dg[1];
            if (it > 0) {
                const double nrm = sqrt(gam);
                rz_new = gam;
                if (nrm < tol || it >= max_iter) {
                    if (L == 0 && threadIdx.x == 0 && a.hist && it - 1 < a.hist_len) a.hist[it - 1] = nrm;
                    if (nrm < tol) {
                        status = FEM_PCG_CONVERGED;
                        stop_iter = it;
                    }
                    halt = 1;
                }
            }
        }
    }
    if (st_loaded) {
#pragma unroll
        for (int j = 0; j < MAXS; ++j) {
            if (GV_ON(j)) {
                const unsigned row = rb + 64u * j;
                a.r[row] = rr[j];
                a.p[row] = pp[j];
                a.s[row] = ss[j];
                a.x[row] = xl[j * 64];
                gv.u[row] = uu[j];
                gv.w[row] = ww[j];
                gv.q[row] = qq[j];
                gv.z[row] = zz[j];
            }
        }
    }
    if (L == 0 && threadIdx.x == 0) {
        if (fail) {
            stop_iter = (int)pk_ld(sy + PK_TMO);
            status = pk_fail_status((unsigned)stop_iter);
            halt = 1;
        }
        st->iter = it;
        st->halt = halt;
        st->status = status;
        st->stop_iter = stop_iter;
        st->rz = gam_old;
        st->rz_new = rz_new;
        st->alpha = alpha_prev;
        st->beta = beta;
        st->pq = pq;
        st->red[1] = gam;
        st->red[2] = del;
        st->pk_epoch = ep;
    }
#undef GV_ON
}

}  // namespace fem
