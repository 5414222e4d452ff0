// Persistent Jacobi-PCG for 3x3-block systems (schedule 3, bs = 3: elasticity), the block counterpart of
// k_pcg_persist (pcg_persist.hpp): the same single-reduction (Chronopoulos–Gear) iteration, slice assignment,
// u hand-off (sc1 stores + drained per-workgroup flags), XCD-hierarchical grid barrier with fixed-order sums, stop
// test / guards and DIST rank exchange, with three dofs per SELL row. A wave keeps up to P3_MAXS slices on chip --
// r, p, s in registers (its own u = w r recomputed, not carried), x, w and v = A u in LDS (3 x 64 doubles per slice
// each) -- and, in the
// overflow build, streams the CG state of its further slices from HBM (r, p, s, x, u, w arrays, v in a.v) inside
// the same launch and barriers. The matrix is the plane-paired layout A copy (sell_pair3.hpp, 9 values per block in
// 5 loads) with 16-bit node-column deltas; the u gathers are agent-scope (sc1) loads, system-scope for columns of
// other ranks (DIST).
//   10M-tet elasticity on one GPU: 27,000 slices over 4,096 waves -> 2 on chip + ~5 streamed per wave (the state,
//   7 x 41.5 MB, exceeds the chip's registers + LDS); the same system over 8 ranks: <= 1 slice per wave, all on chip.
#pragma once
#include "pcg_persist.hpp"
#include "sell_pair3.hpp"

namespace fem {

constexpr int P3_MAXS = 2;   // on-chip slices per wave
constexpr int P3_U = 1;      // blocks in flight per lane in the SpMV (2 spills the slot state)
// LDS: head, then x, w, v of the on-chip slices: [vector][wave][slot][component][lane]
constexpr size_t P3_LDS = PK_LDS_HEAD + sizeof(double) * 3 * PK_WAVES * P3_MAXS * 3 * 64;
static_assert(P3_LDS <= 160 * 1024, "persistent bs=3 PCG: LDS over the 160 KB of a CU");

// y (3 rows) of lane `lane` in slice s, layout A, u gathers in hand-off mode MODE (1: sc1; 3: per column, system
// scope outside this rank's dof range [own_lo, own_hi)); U entries in flight. Summation order = sell3_row_a.
template <int U, int MODE>
__device__ __forceinline__ void sell3_row_pk(int64_t s, int lane, const int64_t* __restrict__ slice_ptr,
                                             const int16_t* __restrict__ cols, const double* __restrict__ vals,
                                             const double* __restrict__ x, int own_lo, int own_hi, double out[3]) {
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
        for (int u = 0; u < U; ++u) cc[u] = (k0 + u < w) ? 3 * (base + (int)c[64 * (k0 + u)]) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double* ch = vb + 576 * (int64_t)(k0 + u);
            const double2* c2 = reinterpret_cast<const double2*>(ch) + lane;
            if (k0 + u < w) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const double2 d = c2[64 * t];
                    vv[u][2 * t] = d.x;
                    vv[u][2 * t + 1] = d.y;
                }
                vv[u][8] = ch[512 + lane];
            } else {
#pragma unroll
                for (int e = 0; e < 9; ++e) vv[u][e] = 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 3; ++j) xv[u][j] = (k0 + u < w) ? ldx_col<MODE>(x, cc[u] + j, own_lo, own_hi) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < w) blk3_fma(out, vv[u], xv[u]);
    }
}

// DIST: the 3 dofs of node row `row` also land in the comm block of every rank in pubmask whose gathered node range
// holds it
__device__ __forceinline__ void p3_publish_row(const PkArgs& a, int L, unsigned pubmask, unsigned row, const double* v) {
    for (int q = 0; q < a.nranks; ++q) {
        if (!(pubmask & (1u << q))) continue;
        const int32_t* pr = a.pub + (L * a.nranks + q) * 2;
        if ((int)row >= pr[0] && (int)row < pr[1])
#pragma unroll
            for (int c = 0; c < 3; ++c)
                __hip_atomic_store(reinterpret_cast<double*>(a.peer[q]) + 3 * (size_t)row + c, v[c], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#define P3_ON(j) ((j) < nreg && lane < nrows - (s0 + (j)) * 64)

template <int MAXS, bool OVF = false, bool DIST = false>
__global__ void __launch_bounds__(PK_T) k_pcg_persist3(PkArgs a) {
    static_assert(!DIST || !OVF, "distributed persistent PCG: no overflow build");
    static_assert(MAXS <= P3_MAXS, "LDS sized for P3_MAXS slices per wave");
    extern __shared__ __attribute__((aligned(16))) double p3_lds_raw[];
    double* lds16 = p3_lds_raw;
    int& lds_ok = *reinterpret_cast<int*>(p3_lds_raw + PK_WAVES);
    double* lds_dg = p3_lds_raw + PK_WAVES + 2;
    double* lds = p3_lds_raw + PK_LDS_HEAD / sizeof(double);
    const int G = gridDim.x;
    const unsigned nper = (unsigned)(G / NXCD);
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;   // XCD-contiguous logical order
    const int grp = L / (int)nper;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // packed slice assignment (k_pcg_persist): a.pack slices per wave in order
    const int m = a.pack;
    const int sL0 = (int)((int64_t)L * a.nslices / G);
    const int nL = (int)((int64_t)(L + 1) * a.nslices / G) - sL0;
    const int lo0 = wv * m < nL ? wv * m : nL;
    const int s0 = sL0 + lo0 + (DIST ? (int)a.sbase : 0);
    const int nsl = nL - lo0 < m ? nL - lo0 : m;
    const int nreg = (OVF && nsl > MAXS) ? MAXS : nsl;
    const int nov = nsl - nreg;
    const int nrows = (int)a.nrows;
    const unsigned rb = (unsigned)s0 * 64u + (unsigned)lane;
    constexpr int VS = PK_WAVES * P3_MAXS * 3 * 64;   // doubles per LDS vector
    double* xl = lds + (wv * P3_MAXS * 3) * 64 + lane;   // component c of slot j at [(j * 3 + c) * 64]
    double* wl = xl + VS;
    double* vl = xl + 2 * VS;
    unsigned* sy = a.sync;
    PcgState* st = a.st;
    unsigned* uf = DIST ? reinterpret_cast<unsigned*>(a.peer[a.rank] + a.off_flag) : sy + PK_UFLAG;
    const int Lg = DIST ? a.rank * G + L : L;
    const int olo = DIST ? (int)(a.sbase * 64) * 3 : 0;   // this rank's dofs [olo, ohi)
    const int ohi = DIST ? (int)((a.sbase + a.nslices) * 64 < a.nrows ? (a.sbase + a.nslices) * 64 : a.nrows) * 3 : 0;
    unsigned pubmask = 0;
    bool ghost = false;
    if constexpr (DIST) {
        for (int q = 0; q < a.nranks; ++q)
            if (q != a.rank && a.pub[(L * a.nranks + q) * 2] >= 0) pubmask |= 1u << q;
        ghost = a.win[L] < a.rank * G || a.win[G + L] >= (a.rank + 1) * G;
    }

    const bool cg = st->mode != FEM_MODE_PCG;
    const double tol = st->tol, eps = st->eps;
    const int max_iter = st->max_iter;
    int it = st->iter, halt = st->halt, status = st->status, stop_iter = st->stop_iter;
    double rz = st->rz, alpha_prev = st->alpha, beta = st->beta, pq = st->pq, rz_new = st->rz_new;
    double g = st->red[1];
    unsigned ebase = st->pk_epoch;
    unsigned elast = ebase;

    // own u = w r is not carried: recomputed from w (LDS) and r, the same product that formed every stored u
    double rr[MAXS][3], pp[MAXS][3], ss[MAXS][3];
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
        const bool on = P3_ON(j);
        const size_t d0 = 3 * (size_t)(rb + 64u * j);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            rr[j][c] = on ? a.r[d0 + c] : 0.0;
            pp[j][c] = on ? a.p[d0 + c] : 0.0;
            ss[j][c] = on ? a.s[d0 + c] : 0.0;
            xl[(j * 3 + c) * 64] = on ? a.x[d0 + c] : 0.0;
            const double wj = on ? a.w[d0 + c] : 0.0;
            wl[(j * 3 + c) * 64] = wj;
            vl[(j * 3 + c) * 64] = 0.0;
        }
    }
    // clamped to the flag array (nranks * G workgroups): a window is never an index outside it, whatever the
    // array holds; a window outside it is reported (FEM_PCG_BAD_WINDOW, every spinner released), not run
    const int nflags = (DIST ? a.nranks : 1) * G;
    const int wraw0 = a.win[L], wraw1 = a.win[G + L];
    const int wlo = max(wraw0, 0), whi = min(wraw1, nflags - 1);
    bool fail = false;
    if (pk_window_bad(wraw0, wraw1, nflags)) {
        if (threadIdx.x == 0) pk_st(sy + PK_TMO, PK_SITE_WINDOW);
        fail = true;
    }
    bool st_loaded = !halt;
    int k = 0;
    if constexpr (DIST) {
        // first launch of a distributed solve: r0 = b - A x0 over the own rows, u0 = w r0 published, r0.u0 summed
        if (a.init && !halt) {
            const int64_t* slp = pk_launder(a.slice_ptr);
            const int16_t* cop = pk_launder(a.cols);
            const double* vap = pk_launder(a.vals);
            const double* xvp = pk_launder(a.x);
            double gp = 0.0;
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) {
                    double q[3];
                    sell3_row_pk<1, 0>(s0 + j, lane, slp, cop, vap, xvp, 0, 0, q);
                    const unsigned row = rb + 64u * j;
                    const bool on = P3_ON(j);
                    double uv[3];
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const size_t d = 3 * (size_t)row + c;
                        double rv = on ? a.b[d] - q[c] : 0.0;
                        const double wj = wl[(j * 3 + c) * 64];
                        if (cg && wj == 0.0) rv = 0.0;
                        rr[j][c] = rv;
                        pp[j][c] = 0.0;
                        ss[j][c] = 0.0;
                        xl[(j * 3 + c) * 64] = on ? a.x[d] : 0.0;
                        uv[c] = wj * rv;
                        gp += rv * uv[c];
                        if (on) __hip_atomic_store(a.u + d, uv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (on && pubmask) p3_publish_row(a, L, pubmask, row, uv);
                }
                asm volatile("" ::: "memory");
            }
            {
                const double gw = wave_sum(gp);
                if (lane == 0) lds16[wv] = gw;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const unsigned e0 = ebase + 1;
            double* pg0 = a.part + 2 * (size_t)G;
            if (threadIdx.x == 0) {
                double gsum = 0.0;
#pragma unroll
                for (int i = 0; i < PK_WAVES; ++i) gsum += lds16[i];
                __hip_atomic_store(pg0 + L, gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                pk_st(uf + Lg * PK_LINE, e0);
                if (pubmask) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    pk_publish_flag(a, Lg, pubmask, e0);
                }
            }
            st_loaded = true;
            if (!pk_barrier_dist(a, sy, grp, nper, e0, &lds_ok, pg0, nullptr, G, lds_dg)) {
                fail = true;
            } else {
                g = lds_dg[0];
                rz = g;
                ebase = e0;
                elast = e0;
            }
        }
    }
    if (!halt && !fail) {
        for (k = 0; k < a.kmax; ++k) {
            const unsigned e = ebase + (unsigned)k + 1;
            if (k > 0 || (DIST && a.init)) {   // u of the gather window (previous update, or the DIST init)
                if (wv == 0) {
                    bool ok = true;
                    for (int b0 = wlo; b0 <= whi && ok; b0 += 64) {
                        const int jw = b0 + lane;
                        bool done = jw > whi;
                        const uint64_t t0 = pk_now();
                        for (unsigned spins = 0; !__all(done); ++spins) {
                            if (!done)
                                done = (DIST ? __hip_atomic_load(uf + jw * PK_LINE, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_SYSTEM)
                                             : pk_ld(uf + jw * PK_LINE)) >= e - 1;
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
                if (!lds_ok) {
                    fail = true;
                    break;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            // ---- v = A u over the own slices (sweep direction alternating by iteration parity), d partial
            const bool rv = a.rev && ((it & 1) != 0);
            const int64_t* slp = pk_launder(a.slice_ptr);
            const int16_t* cop = pk_launder(a.cols);
            const double* vap = pk_launder(a.vals);
            const double* uvp = pk_launder(a.u);
#define P3_SPMV(MODE)                                                                              \
    _Pragma("unroll") for (int jj = 0; jj < MAXS; ++jj) {                                          \
        const int j = rv ? MAXS - 1 - jj : jj;                                                     \
        if (j < nreg) {                                                                            \
            double v[3];                                                                           \
            sell3_row_pk<P3_U, MODE>(s0 + j, lane, slp, cop, vap, uvp, olo, ohi, v);                  \
            _Pragma("unroll") for (int c = 0; c < 3; ++c) vl[(j * 3 + c) * 64] = v[c];             \
        }                                                                                          \
        asm volatile("" ::: "memory");                                                             \
    }
            if (DIST && ghost) {
                P3_SPMV(3)
            } else {
                P3_SPMV(1)
            }
#undef P3_SPMV
            double dp = 0.0;
#pragma unroll
            for (int j = 0; j < MAXS; ++j)
#pragma unroll
                for (int c = 0; c < 3; ++c)   // absent rows: w = r = 0
                    dp += (wl[(j * 3 + c) * 64] * rr[j][c]) * vl[(j * 3 + c) * 64];
            if constexpr (OVF) {   // overflow slices: v to HBM, u.v from the own u (this lane stored it last update)
                __builtin_amdgcn_sched_barrier(0);
                for (int q = 0; q < nov; ++q) {
                    const int sq = s0 + MAXS + q;
                    double v[3];
                    sell3_row_pk<P3_U, 1>(sq, lane, slp, cop, vap, uvp, 0, 0, v);
                    const int row = sq * 64 + lane;
                    if (row < nrows)
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            a.v[3 * (size_t)row + c] = v[c];
                            dp += a.u[3 * (size_t)row + c] * v[c];
                        }
                }
            }
            const int bank = k & 1;
            double* pd = a.part + (size_t)bank * 2 * G;
            __builtin_amdgcn_sched_barrier(0);
            const double dsum = pk_block_sum(dp, lds16);
            if (threadIdx.x == 0) __hip_atomic_store(pd + L, dsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!(DIST ? pk_barrier_dist(a, sy, grp, nper, e, &lds_ok, pd, k > 0 ? pd + G : nullptr, G, lds_dg, false)
                       : pk_barrier(sy, grp, nper, e, &lds_ok, pd, k > 0 ? pd + G : nullptr, G, lds_dg, false))) {
                fail = true;
                break;
            }
            elast = e;
            const double d = lds_dg[0];
            if (k > 0) g = lds_dg[1];
            // ---- step (k_cg1_step; identical to k_pcg_persist)
            double bnew = 0.0;
            bool stop = false;
            if (it > 0) {
                rz_new = g;
                const double nrm = sqrt(g);
                if (L == 0 && threadIdx.x == 0 && a.hist && it - 1 < a.hist_len) a.hist[it - 1] = nrm;
                if (nrm < tol) {
                    status = FEM_PCG_CONVERGED;
                    stop_iter = it;
                    stop = true;
                } else {
                    bnew = cg ? g / (rz + eps) : g / rz;
                    if (cg && (isnan(bnew) || isinf(bnew))) {
                        status = FEM_PCG_BETA_NAN;
                        stop_iter = it;
                        stop = true;
                    }
                }
            }
            if (!stop && it >= max_iter) stop = true;
            double al = 0.0;
            if (!stop) {
                pq = (it == 0) ? d : d - bnew * g / alpha_prev;
                if (cg) {
                    if (fabs(pq) < eps || pq < 0.0) {
                        status = FEM_PCG_BREAKDOWN;
                        stop_iter = it + 1;
                        stop = true;
                    } else {
                        al = g / (pq + eps);
                        if (isnan(al) || isinf(al)) {
                            status = FEM_PCG_ALPHA_NAN;
                            stop_iter = it + 1;
                            stop = true;
                        }
                    }
                } else {
                    al = g / pq;
                }
            }
            if (stop) {
                halt = 1;
                break;
            }
            rz = g;
            alpha_prev = al;
            beta = bnew;
            it += 1;
            __builtin_amdgcn_sched_barrier(0);
            // ---- update the own rows, publish u and the g partial
            double gp = 0.0;
            unsigned rbi = rb;
            double* ust = pk_launder(a.u);
            asm volatile("" : "+v"(rbi));
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) {
                    double uv[3];
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const int o = (j * 3 + c) * 64;
                        const double wi = wl[o];
                        const double pi = wi * rr[j][c] + bnew * pp[j][c];
                        const double si = vl[o] + bnew * ss[j][c];
                        pp[j][c] = pi;
                        ss[j][c] = si;
                        xl[o] += al * pi;
                        double ri = rr[j][c] - al * si;
                        if (cg && wi == 0.0) ri = 0.0;
                        rr[j][c] = ri;
                        const double ui = wi * ri;
                        uv[c] = ui;
                        gp += ri * ui;
                    }
                    if (P3_ON(j)) {
                        const size_t d0 = 3 * (size_t)(rbi + 64u * j);
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            __hip_atomic_store(ust + d0 + c, uv[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if constexpr (DIST) {
                            if (pubmask) p3_publish_row(a, L, pubmask, rbi + 64u * j, uv);
                        }
                    }
                }
            }
            if constexpr (OVF) {
                __builtin_amdgcn_sched_barrier(0);
                for (int q = 0; q < nov; ++q) {
                    const int row = (s0 + MAXS + q) * 64 + lane;
                    if (row < nrows)
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const size_t i = 3 * (size_t)row + c;
                            const double pi = a.u[i] + bnew * a.p[i];
                            const double si = a.v[i] + bnew * a.s[i];
                            a.p[i] = pi;
                            a.s[i] = si;
                            a.x[i] += al * pi;
                            double ri = a.r[i] - al * si;
                            const double wi = a.w[i];
                            if (cg && wi == 0.0) ri = 0.0;
                            a.r[i] = ri;
                            const double ui = wi * ri;
                            __hip_atomic_store(ust + i, ui, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            gp += ri * ui;
                        }
                }
            }
            {
                const double gw = wave_sum(gp);
                if (lane == 0) lds16[wv] = gw;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                double gsum = 0.0;
#pragma unroll
                for (int i = 0; i < PK_WAVES; ++i) gsum += lds16[i];
                __hip_atomic_store(a.part + (size_t)(bank ^ 1) * 2 * G + G + L, gsum, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                pk_st(uf + Lg * PK_LINE, e);
                if constexpr (DIST) {
                    if (pubmask) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        pk_publish_flag(a, Lg, pubmask, e);
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    auto store_state = [&]() {
        if (!st_loaded) return;
#pragma unroll
        for (int j = 0; j < MAXS; ++j) {
            if (P3_ON(j)) {
                const size_t d0 = 3 * (size_t)(rb + 64u * j);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    a.r[d0 + c] = rr[j][c];
                    a.p[d0 + c] = pp[j][c];
                    a.s[d0 + c] = ss[j][c];
                    a.x[d0 + c] = xl[(j * 3 + c) * 64];
                }
            }
        }
    };
    if (wv != 0) store_state();
    if (!fail && !halt && k == a.kmax && a.kmax > 0) {   // chunk end: the last g partials, stop test of that g
        const unsigned e = ebase + (unsigned)a.kmax + 1;
        const double* pgl = a.part + (size_t)(a.kmax & 1) * 2 * G + G;
        const bool okb = DIST ? pk_barrier_dist(a, sy, grp, nper, e, &lds_ok, pgl, nullptr, G, lds_dg)
                              : pk_barrier(sy, grp, nper, e, &lds_ok, pgl, nullptr, G, lds_dg);
        if (!okb) {
            fail = true;
        } else {
            elast = e;
            g = lds_dg[0];
            if (it > 0) {
                const double nrm = sqrt(g);
                const bool conv = nrm < tol;
                rz_new = g;
                if (conv || it >= max_iter) {
                    if (L == 0 && threadIdx.x == 0 && a.hist && it - 1 < a.hist_len) a.hist[it - 1] = nrm;
                    if (conv) {
                        status = FEM_PCG_CONVERGED;
                        stop_iter = it;
                    }
                    halt = 1;
                }
            }
        }
    }
    if (wv == 0) store_state();
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
        st->rz = rz;
        st->rz_new = rz_new;
        st->alpha = alpha_prev;
        st->beta = beta;
        st->pq = pq;
        st->red[1] = g;
        st->pk_epoch = elast;
    }
}
#undef P3_ON

}  // namespace fem
