// Persistent PIPELINED Jacobi-PCG (schedule 4, bs = 1 with the lane-paired matrix copy).
//
// The same Jacobi-PCG as schedule 3 (pcg_persist.hpp) in its pipelined form (Ghysels & Vanroose 2014, "Hiding
// global synchronization latency in the preconditioned Conjugate Gradient algorithm", Alg. 3, with the diagonal
// preconditioner D = w folded in: u = D r, m = D a, q = D s are never stored). Carried per row: x, r, a (= A u by
// recurrence), s, p, z; the SpMV of an iteration is n = A m, and the two dot products it needs,
//     gamma = r.u and delta = a.u,
// are formed by the PREVIOUS update. So the grid-wide sum no longer sits between the SpMV and the update: every
// workgroup publishes its partials together with its m rows, and by the time any workgroup has finished its own
// SpMV the partials of all the others are (almost always) there. There is no grid barrier at all:
//
//   per iteration (epoch E = ebase + local iteration + 1):
//     wait   : one wave polls the flags of the workgroups in this workgroup's gather window (>= E - 1: their m of
//              the last update is stored)
//     SpMV   : n = A m over the own slices (m double-buffered by epoch parity: a workgroup may already write the
//              next m while a slower neighbour still gathers this one; the next write after that waits for the
//              neighbour's flag, so two buffers suffice)
//     reduce : the last wave (fewest slices) polls ALL G flags >= E - 1, then sums the G partials of gamma and delta
//              in fixed order (identical bits in every workgroup) and leaves them in LDS
//     step   : stop test on gamma (`solver/solver.py:210` / `:805`), beta = gamma / gamma_prev,
//              alpha = gamma / (delta - beta gamma / alpha_prev), the same scalar recurrence and guards as schedule 3
//     update : z = n + beta z, s = a + beta s, p = D r + beta p, x += alpha p, r -= alpha s (CG: masked),
//              a -= alpha z, m = D a stored sc1; gamma / delta partials stored sc1; drain; flag = E
// Partials are banked by epoch parity for the same reason as m (the reduce wait of the next iteration proves that
// every reader of the older bank is done). Rounding differs from schedule 3 (a = A u is carried by recurrence); the
// contract is the survey's: iterations +-2, solutions 1e-10 (tests/test_gpu_parity.py).
// Geometry: NW waves per workgroup, one workgroup per CU (LDS pins it), MAXS register slots of 64 rows per wave;
// r, a, s, p, z and (MAXS - VL) n slots in registers; x, D and VL n slots in LDS.
#pragma once
#include "pcg_persist.hpp"

namespace fem {

struct PpArgs {
    int64_t nslices, nrows;
    const int64_t* slice_ptr;
    const int16_t* cols;    // lane-paired copy (sell_pair.hpp)
    const double* vals;
    double* x;
    double* r;
    double* av;             // a = A u (carried)
    double* s;
    double* p;
    double* z;
    double* m0;             // m = D a, double-buffered by epoch parity (gathered by the SpMV)
    double* m1;
    const double* w;
    const int32_t* win;     // [2 G] gather window per logical workgroup
    double* part;           // [2 banks][2 (gamma, delta)][G]
    unsigned* flag;         // [G] lines: epoch of the workgroup's last published update
    unsigned* tmo;          // give-up word
    PcgState* st;
    double* hist;
    int64_t hist_len;
    int kmax;
    int rev;
    int pack;               // slices per wave (packed assignment, <= MAXS)
    unsigned long long* prof;
};

constexpr int PP_NPROF = 8;   // phases: wait, SpMV, reduce, (unused), step, update + publish, prologue, epilogue
// LDS head: [16] wave sums of gamma, [16] of delta, the verdict word (own 16-byte slot), reduced gamma / delta
constexpr size_t PP_LDS_HEAD = 512;

template <int NW, int MAXS, int VL>
constexpr size_t pp_lds_bytes() {
    return PP_LDS_HEAD + sizeof(double) * (size_t)(2 * MAXS + VL) * NW * 64;
}

// one wave: all G flags >= target (bounded spin; false on give-up), then the fixed-order sums of the two partial
// vectors of `bank` into out[0] (gamma), out[1] (delta)
__device__ __forceinline__ bool pp_reduce(const unsigned* flag, unsigned* tmo, unsigned target, const double* pb,
                                          int G, double* out) {
    const int lane = threadIdx.x & 63;
    for (int b0 = 0; b0 < G; b0 += 64) {
        const int j = b0 + lane;
        bool done = j >= G;
        for (unsigned spins = 0; !__all(done); ++spins) {
            if (!done) done = pk_ld(flag + (size_t)j * PK_LINE) >= target;
            if ((spins & 63) == 63 && pk_ld(tmo)) return false;
            if (spins >= PK_SPIN_LIMIT) {
                pk_st(tmo, 1u);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    double vg = 0.0, vd = 0.0;
#pragma unroll 4
    for (int i = lane; i < G; i += 64) {
        vg += __hip_atomic_load(pb + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vd += __hip_atomic_load(pb + G + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    vg = wave_sum(vg);
    vd = wave_sum(vd);
    if (lane == 0) {
        out[0] = vg;
        out[1] = vd;
    }
    return true;
}

#define PP_ON(j) ((j) < nreg && lane < nrows - (s0 + (j)) * 64)

template <int NW, int MAXS, int VL, int U, bool PROF>
__global__ void __launch_bounds__(NW * 64) k_pcg_pipe(PpArgs a) {
    static_assert(VL <= MAXS && NW <= 16, "n slots in LDS, wave sums in the head");
    static_assert(pp_lds_bytes<NW, MAXS, VL>() <= 160 * 1024, "pipelined PCG: LDS over the 160 KB of a CU");
    unsigned long long pacc[PROF ? PP_NPROF : 1] = {};
    unsigned long long pt = 0;
    if constexpr (PROF) pt = __builtin_amdgcn_s_memtime();
#define PP_MARK(i)                                                         \
    __builtin_amdgcn_sched_barrier(0);                                     \
    if constexpr (PROF) {                                                  \
        const unsigned long long now = __builtin_amdgcn_s_memtime();       \
        pacc[i] += now - pt;                                               \
        pt = now;                                                          \
    }
    extern __shared__ __attribute__((aligned(16))) double pp_lds_raw[];
    double* lds16 = pp_lds_raw;                                  // [NW] wave sums of gamma, [NW] of delta
    int& lds_ok = *reinterpret_cast<int*>(pp_lds_raw + 2 * 16);
    double* lds_gd = pp_lds_raw + 2 * 16 + 2;                    // reduced gamma, delta
    double* pl = pp_lds_raw + PP_LDS_HEAD / sizeof(double);
    const int G = gridDim.x;
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;   // XCD-contiguous logical order
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // packed slice assignment: workgroup L owns [L S / G, (L+1) S / G); its waves take a.pack slices each in order
    int s0, nsl;
    {
        const int m = a.pack;
        const int sL0 = (int)((int64_t)L * a.nslices / G);
        const int nL = (int)((int64_t)(L + 1) * a.nslices / G) - sL0;
        const int lo = wv * m < nL ? wv * m : nL;
        s0 = sL0 + lo;
        nsl = nL - lo < m ? nL - lo : m;
    }
    const int nreg = nsl;   // <= MAXS (host)
    const int nrows = (int)a.nrows;
    const unsigned rb = (unsigned)s0 * 64u + (unsigned)lane;
    double* xl = pl + wv * MAXS * 64 + lane;
    double* dl = pl + NW * MAXS * 64 + wv * MAXS * 64 + lane;
    double* nl = pl + 2 * NW * MAXS * 64 + wv * VL * 64 + lane;
    PcgState* st = a.st;

    const bool cg = st->mode != FEM_MODE_PCG;
    const double tol = st->tol, eps = st->eps;
    const int max_iter = st->max_iter;
    int it = st->iter, halt = st->halt, status = st->status, stop_iter = st->stop_iter;
    double rz = st->rz, alpha_prev = st->alpha, beta = st->beta, pq = st->pq, rz_new = st->rz_new;
    double g = st->red[1];
    const unsigned ebase = st->pk_epoch;
    unsigned elast = ebase;

    double rr[MAXS], av[MAXS], ss[MAXS], pp[MAXS], zz[MAXS], nv[MAXS];
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
        const unsigned row = rb + 64u * j;
        const bool on = PP_ON(j);
        rr[j] = on ? a.r[row] : 0.0;
        av[j] = on ? a.av[row] : 0.0;
        ss[j] = on ? a.s[row] : 0.0;
        pp[j] = on ? a.p[row] : 0.0;
        zz[j] = on ? a.z[row] : 0.0;
        nv[j] = 0.0;
        if (j < VL) nl[j * 64] = 0.0;
        xl[j * 64] = on ? a.x[row] : 0.0;
        dl[j * 64] = on ? a.w[row] : 0.0;
    }
    const int wlo = a.win[L], whi = a.win[G + L];
    const bool red_wave = wv == NW - 1;
    bool fail = false;
    int k = 0;
    if constexpr (PROF) {
        __syncthreads();
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        pacc[6] += now - pt;
        pt = now;
    }
    if (!halt) {
        for (k = 0; k < a.kmax; ++k) {
            const unsigned e = ebase + (unsigned)k + 1;
            // ---- the m of the gather window (the previous update; the previous launch's is complete at k = 0)
            if (k > 0) {
                if (wv == 0) {
                    bool ok = true;
                    for (int b0 = wlo; b0 <= whi && ok; b0 += 64) {
                        const int jw = b0 + lane;
                        bool done = jw > whi;
                        for (unsigned spins = 0; !__all(done); ++spins) {
                            if (!done) done = pk_ld(a.flag + (size_t)jw * PK_LINE) >= e - 1;
                            if ((spins & 63) == 63 && pk_ld(a.tmo)) {
                                ok = false;
                                break;
                            }
                            if (spins >= PK_SPIN_LIMIT) {
                                pk_st(a.tmo, 1u);
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
            PP_MARK(0);
            // ---- n = A m over the own slices
            const bool rv = a.rev && ((it & 1) != 0);
            const int64_t* slp = pk_launder(a.slice_ptr);
            const int16_t* cop = pk_launder(a.cols);
            const double* vap = pk_launder(a.vals);
            const double* mvp = pk_launder(((e - 1) & 1) ? a.m1 : a.m0);
            if (!rv) {
#pragma unroll
                for (int j = 0; j < MAXS; ++j) {
                    if (j < nreg) {
                        const double v = sell_row_pair<U, true>(s0 + j, lane, slp, cop, vap, mvp);
                        if (j < VL) nl[j * 64] = v; else nv[j] = v;
                    }
                    asm volatile("" ::: "memory");
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < MAXS; ++jj) {
                    const int j = MAXS - 1 - jj;
                    if (j < nreg) {
                        const double v = sell_row_pair<U, true>(s0 + j, lane, slp, cop, vap, mvp);
                        if (j < VL) nl[j * 64] = v; else nv[j] = v;
                    }
                    asm volatile("" ::: "memory");
                }
            }
            PP_MARK(1);
            // ---- gamma, delta of the current iterate: every workgroup's partials of the previous update
            if (red_wave) {
                const bool ok = pp_reduce(a.flag, a.tmo, e - 1, a.part + (size_t)((e - 1) & 1) * 2 * G, G, lds_gd);
                if (lane == 0) lds_ok = ok;
            }
            __syncthreads();
            if (!lds_ok) {
                fail = true;
                break;
            }
            g = lds_gd[0];
            const double d = lds_gd[1];
            elast = e;
            PP_MARK(2);
            // ---- step (k_cg1_step / pcg_persist.hpp)
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
            PP_MARK(4);
            // ---- update the own rows, publish m and the partials of the next iteration
            double gp = 0.0, dp = 0.0;
            unsigned rbi = rb;
            double* mst = pk_launder((e & 1) ? a.m1 : a.m0);
            asm volatile("" : "+v"(rbi));
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) {
                    const double dj = dl[j * 64];
                    const double nj = j < VL ? nl[j * 64] : nv[j];
                    const double zi = nj + bnew * zz[j];
                    const double si = av[j] + bnew * ss[j];
                    const double pi = dj * rr[j] + bnew * pp[j];
                    zz[j] = zi;
                    ss[j] = si;
                    pp[j] = pi;
                    xl[j * 64] += al * pi;
                    double ri = rr[j] - al * si;
                    if (cg && dj == 0.0) ri = 0.0;
                    rr[j] = ri;
                    const double ai = av[j] - al * zi;
                    av[j] = ai;
                    const double ui = dj * ri;
                    if (PP_ON(j)) __hip_atomic_store(mst + (rbi + 64u * j), dj * ai, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    gp += ri * ui;
                    dp += ai * ui;
                }
            }
            {
                const double gw = wave_sum(gp), dw = wave_sum(dp);
                if (lane == 0) {
                    lds16[wv] = gw;
                    lds16[16 + wv] = dw;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its m stores
            __syncthreads();
            if (threadIdx.x == 0) {
                double gs = 0.0, ds = 0.0;
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    gs += lds16[i];
                    ds += lds16[16 + i];
                }
                double* pb = a.part + (size_t)(e & 1) * 2 * G;
                __hip_atomic_store(pb + L, gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pb + G + L, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // partials before the flag
                pk_st(a.flag + (size_t)L * PK_LINE, e);
            }
            PP_MARK(5);
        }
    }
    // ---- chunk end without a stop: gamma of the last update for the stop test and the host's poll
    if (!fail && !halt && k == a.kmax && a.kmax > 0) {
        const unsigned e = ebase + (unsigned)a.kmax;   // epoch of the last update
        if (red_wave) {
            const bool ok = pp_reduce(a.flag, a.tmo, e, a.part + (size_t)(e & 1) * 2 * G, G, lds_gd);
            if (lane == 0) lds_ok = ok;
        }
        __syncthreads();
        if (!lds_ok) {
            fail = true;
        } else {
            g = lds_gd[0];
            elast = e;
            const double nrm = sqrt(g);
            rz_new = g;
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
    // ---- state back to memory (m and the partials are already there)
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
        if (PP_ON(j)) {
            const unsigned row = rb + 64u * j;
            a.r[row] = rr[j];
            a.av[row] = av[j];
            a.s[row] = ss[j];
            a.p[row] = pp[j];
            a.z[row] = zz[j];
            a.x[row] = xl[j * 64];
        }
    }
    if constexpr (PROF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        pacc[7] += __builtin_amdgcn_s_memtime() - pt;
        if (threadIdx.x == 0)
            for (int i = 0; i < PP_NPROF; ++i) a.prof[(size_t)L * PP_NPROF + i] = pacc[i];
    }
    if (L == 0 && threadIdx.x == 0) {
        if (fail) {
            status = FEM_PCG_SYNC_TIMEOUT;
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
        st->pk_epoch = elast;   // the epoch of the last published update (its m buffer and partial bank)
    }
#undef PP_MARK
}
#undef PP_ON

// start of the pipelined iteration: r0 = b - q (q = A x0; CG: masked rows 0), u0 = w r0 into u, p = s = z = 0
__global__ void k_pipe_init1(int64_t n, const double* __restrict__ b, const double* __restrict__ q,
                             const double* __restrict__ w, double* __restrict__ r, double* __restrict__ u,
                             double* __restrict__ p, double* __restrict__ s, double* __restrict__ z, int cg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double rv = b[i] - q[i];
        if (cg && w[i] == 0.0) rv = 0.0;
        r[i] = rv;
        u[i] = w[i] * rv;
        p[i] = 0.0;
        s[i] = 0.0;
        z[i] = 0.0;
    }
}

// a0 = q (= A u0), m0 = w a0 (buffer of epoch 0), and the epoch-0 partials gamma0 = r.u, delta0 = a.u: block sums in
// fixed order into gd[2 * block], then k_pipe_init3 sums the blocks in fixed order into bank 0 of the partials
__global__ void __launch_bounds__(256) k_pipe_init2(int64_t n, const double* __restrict__ q,
                                                    const double* __restrict__ w, const double* __restrict__ r,
                                                    double* __restrict__ av, double* __restrict__ m0,
                                                    double* __restrict__ gd) {
    __shared__ double sh[2][4];
    double gp = 0.0, dp = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double a0 = q[i];
        const double ui = w[i] * r[i];
        av[i] = a0;
        m0[i] = w[i] * a0;
        gp += r[i] * ui;
        dp += a0 * ui;
    }
    gp = wave_sum(gp);
    dp = wave_sum(dp);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[0][wv] = gp;
        sh[1][wv] = dp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        gd[2 * blockIdx.x] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
        gd[2 * blockIdx.x + 1] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    }
}

__global__ void k_pipe_init3(const double* __restrict__ gd, int nb, double* __restrict__ part, int G,
                             PcgState* __restrict__ st) {
    // one wave: fixed-order sums of the nb block partials; bank 0 = {gamma0 at [0], delta0 at [G]}, rest zero
    const int lane = threadIdx.x;
    double vg = 0.0, vd = 0.0;
    for (int i = lane; i < nb; i += 64) {
        vg += gd[2 * i];
        vd += gd[2 * i + 1];
    }
    vg = wave_sum(vg);
    vd = wave_sum(vd);
    for (int i = lane; i < 4 * G; i += 64) part[i] = 0.0;
    __syncthreads();
    if (lane == 0) {
        part[0] = vg;
        part[G] = vd;
        st->red[1] = vg;
        st->rz = vg;
    }
}

}  // namespace fem
