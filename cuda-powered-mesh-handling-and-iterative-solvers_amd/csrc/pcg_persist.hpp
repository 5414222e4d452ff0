// Persistent register-resident Jacobi-PCG (schedule 3, bs = 1 with the lane-paired matrix copy).
//
// The single-reduction (Chronopoulos–Gear) form of k_cg1_* run as ONE launch per chunk of iterations: every wave
// owns a fixed contiguous range of at most PK_MAXS slices for the whole launch and keeps its rows' CG state on the
// chip — r, p, s = A p, its own u and 2 of 7 v = A u slots in registers, x, w and 5 v slots in LDS — so an
// iteration moves the matrix once,
// gathers u, and writes u: (8 + 2) nnz + 16 n bytes instead of the deferred schedule's (8 + 2) nnz + 96 n.
//
//   per iteration (epoch e = local iteration + 1):
//     wait   : one wave polls the u-flags of the workgroups whose rows this workgroup's columns reach
//              (gather window, computed once per matrix); workgroup barrier (GSC1 = 0: one agent acquire first)
//     SpMV   : v = A u over the own slices (paired layout; u gathers as global sc1 loads, GSC1 = 1, the default),
//              d partial = u.v
//     reduce : workgroup partials of d (and g of the last update) stored sc1 into a parity bank; hierarchical
//              grid barrier (8 group counters -> 8 replicas of the top counter), wave 0 then sums
//              the G partials in the same fixed order -> identical scalars in every workgroup
//     step   : stop test on g (`solver/solver.py:210` / `:805`), beta, p.Ap = d - beta g / alpha_prev, alpha,
//              guards (`:187-198`, `:214`) -- the single-reduction step (pcg.hip cg1_eval), by every thread
//     update : p = u + beta p, s = v + beta s, x += alpha p, r -= alpha s (CG: masked), u = w r stored sc1,
//              g partial; every wave drains its stores, then one lane raises the workgroup's u-flag to e
// The hand-offs follow MI355X_MICROARCH.md "Valid forms" (sc1 stores + drain + relaxed flag / counter; global sc1
// loads of the partials and of the u gathers, or an agent acquire before plain gathers). Every spin is bounded: a
// give-up sets a word all
// spinners check, the launch then ends with status FEM_PCG_SYNC_TIMEOUT instead of hanging.
// Exactly one workgroup of PK_T threads per CU (LDS pins it): the grid is resident by construction (the host
// checks the occupancy query; a plain launch: a cooperative one adds ~17 us per launch and buys only that check).
#pragma once
#include "sell_pair.hpp"

namespace fem {

// PK_T / PK_WAVES (threads / waves per workgroup) and pk_slice_span live in sell_pair.hpp: the pattern pass that
// forms the gather windows (sl_pattern_slice) needs them outside this header
#ifndef FEM_PK_PF
#define FEM_PK_PF 0   // L2 prefetch of the next SpMV's first slice under the grid barrier: measured slower (r06v), off
#endif
constexpr int PK_MAXS = 7;               // slices per wave (10M Poisson: 27,000 slices over 4,096 waves -> 7)
constexpr int PK_U = 2;                  // pairs in flight per lane (4 spills the slot state; persist_probe: 4 = 8)
// pairs in flight of a build: one slot per wave (small systems: every wave owns at most one slice, e.g. 1M tets or
// a rank's share at N = 8) leaves the registers for 8 pairs, so a slice's loads go out in one round instead of 4;
// up to four slots for 4 pairs (the instrumented builds keep PK_U there: their clock registers would spill)
template <int MAXS, bool PROF>
constexpr int pk_u() { return MAXS <= 1 ? 8 : (MAXS <= 4 && !PROF) ? 4 : PK_U; }
constexpr int PK_LINE = 32;              // unsigned words per 128-byte line
// sync words (zeroed by fem_pcg_start; epochs continue across launches from PcgState::pk_epoch), in lines: [0, 8) group arrivals, 8 (unused), [9, 17) replicas of the
// top counter (one per group),
// 17 give-up word, 18 + L: u-flag of workgroup L
enum { PK_GRP = 0, PK_TOP = 8 * PK_LINE, PK_GEN = 9 * PK_LINE, PK_TMO = 17 * PK_LINE, PK_UFLAG = 18 * PK_LINE };
// every spin is bounded in TIME (s_memrealtime, 100 MHz on gfx9 parts: hipDeviceAttributeWallClockRate), checked
// every 64 polls: 2 s for a wait inside one GPU (the longest legitimate one is a grid barrier behind one ~50 us
// SpMV phase), 5 s for the rank exchange of the DIST build (ranks start their launches up to milliseconds apart).
// A give-up therefore costs at most ~5 s per launch whatever the poll latency (xGMI system-scope loads included);
// the spin-count bound this replaces scaled with that latency (4M polls: 4-50 s)
constexpr uint64_t PK_WAIT_TICKS = 200000000ull;
constexpr uint64_t PK_RANK_WAIT_TICKS = 500000000ull;
__device__ __forceinline__ uint64_t pk_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool pk_expired(uint64_t t0, uint64_t ticks) { return pk_now() - t0 > ticks; }
constexpr int PK_NPROF = 8;   // phases: u wait, SpMV, block sum, barrier + sums, step, update + drain + flag,
                               // prologue (state loads), epilogue (chunk-end barrier + state stores)
// dynamic LDS (statics would shift the dynamic base off 16 B, cdna_hip_programming.md Guideline 17): 16 wave sums,
// the barrier verdict (own 16-byte slot), then x and w of the workgroup's rows
constexpr size_t PK_LDS_HEAD = 256;
constexpr int PK_VL = 5;                 // slots of v = A u kept in LDS (the rest in registers): fills the LDS left
                                         // by x and w, frees 2 PK_VL VGPRs for the SpMV (no spills at PK_U = 2)
constexpr size_t PK_LDS = PK_LDS_HEAD + sizeof(double) * (2 * PK_MAXS + PK_VL) * PK_WAVES * 64;
static_assert(PK_LDS <= 160 * 1024, "persistent PCG: LDS over the 160 KB of a CU");

// an opaque copy of a global pointer (the compiler cannot hoist address arithmetic on it out of the iteration loop)
// that keeps its address space: laundering a generic pointer turns every access through it into a FLAT access
// (lgkmcnt-coupled, and `flat_` sc1 loads are not a valid hand-off form, MI355X_MICROARCH.md)
template <class T>
__device__ __forceinline__ T* pk_launder(T* p) {
    __attribute__((address_space(1))) T* q = (__attribute__((address_space(1))) T*)p;
    asm volatile("" : "+s"(q));
    return (T*)q;
}

__device__ __forceinline__ unsigned pk_ld(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pk_st(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one lane spins until *p >= target; false on give-up (own or another spinner's)
// the give-up word holds the site of the first give-up (diagnostics, reported by fem_pcg_sync_site for a
// FEM_PCG_SYNC_TIMEOUT): 1 + 16 * epoch local grid barrier, 2 + 16 * epoch u-flag window, 3 + 16 * epoch
// rank sums (DIST), PK_SITE_WINDOW: a gather window outside the flag array (status FEM_PCG_BAD_WINDOW)
// (PK_SITE_WINDOW, pk_window_bad, pk_fail_status: common.hpp)
__device__ __forceinline__ bool pk_wait_ge(const unsigned* p, unsigned target, unsigned* tmo) {
    const uint64_t t0 = pk_now();
    for (unsigned spins = 0;; ++spins) {
        if (pk_ld(p) >= target) return true;
        if ((spins & 63) == 63 && pk_ld(tmo)) return false;
        if ((spins & 63) == 63 && pk_expired(t0, PK_WAIT_TICKS)) {
            pk_st(tmo, 1u + 16u * (target / NXCD));
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// fixed-order sum of n sc1-loaded partials by one wave (identical result in every lane)
__device__ __forceinline__ double pk_sum(const double* part, int n) {
    const int lane = threadIdx.x & 63;
    double v = 0.0;
    for (int i = lane; i < n; i += 64) v += __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return wave_sum(v);
}

// grid barrier of epoch e over 8 groups of nper workgroups, then the fixed-order sums of the partial vectors pd
// (and pg when given) by wave 0 alone, handed to the other waves through LDS (out[0], out[1]). One wave per
// workgroup reads the G partials instead of all 16 (4,096 waves loading the same 4 KB with sc1 loads queue on the
// memory channels that hold those lines).
// entry_sync = false: the caller's own workgroup barrier (pk_block_sum's) already separates every wave's prior work
__device__ __forceinline__ bool pk_barrier(unsigned* sy, int grp, unsigned nper, unsigned e, int* lds_ok,
                                           const double* pd, const double* pg, int G, double* out,
                                           bool entry_sync = true) {
    if (entry_sync) __syncthreads();
    if (threadIdx.x < 64) {
        int okv = 0;
        if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned* tmo = sy + PK_TMO;
            bool ok;
            const unsigned old = __hip_atomic_fetch_add(sy + PK_GRP + grp * PK_LINE, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            // last of its group: arrive on all 8 replicas of the top counter (one line each); every workgroup polls
            // its group's replica (32 pollers per line, no leader -> generation hop)
#if FEM_PK_PROBE_NOBAR
            // (probe: workgroups reach the chunk-end barrier while others of their group still iterate, so the add
            // that completes any epoch's count bumps the replicas, whoever makes it)
            if ((old + 1) % nper == 0)
#else
            if (old == e * nper - 1)
#endif
                for (int r = 0; r < NXCD; ++r)
                    __hip_atomic_fetch_add(sy + PK_GEN + r * PK_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = pk_wait_ge(sy + PK_GEN + grp * PK_LINE, e * NXCD, tmo);
            okv = ok ? 1 : 0;
        }
        okv = __builtin_amdgcn_readfirstlane(okv);
        if (okv && pd) {   // both partial vectors in one round of loads (same per-lane order as two pk_sums)
            const int lane = threadIdx.x & 63;
            double vd = 0.0, vg = 0.0;
            if (pg) {
#pragma unroll 4
                for (int i = lane; i < G; i += 64) {
                    const double a = __hip_atomic_load(pd + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const double b = __hip_atomic_load(pg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vd += a;
                    vg += b;
                }
            } else {
#pragma unroll 4
                for (int i = lane; i < G; i += 64) vd += __hip_atomic_load(pd + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const double d = wave_sum(vd);
            const double g = pg ? wave_sum(vg) : 0.0;
            if (threadIdx.x == 0) {
                out[0] = d;
                out[1] = g;
            }
        }
        if (threadIdx.x == 0) *lds_ok = okv;
    }
    __syncthreads();
    return *lds_ok != 0;
}

// fixed-order workgroup sum (PK_WAVES waves), valid in thread 0
__device__ __forceinline__ double pk_block_sum(double v, double* lds16) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds16[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < PK_WAVES; ++i) t += lds16[i];
    }
    return t;
}

constexpr int PK_MAX_RANKS = 8;

struct PkArgs {
    int64_t nslices, nrows;
    const int64_t* slice_ptr;
    const int16_t* cols;    // lane-paired copy (sell_pair.hpp)
    const double* vals;
    const int32_t* uoff;    // slice-uniform deltas (k_sell_uniform; nullptr: per-lane deltas everywhere)
    const int16_t* ucol;
    double* x;
    double* r;
    double* p;
    double* s;
    double* u;              // gathered by the SpMV: the hand-off between workgroups
    const double* w;
    const int32_t* win;     // [2 G] gather window per logical workgroup: first workgroups, then last ones
    double* part;           // [2 banks][2 (d, g)][G]
    unsigned* sync;
    PcgState* st;
    double* hist;
    int64_t hist_len;
    int kmax;               // iterations of this launch
    int rev;                // FEM_TUNE_REVERSE: odd iterations walk the own slices backwards
    int pack;               // FEM_TUNE_PK_PACK: slices per wave in order (0: spread; see k_pcg_persist)
    double* v;              // OVF: v = A u of the overflow rows (their state stays in r, p, s, x, u, w in HBM)
    unsigned long long* prof;   // PROF instantiation: [G][PK_NPROF] shader-clock sums per phase (thread 0 of each WG),
                                // then [G][PK_WAVES] SpMV-phase clock sums of every wave (its own slices only)
    // DIST build (one rank per GPU, rows partitioned): this rank owns the global slices [sbase, sbase + nslices) of
    // a matrix whose rows are global; every vector is global-length. Each rank's comm block (peer[rank]; the other
    // ranks' blocks mapped through IPC) holds: u at offset 0 (the gathered vector: own rows written here, the rows
    // other ranks gather from this rank also written into THEIR blocks), the u-flags of all nranks * G workgroups
    // (off_flag, one line each, written by the owning workgroup wherever its rows are gathered), the rank sums
    // [2 banks][PK_MAX_RANKS][d, g] (off_red) and one epoch line per rank announcing them (off_rflag).
    int64_t sbase;
    int rank, nranks;
    char* peer[PK_MAX_RANKS];
    int64_t off_flag, off_red, off_rflag;
    const int32_t* pub;     // [G][nranks][2]: rows [lo, hi) of logical workgroup L gathered by rank Q; lo < 0: Q
                            // never waits on L (lo >= 0 with lo == hi: L raises its flag in Q, no rows)
    const double* b;        // init launch: r0 = b - A x0 over the own rows (x0 global-length, the same on every rank)
    int init;
};

// DIST grid barrier with the rank exchange folded in. Arrivals as in pk_barrier (group counter, the last of a group
// adds to ONE top counter); the add on the top counter that returns e * 8 - 1 tells its workgroup that the whole
// rank has arrived: its wave 0 alone sums the G partials (fixed order) and announces the rank's (d, g) to every
// rank -- system-scope stores into bank e & 1 of each rank's comm block, a system release, then epoch e on the
// rank's 8 replica lines there (one per XCD group: 32 pollers per line). Every workgroup's wave 0 waits for epoch e
// from all ranks on its group's replicas and sums the ranks' pairs in rank order 0..N-1 (identical bits on every
// rank). Banked by epoch parity: a rank announces e + 2 only after all ranks announced e + 1, i.e. after every
// reader of bank e is done. The give-up word records 3 + 16 e.
__device__ __forceinline__ bool pk_barrier_dist(const PkArgs& a, unsigned* sy, int grp, unsigned nper, unsigned e,
                                                int* lds_ok, const double* pd, const double* pg, int G, double* out,
                                                bool entry_sync = true) {
    if (entry_sync) __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        unsigned* tmo = sy + PK_TMO;
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
        const int bank = (int)(e & 1u);
        if (last) {
            double vd = 0.0, vg = 0.0;
#pragma unroll 4
            for (int i = lane; i < G; i += 64) {
                vd += __hip_atomic_load(pd + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (pg) vg += __hip_atomic_load(pg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const double d = wave_sum(vd), g = wave_sum(vg);
            if (lane < a.nranks) {
                double* red = reinterpret_cast<double*>(a.peer[lane] + a.off_red) + (bank * PK_MAX_RANKS + a.rank) * 2;
                __hip_atomic_store(red, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(red + 1, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane < a.nranks * NXCD)   // rank (lane / 8)'s replica (lane % 8) of this rank's epoch line
                __hip_atomic_store(reinterpret_cast<unsigned*>(a.peer[lane / NXCD] + a.off_rflag) +
                                       (a.rank * NXCD + lane % NXCD) * PK_LINE,
                                   e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
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
            const double* red = reinterpret_cast<const double*>(a.peer[a.rank] + a.off_red) + bank * PK_MAX_RANKS * 2;
            double d = 0.0, g = 0.0;
            for (int q = 0; q < a.nranks; ++q) {   // rank order: the same sum on every rank
                d += __hip_atomic_load(red + 2 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                g += __hip_atomic_load(red + 2 * q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (lane == 0) {
                out[0] = d;
                out[1] = g;
            }
        }
        if (lane == 0) *lds_ok = okv;
    }
    __syncthreads();
    return *lds_ok != 0;
}

// DIST: row `row` of this rank's u also lands in the comm block of every rank in pubmask whose gathered range holds it
__device__ __forceinline__ void pk_publish_row(const PkArgs& a, int L, unsigned pubmask, unsigned row, double v) {
    for (int q = 0; q < a.nranks; ++q) {
        if (!(pubmask & (1u << q))) continue;
        const int32_t* pr = a.pub + (L * a.nranks + q) * 2;
        if ((int)row >= pr[0] && (int)row < pr[1])
            __hip_atomic_store(reinterpret_cast<double*>(a.peer[q]) + row, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// DIST: after every wave drained its stores (and, where it published rows to other ranks, ran a system release),
// thread 0 raises this workgroup's u-flag in every rank that gathers its rows
__device__ __forceinline__ void pk_publish_flag(const PkArgs& a, int Lg, unsigned pubmask, unsigned e) {
    for (int q = 0; q < a.nranks; ++q)
        if (pubmask & (1u << q))
            __hip_atomic_store(reinterpret_cast<unsigned*>(a.peer[q] + a.off_flag) + Lg * PK_LINE, e, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
}


// the 64 rows of slot j of this wave: row = rb + 64 j (32-bit; the host checks nrows < 2^31); `lim` = rows of the
// slot that exist (wave-uniform; < 64 only in the matrix's last slice)
#define PK_ON(j) ((j) < nreg && lane < nrows - (s0 + (j)) * 64)

// GSC1: the u gathers are sc1 loads and the u-flag wait needs no agent acquire (whose L2 invalidation by every
// workgroup of an XCD can drop the gather window other workgroups are still reading)
// OVF: meshes past MAXS slices per wave (packed assignment only): a wave's slices beyond its MAXS register slots keep
// their CG state in HBM (the r, p, s, x, u, w arrays, v in a.v) and are streamed every iteration like the deferred
// schedule's rows, inside the same launch and the same barriers
// DIST: see PkArgs (GSC1 and !OVF implied)
template <int MAXS, bool PROF, bool GSC1, bool OVF = false, bool DIST = false>
__global__ void __launch_bounds__(PK_T) k_pcg_persist(PkArgs a) {
    static_assert(!DIST || (GSC1 && !OVF), "distributed persistent PCG: sc1 gathers, no overflow build");
    unsigned long long pacc[PROF ? PK_NPROF : 1] = {};
    unsigned long long pt = 0, wspmv = 0;
    if constexpr (PROF) pt = __builtin_amdgcn_s_memtime();
// phase boundary: a scheduling barrier in every build (instructions hoisted across phases lengthen the live ranges
// of the slot arrays: ~180 spilled VGPRs without it), plus the phase clock in the PROF build
#define PK_MARK(i)                                                         \
    __builtin_amdgcn_sched_barrier(0);                                     \
    if constexpr (PROF) {                                                  \
        const unsigned long long now = __builtin_amdgcn_s_memtime();       \
        pacc[i] += now - pt;                                               \
        pt = now;                                                          \
    }
    extern __shared__ __attribute__((aligned(16))) double pk_lds_raw[];
    double* lds16 = pk_lds_raw;
    int& lds_ok = *reinterpret_cast<int*>(pk_lds_raw + PK_WAVES);
    double* lds_dg = pk_lds_raw + PK_WAVES + 2;   // barrier sums (bytes 144..159 of the 256-byte head)
    double* pk_lds = pk_lds_raw + PK_LDS_HEAD / sizeof(double);
    const int G = gridDim.x;
    const unsigned nper = (unsigned)(G / NXCD);
    const int L = (blockIdx.x % NXCD) * (G / NXCD) + blockIdx.x / NXCD;   // XCD-contiguous logical order
    const int grp = L / (int)nper;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform -> scalar slot bounds
    // slices of this wave (wave-uniform): workgroup L owns [L S / G, (L+1) S / G) either way; spread: the
    // workgroup's slices evenly over its 16 waves (6 or 7 each at 10M); packed (FEM_TUNE_PK_PACK): a.pack =
    // ceil(max slices per workgroup / 16) per wave in order, the remainder on the last busy wave (10M: 15 waves x 7
    // + 0 or 1 -- every busy wave streams to the end of the phase instead of 41 % of them idling through the 7th)
    int s0, nsl;
    if (a.pack) {
        const int m = a.pack;   // <= MAXS (host)
        const int sL0 = (int)((int64_t)L * a.nslices / G);
        const int nL = (int)((int64_t)(L + 1) * a.nslices / G) - sL0;
        const int lo = wv * m < nL ? wv * m : nL;
        s0 = sL0 + lo + (DIST ? (int)a.sbase : 0);   // DIST: this rank's slices start at global slice sbase
        nsl = nL - lo < m ? nL - lo : m;
    } else {
        const int64_t W = (int64_t)G * PK_WAVES;
        const int64_t gw = (int64_t)L * PK_WAVES + wv;
        s0 = (int)(gw * a.nslices / W);
        nsl = (int)((gw + 1) * a.nslices / W) - s0;   // <= MAXS (host check)
    }
    const int nreg = (OVF && nsl > MAXS) ? MAXS : nsl;   // register / LDS slots
    const int nov = nsl - nreg;                          // overflow slices (OVF only; host-checked 0 otherwise)
    const int nrows = (int)a.nrows;
    const unsigned rb = (unsigned)s0 * 64u + (unsigned)lane;
    double* xl = pk_lds + wv * MAXS * 64 + lane;
    double* wl = pk_lds + PK_WAVES * MAXS * 64 + wv * MAXS * 64 + lane;
    double* vl = pk_lds + 2 * PK_WAVES * MAXS * 64 + wv * PK_VL * 64 + lane;   // v of slots j < PK_VL
    unsigned* sy = a.sync;
    PcgState* st = a.st;
    // u-flags: this rank's own lines (single GPU), or the comm block's lines of all ranks' workgroups (DIST)
    unsigned* uf = DIST ? reinterpret_cast<unsigned*>(a.peer[a.rank] + a.off_flag) : sy + PK_UFLAG;
    const int Lg = DIST ? a.rank * G + L : L;   // global logical workgroup
    const int olo = DIST ? (int)(a.sbase * 64) : 0;                         // this rank's rows [olo, ohi)
    const int ohi = DIST ? (int)((a.sbase + a.nslices) * 64 < a.nrows ? (a.sbase + a.nslices) * 64 : a.nrows) : 0;
    unsigned pubmask = 0;                       // DIST: ranks that gather rows of this workgroup
    bool ghost = false;                         // DIST: this workgroup gathers rows of other ranks
    if constexpr (DIST) {
        for (int q = 0; q < a.nranks; ++q)
            if (q != a.rank && a.pub[(L * a.nranks + q) * 2] >= 0) pubmask |= 1u << q;
        ghost = a.win[L] < a.rank * G || a.win[G + L] >= (a.rank + 1) * G;
    }

    // scalars (every thread; WG 0 thread 0 writes them back)
    const bool cg = st->mode != FEM_MODE_PCG;
    const double tol = st->tol, eps = st->eps;
    const int max_iter = st->max_iter;
    int it = st->iter, halt = st->halt, status = st->status, stop_iter = st->stop_iter;
    double rz = st->rz, alpha_prev = st->alpha, beta = st->beta, pq = st->pq, rz_new = st->rz_new;
    double g = st->red[1];   // r.z of the current iterate (init or the last launch's last update)
    unsigned ebase = st->pk_epoch;         // barriers of earlier launches (sync words count on from there)
    unsigned elast = ebase;                // last barrier epoch of this launch

    double rr[MAXS], pp[MAXS], ss[MAXS], vv[MAXS], uo[MAXS];
#pragma unroll
    for (int j = 0; j < MAXS; ++j) {
        const unsigned row = rb + 64u * j;
        const bool on = PK_ON(j);
        rr[j] = on ? a.r[row] : 0.0;
        pp[j] = on ? a.p[row] : 0.0;
        ss[j] = on ? a.s[row] : 0.0;
        vv[j] = 0.0;
        xl[j * 64] = on ? a.x[row] : 0.0;
        if (j < PK_VL) vl[j * 64] = 0.0;
        const double wj = on ? a.w[row] : 0.0;
        wl[j * 64] = wj;
        uo[j] = wj * rr[j];   // u = w r is how every u was formed (k_cg1_init, the update): bit-identical, no load
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
    bool st_loaded = !halt;   // the state is on chip and may have changed (nothing to store after a halt)
    int k = 0;
    if constexpr (DIST) {
        // first launch of a distributed solve: r0 = b - A x0 over the own rows (x0 global-length, identical on every
        // rank), u0 = w r0 published like an update (epoch ebase + 1), r0.u0 summed by a full barrier (local, then
        // across ranks) -- the distributed counterpart of k_cg1_init
        if (a.init && !halt) {
            const int64_t* slp = pk_launder(a.slice_ptr);
            const int16_t* cop = pk_launder(a.cols);
            const double* vap = pk_launder(a.vals);
            const double* xvp = pk_launder(a.x);
            double gp = 0.0;
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                if (j < nreg) {
                    const double q = sell_row_pair<pk_u<MAXS, PROF>(), 0>(s0 + j, lane, slp, cop, vap, xvp, 0, 0, a.uoff, a.ucol);
                    const unsigned row = rb + 64u * j;
                    const bool on = PK_ON(j);
                    double rv = on ? a.b[row] - q : 0.0;
                    const double wj = wl[j * 64];
                    if (cg && wj == 0.0) rv = 0.0;
                    rr[j] = rv;
                    pp[j] = 0.0;
                    ss[j] = 0.0;
                    xl[j * 64] = on ? a.x[row] : 0.0;
                    const double ui = wj * rv;
                    uo[j] = ui;
                    gp += rv * ui;
                    if (on) {
                        __hip_atomic_store(a.u + row, ui, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (pubmask) pk_publish_row(a, L, pubmask, row, ui);
                    }
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
            double* pg0 = a.part + 2 * (size_t)G;   // bank 1's d slots: first written at local iteration 1
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
    if constexpr (PROF) {
        __syncthreads();
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        pacc[6] += now - pt;
        pt = now;
    }
    if (!halt && !fail) {
        for (k = 0; k < a.kmax; ++k) {
            const unsigned e = ebase + (unsigned)k + 1;
            // ---- wait for the u of the gather window (written by the previous update of this launch, or by the
            // distributed init above)
            if (k > 0 || (DIST && a.init)) {
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
                        if constexpr (!GSC1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                }
                __syncthreads();
                if (!lds_ok) {
                    fail = true;
                    break;
                }
            }
            PK_MARK(0);
            // ---- v = A u over the own slices, d partial. Slots unrolled (register-resident state needs
            // compile-time indices); the empty asm keeps the compiler from interleaving slots (register blow-up)
            const bool rv = a.rev && ((it & 1) != 0);
            unsigned long long tw0 = 0;
            if constexpr (PROF) tw0 = __builtin_amdgcn_s_memtime();
            // launder the matrix pointers every iteration: otherwise the per-slot addresses are hoisted out of the
            // k loop and held in VGPRs across it (7 slots x ~6 registers -> spills)
            const int64_t* slp = pk_launder(a.slice_ptr);
            const int16_t* cop = pk_launder(a.cols);
            const double* vap = pk_launder(a.vals);
            const double* uvp = pk_launder(a.u);
            const int32_t* uop = a.uoff ? pk_launder(a.uoff) : nullptr;
            const int16_t* ucp = a.uoff ? pk_launder(a.ucol) : nullptr;
#define PK_SPMV(MODE)                                                                              \
    if (!rv) {                                                                                     \
        _Pragma("unroll") for (int j = 0; j < MAXS; ++j) {                                         \
            if (j < nreg) {                                                                        \
                const double v = sell_row_pair<pk_u<MAXS, PROF>(), MODE>(s0 + j, lane, slp, cop, vap, uvp, olo, ohi, uop, ucp); \
                if (j < PK_VL) vl[j * 64] = v; else vv[j] = v;                                     \
            }                                                                                      \
            asm volatile("" ::: "memory");                                                         \
        }                                                                                          \
    } else {                                                                                       \
        _Pragma("unroll") for (int jj = 0; jj < MAXS; ++jj) {                                      \
            const int j = MAXS - 1 - jj;                                                           \
            if (j < nreg) {                                                                        \
                const double v = sell_row_pair<pk_u<MAXS, PROF>(), MODE>(s0 + j, lane, slp, cop, vap, uvp, olo, ohi, uop, ucp); \
                if (j < PK_VL) vl[j * 64] = v; else vv[j] = v;                                     \
            }                                                                                      \
            asm volatile("" ::: "memory");                                                         \
        }                                                                                          \
    }
            // DIST: a workgroup whose gather window reaches other ranks reads the rows of other ranks past this GPU's
            // L2 (they arrive from other GPUs; the L2 may hold the previous iteration's copy), its own rank's rows
            // as usual (mode 3 picks per element)
            if (DIST && ghost) {
                PK_SPMV(3)
            } else {
                PK_SPMV((GSC1 ? 1 : 0))
            }
#undef PK_SPMV
            if constexpr (PROF) {   // this wave's own SpMV time (results back: the v slots are written)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                wspmv += __builtin_amdgcn_s_memtime() - tw0;
            }
            double dp = 0.0;
#pragma unroll
            for (int j = 0; j < MAXS; ++j) dp += uo[j] * (j < PK_VL ? vl[j * 64] : vv[j]);   // absent rows: uo = 0
            if constexpr (OVF) {   // overflow slices: v to HBM, u.v from the own u (this lane stored it last update)
                __builtin_amdgcn_sched_barrier(0);
                for (int q = 0; q < nov; ++q) {
                    const int sq = s0 + MAXS + q;
                    const double v = sell_row_pair<pk_u<MAXS, PROF>(), GSC1>(sq, lane, slp, cop, vap, uvp, 0, 0, uop, ucp);
                    const int row = sq * 64 + lane;
                    if (row < nrows) {
                        a.v[row] = v;
                        dp += a.u[row] * v;
                    }
                }
            }
            // ---- publish d (and g of the last update), grid barrier, fixed-order sums
            const int bank = k & 1;
            double* pd = a.part + (size_t)bank * 2 * G;
            PK_MARK(1);
            const double dsum = pk_block_sum(dp, lds16);
            PK_MARK(2);
            // FEM_PK_PF: waves 1..15 load one 8-byte word of every 128-byte line of the first 8 KB of the slice the
            // next SpMV starts with (the matrix never changes), so those lines sit in L2 when the barrier releases
            // and the memory-side cache streams part of the next SpMV while every workgroup waits; nothing computed
            // from them (the results are unchanged), and wave 0 -- the one that polls -- issues none
            double pfv = 0.0;
            if (FEM_PK_PF && wv != 0 && nreg > 0) {
                const int jf = (a.rev && (((it + 1) & 1) != 0)) ? nreg - 1 : 0;
                const int64_t q0 = slp[s0 + jf], q1 = slp[s0 + jf + 1];
                if ((int64_t)lane * 16 < q1 - q0) pfv = vap[q0 + (int64_t)lane * 16];
            }
            if (threadIdx.x == 0) __hip_atomic_store(pd + L, dsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // (pk_block_sum ended on a workgroup barrier: the grid barrier needs no entry barrier of its own)
#if FEM_PK_PROBE_NOBAR
            // timing probe only (wrong scalars): no grid barrier, every workgroup steps on its own partial -- the
            // neighbour-only coupling (u-flags) a pipelined iteration would leave, i.e. its speed bound
            // (the arrivals still count, without the wait, so the chunk-end barrier's epochs stay consistent)
            if (threadIdx.x == 0) {
                lds_dg[0] = dsum;
                lds_dg[1] = g;
                const unsigned old = __hip_atomic_fetch_add(sy + PK_GRP + grp * PK_LINE, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                if ((old + 1) % nper == 0)   // workgroups desynchronise: every nper-th arrival of the group
                    for (int r = 0; r < NXCD; ++r)
                        __hip_atomic_fetch_add(sy + PK_GEN + r * PK_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
#else
            if (!(DIST ? pk_barrier_dist(a, sy, grp, nper, e, &lds_ok, pd, k > 0 ? pd + G : nullptr, G, lds_dg, false)
                       : pk_barrier(sy, grp, nper, e, &lds_ok, pd, k > 0 ? pd + G : nullptr, G, lds_dg, false))) {
                fail = true;
                break;
            }
#endif
            if (FEM_PK_PF) asm volatile("" ::"v"(pfv));   // (keeps the loads; they completed under the barrier)
            elast = e;
            const double d = lds_dg[0];
            if (k > 0) g = lds_dg[1];
            PK_MARK(3);
            // ---- step (k_cg1_step)
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
            if (!stop && it >= max_iter) stop = true;   // poll reports FEM_PCG_MAXITER
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
            PK_MARK(4);
            // ---- update the own rows, publish u and the g partial (bank of the next iteration)
            double gp = 0.0;
            // per-slot store addresses recomputed every iteration (hoisted out of the k loop they are spilled)
            unsigned rbi = rb;
            double* ust = pk_launder(a.u);
            asm volatile("" : "+v"(rbi));
#pragma unroll
            for (int j = 0; j < MAXS; ++j) {
                // branch-free over the lanes (rows past nrows hold zeros: their SpMV rows are zero padding); only
                // the u store is masked. Exec-masked updates of the loop-carried arrays cost register copies.
                if (j < nreg) {
                    const double pi = uo[j] + bnew * pp[j];
                    const double si = (j < PK_VL ? vl[j * 64] : vv[j]) + bnew * ss[j];
                    pp[j] = pi;
                    ss[j] = si;
                    xl[j * 64] += al * pi;
                    double ri = rr[j] - al * si;
                    const double wi = wl[j * 64];
                    if (cg && wi == 0.0) ri = 0.0;
                    rr[j] = ri;
                    const double ui = wi * ri;
                    uo[j] = ui;
                    if (PK_ON(j)) {
                        __hip_atomic_store(ust + (rbi + 64u * j), ui, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if constexpr (DIST) {
                            if (pubmask) pk_publish_row(a, L, pubmask, rbi + 64u * j, ui);
                        }
                    }
                    gp += ri * ui;
                }
            }
            if constexpr (OVF) {   // overflow rows: the same update on the HBM-resident state
                __builtin_amdgcn_sched_barrier(0);
                for (int q = 0; q < nov; ++q) {
                    const int row = (s0 + MAXS + q) * 64 + lane;
                    if (row < nrows) {
                        const double pi = a.u[row] + bnew * a.p[row];
                        const double si = a.v[row] + bnew * a.s[row];
                        a.p[row] = pi;
                        a.s[row] = si;
                        a.x[row] += al * pi;
                        double ri = a.r[row] - al * si;
                        const double wi = a.w[row];
                        if (cg && wi == 0.0) ri = 0.0;
                        a.r[row] = ri;
                        const double ui = wi * ri;
                        __hip_atomic_store(ust + row, ui, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        gp += ri * ui;
                    }
                }
            }
            // one workgroup barrier for both the g block sum and the u hand-off: every wave leaves its g wave sum
            // in LDS and drains its u stores, then thread 0 sums (wave order, as pk_block_sum), stores the g
            // partial and raises the u-flag (the g partial is covered by the next grid barrier's drain, not by
            // this flag)
            {
                const double gw = wave_sum(gp);
                if (lane == 0) lds16[wv] = gw;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its u stores
            __syncthreads();
            if (threadIdx.x == 0) {
                double gsum = 0.0;
#pragma unroll
                for (int i = 0; i < PK_WAVES; ++i) gsum += lds16[i];
                __hip_atomic_store(a.part + (size_t)(bank ^ 1) * 2 * G + G + L, gsum, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                pk_st(uf + Lg * PK_LINE, e);
                if constexpr (DIST) {
                    if (pubmask) {   // rows published to other GPUs (every wave drained them): one system release
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // for the XCD's L2, then the flags there
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        pk_publish_flag(a, Lg, pubmask, e);
                    }
                }
            }
            PK_MARK(5);
        }
    }
    // ---- state back to memory (u is already there; nothing to store when no iteration ran). The chunk-end barrier
    // below changes none of it, so every wave but wave 0 (which arrives for its workgroup after draining its own
    // stores) writes it before the barrier and the traffic drains under the barrier's latency
    auto store_state = [&]() {
        if (!st_loaded) return;
#pragma unroll
        for (int j = 0; j < MAXS; ++j) {
            if (PK_ON(j)) {
                const unsigned row = rb + 64u * j;
                a.r[row] = rr[j];
                a.p[row] = pp[j];
                a.s[row] = ss[j];
                a.x[row] = xl[j * 64];
            }
        }
    };
    if (wv != 0) store_state();
    // ---- chunk end without a stop: one more barrier makes the last g partials visible; stop test of that g
    if (!fail && !halt && k == a.kmax && a.kmax > 0) {
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
                rz_new = g;   // r.z of the current iterate, what fem_pcg_poll reports between chunks
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
    if constexpr (PROF) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        pacc[7] += __builtin_amdgcn_s_memtime() - pt;
        if (threadIdx.x == 0)
            for (int i = 0; i < PK_NPROF; ++i) a.prof[(size_t)L * PK_NPROF + i] = pacc[i];
        if (lane == 0) a.prof[(size_t)G * PK_NPROF + (size_t)L * PK_WAVES + wv] = wspmv;
    }
    if (L == 0 && threadIdx.x == 0) {
        if (fail) {
            stop_iter = (int)pk_ld(sy + PK_TMO);   // where the first give-up happened (see pk_wait_ge)
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
        st->pk_epoch = elast;   // every workgroup read the base before its first barrier of this launch
    }
}
#undef PK_ON
#undef PK_MARK

// empty gather windows before k_pk_window: lo = lo_empty, hi = -1 for every logical workgroup
__global__ void k_pk_window_init(int G, int lo_empty, int* __restrict__ win) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < G) {
        win[i] = lo_empty;
        win[G + i] = -1;
    }
}

__global__ void k_pk_window(int64_t nslices, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                            const int16_t* __restrict__ dcols, int G, int* __restrict__ lo, int* __restrict__ hi) {
    const int64_t W = (int64_t)G * PK_WAVES;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nslices * 64;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t >> 6;
        const int l = (int)(t & 63);
        const int64_t row = s * 64 + l;
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        int dmin = 0, dmax = 0;
        if (row < nrows) {
#pragma unroll 8
            for (int kk = 0; kk < w; ++kk) {   // unrolled: the delta loads of a row in flight together
                const int d = dcols[p0 + 64 * kk + l];
                dmin = d < dmin ? d : dmin;
                dmax = d > dmax ? d : dmax;
            }
        }
        int64_t cmin, cmax;
        pk_slice_span(s, nrows, dmin, dmax, &cmin, &cmax);   // wave-uniform
        auto owner = [&](int64_t r) {   // logical workgroup owning row r: largest wave gw with gw S / W <= slice
            const int64_t sl = r >> 6;
            const int64_t gw = ((sl + 1) * W - 1) / nslices;
            return (int)(gw / PK_WAVES);
        };
        // the 64 lanes of a wave hold the 64 rows of one slice (same owner): one atomic pair per wave (1.7M-thread
        // atomics on 2 G words cost 4.4 ms)
        if (l == 0) {
            const int me = owner(row);
            atomicMin(lo + me, owner(cmin));
            atomicMax(hi + me, owner(cmax));
        }
    }
}

// DIST gather windows: for every own slice of this rank (global slices [sbase, sbase + nloc)), the first and last
// GLOBAL logical workgroup (rank * G + L) owning a column of its rows; ranks own the slice ranges split[r..r+1)
struct PkSplit {
    int64_t b[PK_MAX_RANKS + 1];
};
__global__ void k_pk_window_dist(int64_t sbase, int64_t nloc, int64_t nrows, const int64_t* __restrict__ slice_ptr,
                                 const int32_t* __restrict__ cols, int G, PkSplit split, int nranks,
                                 int* __restrict__ lo, int* __restrict__ hi, int* __restrict__ cwin) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nloc * 64; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = sbase + (t >> 6);
        const int l = (int)(t & 63);
        const int64_t row = s * 64 + l;
        const int64_t p0 = slice_ptr[s];
        const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
        int dmin = 0, dmax = 0;   // the slice's delta union (k_pk_window)
        if (row < nrows)
            for (int kk = 0; kk < w; ++kk) {
                const int d = (int)(cols[p0 + 64 * kk + l] - row);
                dmin = d < dmin ? d : dmin;
                dmax = d > dmax ? d : dmax;
            }
        int64_t cmin, cmax;
        pk_slice_span(s, nrows, dmin, dmax, &cmin, &cmax);
        auto owner = [&](int64_t r) {   // global logical workgroup owning row r
            const int64_t sl = r >> 6;
            int q = 0;
            while (q + 1 < nranks && split.b[q + 1] <= sl) ++q;
            const int64_t S = split.b[q + 1] - split.b[q];
            const int64_t tl = sl - split.b[q];
            const int64_t L = S > 0 ? ((tl + 1) * G - 1) / S : 0;
            return (int)(q * G + (L < G ? L : G - 1));
        };
        const int me = owner(s * 64) - (int)(owner(sbase * 64) / G) * G;   // local logical workgroup of slice s
        if (l == 0) {
            atomicMin(lo + me, owner(cmin));
            atomicMax(hi + me, owner(cmax));
            atomicMin(cwin, (int)cmin);   // the rank's column window: rows of other ranks it gathers
            atomicMax(cwin + 1, (int)cmax);
        }
    }
}

}  // namespace fem
