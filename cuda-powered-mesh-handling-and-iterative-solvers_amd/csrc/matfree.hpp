// Element-chunk (matrix-free) c3d4 operator: y = K x = sum_e P_e^T K_e P_e x formed from the vertex coordinates in
// every application, never stored -- the reference's element-by-element product (`compute_nodal_forces`,
// `solver/element.py:429-464`) with K_e of `compute_c3d4_K_matrix` (`:883-903`) evaluated in closed form:
//   elasticity  f_a = V sigma(H) g_a,  H = sum_b x_b g_b^T,  sigma = lambda tr(H) I + mu (H + H^T)
//               (= sum_b K_ab x_b with K_ab = V (lambda g_a g_b^T + mu g_b g_a^T + mu (g_a . g_b) I));
//   Poisson     f_a = kappa V g_a . (sum_b g_b x_b).
// Layout (built once per mesh by fem_mf_create, matfree.hip): the elements in Morton order of their centroids, cut
// into chunks of <= MF_EC elements touching <= MF_NC nodes; per chunk its local nodes (ascending global id) and, per
// local node, the (element, corner) pairs that touch it in ascending order. One workgroup per chunk gathers the local
// nodes' coordinates and x into LDS, forms the element vectors f (MF_PASS elements at a time), and every local node
// sums its pairs in that fixed order into a slot (chunk-major); a node's value is the sum of its slots in ascending
// chunk order (k_mf_gather). Deterministic: no atomics, every sum in a fixed order.
#pragma once
#include "common.hpp"
#include "element.hpp"

#include <stdlib.h>

namespace fem {

// slot stores (FEM_MF_NT = 1: non-temporal, the merged update reads them once after the kernel boundary)
#ifndef FEM_MF_NT
#define FEM_MF_NT 0
#endif
__device__ __forceinline__ void mf_store_slot(double* p, double v) {
#if FEM_MF_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}


// Chunk geometry. FEM_MF_WAVE (default): a chunk per WAVE -- <= 64 elements / <= 64 nodes (pieces of 16 elements when
// more), every wave of a workgroup walking its own chunks with no workgroup barrier, ~10 KB of LDS per wave. Else a
// chunk per workgroup: <= 512 elements / <= 256 nodes (pieces of 64), two passes of 256 elements, 41.6 KB per
// workgroup and its barriers.
#ifndef FEM_MF_WAVE
#define FEM_MF_WAVE 0
#endif
#if FEM_MF_WAVE
constexpr int MF_EC = 64;       // elements per chunk (at most)
constexpr int MF_NC = 64;       // local nodes per chunk (at most)
constexpr int MF_PIECE = 16;    // elements per piece of a chunk that touched more than MF_NC nodes
#else
// 240 nodes (not 256): with the pair pointers in registers and the element vectors unpadded the chunk's LDS is
// 40,192 bytes, so 4 workgroups (16 waves) share a CU instead of 3 (41.6 KB each)
constexpr int MF_EC = 512;
constexpr int MF_NC = 240;      // local ids are bytes
constexpr int MF_PIECE = 32;
#endif
static_assert(4 * MF_PIECE <= MF_NC, "a piece of MF_PIECE elements always fits the node cap");
// FEM_MF_W512 = 1 (A/B): 512-thread workgroups -- the chunk's 512 element vectors formed in one pass (64 KB of LDS,
// 2 workgroups per CU: the same 16 waves) and two lanes per local node in the node sums (each sums half of the
// node's pairs in order, the halves added once: a node's sum no longer waits for its longest-walking neighbour lane)
#ifndef FEM_MF_W512
#define FEM_MF_W512 0
#endif
#if FEM_MF_W512 && !FEM_MF_WAVE
constexpr int MF_PASS = 512;
constexpr int MF_BLOCK = 512;
constexpr int MF_LPN = 2;       // lanes per local node
#else
constexpr int MF_PASS = 256;    // elements formed per pass (= threads of the workgroup; workgroup chunks)
constexpr int MF_BLOCK = 256;
constexpr int MF_LPN = 1;
#endif
#ifndef FEM_MF_UNROLL
#define FEM_MF_UNROLL 4
#endif
constexpr int MF_U = FEM_MF_UNROLL;   // pairs whose LDS reads are issued together in the node sums
// FEM_MF_F0 = 1: corner 0's element vector not staged, f_0 = -(f_1 + f_2 + f_3) (mf_element's own formula) re-formed by
// the node sums that need it -- 3 of 4 vectors in LDS, 4 instead of 3 workgroups per CU for bs = 3; measured slower
// (10M elastic chunk kernel 326 vs 231 us: the corner-0 branch diverges inside every wave's node sums), off
#ifndef FEM_MF_F0
#define FEM_MF_F0 0
#endif

enum { MF_APPLY = 0, MF_DOT = 1, MF_DIAG = 2 };

// FEM_MF_SPCHECK = 1 (debug build, tools/mf_spcheck.py; never the default): the slot position ALSO carried through
// the prefetch records, as the walk did before commit c83e619, and compared at every slot store with the position
// read under the chunk's work. mf_spcheck: [0] stores checked, [1] mismatches, [2] first mismatch (chunk << 16 | tid),
// [3] its carried value, [4] the expected one, [5] its walk step (0 = first chunk of the workgroup)
#ifndef FEM_MF_SPCHECK
#define FEM_MF_SPCHECK 0
#endif
#if FEM_MF_SPCHECK
__device__ unsigned long long mf_spcheck[8];
#endif
// FEM_MF_PROF (timing builds only, wrong results): bit 0 skips the element formation (the staged vectors are the
// nodes' x), bit 1 the node sums (each slot gets one pair value) -- what the chunk kernel costs without each phase
#ifndef FEM_MF_PROF
#define FEM_MF_PROF 0
#endif

// staged corners of a mode (the diagonal's corner-0 values are not -(f_1 + f_2 + f_3))
template <int MODE>
constexpr int mf_fc() { return (FEM_MF_F0 && MODE != MF_DIAG) ? 3 : 4; }

// device view of the operator
struct MfOp {
    int64_t nchunks, nslots, nnodes;
    int bs;
    const int32_t* cptr;    // [nchunks + 1] element offsets (into the Morton-ordered arrays)
    const int32_t* sbase;   // [nchunks + 1] slot offsets (= local node counts, prefix summed)
    const int32_t* cnode;   // [nslots] global node of each slot (ascending within a chunk)
    const uint32_t* eloc;   // [M] the element's 4 local node ids, one byte each (corner b in byte b)
    const uint16_t* lptr;   // [nslots + nchunks] per chunk c at sbase[c] + c: first pair of local node l, + end
    const uint16_t* lent;   // [4 M] per chunk at 4 cptr[c]: pairs (element_in_chunk << 2 | corner), node-major
    const int32_t* nptr;    // [nnodes + 1] node -> its slots
    const int32_t* nslot;   // [nslots] slots of each node, ascending (= ascending chunk)
    const int32_t* spos;    // [nslots] or null: node-major slot storage -- slot s stored at spos[s], a node's slots at
                            // [nptr[a], nptr[a + 1]) (readers stream them; nslot unused)
    const double* X;        // [nnodes, 3] coordinates
    double lam, mu, kappa;
};

// the host object (fem_mf of the C-ABI, matfree.hip) as pcg.hip's K1 sees it
MfOp mf_op(const fem_mf* m);
double* mf_slots(const fem_mf* m);
int mf_bs(const fem_mf* m);
int64_t mf_nodes(const fem_mf* m);
int64_t mf_nslots(const fem_mf* m);
// y = K x / d = diag K through the caller's slot buffer ([mf_nslots * bs] doubles)
int mf_apply(fem_mf* m, const double* x, double* y, double* slots, hipStream_t st);
int mf_diag(fem_mf* m, double* d, double* slots, hipStream_t st);

// 1 / x to full precision without the IEEE division sequence: v_rcp_f64 and two Newton steps (within an ulp)
__device__ __forceinline__ double mf_rcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

// Element vectors of one element: f[a][c] for the 4 corners (BS = 3: c = 0..2; BS = 1: c = 0). DIAG: the diagonal of
// the corner's own block (K_aa)_cc instead of (K_e x)_a. In cofactor form: with the edge vectors e_b = x_b - x_0 and
// their cofactors c_1 = e_2 x e_3, c_2 = e_3 x e_1, c_3 = e_1 x e_2, c_0 = -(c_1 + c_2 + c_3), the gradients are
// g_b = c_b / det and V = |det| / 6, so V g_a g_b^T = c_a c_b^T / (6 |det|): every product is formed from the
// unscaled cofactors and scaled once by s = 1 / (6 |det|).
template <int BS, int MODE>
__device__ __forceinline__ void mf_element(const double xc[4][3], const double xv[4][BS], double lam, double mu,
                                           double kappa, double f[4][BS]) {
    double e[3][3], c[4][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        e[0][k] = xc[1][k] - xc[0][k];
        e[1][k] = xc[2][k] - xc[0][k];
        e[2][k] = xc[3][k] - xc[0][k];
    }
#pragma unroll
    for (int b = 0; b < 3; ++b) {   // c_{b+1} = e_{b+1} x e_{b+2} (indices mod 3)
        const double* u = e[(b + 1) % 3];
        const double* v = e[(b + 2) % 3];
        c[b + 1][0] = u[1] * v[2] - u[2] * v[1];
        c[b + 1][1] = u[2] * v[0] - u[0] * v[2];
        c[b + 1][2] = u[0] * v[1] - u[1] * v[0];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) c[0][k] = -(c[1][k] + c[2][k] + c[3][k]);
    const double det = e[0][0] * c[1][0] + e[0][1] * c[1][1] + e[0][2] * c[1][2];
    const double sc = mf_rcp(6.0 * fabs(det));
    if constexpr (MODE == MF_DIAG) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const double cc = c[a][0] * c[a][0] + c[a][1] * c[a][1] + c[a][2] * c[a][2];
            if constexpr (BS == 1) {
                f[a][0] = kappa * cc * sc;
            } else {
#pragma unroll
                for (int q = 0; q < 3; ++q) f[a][q] = sc * ((lam + mu) * (c[a][q] * c[a][q]) + mu * cc);
            }
        }
        return;
    }
    if constexpr (BS == 1) {
        double gu[3];   // det x the gradient of x
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double d1 = xv[1][0] - xv[0][0], d2 = xv[2][0] - xv[0][0], d3 = xv[3][0] - xv[0][0];
            gu[k] = c[1][k] * d1 + c[2][k] * d2 + c[3][k] * d3;
        }
        const double s = kappa * sc;
#pragma unroll
        for (int a = 1; a < 4; ++a) f[a][0] = s * (c[a][0] * gu[0] + c[a][1] * gu[1] + c[a][2] * gu[2]);
        f[0][0] = -(f[1][0] + f[2][0] + f[3][0]);
    } else {
        // H[i][j] = sum_b (x_b - x_0)[i] c_b[j]   (det x the displacement gradient)
        double d[3][3];
#pragma unroll
        for (int b = 0; b < 3; ++b)
#pragma unroll
            for (int i = 0; i < 3; ++i) d[b][i] = xv[b + 1][i] - xv[0][i];
        double H[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) H[i][j] = d[0][i] * c[1][j] + d[1][i] * c[2][j] + d[2][i] * c[3][j];
        const double lt = lam * (H[0][0] + H[1][1] + H[2][2]);
        const double m2 = 2.0 * mu;
        // s sigma(H), symmetric
        const double s00 = sc * (lt + m2 * H[0][0]);
        const double s11 = sc * (lt + m2 * H[1][1]);
        const double s22 = sc * (lt + m2 * H[2][2]);
        const double s01 = sc * (mu * (H[0][1] + H[1][0]));
        const double s02 = sc * (mu * (H[0][2] + H[2][0]));
        const double s12 = sc * (mu * (H[1][2] + H[2][1]));
#pragma unroll
        for (int a = 1; a < 4; ++a) {
            f[a][0] = s00 * c[a][0] + s01 * c[a][1] + s02 * c[a][2];
            f[a][1] = s01 * c[a][0] + s11 * c[a][1] + s12 * c[a][2];
            f[a][2] = s02 * c[a][0] + s12 * c[a][1] + s22 * c[a][2];
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) f[0][q] = -(f[1][q] + f[2][q] + f[3][q]);
    }
}

// FEM_MF_ELC = 1 (A/B): the element vectors of a pass staged [element][corner][component] (one
// element's 4 BS values contiguous: its thread stores them as 16-byte writes, a node's pair read is one 16-byte and
// one 8-byte LDS read for BS = 3 instead of three 8-byte reads 2 KB apart). Measured slower on the 10M elastic cube:
// chunk kernel 220.4 / 221.3 vs 195.9 / 196.9 us (profiles/r06f_mf_elc_ab.txt): the select between the two read
// shapes costs VALU and the 16-byte reads at 24-byte strides conflict more; 0 (default): [corner * BS + c][element].
#ifndef FEM_MF_ELC
#define FEM_MF_ELC 0
#endif
template <int FC>
constexpr bool mf_elc() { return FEM_MF_ELC && FC == 4; }

// LDS of one chunk application (a local node's pair range [lp, lp1) travels in its thread's registers)
// FEM_MF_NDSKEW = 1 (A/B): the local-node rows of nd skewed by one 16-byte unit every 16 rows (a row is 3 (BS = 3) or
// 2 (BS = 1) 16-byte units, so rows l and l + 16 start in the same 16-byte bank group). Measured slower on the 10M
// elastic cube: chunk kernel 185-186 vs 179-180 us (profiles/r06h_mf_ndskew_ab.txt); off
#ifndef FEM_MF_NDSKEW
#define FEM_MF_NDSKEW 0
#endif
template <int BS, int FC>
struct MfLds {
    static constexpr int NDU = (3 + BS) / 2;   // 16-byte units per node row
    // per local node: coordinates, then x (rows of NDU 16-byte units; row l at unit l NDU (+ l / 16 skewed))
    double2 ndu[MF_NC * NDU + (FEM_MF_NDSKEW ? MF_NC / 16 + 1 : 0)];
    __device__ __forceinline__ double2* nd_row(int l) { return ndu + l * NDU + (FEM_MF_NDSKEW ? (l >> 4) : 0); }
    __device__ __forceinline__ const double2* nd_row(int l) const {
        return ndu + l * NDU + (FEM_MF_NDSKEW ? (l >> 4) : 0);
    }
    // element vectors of the current pass: [staged corner * BS + c][element], or (mf_elc) fe[element][corner][c].
    // Row stride MF_PASS + FEM_MF_FSPAD (default 1): the node sums' lanes read the corners of SHARED elements in the
    // same step -- same element, rows 3 apart -- which a stride of 256 doubles (= 0 mod the 32 eight-byte bank pairs)
    // put into one bank; an odd stride spreads them
#ifndef FEM_MF_FSPAD
#define FEM_MF_FSPAD 1
#endif
    alignas(16) double fs[FC * BS][MF_PASS + FEM_MF_FSPAD];
    alignas(16) uint16_t ent[4 * MF_EC];   // the chunk's pairs, node-major
};

// the element vector of pair pe (element << 2 | corner) of the pass starting at element h
template <int BS, int FC>
__device__ __forceinline__ void mf_pair_value(const MfLds<BS, FC>& L, int pe, int h, double v[BS]) {
    const int el = (pe >> 2) - h, b = pe & 3;
    if constexpr (mf_elc<FC>()) {
        const double* fe = &L.fs[0][0];
        const int base = (el * 4 + b) * BS;
        if constexpr (BS == 3) {   // 24 bytes at 8 (mod 16) when b is odd: the 16-byte read one double later
            const int odd = b & 1;
            const double2 d = *reinterpret_cast<const double2*>(fe + base + odd);
            const double sgl = fe[base + (odd ? 0 : 2)];
            v[0] = odd ? sgl : d.x;
            v[1] = odd ? d.x : d.y;
            v[2] = odd ? d.y : sgl;
        } else {
#pragma unroll
            for (int q = 0; q < BS; ++q) v[q] = fe[base + q];
        }
        return;
    }
    if (FC == 3 && b == 0) {
#pragma unroll
        for (int q = 0; q < BS; ++q) v[q] = -(L.fs[q][el] + L.fs[BS + q][el] + L.fs[2 * BS + q][el]);
    } else {
        const int row = (b - (4 - FC)) * BS;
#pragma unroll
        for (int q = 0; q < BS; ++q) v[q] = L.fs[row + q][el];
    }
}

// What a thread loads for one chunk ahead of its use (software pipeline over a workgroup's chunks): the chunk's
// ranges, this thread's local node (id, slot position, pair range, coordinates, x), 8 pairs and the local ids of its
// 2 elements; and the ranges of the chunk this record carries next (three chunks on).
//
// Every load is issued unconditionally (lanes past the chunk's nodes / pairs / elements read a clamped in-range
// index, their values unused), nothing is computed from a loaded value before its use, and the three records rotate
// by name (mf_walk unrolls its loop by three), never by copy. A copy of a record, or a select / zero-fill of a field,
// makes the compiler wait for the loads in flight into it, and a load under a branch makes its wait counts
// conservative past the branch (s_waitcnt vmcnt(0)): the round-4/5 walk, whose records were copied (cur = n1; n1 =
// n2) and loaded under `tid < nn`, waited for each prefetch right after issuing it -- ~4 exposed memory latencies per
// chunk (a FEM_MF_PROF = 3 build, no element formation and no node sums, still took 125 of the kernel's 217 us).
// Every field is defined in every lane (copying indeterminate values was the round-4 NaN).
typedef unsigned int mf_u32x4 __attribute__((ext_vector_type(4)));   // a native vector (HIP's uint4 is a union
                                                                        // wrapper that kept the records in scratch)
template <int BS>
struct MfPf {
    int e0, ne, s0, nn;             // this record's chunk: elements [e0, e0 + ne), slots [s0, s0 + nn)
    int b_e, b_s;                   // ranges of the chunk this record carries next: lane 0 its first element /
                                    // slot, lane 1 its end (lane-varying addresses keep the loads off the scalar
                                    // path, whose v_readfirstlane the compiler places right after the load)
    int node, sp, lp, lp1;          // local node tid: global id, slot position (spos; or unused), its pairs [lp, lp1)
    mf_u32x4 ent;
    uint32_t el[MF_EC / MF_PASS];
    double xv[3], pv[BS];
};

// stage 0: the ranges of chunk c (cptr / sbase), into the record's b_* (consumed by mf_pf1 a step later)
template <int BS>
__device__ __forceinline__ void mf_pf0(const MfOp& op, int64_t c, MfPf<BS>& f) {
    const int h = threadIdx.x & 1;
    f.b_e = op.cptr[c + h];
    f.b_s = op.sbase[c + h];
}

// stage 1: the chunk's ids / pairs / local ids, after its ranges arrived
template <int BS>
__device__ __forceinline__ void mf_pf1(const MfOp& op, int64_t c, MfPf<BS>& f) {
    const int tid = threadIdx.x;
    f.e0 = __builtin_amdgcn_readlane(f.b_e, 0);
    f.ne = __builtin_amdgcn_readlane(f.b_e, 1) - f.e0;
    f.s0 = __builtin_amdgcn_readlane(f.b_s, 0);
    f.nn = __builtin_amdgcn_readlane(f.b_s, 1) - f.s0;
    const int tn = tid / MF_LPN;                  // this lane's local node (MF_LPN lanes per node)
    const int t = tn < f.nn ? tn : f.nn - 1;      // a chunk has >= 1 node and >= 1 element
    f.node = op.cnode[f.s0 + t];
    f.lp = op.lptr[f.s0 + c + t];
    f.lp1 = op.lptr[f.s0 + c + t + 1];           // the chunk's end marker for its last node
    f.sp = (op.spos ? op.spos : op.cnode)[f.s0 + t];   // unconditional (chunk-major slots: unused, s0 + tid)
    const int q = 8 * tid < 4 * f.ne ? tid : (4 * f.ne - 1) >> 3;
    f.ent = reinterpret_cast<const mf_u32x4*>(op.lent + 4 * (int64_t)f.e0)[q];
#pragma unroll
    for (int j = 0; j < MF_EC / MF_PASS; ++j) {
        const int e = tid + MF_PASS * j < f.ne ? tid + MF_PASS * j : f.ne - 1;
        f.el[j] = op.eloc[f.e0 + e];
    }
}

// stage 2: the local node's coordinates and x (after stage 1's node id arrived)
template <int BS, int MODE>
__device__ __forceinline__ void mf_pf2(const MfOp& op, const double* __restrict__ x, MfPf<BS>& f) {
    const int64_t g = f.node;
#pragma unroll
    for (int k = 0; k < 3; ++k) f.xv[k] = op.X[3 * g + k];
#pragma unroll
    for (int k = 0; k < BS; ++k) f.pv[k] = MODE == MF_DIAG ? 0.0 : x[BS * g + k];
}

// One chunk of the walk: cur is formed and stored, n1 (next chunk) gets its node gathers, n2 (the one after) its ids /
// pairs / local ids, cur its ranges for three chunks on. Returns whether this workgroup has a next chunk.
template <int BS, int MODE>
__device__ __forceinline__ bool mf_step(const MfOp& op, const double* __restrict__ x, double* __restrict__ slots,
                                        MfLds<BS, mf_fc<MODE>()>& L, int64_t base, int64_t per, int64_t nb,
                                        int64_t last, int64_t& k, MfPf<BS>& cur, MfPf<BS>& n1, MfPf<BS>& n2,
                                        double& dot) {
    constexpr int FC = mf_fc<MODE>();
    const int tid = threadIdx.x;
    // chunks past this workgroup's range load its last chunk's data again (in range and in L2, never used)
    const auto chunk = [&](int64_t kk) { return kk < per && base + kk < op.nchunks ? base + kk : last; };
    __syncthreads();   // the previous chunk's LDS reads are done
    const int tn = tid / MF_LPN;                   // this lane's local node
    const bool own = tn < cur.nn && tid % MF_LPN == 0;   // the lane that installs and stores the node
    if (own) {
#pragma unroll
        for (int q = 0; q < 3; ++q) reinterpret_cast<double*>(L.nd_row(tn))[q] = cur.xv[q];
#pragma unroll
        for (int q = 0; q < BS; ++q) reinterpret_cast<double*>(L.nd_row(tn))[3 + q] = cur.pv[q];
    }
    if (8 * tid < 4 * cur.ne) reinterpret_cast<mf_u32x4*>(L.ent)[tid] = cur.ent;
    // issue order: every load a later wait needs has the same younger loads behind it on every path (the prologue's
    // order matches), so the waits stay partial: s_waitcnt vmcnt(N > 0)
    mf_pf2<BS, MODE>(op, x, n1);
    mf_pf0<BS>(op, chunk(k + 3 * nb), cur);
    mf_pf1<BS>(op, chunk(k + 2 * nb), n2);
    __syncthreads();
    double acc[BS];
#pragma unroll
    for (int q = 0; q < BS; ++q) acc[q] = 0.0;
    int pos = tn < cur.nn ? cur.lp : 0;
    int end = tn < cur.nn ? cur.lp1 : 0;
    if constexpr (MF_LPN == 2) {   // lane 0 of the node: the first half of its pairs, lane 1 the rest
        const int half = (end - pos + 1) >> 1;
        if (tid & 1) pos += half;
        else end = pos + half;
    }
    // the node's pairs split at the pass boundary (pairs ascend by element): lower bound of 4 MF_PASS
    int mid = end;
    if (cur.ne > MF_PASS) {
        int lo = pos, len = end - pos;
        while (len > 0) {
            const int half = len >> 1;
            if (L.ent[lo + half] < 4 * MF_PASS) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        mid = lo;
    }
#pragma unroll
    for (int j = 0; j < MF_EC / MF_PASS; ++j) {
        const int h = MF_PASS * j;
        if (h >= cur.ne) break;
        if (h + tid < cur.ne) {
            const uint32_t w = cur.el[j];
            double xc[4][3], xv[4][BS], f[4][BS];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int l = (w >> (8 * b)) & 0xff;
                const double2* r = L.nd_row(l);
                const double2 a0 = r[0], a1 = r[1];
                xc[b][0] = a0.x;
                xc[b][1] = a0.y;
                xc[b][2] = a1.x;
                if constexpr (BS == 1) {
                    xv[b][0] = a1.y;
                } else {
                    const double2 a2 = r[2];
                    xv[b][0] = a1.y;
                    xv[b][1] = a2.x;
                    xv[b][2] = a2.y;
                }
            }
#if FEM_MF_PROF & 1
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int q = 0; q < BS; ++q) f[b][q] = xv[b][q] + xc[b][q];
#else
            mf_element<BS, MODE>(xc, xv, op.lam, op.mu, op.kappa, f);
#endif
            if constexpr (mf_elc<FC>()) {   // the element's 4 BS values contiguous (16-byte stores)
                double2* fe2 = reinterpret_cast<double2*>(&L.fs[0][0] + tid * 4 * BS);
                double fl[4 * BS];
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int q = 0; q < BS; ++q) fl[b * BS + q] = f[b][q];
#pragma unroll
                for (int t = 0; t < 2 * BS; ++t) fe2[t] = make_double2(fl[2 * t], fl[2 * t + 1]);
            } else {
#pragma unroll
                for (int b = 4 - FC; b < 4; ++b)
#pragma unroll
                    for (int q = 0; q < BS; ++q) L.fs[(b - (4 - FC)) * BS + q][tid] = f[b][q];
            }
        }
        __syncthreads();
        // every local node adds its pairs of this pass in ascending (element, corner) order; the pair reads of
        // four steps are issued before their adds (independent LDS loads, one latency per four pairs)
        const int stop = j == 0 ? mid : end;
#if FEM_MF_PROF & 2
        if (pos < stop) {
            double v[BS];
            mf_pair_value<BS, FC>(L, L.ent[pos], h, v);
#pragma unroll
            for (int q = 0; q < BS; ++q) acc[q] += v[q];
            pos = stop;
        }
#endif
        for (; pos + MF_U <= stop; pos += MF_U) {
            int pe[MF_U];
#pragma unroll
            for (int u = 0; u < MF_U; ++u) pe[u] = L.ent[pos + u];
            double v[MF_U][BS];
#pragma unroll
            for (int u = 0; u < MF_U; ++u) mf_pair_value<BS, FC>(L, pe[u], h, v[u]);
#pragma unroll
            for (int u = 0; u < MF_U; ++u)
#pragma unroll
                for (int q = 0; q < BS; ++q) acc[q] += v[u][q];
        }
        for (; pos < stop; ++pos) {
            double v[BS];
            mf_pair_value<BS, FC>(L, L.ent[pos], h, v);
#pragma unroll
            for (int q = 0; q < BS; ++q) acc[q] += v[q];
        }
        __syncthreads();
    }
    if constexpr (MF_LPN == 2) {   // the halves added once (a + b == b + a: both lanes hold the same sum)
#pragma unroll
        for (int q = 0; q < BS; ++q) acc[q] += __shfl_xor(acc[q], 1, 64);
    }
    if (own) {
#pragma unroll
        for (int q = 0; q < BS; ++q) {
            mf_store_slot(&slots[(int64_t)(op.spos ? cur.sp : cur.s0 + tn) * BS + q], acc[q]);
            if constexpr (MODE == MF_DOT) dot += cur.pv[q] * acc[q];
        }
#if FEM_MF_SPCHECK
        // the carried position against one read now (the round-4 question)
        const int spc = op.spos ? op.spos[cur.s0 + tn] : cur.s0 + tn;
        atomicAdd(&mf_spcheck[0], 1ull);
        if (op.spos && cur.sp != spc && atomicAdd(&mf_spcheck[1], 1ull) == 0) {
            mf_spcheck[2] = ((unsigned long long)(base + k) << 16) | (unsigned)tid;
            mf_spcheck[3] = (unsigned)cur.sp;
            mf_spcheck[4] = (unsigned)spc;
            mf_spcheck[5] = 0;
        }
#endif
    }
    k += nb;
    return k < per && base + k < op.nchunks;
}

// Every chunk of this workgroup (chunk ranges per XCD, consecutive chunks -- neighbours in space -- at once on one XCD,
// whose L2 then holds their shared nodes): the slot values of its local nodes (slots[spos[sbase[c] + l] * BS + c]);
// three chunks in flight: cur (installed in LDS and formed now), n1 (its node gathers issued at the top of this
// chunk), n2 (its ids / pairs / local ids issued now, its ranges a chunk earlier): every load has a whole chunk of
// work to arrive (~1-2 us of HBM latency under load). MODE_DOT returns this thread's part of sum_l x_l . slot_l over
// its chunks (0 elsewhere). x unused for MF_DIAG.
template <int BS, int MODE>
__device__ __forceinline__ double mf_walk(const MfOp& op, const double* __restrict__ x, double* __restrict__ slots,
                                          MfLds<BS, mf_fc<MODE>()>& L) {
    const int64_t per = (op.nchunks + NXCD - 1) / NXCD;
    const int64_t base = (int64_t)(blockIdx.x % NXCD) * per;
    const int64_t nb = gridDim.x / NXCD;
    int64_t k = blockIdx.x / NXCD;
    double dot = 0.0;
    if (k >= per || base + k >= op.nchunks) return dot;
    // this workgroup's last chunk: the stand-in for the chunks past its range (mf_step)
    const int64_t cnt = (per < op.nchunks - base ? per : op.nchunks - base);
    const int64_t last = base + k + ((cnt - 1 - k) / nb) * nb;
    const auto chunk = [&](int64_t kk) { return kk < per && base + kk < op.nchunks ? base + kk : last; };
    MfPf<BS> A, B, C;   // records rotate by name: the loop body is three steps
    mf_pf0<BS>(op, chunk(k), A);
    mf_pf0<BS>(op, chunk(k + nb), B);
    mf_pf1<BS>(op, chunk(k), A);
    mf_pf2<BS, MODE>(op, x, A);
    mf_pf0<BS>(op, chunk(k + 2 * nb), C);
    mf_pf1<BS>(op, chunk(k + nb), B);
    for (;;) {
        if (!mf_step<BS, MODE>(op, x, slots, L, base, per, nb, last, k, A, B, C, dot)) break;
        if (!mf_step<BS, MODE>(op, x, slots, L, base, per, nb, last, k, B, C, A, dot)) break;
        if (!mf_step<BS, MODE>(op, x, slots, L, base, per, nb, last, k, C, A, B, dot)) break;
    }
    return dot;
}

// LDS of one wave's chunk (FEM_MF_WAVE)
template <int BS, int FC>
struct MfLdsW {
    double nd[MF_NC][3 + BS];
    double fs[FC * BS][MF_EC + 1];
    uint16_t lp[MF_NC + 1];
    alignas(16) uint16_t ent[4 * MF_EC];
};

// LDS hand-off between the lanes of one wave: program order for the compiler (the hardware runs a wave's LDS
// operations in order)
__device__ __forceinline__ void mf_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int BS>
struct MfPfW {
    int e0, ne, s0, nn;
    int node;
    uint16_t lp;
    uint2 ent;
    uint32_t el;
    double xv[3], pv[BS];
};

template <int BS>
__device__ __forceinline__ void mf_pfw1(const MfOp& op, int64_t c, MfPfW<BS>& f) {
    const int lane = threadIdx.x & 63;
    f.e0 = __builtin_amdgcn_readfirstlane(op.cptr[c]);
    f.ne = __builtin_amdgcn_readfirstlane(op.cptr[c + 1]) - f.e0;
    f.s0 = __builtin_amdgcn_readfirstlane(op.sbase[c]);
    f.nn = __builtin_amdgcn_readfirstlane(op.sbase[c + 1]) - f.s0;
    f.node = 0;
    f.lp = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) f.xv[k] = 0.0;
#pragma unroll
    for (int k = 0; k < BS; ++k) f.pv[k] = 0.0;
    if (lane < f.nn) {
        f.node = op.cnode[f.s0 + lane];
        f.lp = op.lptr[f.s0 + c + lane];
    }
    f.ent = make_uint2(0, 0);
    if (4 * lane < 4 * f.ne) f.ent = reinterpret_cast<const uint2*>(op.lent + 4 * (int64_t)f.e0)[lane];
    f.el = lane < f.ne ? op.eloc[f.e0 + lane] : 0u;
}

template <int BS, int MODE>
__device__ __forceinline__ void mf_pfw2(const MfOp& op, const double* __restrict__ x, MfPfW<BS>& f) {
    if ((int)(threadIdx.x & 63) < f.nn) {
        const int64_t g = f.node;
#pragma unroll
        for (int k = 0; k < 3; ++k) f.xv[k] = op.X[3 * g + k];
#pragma unroll
        for (int k = 0; k < BS; ++k) f.pv[k] = MODE == MF_DIAG ? 0.0 : x[BS * g + k];
    }
}

// Every chunk of this WAVE (chunk ranges per XCD; consecutive chunks on one XCD at once), three chunks in flight as in
// mf_walk; lane l < nn owns local node l, lane e < ne element e. No workgroup barrier: the waves of a workgroup only
// share the CU.
template <int BS, int MODE>
__device__ __forceinline__ double mf_walk_w(const MfOp& op, const double* __restrict__ x, double* __restrict__ slots,
                                            MfLdsW<BS, mf_fc<MODE>()>& L) {
    constexpr int FC = mf_fc<MODE>();
    const int lane = threadIdx.x & 63;
    constexpr int WPB = MF_BLOCK / 64;
    const int64_t per = (op.nchunks + NXCD - 1) / NXCD;
    const int64_t base = (int64_t)(blockIdx.x % NXCD) * per;
    const int64_t nb = (int64_t)(gridDim.x / NXCD) * WPB;
    int64_t k = (int64_t)(blockIdx.x / NXCD) * WPB + (threadIdx.x >> 6);
    double dot = 0.0;
    if (k >= per || base + k >= op.nchunks) return dot;
    MfPfW<BS> cur, n1, n2;
    mf_pfw1<BS>(op, base + k, cur);
    bool has1 = k + nb < per && base + k + nb < op.nchunks;
    if (has1) mf_pfw1<BS>(op, base + k + nb, n1);
    mf_pfw2<BS, MODE>(op, x, cur);
    for (;;) {
        mf_wave_sync();   // the previous chunk's LDS reads are done
        if (lane < cur.nn) {
#pragma unroll
            for (int q = 0; q < 3; ++q) L.nd[lane][q] = cur.xv[q];
#pragma unroll
            for (int q = 0; q < BS; ++q) L.nd[lane][3 + q] = cur.pv[q];
            L.lp[lane] = cur.lp;
        }
        if (lane == 0) L.lp[cur.nn] = (uint16_t)(4 * cur.ne);
        if (lane < cur.ne) reinterpret_cast<uint2*>(L.ent)[lane] = cur.ent;
        const int64_t k2 = k + 2 * nb;
        const bool has2 = has1 && k2 < per && base + k2 < op.nchunks;
        if (has1) mf_pfw2<BS, MODE>(op, x, n1);
        if (has2) mf_pfw1<BS>(op, base + k2, n2);
        int spc = 0;   // this lane's slot position (see mf_walk)
        if (lane < cur.nn) spc = op.spos ? op.spos[cur.s0 + lane] : cur.s0 + lane;
        mf_wave_sync();
        if (lane < cur.ne) {
            const uint32_t w = cur.el;
            double xc[4][3], xv[4][BS], f[4][BS];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int l = (w >> (8 * b)) & 0xff;
                const double2* r = reinterpret_cast<const double2*>(&L.nd[l][0]);
                const double2 a0 = r[0], a1 = r[1];
                xc[b][0] = a0.x;
                xc[b][1] = a0.y;
                xc[b][2] = a1.x;
                if constexpr (BS == 1) {
                    xv[b][0] = a1.y;
                } else {
                    const double2 a2 = r[2];
                    xv[b][0] = a1.y;
                    xv[b][1] = a2.x;
                    xv[b][2] = a2.y;
                }
            }
            mf_element<BS, MODE>(xc, xv, op.lam, op.mu, op.kappa, f);
#pragma unroll
            for (int b = 4 - FC; b < 4; ++b)
#pragma unroll
                for (int q = 0; q < BS; ++q) L.fs[(b - (4 - FC)) * BS + q][lane] = f[b][q];
        }
        mf_wave_sync();
        if (lane < cur.nn) {
            double acc[BS];
#pragma unroll
            for (int q = 0; q < BS; ++q) acc[q] = 0.0;
            int pos = L.lp[lane];
            const int end = L.lp[lane + 1];
            for (; pos + MF_U <= end; pos += MF_U) {
                int pe[MF_U];
#pragma unroll
                for (int u = 0; u < MF_U; ++u) pe[u] = L.ent[pos + u];
                double v[MF_U][BS];
#pragma unroll
                for (int u = 0; u < MF_U; ++u) {
                    const int el = pe[u] >> 2, b = pe[u] & 3;
                    if (FC == 3 && b == 0) {
#pragma unroll
                        for (int q = 0; q < BS; ++q) v[u][q] = -(L.fs[q][el] + L.fs[BS + q][el] + L.fs[2 * BS + q][el]);
                    } else {
#pragma unroll
                        for (int q = 0; q < BS; ++q) v[u][q] = L.fs[(b - (4 - FC)) * BS + q][el];
                    }
                }
#pragma unroll
                for (int u = 0; u < MF_U; ++u)
#pragma unroll
                    for (int q = 0; q < BS; ++q) acc[q] += v[u][q];
            }
            for (; pos < end; ++pos) {
                const int pe = L.ent[pos];
                const int el = pe >> 2, b = pe & 3;
#pragma unroll
                for (int q = 0; q < BS; ++q) {
                    const double v = (FC == 3 && b == 0)
                                         ? -(L.fs[q][el] + L.fs[BS + q][el] + L.fs[2 * BS + q][el])
                                         : L.fs[(b - (4 - FC)) * BS + q][el];
                    acc[q] += v;
                }
            }
#pragma unroll
            for (int q = 0; q < BS; ++q) {
                mf_store_slot(&slots[(int64_t)spc * BS + q], acc[q]);
                if constexpr (MODE == MF_DOT) dot += cur.pv[q] * acc[q];
            }
        }
        if (!has1) break;
        k += nb;
        cur = n1;
        n1 = n2;
        has1 = has2;
    }
    return dot;
}

// the walker of the build's geometry, with its LDS
template <int BS, int MODE>
struct MfKernelLds {
#if FEM_MF_WAVE
    MfLdsW<BS, mf_fc<MODE>()> w[MF_BLOCK / 64];
#else
    MfLds<BS, mf_fc<MODE>()> b;
#endif
};
template <int BS, int MODE>
__device__ __forceinline__ double mf_walk_any(const MfOp& op, const double* __restrict__ x, double* __restrict__ slots,
                                              MfKernelLds<BS, MODE>& L) {
#if FEM_MF_WAVE
    return mf_walk_w<BS, MODE>(op, x, slots, L.w[threadIdx.x >> 6]);
#else
    return mf_walk<BS, MODE>(op, x, slots, L.b);
#endif
}

// resident workgroups of a chunk kernel (one pass of the grid over the chunks), cached per kernel
inline int mf_resident_grid(const void* fn, int block, int64_t nchunks) {
    static int cache[8] = {0};
    static const void* keys[8] = {nullptr};
    int per_cu = 0;
    for (int i = 0; i < 8; ++i)
        if (keys[i] == fn) per_cu = cache[i];
    if (per_cu == 0) {
        int dev = 0, ncu = 0, nb = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, block, 0) != hipSuccess || nb < 1)
            nb = 1, ncu = 256;
        per_cu = ((ncu / NXCD) * NXCD) * nb;
        for (int i = 0; i < 8; ++i)
            if (!keys[i] || keys[i] == fn) {
                keys[i] = fn;
                cache[i] = per_cu;
                break;
            }
    }
    static const int mult = [] {
        const char* e = getenv("FEM355_MF_GRID_MULT");   // A/B: workgroups per resident slot
        const int m = e ? atoi(e) : 1;
        return m < 1 ? 1 : m;
    }();
    int64_t g = (int64_t)per_cu * mult;
    if (const char* cap = getenv("FEM355_MF_GRID_CAP")) {   // tests: a small grid walks many chunks per workgroup
        const int64_t c = atoll(cap);
        if (c >= NXCD && c < g) g = (c / NXCD) * NXCD;
    }
    const int64_t want = ((nchunks + NXCD - 1) / NXCD) * NXCD;
    if (want < g) g = want;
    return (int)(g < NXCD ? NXCD : g);
}

// y[node] = sum of the node's slots in ascending chunk order (0 for a node of no element)
template <int BS>
__global__ void __launch_bounds__(256) k_mf_gather(MfOp op, const double* __restrict__ slots, double* __restrict__ y) {
    for (int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; a < op.nnodes;
         a += (int64_t)gridDim.x * blockDim.x) {
        const int k0 = op.nptr[a], k1 = op.nptr[a + 1];
        double s[BS];
#pragma unroll
        for (int k = 0; k < BS; ++k) s[k] = 0.0;
        for (int k = k0; k < k1; ++k) {
            const int64_t sl = op.spos ? k : op.nslot[k];
#pragma unroll
            for (int c = 0; c < BS; ++c) s[c] += slots[sl * BS + c];
        }
#pragma unroll
        for (int c = 0; c < BS; ++c) y[a * BS + c] = s[c];
    }
}

}  // namespace fem
