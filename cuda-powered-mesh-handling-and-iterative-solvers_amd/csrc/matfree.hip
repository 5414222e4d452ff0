// Element-chunk (matrix-free) c3d4 operator: build (fem_mf_create) and stand-alone application (fem_mf_apply,
// fem_mf_diag). The chunk kernels themselves are in matfree.hpp (shared with the PCG's K1 in pcg.hip).
//
// Build, all on the device except two small host reads of the per-chunk node counts:
//   1. node bounding box; per element the Morton key of its centroid's cell (cubic cells ~one element cluster wide, at
//      most 10 bits per axis), the connectivity range check
//      and the singular check (|det| < 1e-12, `solver/element.py:857-858`, the smallest such element reported);
//   2. elements sorted by key (stable radix sort: equal keys keep their file order);
//   3. chunks of MF_EC consecutive sorted elements; a chunk touching more than MF_NC nodes is halved, and each half
//      that still does halved again, down to MF_PIECE elements (<= MF_NC nodes each, always);
//   4. per chunk (one workgroup): the (node << 11 | element << 2 | corner) keys of its 4 ne corners sorted in LDS, the
//      local node list, the node-major pair list and every element's 4 local ids;
//   5. node -> slots: the (node, slot) pairs sorted by node (stable: slots ascend within a node).
#include <hipcub/hipcub.hpp>

#include <vector>

#include "matfree.hpp"

struct fem_mf {
    int bs = 3;
    int64_t M = 0, N = 0, nchunks = 0, nslots = 0;
    double lam = 0, mu = 0, kappa = 0;
    const double* X = nullptr;
    int32_t* eorder = nullptr;   // [M] element ids in Morton order
    int32_t* cptr = nullptr;
    int32_t* sbase = nullptr;
    int32_t* cnode = nullptr;
    uint32_t* eloc = nullptr;
    uint16_t* lptr = nullptr;
    uint16_t* lent = nullptr;
    int32_t* nptr = nullptr;
    int32_t* nslot = nullptr;
    int32_t* spos = nullptr;     // node-major slot positions (null: chunk-major slots)
    double* slots = nullptr;     // [nslots * bs] scratch of the stand-alone applications (fem_mf_apply / fem_mf_diag:
                                 // one stream at a time); every (P)CG context has its own (fem_pcg_set_operator_mf)
    fem::MfOp op() const {
        fem::MfOp o{};
        o.nchunks = nchunks;
        o.nslots = nslots;
        o.nnodes = N;
        o.bs = bs;
        o.cptr = cptr;
        o.sbase = sbase;
        o.cnode = cnode;
        o.eloc = eloc;
        o.lptr = lptr;
        o.lent = lent;
        o.nptr = nptr;
        o.nslot = nslot;
        o.spos = spos;
        o.X = X;
        o.lam = lam;
        o.mu = mu;
        o.kappa = kappa;
        return o;
    }
};

namespace fem {

// ---------------------------------------------------------------- build kernels
__global__ void __launch_bounds__(256) k_mf_bbox(const double* __restrict__ X, int64_t N, double* __restrict__ part) {
    __shared__ double red[6][256];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double v = X[3 * i + k];
            lo[k] = fmin(lo[k], v);
            hi[k] = fmax(hi[k], v);
        }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        red[k][threadIdx.x] = lo[k];
        red[3 + k][threadIdx.x] = hi[k];
    }
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                red[k][threadIdx.x] = fmin(red[k][threadIdx.x], red[k][threadIdx.x + o]);
                red[3 + k][threadIdx.x] = fmax(red[3 + k][threadIdx.x], red[3 + k][threadIdx.x + o]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

__device__ __forceinline__ uint32_t mf_spread10(uint32_t v) {   // 10 bits -> every third bit of 30
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// Morton keys, element ids, range and singular checks. bad[0]: smallest element with a node outside [0, N);
// bad[1]: smallest singular element
__global__ void __launch_bounds__(256) k_mf_keys(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                 int64_t M, int64_t N, const double* __restrict__ part, int nparts,
                                                 double cells, uint32_t* __restrict__ keys, int32_t* __restrict__ ids,
                                                 unsigned long long* __restrict__ bad) {
    __shared__ double box[6];
    if (threadIdx.x < 6) {
        double v = threadIdx.x < 3 ? INFINITY : -INFINITY;
        for (int i = 0; i < nparts; ++i) {
            const double p = part[i * 6 + threadIdx.x];
            v = threadIdx.x < 3 ? fmin(v, p) : fmax(v, p);
        }
        box[threadIdx.x] = v;
    }
    __syncthreads();
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < M; e += (int64_t)gridDim.x * 256) {
        int64_t c[4];
        bool ok = true;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            c[b] = conn[4 * e + b];
            ok = ok && c[b] >= 0 && c[b] < N;
        }
        ids[e] = (int32_t)e;
        if (!ok) {
            atomicMin(&bad[0], (unsigned long long)e);
            keys[e] = 0;
            continue;
        }
        double p[4][3], g[4][3];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int k = 0; k < 3; ++k) p[b][k] = X[3 * c[b] + k];
        const double det = tet4_grads_p(p, g);
        if (!(fabs(det) >= 1e-12)) atomicMin(&bad[1], (unsigned long long)e);
        // cubic cells, `cells` of them along the longest extent (capped at 1024 per axis)
        const double ext = fmax(box[3] - box[0], fmax(box[4] - box[1], box[5] - box[2]));
        uint32_t q[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double cen = 0.25 * (p[0][k] + p[1][k] + p[2][k] + p[3][k]);
            double t = ext > 0.0 ? (cen - box[k]) / ext * cells : 0.0;
            t = fmin(fmax(t, 0.0), 1023.0);
            q[k] = (uint32_t)t;
        }
        keys[e] = mf_spread10(q[0]) | (mf_spread10(q[1]) << 1) | (mf_spread10(q[2]) << 2);
    }
}

// bitonic sort of MF_SORT keys in LDS (256 threads)
constexpr int MF_SORT = 4 * MF_EC < 256 ? 256 : 4 * MF_EC;   // a chunk's (element, corner) pairs, padded
constexpr int MF_SPT = MF_SORT / 256;                        // pairs per thread in the scans
template <typename T>
__device__ __forceinline__ void mf_bitonic(T* s) {
    for (int k = 2; k <= MF_SORT; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < MF_SORT; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const T a = s[i], b = s[ixj];
                    if ((a > b) == ((i & k) == 0)) {
                        s[i] = b;
                        s[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// exclusive scan over the block of one int per thread (256 threads); returns the exclusive prefix, *total the sum
__device__ __forceinline__ int mf_block_scan(int v, int* sc, int* total) {
    sc[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int a = threadIdx.x >= (unsigned)o ? sc[threadIdx.x - o] : 0;
        __syncthreads();
        sc[threadIdx.x] += a;
        __syncthreads();
    }
    const int incl = sc[threadIdx.x];
    *total = sc[255];
    __syncthreads();
    return incl - v;
}

__device__ __forceinline__ void mf_chunk_range(const int32_t* cptr, int64_t c, int64_t M, int ec, int* e0, int* ne) {
    if (cptr) {
        *e0 = cptr[c];
        *ne = cptr[c + 1] - cptr[c];
    } else {
        const int64_t a = c * ec;
        *e0 = (int)a;
        *ne = (int)((M - a) < ec ? (M - a) : ec);
    }
}

// local node count of every chunk (cptr null: uniform chunks of ec <= MF_EC elements)
__global__ void __launch_bounds__(256) k_mf_count(const int64_t* __restrict__ conn, const int32_t* __restrict__ order,
                                                  int64_t M, const int32_t* __restrict__ cptr, int64_t nchunks,
                                                  int32_t* __restrict__ count, int ec) {
    __shared__ uint32_t s[MF_SORT];
    __shared__ int sc[256];
    const int64_t c = blockIdx.x;
    if (c >= nchunks) return;
    int e0, ne;
    mf_chunk_range(cptr, c, M, ec, &e0, &ne);
    for (int k = threadIdx.x; k < MF_SORT; k += 256)
        s[k] = k < 4 * ne ? (uint32_t)conn[4 * (int64_t)order[e0 + (k >> 2)] + (k & 3)] : 0xffffffffu;
    __syncthreads();
    mf_bitonic(s);
    int h = 0;
    for (int k = MF_SPT * threadIdx.x; k < MF_SPT * threadIdx.x + MF_SPT; ++k)
        h += (k < 4 * ne && (k == 0 || s[k] != s[k - 1])) ? 1 : 0;
    int total;
    (void)mf_block_scan(h, sc, &total);
    if (threadIdx.x == 0) count[c] = total;
}

// the chunk's local nodes, pair lists and element local ids
__global__ void __launch_bounds__(256) k_mf_fill(const int64_t* __restrict__ conn, const int32_t* __restrict__ order,
                                                 const int32_t* __restrict__ cptr, const int32_t* __restrict__ sbase,
                                                 int64_t nchunks, int32_t* __restrict__ cnode,
                                                 uint16_t* __restrict__ lptr, uint16_t* __restrict__ lent,
                                                 uint8_t* __restrict__ eloc) {
    __shared__ uint64_t s[MF_SORT];
    __shared__ int sc[256];
    const int64_t c = blockIdx.x;
    if (c >= nchunks) return;
    const int e0 = cptr[c], ne = cptr[c + 1] - e0;
    const int s0 = sbase[c];
    for (int k = threadIdx.x; k < MF_SORT; k += 256)
        s[k] = k < 4 * ne ? ((uint64_t)conn[4 * (int64_t)order[e0 + (k >> 2)] + (k & 3)] << 11) | (uint64_t)k
                          : ~(uint64_t)0;
    __syncthreads();
    mf_bitonic(s);
    const int k0 = MF_SPT * threadIdx.x;
    int h = 0;
    for (int k = k0; k < k0 + MF_SPT; ++k) h += (k < 4 * ne && (k == 0 || (s[k] >> 11) != (s[k - 1] >> 11))) ? 1 : 0;
    int total;
    int lid = mf_block_scan(h, sc, &total) - 1;
    uint16_t* lp = lptr + s0 + c;
    for (int k = k0; k < k0 + MF_SPT && k < 4 * ne; ++k) {
        const uint64_t key = s[k];
        if (k == 0 || (key >> 11) != (s[k - 1] >> 11)) {
            ++lid;
            cnode[s0 + lid] = (int32_t)(key >> 11);
            lp[lid] = (uint16_t)k;
        }
        const int pe = (int)(key & 2047);
        lent[4 * (int64_t)e0 + k] = (uint16_t)pe;
        eloc[4 * ((int64_t)e0 + (pe >> 2)) + (pe & 3)] = (uint8_t)lid;
    }
    if (threadIdx.x == 0) lp[total] = (uint16_t)(4 * ne);
}

__global__ void k_mf_slot_keys(const int32_t* __restrict__ cnode, int64_t nslots, int32_t* __restrict__ sid) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nslots; k += (int64_t)gridDim.x * 256)
        sid[k] = (int32_t)k;
}

// nptr from the node-sorted slot keys: nptr[j] = first k with key[k] >= j
__global__ void k_mf_nptr(const int32_t* __restrict__ skey, int64_t nslots, int64_t N, int32_t* __restrict__ nptr) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k <= nslots; k += (int64_t)gridDim.x * 256) {
        const int64_t prev = k == 0 ? -1 : skey[k - 1];
        const int64_t cur = k == nslots ? N : skey[k];
        for (int64_t j = prev + 1; j <= cur; ++j) nptr[j] = (int32_t)k;
    }
}

// spos[nslot[k]] = k: where each slot is stored in the node-major order
__global__ void k_mf_spos(const int32_t* __restrict__ nslot, int64_t nslots, int32_t* __restrict__ spos) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nslots; k += (int64_t)gridDim.x * 256)
        spos[nslot[k]] = (int32_t)k;
}

// ---------------------------------------------------------------- application
template <int BS, int MODE>
__global__ void __launch_bounds__(MF_BLOCK) k_mf_apply(MfOp op, const double* __restrict__ x,
                                                       double* __restrict__ slots) {
    __shared__ MfKernelLds<BS, MODE> L;
    (void)mf_walk_any<BS, MODE>(op, x, slots, L);
}

// one application into y through the slot buffer `slots` ([nslots * bs]: the operator's own for the stand-alone
// calls, a (P)CG context's own inside a solve, so applications on different streams never share scratch)
static int mf_run(fem_mf* m, int mode, const double* x, double* y, double* slots, hipStream_t st) {
    const MfOp op = m->op();
    if (m->nchunks > 0) {
#define FEM_MFA(B, MD)                                                                                              \
    hipLaunchKernelGGL((k_mf_apply<B, MD>),                                                                          \
                       dim3(mf_resident_grid((const void*)k_mf_apply<B, MD>, MF_BLOCK, m->nchunks)), dim3(MF_BLOCK), \
                       0, st, op, x, slots)
        if (m->bs == 3) {
            if (mode == MF_DIAG) FEM_MFA(3, MF_DIAG);
            else FEM_MFA(3, MF_APPLY);
        } else {
            if (mode == MF_DIAG) FEM_MFA(1, MF_DIAG);
            else FEM_MFA(1, MF_APPLY);
        }
#undef FEM_MFA
        FEM_LAUNCHED();
    }
    if (m->N > 0) {
        if (m->bs == 3) hipLaunchKernelGGL(k_mf_gather<3>, dim3(stream_grid(m->N, 256)), dim3(256), 0, st, op, slots, y);
        else hipLaunchKernelGGL(k_mf_gather<1>, dim3(stream_grid(m->N, 256)), dim3(256), 0, st, op, slots, y);
        FEM_LAUNCHED();
    }
    return FEM_OK;
}

// used by pcg.hip (the PCG's K1 on this operator)
MfOp mf_op(const fem_mf* m) { return m->op(); }
double* mf_slots(const fem_mf* m) { return m->slots; }
int mf_bs(const fem_mf* m) { return m->bs; }
int64_t mf_nodes(const fem_mf* m) { return m->N; }
int64_t mf_nslots(const fem_mf* m) { return m->nslots; }
int mf_apply(fem_mf* m, const double* x, double* y, double* slots, hipStream_t st) {
    return mf_run(m, MF_APPLY, x, y, slots, st);
}
int mf_diag(fem_mf* m, double* d, double* slots, hipStream_t st) { return mf_run(m, MF_DIAG, nullptr, d, slots, st); }

static void mf_free(fem_mf* m) {
    if (!m) return;
    void* ps[] = {m->eorder, m->cptr, m->sbase, m->cnode, m->eloc, m->lptr, m->lent, m->nptr, m->nslot, m->spos,
                  m->slots};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete m;
}

}  // namespace fem

using namespace fem;

extern "C" {

int fem_mf_create(const double* coords, const int64_t* conn, int64_t M, int64_t N, int kind, double E, double nu,
                  int64_t* bad_idx, fem_stream_t stream, fem_mf** out) {
    if (!out || (M > 0 && (!coords || !conn)) || M < 0 || N < 0) {
        set_error("fem_mf_create: bad arguments");
        return FEM_EARG;
    }
    if (kind != FEM_KIND_ELASTIC && kind != FEM_KIND_POISSON) {
        set_error("fem_mf_create: kind %d unsupported (elastic or Poisson)", kind);
        return FEM_EARG;
    }
    if (M >= (int64_t)1 << 29 || N >= (int64_t)1 << 31) {
        set_error("fem_mf_create: mesh too large for 32-bit element / slot indices");
        return FEM_EARG;
    }
    hipStream_t st = S(stream);
    fem_mf* m = new fem_mf();
    *out = nullptr;
    m->bs = kind == FEM_KIND_ELASTIC ? 3 : 1;
    m->M = M;
    m->N = N;
    m->X = coords;
    const Lame L = lame(E, nu);
    m->lam = L.lam;
    m->mu = L.mu;
    m->kappa = E;
    int rc = FEM_OK;
    void* tmp = nullptr;
    uint32_t *keys = nullptr, *keys2 = nullptr;
    int32_t *ids = nullptr, *skey = nullptr, *sid = nullptr;
    double* part = nullptr;
    unsigned long long* bad = nullptr;
#define MF_TRY(call)                                                                   \
    do {                                                                               \
        hipError_t _e = (call);                                                        \
        if (_e != hipSuccess) {                                                        \
            set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(_e)); \
            rc = FEM_EHIP;                                                             \
            goto done;                                                                 \
        }                                                                              \
    } while (0)
    MF_TRY(hipMalloc(&m->nptr, sizeof(int32_t) * (size_t)(N + 1)));
    if (M == 0) {
        MF_TRY(hipMemsetAsync(m->nptr, 0, sizeof(int32_t) * (size_t)(N + 1), st));
        MF_TRY(hipStreamSynchronize(st));
        *out = m;
        return FEM_OK;
    }
    {
        const int nparts = N > 0 ? stream_grid(N, 256) : 1;
        MF_TRY(hipMalloc(&part, sizeof(double) * 6 * (size_t)nparts));
        MF_TRY(hipMalloc(&bad, sizeof(unsigned long long) * 2));
        MF_TRY(hipMemsetAsync(bad, 0xff, sizeof(unsigned long long) * 2, st));
        MF_TRY(hipMalloc(&keys, sizeof(uint32_t) * (size_t)M));
        MF_TRY(hipMalloc(&keys2, sizeof(uint32_t) * (size_t)M));
        MF_TRY(hipMalloc(&ids, sizeof(int32_t) * (size_t)M));
        MF_TRY(hipMalloc(&m->eorder, sizeof(int32_t) * (size_t)M));
        if (N > 0) hipLaunchKernelGGL(k_mf_bbox, dim3(nparts), dim3(256), 0, st, coords, N, part);
        else MF_TRY(hipMemsetAsync(part, 0, sizeof(double) * 6, st));
        // Morton cells about one element cluster wide: (M / 6)^(1/3) along the longest extent -- one hex of a Kuhn
        // cube per cell (its 6 tets share a key and keep their file order), so chunks are compact blocks of whole
        // clusters and their boundary nodes (the slots shared with other chunks) few. FEM355_MF_CELLS overrides.
        double cells = cbrt((double)M / 6.0);
        if (const char* ev = getenv("FEM355_MF_CELLS")) cells = atof(ev);
        cells = cells < 1.0 ? 1.0 : (cells > 1024.0 ? 1024.0 : cells);
        hipLaunchKernelGGL(k_mf_keys, dim3(stream_grid(M, 256)), dim3(256), 0, st, coords, conn, M, N, part, nparts,
                           cells, keys, ids, bad);
        MF_TRY(hipGetLastError());
        unsigned long long hb[2];
        MF_TRY(hipMemcpyAsync(hb, bad, sizeof(hb), hipMemcpyDeviceToHost, st));
        MF_TRY(hipStreamSynchronize(st));
        if (hb[0] != ~0ull) {
            set_error("fem_mf_create: element %llu has a node outside [0, %lld)", hb[0], (long long)N);
            rc = FEM_EARG;
            goto done;
        }
        if (hb[1] != ~0ull) {
            if (bad_idx) *bad_idx = (int64_t)hb[1];
            set_error("Singular matrix encountered while computing B matrix.");
            rc = FEM_ESINGULAR;
            goto done;
        }
        size_t tb = 0;
        MF_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys2, ids, m->eorder, (int)M, 0, 30, st));
        MF_TRY(hipMalloc(&tmp, tb));
        MF_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys2, ids, m->eorder, (int)M, 0, 30, st));
        (void)hipFree(tmp);
        tmp = nullptr;
        // chunk sizes: uniform MF_EC; a chunk touching more than MF_NC nodes is halved, a half that still does
        // halved again, down to MF_PIECE (4 MF_PIECE <= MF_NC nodes). The node counts of the uniform chunkings of
        // MF_EC >> l elements, level by level while some chunk of the level above is over (hcl[l]).
        int32_t* cnt = ids;   // reused (chunks <= M)
        constexpr int LMAX = [] { int l = 0; while ((MF_EC >> l) > MF_PIECE) ++l; return l; }();
        std::vector<std::vector<int32_t>> hcl;
        for (int l = 0; l <= LMAX; ++l) {
            const int ec = MF_EC >> l;
            const int64_t ncl = cdiv(M, ec);
            hipLaunchKernelGGL(k_mf_count, dim3((unsigned)ncl), dim3(256), 0, st, conn, m->eorder, M,
                               (const int32_t*)nullptr, ncl, cnt, ec);
            MF_TRY(hipGetLastError());
            hcl.emplace_back((size_t)ncl);
            MF_TRY(hipMemcpyAsync(hcl.back().data(), cnt, sizeof(int32_t) * (size_t)ncl, hipMemcpyDeviceToHost, st));
            MF_TRY(hipStreamSynchronize(st));
            bool over = false;
            for (int32_t v : hcl.back()) over |= v > MF_NC;
            if (!over) break;
        }
        std::vector<int32_t> hcp, hn;
        hcp.reserve((size_t)hcl[0].size() + 1);
        hn.reserve((size_t)hcl[0].size());
        bool split = false;
        // emit level-l chunk idx: whole if it fits (or is a piece), else its two halves of level l + 1
        std::vector<std::pair<int, int64_t>> todo;
        for (int64_t c = (int64_t)hcl[0].size() - 1; c >= 0; --c) todo.emplace_back(0, c);
        while (!todo.empty()) {
            const auto [l, idx] = todo.back();
            todo.pop_back();
            const int64_t a = idx * (int64_t)(MF_EC >> l);
            if (a >= M) continue;
            const int32_t nodes = hcl[(size_t)l][(size_t)idx];
            if (nodes <= MF_NC || l == LMAX || l + 1 >= (int)hcl.size()) {
                hcp.push_back((int32_t)a);
                hn.push_back(nodes);
                split |= l > 0;
            } else {
                todo.emplace_back(l + 1, 2 * idx + 1);
                todo.emplace_back(l + 1, 2 * idx);
            }
        }
        hcp.push_back((int32_t)M);
        const int64_t nch = (int64_t)hcp.size() - 1;
        m->nchunks = nch;
        MF_TRY(hipMalloc(&m->cptr, sizeof(int32_t) * (size_t)(nch + 1)));
        MF_TRY(hipMalloc(&m->sbase, sizeof(int32_t) * (size_t)(nch + 1)));
        MF_TRY(hipMemcpyAsync(m->cptr, hcp.data(), sizeof(int32_t) * (size_t)(nch + 1), hipMemcpyHostToDevice, st));
        (void)split;
        std::vector<int32_t> hs((size_t)nch + 1);
        int64_t tot = 0;
        for (int64_t c = 0; c < nch; ++c) {
            hs[(size_t)c] = (int32_t)tot;
            tot += hn[(size_t)c];
        }
        hs[(size_t)nch] = (int32_t)tot;
        m->nslots = tot;
        MF_TRY(hipMemcpyAsync(m->sbase, hs.data(), sizeof(int32_t) * (size_t)(nch + 1), hipMemcpyHostToDevice, st));
        MF_TRY(hipMalloc(&m->cnode, sizeof(int32_t) * (size_t)tot));
        MF_TRY(hipMalloc(&m->eloc, sizeof(uint32_t) * (size_t)M));
        MF_TRY(hipMalloc(&m->lptr, sizeof(uint16_t) * (size_t)(tot + nch)));
        MF_TRY(hipMalloc(&m->lent, sizeof(uint16_t) * (4 * (size_t)M + 4 * MF_EC)));   // + a chunk: 16-byte reads
        MF_TRY(hipMalloc(&m->nslot, sizeof(int32_t) * (size_t)tot));
        MF_TRY(hipMalloc(&m->slots, sizeof(double) * (size_t)m->bs * (size_t)tot));
        hipLaunchKernelGGL(k_mf_fill, dim3((unsigned)nch), dim3(256), 0, st, conn, m->eorder, m->cptr, m->sbase, nch,
                           m->cnode, m->lptr, m->lent, reinterpret_cast<uint8_t*>(m->eloc));
        MF_TRY(hipGetLastError());
        // node -> slots (stable sort by node keeps the slots of a node ascending)
        MF_TRY(hipMalloc(&skey, sizeof(int32_t) * (size_t)tot));
        MF_TRY(hipMalloc(&sid, sizeof(int32_t) * (size_t)tot));
        hipLaunchKernelGGL(k_mf_slot_keys, dim3(stream_grid(tot, 256)), dim3(256), 0, st, m->cnode, tot, sid);
        MF_TRY(hipGetLastError());
        int bits = 1;
        while (bits < 31 && ((int64_t)1 << bits) < N) ++bits;
        MF_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, m->cnode, skey, sid, m->nslot, (int)tot, 0, bits, st));
        MF_TRY(hipMalloc(&tmp, tb));
        MF_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, m->cnode, skey, sid, m->nslot, (int)tot, 0, bits, st));
        hipLaunchKernelGGL(k_mf_nptr, dim3(stream_grid(tot + 1, 256)), dim3(256), 0, st, skey, tot, N, m->nptr);
        MF_TRY(hipGetLastError());
        // node-major slot storage (default): the chunk kernel writes each slot where its node's slots are contiguous,
        // so the readers (merged update, gather) stream them instead of following nslot. FEM355_MF_NODEMAJOR=0: the
        // chunk-major slots (A/B)
        const char* nm = getenv("FEM355_MF_NODEMAJOR");
        if (!nm || atoi(nm) != 0) {
            MF_TRY(hipMalloc(&m->spos, sizeof(int32_t) * (size_t)tot));
            hipLaunchKernelGGL(k_mf_spos, dim3(stream_grid(tot, 256)), dim3(256), 0, st, m->nslot, tot, m->spos);
            MF_TRY(hipGetLastError());
        }
        MF_TRY(hipStreamSynchronize(st));
    }
done:
#undef MF_TRY
    if (tmp) (void)hipFree(tmp);
    void* scratch[] = {keys, keys2, ids, skey, sid, part, bad};
    for (void* p : scratch)
        if (p) (void)hipFree(p);
    if (rc != FEM_OK) {
        mf_free(m);
        return rc;
    }
    *out = m;
    return FEM_OK;
}

int fem_mf_destroy(fem_mf* m) {
    mf_free(m);
    return FEM_OK;
}

int fem_mf_apply(fem_mf* m, const double* x, double* y, fem_stream_t stream) {
    if (!m || (m->N > 0 && (!x || !y))) {
        set_error("fem_mf_apply: bad arguments");
        return FEM_EARG;
    }
    return mf_run(m, MF_APPLY, x, y, m->slots, S(stream));
}

int fem_mf_diag(fem_mf* m, double* d, fem_stream_t stream) {
    if (!m || (m->N > 0 && !d)) {
        set_error("fem_mf_diag: bad arguments");
        return FEM_EARG;
    }
    return mf_run(m, MF_DIAG, nullptr, d, m->slots, S(stream));
}

// debug build only (FEM_MF_SPCHECK = 1): read and reset the carried-vs-reread slot position counters (out8); FEM_EARG
// in a normal build
int fem_mf_spcheck(uint64_t* out8) {
#if FEM_MF_SPCHECK
    FEM_HIP(hipDeviceSynchronize());
    FEM_HIP(hipMemcpyFromSymbol(out8, HIP_SYMBOL(mf_spcheck), sizeof(unsigned long long) * 8));
    unsigned long long z[8] = {0};
    FEM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mf_spcheck), z, sizeof(z)));
    return FEM_OK;
#else
    (void)out8;
    set_error("fem_mf_spcheck: not a FEM_MF_SPCHECK build");
    return FEM_EARG;
#endif
}

int fem_mf_info(fem_mf* m, int64_t* out6) {
    if (!m || !out6) {
        set_error("fem_mf_info: bad arguments");
        return FEM_EARG;
    }
    out6[0] = m->nchunks;
    out6[1] = m->nslots;
    out6[2] = m->bs;
    // static bytes one application streams: element local ids, pair lists, chunk tables, node -> slot lists
    out6[3] = 4 * m->M + 8 * m->M + 2 * (m->nslots + m->nchunks) + 8 * (m->nchunks + 1) + 4 * m->nslots +
              4 * (m->N + 1) + 4 * m->nslots;
    out6[4] = m->M;
    out6[5] = m->N;
    return FEM_OK;
}

int fem_mf_order(fem_mf* m, int32_t* eorder, int32_t* cptr, int32_t* sbase, int32_t* cnode, fem_stream_t stream) {
    if (!m) {
        set_error("fem_mf_order: bad arguments");
        return FEM_EARG;
    }
    hipStream_t st = S(stream);
    if (eorder && m->M) FEM_HIP(hipMemcpyAsync(eorder, m->eorder, sizeof(int32_t) * m->M, hipMemcpyDeviceToDevice, st));
    if (cptr && m->nchunks)
        FEM_HIP(hipMemcpyAsync(cptr, m->cptr, sizeof(int32_t) * (m->nchunks + 1), hipMemcpyDeviceToDevice, st));
    if (sbase && m->nchunks)
        FEM_HIP(hipMemcpyAsync(sbase, m->sbase, sizeof(int32_t) * (m->nchunks + 1), hipMemcpyDeviceToDevice, st));
    if (cnode && m->nslots)
        FEM_HIP(hipMemcpyAsync(cnode, m->cnode, sizeof(int32_t) * m->nslots, hipMemcpyDeviceToDevice, st));
    return FEM_OK;
}

}  // extern "C"
