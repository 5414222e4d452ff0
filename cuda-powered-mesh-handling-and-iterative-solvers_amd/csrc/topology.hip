// Mesh topology on the device: face / edge matching by radix sort of packed node keys.
//
// The reference forms every element face (or edge) from a local node table, sorts the nodes of each face, and
// groups equal faces with torch.unique(dim=0) (`solver/element.py:543-579`, `:707-762`, `:1293-1334`,
// `:1474-1532`, `:2234-2283`, `:2687-2713`). Here one context does the grouping once:
//   1. key kernel: the face's node ids sorted ascending, packed at ceil(log2 N) bits per node into one 64-bit
//      key, or two (hi, lo) when fpn * bits > 64 -> the packed order is the lexicographic row order of unique;
//   2. stable LSD radix sort (rocPRIM via hipCUB) of (key, flat face id): lo pass, then hi pass;
//   3. segment pass: head flags, per-face multiplicity, and counts of unique / single / paired keys.
// Queries then compact in the order each reference function returns: pairs in key order (shared faces, the
// element graph), single faces in the caller's face-major table order (surfaces), unique keys decoded (edges).
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace fem {

constexpr int TOPO_MAX_FPN = 4;
constexpr int TOPO_MAX_F = 12;

struct FaceTab {
    int8_t node[TOPO_MAX_F][TOPO_MAX_FPN];
};

__device__ __forceinline__ void sort_small(int64_t* v, int n) {
    for (int i = 1; i < n; ++i) {
        const int64_t x = v[i];
        int j = i - 1;
        while (j >= 0 && v[j] > x) {
            v[j + 1] = v[j];
            --j;
        }
        v[j + 1] = x;
    }
}

// flat face id i = e * F + f (element-major, the shared-face order of the reference)
__global__ void k_face_keys(const int64_t* __restrict__ conn, int64_t M, int npe, FaceTab tab, int F, int fpn,
                            int bits, int split, uint64_t* __restrict__ khi, uint64_t* __restrict__ klo,
                            int32_t* __restrict__ ids) {
    const int64_t nf = M * F;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i / F;
        const int f = (int)(i - e * F);
        int64_t v[TOPO_MAX_FPN];
        for (int k = 0; k < fpn; ++k) v[k] = conn[e * npe + tab.node[f][k]];
        sort_small(v, fpn);
        uint64_t hi = 0, lo = 0;
        for (int k = 0; k < split; ++k) hi = (hi << bits) | (uint64_t)v[k];
        for (int k = split; k < fpn; ++k) lo = (lo << bits) | (uint64_t)v[k];
        khi[i] = hi;
        if (klo) klo[i] = lo;
        ids[i] = (int32_t)i;
    }
}

__global__ void k_gather_u64(const uint64_t* __restrict__ src, const int32_t* __restrict__ perm, int64_t n,
                             uint64_t* __restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[perm[i]];
}

__device__ __forceinline__ bool key_eq(const uint64_t* hi, const uint64_t* lo, int64_t a, int64_t b) {
    return hi[a] == hi[b] && (!lo || lo[a] == lo[b]);
}

// head[p] = 1 at the first position of every key run (sorted order)
__global__ void k_heads(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo, int64_t n,
                        int32_t* __restrict__ head) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
        head[p] = (p == 0 || !key_eq(hi, lo, p, p - 1)) ? 1 : 0;
}

// run length at every run head -> mult[flat id] for every member; single / pair head flags
__global__ void k_runs(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo, const int32_t* __restrict__ perm,
                       const int32_t* __restrict__ head, int64_t n, int32_t* __restrict__ mult,
                       int32_t* __restrict__ single_head, int32_t* __restrict__ pair_head) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        int len = 0;
        if (head[p]) {
            len = 1;
            while (p + len < n && !head[p + len]) ++len;
            for (int k = 0; k < len; ++k) mult[perm[p + k]] = len;
        }
        single_head[p] = len == 1;
        pair_head[p] = len == 2;
    }
}

// exclusive scan of int32 flags (int64 output) via hipCUB
static int scan_flags(const int32_t* flags, int64_t* out, int64_t n, hipStream_t st) {
    size_t tb = 0;
    FEM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flags, out, (int)n, st));
    void* tmp = nullptr;
    FEM_HIP(::fem::malloc_async(&tmp, tb, st));
    FEM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, flags, out, (int)n, st));
    FEM_HIP(hipFreeAsync(tmp, st));
    return FEM_OK;
}

__global__ void k_emit_pairs(const int32_t* __restrict__ perm, const int32_t* __restrict__ pair_head,
                             const int64_t* __restrict__ pos, int64_t n, int F, int64_t* __restrict__ out) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        if (!pair_head[p]) continue;
        const int64_t s = pos[p];
        const int32_t a = perm[p], b = perm[p + 1];   // stable sort: a < b (element-major flat ids)
        out[4 * s + 0] = a / F;
        out[4 * s + 1] = a % F;
        out[4 * s + 2] = b / F;
        out[4 * s + 3] = b % F;
    }
}

__global__ void k_emit_unique(const uint64_t* __restrict__ hi, const uint64_t* __restrict__ lo,
                              const int32_t* __restrict__ head, const int64_t* __restrict__ pos, int64_t n, int fpn,
                              int bits, int split, int64_t* __restrict__ out) {
    const uint64_t mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        if (!head[p]) continue;
        const int64_t u = pos[p];
        uint64_t h = hi[p], l = lo ? lo[p] : 0;
        for (int k = fpn - 1; k >= split; --k) {
            out[u * fpn + k] = (int64_t)(l & mask);
            l >>= bits;
        }
        for (int k = split - 1; k >= 0; --k) {
            out[u * fpn + k] = (int64_t)(h & mask);
            h >>= bits;
        }
    }
}

// boundary faces in face-major order j = fs * M + e of the caller's table: flag where the matching context face
// (row smap[fs]) occurs once
__global__ void k_boundary_flags(const int32_t* __restrict__ mult, int64_t M, int F, int Fs, FaceTab smap1,
                                 int32_t* __restrict__ flag) {
    const int64_t n = M * Fs;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t fs = j / M, e = j - fs * M;
        flag[j] = mult[e * F + smap1.node[fs][0]] == 1;
    }
}

__global__ void k_boundary_emit(const int64_t* __restrict__ conn, int64_t M, int npe, const int32_t* __restrict__ flag,
                                const int64_t* __restrict__ pos, int Fs, int fpn, FaceTab stab, FaceTab xtab,
                                int has_extra, int64_t* __restrict__ faces, int64_t* __restrict__ extra) {
    const int64_t n = M * Fs;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[j]) continue;
        const int64_t fs = j / M, e = j - fs * M;
        const int64_t k = pos[j];
        for (int t = 0; t < fpn; ++t) faces[k * fpn + t] = conn[e * npe + stab.node[fs][t]];
        if (has_extra && extra) extra[k] = conn[e * npe + xtab.node[fs][0]];
    }
}

// sub-element split: out[(e * T + t) * spe + k] = conn[e * npe + tab[t][k]] (c3d8/c3d6/c3d10 -> c3d4)
__global__ void k_sub_elements(const int64_t* __restrict__ conn, int64_t M, int npe, FaceTab tab, int T, int spe,
                               int64_t* __restrict__ out) {
    const int64_t n = M * T * spe;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t et = i / spe;
        const int k = (int)(i - et * spe);
        const int64_t e = et / T;
        const int t = (int)(et - e * T);
        out[i] = conn[e * npe + tab.node[t][k]];
    }
}

// ---------------------------------------------------------------- face normals
// per element and face row: n = (p[a1] - p[a0]) x (p[a2] - p[a0]) * scale; flip so that n points away from the
// row's extra node (dot(n, x_extra - centroid) > 0 -> -n) when flip; unit = normalise
struct NormalTab {
    int8_t a[TOPO_MAX_F][3];      // vertex rows for the two edges
    int8_t cen[TOPO_MAX_F][TOPO_MAX_FPN];
    int8_t ncen[TOPO_MAX_F];
    int8_t extra[TOPO_MAX_F];
};

__global__ void k_element_face_normals(const double* __restrict__ X, const int64_t* __restrict__ conn, int64_t M,
                                       int npe, NormalTab tab, int F, double scale, int flip, int unit,
                                       double* __restrict__ out) {
    const int64_t n = M * F;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i / F;
        const int f = (int)(i - e * F);
        const int64_t* c = conn + e * npe;
        const double* p0 = X + 3 * c[tab.a[f][0]];
        const double* p1 = X + 3 * c[tab.a[f][1]];
        const double* p2 = X + 3 * c[tab.a[f][2]];
        const double u[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
        const double v[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
        double nn[3] = {(u[1] * v[2] - u[2] * v[1]) * scale, (u[2] * v[0] - u[0] * v[2]) * scale,
                        (u[0] * v[1] - u[1] * v[0]) * scale};
        if (unit) {
            const double r = sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
            nn[0] /= r;
            nn[1] /= r;
            nn[2] /= r;
        }
        if (flip) {
            double cx = 0, cy = 0, cz = 0;
            for (int k = 0; k < tab.ncen[f]; ++k) {
                const double* q = X + 3 * c[tab.cen[f][k]];
                cx += q[0];
                cy += q[1];
                cz += q[2];
            }
            const double nc = (double)tab.ncen[f];
            const double* x4 = X + 3 * c[tab.extra[f]];
            const double d = nn[0] * (x4[0] - cx / nc) + nn[1] * (x4[1] - cy / nc) + nn[2] * (x4[2] - cz / nc);
            if (d > 0) {
                nn[0] = -nn[0];
                nn[1] = -nn[1];
                nn[2] = -nn[2];
            }
        }
        out[3 * i] = nn[0];
        out[3 * i + 1] = nn[1];
        out[3 * i + 2] = nn[2];
    }
}

// surface-face normals (`compute_*_surface_normals`): faces [K, fpn] + extra [K]; second edge to vertex `v2`;
// unit normal flipped against the normalised centroid -> extra vector
__global__ void k_surface_normals(const double* __restrict__ X, const int64_t* __restrict__ faces,
                                  const int64_t* __restrict__ extra, int64_t K, int fpn, int v2,
                                  double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < K; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* fc = faces + i * fpn;
        const double* p0 = X + 3 * fc[0];
        const double* p1 = X + 3 * fc[1];
        const double* p2 = X + 3 * fc[v2];
        const double u[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
        const double v[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
        double nn[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
        const double r = sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        nn[0] /= r;
        nn[1] /= r;
        nn[2] /= r;
        double c[3] = {0, 0, 0};
        for (int k = 0; k < fpn; ++k)
            for (int d = 0; d < 3; ++d) c[d] += X[3 * fc[k] + d];
        const double* x4 = X + 3 * extra[i];
        double t[3];
        for (int d = 0; d < 3; ++d) t[d] = x4[d] - c[d] / (double)fpn;
        const double tr = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        const double dot = nn[0] * (t[0] / tr) + nn[1] * (t[1] / tr) + nn[2] * (t[2] / tr);
        const double s = dot > 0 ? -1.0 : 1.0;
        out[3 * i] = s * nn[0];
        out[3 * i + 1] = s * nn[1];
        out[3 * i + 2] = s * nn[2];
    }
}

}  // namespace fem

using namespace fem;

struct fem_topo {
    int64_t M, nf;
    int npe, F, fpn, bits, split;
    hipStream_t stream;
    uint64_t* hi;   // sorted keys
    uint64_t* lo;   // nullptr for one-word keys
    int32_t* perm;  // sorted flat face ids
    int32_t* mult;  // [nf] multiplicity of each flat face
    int32_t* head;
    int32_t* single_head;
    int32_t* pair_head;
    int64_t* pos;   // scratch [nf] exclusive scan
    int64_t n_unique, n_single, n_pair;
};

static int fill_tab(FaceTab* t, const int32_t* src, int rows, int cols) {
    if (rows > TOPO_MAX_F || cols > TOPO_MAX_FPN) return 1;
    *t = FaceTab{};
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) t->node[r][c] = (int8_t)src[r * cols + c];
    return 0;
}

static int64_t count_flags(const int32_t* flags, int64_t n, int64_t* scratch, hipStream_t st, int* rc) {
    *rc = scan_flags(flags, scratch, n, st);
    if (*rc) return 0;
    int64_t last = 0;
    int32_t lf = 0;
    if (hipMemcpyAsync(&last, scratch + n - 1, sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&lf, flags + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        *rc = FEM_EHIP;
        return 0;
    }
    return last + lf;
}

extern "C" {

void fem_topo_destroy(fem_topo* t);

int fem_topo_create(const int64_t* conn, int64_t M, int npe, const int32_t* ftab, int F, int fpn, int64_t N,
                    fem_stream_t stream, fem_topo** out) {
    *out = nullptr;
    FaceTab tab;
    if (M < 0 || F < 1 || fpn < 1 || fill_tab(&tab, ftab, F, fpn) || N < 1 || N > ((int64_t)1 << 32) ||
        M * F >= ((int64_t)1 << 31)) {
        set_error("fem_topo_create: bad table (F <= %d, fpn <= %d), N in [1, 2^32], M*F < 2^31", TOPO_MAX_F,
                  TOPO_MAX_FPN);
        return FEM_EARG;
    }
    for (int r = 0; r < F; ++r)
        for (int c = 0; c < fpn; ++c)
            if (ftab[r * fpn + c] < 0 || ftab[r * fpn + c] >= npe) {
                set_error("fem_topo_create: table entry outside [0, npe)");
                return FEM_EARG;
            }
    const hipStream_t st = S(stream);
    fem_topo* t = new fem_topo();
    t->M = M;
    t->nf = M * F;
    t->npe = npe;
    t->F = F;
    t->fpn = fpn;
    t->stream = st;
    int bits = 1;
    while (((int64_t)1 << bits) < N) ++bits;
    t->bits = bits;
    t->split = (fpn * bits <= 64) ? fpn : (fpn + 1) / 2;   // one-word key when it fits
    const bool two = t->split < fpn;
    const int64_t nf = t->nf;
    *out = t;
    if (nf == 0) return FEM_OK;
    auto fail = [&](int rc) {
        fem_topo_destroy(t);
        *out = nullptr;
        return rc;
    };
    uint64_t *khi = nullptr, *klo = nullptr, *k2 = nullptr;
    int32_t *ids = nullptr, *ids2 = nullptr;
    if (hipMalloc(&khi, 8 * nf) || hipMalloc(&k2, 8 * nf) || hipMalloc(&ids, 4 * nf) || hipMalloc(&ids2, 4 * nf) ||
        (two && hipMalloc(&klo, 8 * nf)) || hipMalloc(&t->mult, 4 * nf) || hipMalloc(&t->head, 4 * nf) ||
        hipMalloc(&t->single_head, 4 * nf) || hipMalloc(&t->pair_head, 4 * nf) || hipMalloc(&t->pos, 8 * nf)) {
        set_error("fem_topo_create: out of device memory");
        (void)hipFree(khi);
        (void)hipFree(klo);
        (void)hipFree(k2);
        (void)hipFree(ids);
        (void)hipFree(ids2);
        return fail(FEM_EHIP);
    }
    const dim3 g(stream_grid(nf, 256)), b(256);
    hipLaunchKernelGGL(k_face_keys, g, b, 0, st, conn, M, npe, tab, F, fpn, bits, t->split, khi, klo, ids);
    // radix sort: one pass on the single key, or lo then (stable) hi
    auto sort = [&](const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout, int end_bit) -> int {
        size_t tb = 0;
        if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, (int)nf, 0, end_bit, st))
            return FEM_EHIP;
        void* tmp = nullptr;
        if (::fem::malloc_async(&tmp, tb, st)) return FEM_EHIP;
        if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, (int)nf, 0, end_bit, st))
            return FEM_EHIP;
        (void)hipFreeAsync(tmp, st);
        return FEM_OK;
    };
    int rc = FEM_OK;
    const int hi_bits = t->split * bits, lo_bits = (fpn - t->split) * bits;
    if (!two) {
        rc = sort(khi, k2, ids, ids2, hi_bits);
        if (!rc) {
            t->hi = k2;
            t->perm = ids2;
            (void)hipFree(khi);
            (void)hipFree(ids);
        }
    } else {
        rc = sort(klo, k2, ids, ids2, lo_bits);                                  // pass 1: perm1 = ids2
        if (!rc) {
            hipLaunchKernelGGL(k_gather_u64, g, b, 0, st, khi, ids2, nf, k2);   // hi in pass-1 order
            rc = sort(k2, khi, ids2, ids, hi_bits);                             // pass 2 (stable): khi, ids
        }
        if (!rc) {
            hipLaunchKernelGGL(k_gather_u64, g, b, 0, st, klo, ids, nf, k2);    // lo aligned with the final order
            t->hi = khi;
            t->lo = k2;
            t->perm = ids;
            (void)hipFree(klo);
            (void)hipFree(ids2);
        }
    }
    if (rc) {
        set_error("fem_topo_create: radix sort failed");
        (void)hipFree(khi);
        (void)hipFree(klo);
        (void)hipFree(k2);
        (void)hipFree(ids);
        (void)hipFree(ids2);
        return fail(rc);
    }
    hipLaunchKernelGGL(k_heads, g, b, 0, st, t->hi, t->lo, nf, t->head);
    hipLaunchKernelGGL(k_runs, g, b, 0, st, t->hi, t->lo, t->perm, t->head, nf, t->mult, t->single_head, t->pair_head);
    if (hipGetLastError() != hipSuccess) {
        set_error("fem_topo_create: kernel launch failed");
        return fail(FEM_EHIP);
    }
    t->n_unique = count_flags(t->head, nf, t->pos, st, &rc);
    if (!rc) t->n_single = count_flags(t->single_head, nf, t->pos, st, &rc);
    if (!rc) t->n_pair = count_flags(t->pair_head, nf, t->pos, st, &rc);
    if (rc) return fail(rc);
    return FEM_OK;
}

int fem_topo_counts(const fem_topo* t, int64_t* n_unique, int64_t* n_single, int64_t* n_pair) {
    if (n_unique) *n_unique = t->n_unique;
    if (n_single) *n_single = t->n_single;
    if (n_pair) *n_pair = t->n_pair;
    return FEM_OK;
}

int fem_topo_pairs(fem_topo* t, int64_t* out) {
    if (t->nf == 0 || t->n_pair == 0) return FEM_OK;
    int rc = scan_flags(t->pair_head, t->pos, t->nf, t->stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_emit_pairs, dim3(stream_grid(t->nf, 256)), dim3(256), 0, t->stream, t->perm, t->pair_head,
                       t->pos, t->nf, t->F, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_topo_unique(fem_topo* t, int64_t* out) {
    if (t->nf == 0) return FEM_OK;
    int rc = scan_flags(t->head, t->pos, t->nf, t->stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_emit_unique, dim3(stream_grid(t->nf, 256)), dim3(256), 0, t->stream, t->hi, t->lo, t->head,
                       t->pos, t->nf, t->fpn, t->bits, t->split, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_topo_boundary(fem_topo* t, const int64_t* conn, int Fs, const int32_t* smap, const int32_t* stab,
                      const int32_t* xtab, int64_t* faces, int64_t* extra, int64_t* count) {
    FaceTab sm, s2, x2;
    if (Fs < 1 || Fs > TOPO_MAX_F || fill_tab(&s2, stab, Fs, t->fpn)) {
        set_error("fem_topo_boundary: bad surface table");
        return FEM_EARG;
    }
    sm = FaceTab{};
    x2 = FaceTab{};
    for (int r = 0; r < Fs; ++r) {
        if (smap[r] < 0 || smap[r] >= t->F) {
            set_error("fem_topo_boundary: smap entry outside the context's face rows");
            return FEM_EARG;
        }
        sm.node[r][0] = (int8_t)smap[r];
        if (xtab) x2.node[r][0] = (int8_t)xtab[r];
    }
    const int64_t n = t->M * Fs;
    if (count) *count = 0;
    if (n == 0) return FEM_OK;
    int32_t* flag = nullptr;
    int64_t* pos = nullptr;
    FEM_HIP(::fem::malloc_async((void**)&flag, 4 * n, t->stream));
    FEM_HIP(::fem::malloc_async((void**)&pos, 8 * n, t->stream));
    const dim3 g(stream_grid(n, 256)), b(256);
    hipLaunchKernelGGL(k_boundary_flags, g, b, 0, t->stream, t->mult, t->M, t->F, Fs, sm, flag);
    int rc = FEM_OK;
    const int64_t k = count_flags(flag, n, pos, t->stream, &rc);
    if (!rc && faces) {
        hipLaunchKernelGGL(k_boundary_emit, g, b, 0, t->stream, conn, t->M, t->npe, flag, pos, Fs, t->fpn, s2, x2,
                           xtab ? 1 : 0, faces, extra);
        if (hipGetLastError() != hipSuccess) rc = FEM_EHIP;
    }
    (void)hipFreeAsync(flag, t->stream);
    (void)hipFreeAsync(pos, t->stream);
    if (count) *count = k;
    return rc;
}

void fem_topo_destroy(fem_topo* t) {
    if (!t) return;
    (void)hipStreamSynchronize(t->stream);
    (void)hipFree(t->hi);
    (void)hipFree(t->lo);
    (void)hipFree(t->perm);
    (void)hipFree(t->mult);
    (void)hipFree(t->head);
    (void)hipFree(t->single_head);
    (void)hipFree(t->pair_head);
    (void)hipFree(t->pos);
    delete t;
}

int fem_sub_elements(const int64_t* conn, int64_t M, int npe, const int32_t* tab, int T, int spe, int64_t* out,
                     fem_stream_t stream) {
    FaceTab tb;
    if (T < 1 || spe < 1 || fill_tab(&tb, tab, T, spe)) {
        set_error("fem_sub_elements: table must be at most %d x %d", TOPO_MAX_F, TOPO_MAX_FPN);
        return FEM_EARG;
    }
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_sub_elements, dim3(stream_grid(M * T * spe, 256)), dim3(256), 0, S(stream), conn, M, npe, tb,
                       T, spe, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_element_face_normals(const double* coords, const int64_t* conn, int64_t M, int npe, const int32_t* edges,
                             const int32_t* cen, const int32_t* ncen, const int32_t* extra, int F, double scale,
                             int flip, int unit, double* out, fem_stream_t stream) {
    if (F < 1 || F > TOPO_MAX_F) {
        set_error("fem_element_face_normals: F must be in [1, %d]", TOPO_MAX_F);
        return FEM_EARG;
    }
    NormalTab tab{};
    for (int f = 0; f < F; ++f) {
        for (int k = 0; k < 3; ++k) tab.a[f][k] = (int8_t)edges[3 * f + k];
        tab.ncen[f] = (int8_t)(ncen ? ncen[f] : 0);
        for (int k = 0; k < tab.ncen[f] && k < TOPO_MAX_FPN; ++k) tab.cen[f][k] = (int8_t)cen[TOPO_MAX_FPN * f + k];
        tab.extra[f] = (int8_t)(extra ? extra[f] : 0);
    }
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_element_face_normals, dim3(stream_grid(M * F, 256)), dim3(256), 0, S(stream), coords, conn, M,
                       npe, tab, F, scale, flip, unit, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_surface_normals(const double* coords, const int64_t* faces, const int64_t* extra, int64_t K, int fpn, int v2,
                        double* out, fem_stream_t stream) {
    if (fpn < 3 || fpn > TOPO_MAX_FPN || v2 < 2 || v2 >= fpn) {
        set_error("fem_surface_normals: fpn in [3, 4], second-edge vertex in [2, fpn)");
        return FEM_EARG;
    }
    if (K <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_surface_normals, dim3(stream_grid(K, 256)), dim3(256), 0, S(stream), coords, faces, extra, K,
                       fpn, v2, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // extern "C"
