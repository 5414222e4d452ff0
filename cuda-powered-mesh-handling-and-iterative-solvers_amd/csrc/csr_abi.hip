// The dof-level CSR entry points named in SURVEY.md §8(b) ("C-ABI the replacement must export"), for callers that
// want the reference's assembled-matrix view (`subdivision.ipynb:118-139`: COO rows dof_i, cols dof_j, values
// K_e row-major, coalesced) rather than the blocked SELL-64 operator the rest of fem355 uses:
//   fem_solid_ke    element matrices of c3d8 / c3d6 / c3d10 from natural points + weights (device dN evaluation)
//   fem_csr_pattern dof CSR pattern (rowptr, colidx sorted, diagpos) of a connectivity block
//   fem_csr_fill    deterministic row-gather of element matrices into that pattern
//   fem_spmv_csr    y = A x on the dof CSR
//   fem_pcg_csr     one-shot (P)CG on the dof CSR: converted to SELL-64 (bs = 1) and run by the device PCG
// Each is a thin layer over the node-level kernels (pattern.hip, assemble.hip, pcg.hip); the node graph is
// expanded to dofs as rows dpn*i + c with columns dpn*j + c' (ascending because the node columns are).
#include "common.hpp"

namespace fem {

// ---------------------------------------------------------------- natural derivatives on the device
// exactly the host tables of element.py (`solver/element.py:1617-1626`, `:2498-2505`, `:1043-1054`), no contraction
#pragma clang fp contract(off)
__global__ void k_dn_table(int npe, const double* __restrict__ ip, int n_ip, double* __restrict__ dN) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_ip) return;
    const double xi = ip[3 * q], eta = ip[3 * q + 1], zeta = ip[3 * q + 2];
    double* d = dN + (int64_t)q * npe * 3;
    if (npe == 8) {
        const int s[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                             {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};
        for (int n = 0; n < 8; ++n) {
            const double a = s[n][0], b = s[n][1], c = s[n][2];
            d[3 * n + 0] = 0.125 * a * (1.0 + b * eta) * (1.0 + c * zeta);
            d[3 * n + 1] = 0.125 * b * (1.0 + a * xi) * (1.0 + c * zeta);
            d[3 * n + 2] = 0.125 * c * (1.0 + a * xi) * (1.0 + b * eta);
        }
    } else if (npe == 6) {
        const double r = xi, s = eta, t = zeta;
        const double v[18] = {-0.5 * (1.0 - t), -0.5 * (1.0 - t), -0.5 * (1.0 - r - s),
                              0.5 * (1.0 - t),  0.0,              -0.5 * r,
                              0.0,              0.5 * (1.0 - t),  -0.5 * s,
                              -0.5 * (1.0 + t), -0.5 * (1.0 + t), 0.5 * (1.0 - r - s),
                              0.5 * (1.0 + t),  0.0,              0.5 * r,
                              0.0,              0.5 * (1.0 + t),  0.5 * s};
        for (int k = 0; k < 18; ++k) d[k] = v[k];
    } else {
        const double L = 1.0 - xi - eta - zeta;
        const double v[30] = {4.0 * xi - 1.0,   0.0,              0.0,
                              0.0,              4.0 * eta - 1.0,  0.0,
                              0.0,              0.0,              4.0 * zeta - 1.0,
                              -4.0 * L + 1.0,   -4.0 * L + 1.0,   -4.0 * L + 1.0,
                              4.0 * eta,        4.0 * xi,         0.0,
                              0.0,              4.0 * zeta,       4.0 * eta,
                              4.0 * zeta,       0.0,              4.0 * xi,
                              4.0 * (1.0 - 2.0 * xi - eta - zeta), -4.0 * xi, -4.0 * xi,
                              -4.0 * eta, 4.0 * (1.0 - xi - 2.0 * eta - zeta), -4.0 * eta,
                              -4.0 * zeta, -4.0 * zeta, 4.0 * (1.0 - xi - eta - 2.0 * zeta)};
        for (int k = 0; k < 30; ++k) d[k] = v[k];
    }
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------- node graph -> dof CSR
__global__ void k_dof_rowptr(const int32_t* __restrict__ nrp, int64_t N, int dpn, int32_t* __restrict__ rp) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= N * dpn; r += (int64_t)gridDim.x * blockDim.x) {
        if (r == N * dpn) {
            rp[r] = dpn * dpn * nrp[N];
            continue;
        }
        const int64_t i = r / dpn;
        const int c = (int)(r - i * dpn);
        const int L = nrp[i + 1] - nrp[i];
        rp[r] = dpn * dpn * nrp[i] + c * dpn * L;
    }
}

__global__ void k_dof_cols(const int32_t* __restrict__ nrp, const int32_t* __restrict__ ncol, int64_t N, int dpn,
                           const int32_t* __restrict__ rp, int32_t* __restrict__ col, int32_t* __restrict__ diag) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N * dpn; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = r / dpn;
        int p = rp[r];
        for (int t = nrp[i]; t < nrp[i + 1]; ++t)
            for (int c2 = 0; c2 < dpn; ++c2) {
                const int v = dpn * ncol[t] + c2;
                if (diag && v == (int)r) diag[r] = p;
                col[p++] = v;
            }
    }
}

__device__ __forceinline__ int find_sorted(const int32_t* __restrict__ c, int lo, int hi, int j) {
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (c[m] < j) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// dof row r = dpn*i + c: every incident (e, a) adds K_e[dpn a + c, dpn b + c'] to column dpn conn[e,b] + c', in
// ascending incidence order (deterministic)
__global__ void k_csr_fill(const double* __restrict__ Ke, const int64_t* __restrict__ conn, int npe, int dpn,
                           const int32_t* __restrict__ inc_ptr, const int32_t* __restrict__ inc, int64_t N,
                           const int32_t* __restrict__ rp, const int32_t* __restrict__ col, double* __restrict__ vals) {
    const int d = npe * dpn;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N * dpn; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = r / dpn;
        const int c = (int)(r - i * dpn);
        const int lo = rp[r], hi = rp[r + 1];
        for (int t = inc_ptr[i]; t < inc_ptr[i + 1]; ++t) {
            const int ea = inc[t];
            const int64_t e = ea / npe;
            const int a = ea - (int)e * npe;
            const double* krow = Ke + (e * d + (int64_t)(dpn * a + c)) * d;
            for (int b = 0; b < npe; ++b) {
                const int jb = dpn * (int)conn[e * npe + b];
                const int p = find_sorted(col, lo, hi, jb);
                for (int c2 = 0; c2 < dpn; ++c2) vals[p + c2] += krow[dpn * b + c2];
            }
        }
    }
}

// CSR SpMV: 8 lanes per row, fixed-order lane partials combined by a fixed shuffle tree (deterministic)
__global__ void __launch_bounds__(256) k_csr_spmv(const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                  const double* __restrict__ vals, const double* __restrict__ x,
                                                  double* __restrict__ y, int64_t n) {
    const int sub = threadIdx.x & 7;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; r < n;
         r += ((int64_t)gridDim.x * blockDim.x) >> 3) {
        double acc = 0.0;
        for (int p = rp[r] + sub; p < rp[r + 1]; p += 8) acc += vals[p] * x[col[p]];
        acc += __shfl_xor(acc, 4, 8);
        acc += __shfl_xor(acc, 2, 8);
        acc += __shfl_xor(acc, 1, 8);
        if (sub == 0) y[r] = acc;
    }
}

__global__ void k_scatter_vals(const double* __restrict__ v, const int64_t* __restrict__ map, int64_t nnz,
                               double* __restrict__ out) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x)
        out[map[p]] = v[p];
}

__global__ void k_pcg_weights(const double* __restrict__ dinv, const uint8_t* __restrict__ fixed, int64_t n,
                              double* __restrict__ w) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        w[i] = (fixed && fixed[i]) ? 0.0 : (dinv ? dinv[i] : 1.0);
}

}  // namespace fem

using namespace fem;

// node graph of conn (internal, stream-ordered temporaries): incidence + node CSR
struct NodeGraph {
    int32_t* inc_ptr = nullptr;
    int32_t* inc = nullptr;
    int32_t* rowptr = nullptr;
    int32_t* colidx = nullptr;
    int64_t nnz = 0;
};

static int node_graph(const int64_t* conn, int64_t M, int npe, int64_t N, hipStream_t st, bool cols, NodeGraph* g) {
    const fem_stream_t fs = reinterpret_cast<fem_stream_t>(st);
    FEM_HIP(::fem::malloc_async((void**)&g->inc_ptr, sizeof(int32_t) * (N + 1), st));
    FEM_HIP(::fem::malloc_async((void**)&g->inc, sizeof(int32_t) * (M * npe > 0 ? M * npe : 1), st));
    int rc = fem_incidence(conn, M, npe, N, g->inc_ptr, g->inc, nullptr, fs);
    if (rc) return rc;
    int32_t *row_len = nullptr, *tmp = nullptr, *work = nullptr;
    FEM_HIP(::fem::malloc_async((void**)&row_len, sizeof(int32_t) * N, st));
    FEM_HIP(::fem::malloc_async((void**)&tmp, sizeof(int32_t) * fem_graph_tmp_len(N), st));
    FEM_HIP(::fem::malloc_async((void**)&g->rowptr, sizeof(int32_t) * (N + 1), st));
    FEM_HIP(::fem::malloc_async((void**)&work, sizeof(int32_t) * (fem_scan_work_len(N) + 1), st));
    if ((rc = fem_graph_count2(conn, npe, g->inc_ptr, g->inc, N, row_len, tmp, nullptr, fs))) return rc;
    if ((rc = fem_scan_i32(row_len, N, g->rowptr, work, fs))) return rc;
    int32_t nnz = 0;
    FEM_HIP(hipMemcpyAsync(&nnz, g->rowptr + N, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FEM_HIP(hipStreamSynchronize(st));
    g->nnz = nnz;
    if (cols) {
        int32_t* diag = nullptr;
        FEM_HIP(::fem::malloc_async((void**)&g->colidx, sizeof(int32_t) * (g->nnz > 0 ? g->nnz : 1), st));
        FEM_HIP(::fem::malloc_async((void**)&diag, sizeof(int32_t) * N, st));
        if ((rc = fem_graph_fill2(conn, npe, g->inc_ptr, g->inc, N, g->rowptr, tmp, g->colidx, diag, fs))) return rc;
        FEM_HIP(hipFreeAsync(diag, st));
    }
    FEM_HIP(hipFreeAsync(row_len, st));
    FEM_HIP(hipFreeAsync(tmp, st));
    FEM_HIP(hipFreeAsync(work, st));
    return FEM_OK;
}

static void free_graph(NodeGraph* g, hipStream_t st) {
    if (g->inc_ptr) (void)hipFreeAsync(g->inc_ptr, st);
    if (g->inc) (void)hipFreeAsync(g->inc, st);
    if (g->rowptr) (void)hipFreeAsync(g->rowptr, st);
    if (g->colidx) (void)hipFreeAsync(g->colidx, st);
}

extern "C" {

int fem_solid_ke(int type, const double* coords, const int64_t* conn, int64_t M, double E, double nu, const double* ip,
                 const double* w, int n_ip, int single, double* Ke, fem_stream_t stream) {
    const int npe = type;
    if (npe != 6 && npe != 8 && npe != 10) {
        set_error("fem_solid_ke: element type %d is not c3d6 / c3d8 / c3d10", type);
        return FEM_EBADTYPE;
    }
    const hipStream_t st = S(stream);
    if (npe == 6 && single) {   // one point (1/3, 1/3, 0) times the wedge volume (`solver/element.py:2656-2659`)
        const double pt[3] = {1.0 / 3.0, 1.0 / 3.0, 0.0};
        double* dip = nullptr;
        double* dN = nullptr;
        FEM_HIP(::fem::malloc_async((void**)&dip, sizeof(pt), st));
        FEM_HIP(::fem::malloc_async((void**)&dN, sizeof(double) * 18, st));
        FEM_HIP(hipMemcpyAsync(dip, pt, sizeof(pt), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_dn_table, dim3(1), dim3(64), 0, st, 6, dip, 1, dN);
        FEM_LAUNCHED();
        const int rc = fem_iso_ke(coords, conn, M, 6, E, nu, dN, nullptr, 1, FEM_ISO_VOLUME, Ke, stream);
        FEM_HIP(hipStreamSynchronize(st));   // pt lives on this stack frame
        (void)hipFreeAsync(dip, st);
        (void)hipFreeAsync(dN, st);
        return rc;
    }
    if (!ip || !w || n_ip < 1) {
        set_error("fem_solid_ke: integration points / weights required");
        return FEM_EARG;
    }
    // the shape-function table in the stream's kept scratch: a hipFreeAsync here would hold the host until the
    // K_e kernel finished (runtime.hip stream_scratch)
    double* dN = nullptr;
    FEM_HIP(::fem::stream_scratch((void**)&dN, sizeof(double) * n_ip * npe * 3, st));
    hipLaunchKernelGGL(k_dn_table, dim3(cdiv(n_ip, 64)), dim3(64), 0, st, npe, ip, n_ip, dN);
    FEM_LAUNCHED();
    // single=False: per-point stack for c3d8 / c3d10 (Q6); c3d6's flag only selects the one-point rule
    const int mode = (single || npe == 6) ? FEM_ISO_SUM : FEM_ISO_STACK;
    return fem_iso_ke(coords, conn, M, npe, E, nu, dN, w, n_ip, mode, Ke, stream);
}

int fem_csr_pattern(const int64_t* conn, int64_t M, int npe, int dofs_per_node, int64_t n_nodes, int32_t* rowptr,
                    int32_t* colidx, int32_t* diagpos, int64_t* nnz_out, fem_stream_t stream) {
    const int dpn = dofs_per_node;
    if (dpn < 1 || dpn > 6 || n_nodes < 1 || n_nodes * dpn >= ((int64_t)1 << 31)) {
        set_error("fem_csr_pattern: bad dofs_per_node %d / n_nodes %lld", dpn, (long long)n_nodes);
        return FEM_EARG;
    }
    const hipStream_t st = S(stream);
    NodeGraph g;
    int rc = node_graph(conn, M, npe, n_nodes, st, colidx != nullptr, &g);
    if (!rc && (int64_t)g.nnz * dpn * dpn >= ((int64_t)1 << 31)) {
        set_error("fem_csr_pattern: %lld nonzeros exceed int32 offsets", (long long)g.nnz * dpn * dpn);
        rc = FEM_EARG;
    }
    if (!rc) {
        const int64_t nr = n_nodes * dpn;
        hipLaunchKernelGGL(k_dof_rowptr, dim3(stream_grid(nr + 1, 256)), dim3(256), 0, st, g.rowptr, n_nodes, dpn,
                           rowptr);
        if (colidx && diagpos && hipMemsetAsync(diagpos, 0xff, sizeof(int32_t) * (size_t)nr, st) != hipSuccess)
            rc = FEM_EHIP;   // -1 = no diagonal (a node no element touches)
        if (colidx)
            hipLaunchKernelGGL(k_dof_cols, dim3(stream_grid(nr, 256)), dim3(256), 0, st, g.rowptr, g.colidx, n_nodes,
                               dpn, rowptr, colidx, diagpos);
        if (hipGetLastError() != hipSuccess) rc = FEM_EHIP;
        if (nnz_out) *nnz_out = g.nnz * dpn * dpn;
    }
    free_graph(&g, st);
    return rc;
}

int fem_csr_fill(const double* Ke, const int64_t* conn, int64_t M, int npe, int dpn, int64_t n_nodes,
                 const int32_t* rowptr, const int32_t* colidx, double* vals, fem_stream_t stream) {
    if (dpn < 1 || dpn > 6 || n_nodes < 1) {
        set_error("fem_csr_fill: bad dpn %d / n_nodes %lld", dpn, (long long)n_nodes);
        return FEM_EARG;
    }
    const hipStream_t st = S(stream);
    NodeGraph g;
    g.inc_ptr = nullptr;
    FEM_HIP(::fem::malloc_async((void**)&g.inc_ptr, sizeof(int32_t) * (n_nodes + 1), st));
    FEM_HIP(::fem::malloc_async((void**)&g.inc, sizeof(int32_t) * (M * npe > 0 ? M * npe : 1), st));
    int rc = fem_incidence(conn, M, npe, n_nodes, g.inc_ptr, g.inc, nullptr, stream);
    if (!rc) {
        hipLaunchKernelGGL(k_csr_fill, dim3(stream_grid(n_nodes * dpn, 256)), dim3(256), 0, st, Ke, conn, npe, dpn,
                           g.inc_ptr, g.inc, n_nodes, rowptr, colidx, vals);
        if (hipGetLastError() != hipSuccess) rc = FEM_EHIP;
    }
    free_graph(&g, st);
    return rc;
}

int fem_spmv_csr(const int32_t* rowptr, const int32_t* colidx, const double* vals, const double* x, double* y,
                 int64_t n, fem_stream_t stream) {
    if (n <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_csr_spmv, dim3(stream_grid(n * 8, 256)), dim3(256), 0, S(stream), rowptr, colidx, vals, x, y,
                       n);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_pcg_csr(const int32_t* rowptr, const int32_t* colidx, const double* vals, int64_t n, const double* b,
                double* x, const double* dinv, const uint8_t* fixed_mask, double tol, int max_iter, double eps,
                int mode, int* iters_out, int* status_out, double* res_hist_out, fem_stream_t stream) {
    if (n <= 0) return FEM_OK;
    if (mode != FEM_MODE_CG_STABLE && mode != FEM_MODE_PCG) {
        set_error("fem_pcg_csr: mode must be FEM_MODE_CG_STABLE or FEM_MODE_PCG");
        return FEM_EARG;
    }
    const hipStream_t st = S(stream);
    const int64_t ns = cdiv(n, 64);
    int64_t *width = nullptr, *slice_ptr = nullptr, *work = nullptr, *csr2sell = nullptr;
    int32_t* cols = nullptr;
    int16_t* d16 = nullptr;
    int32_t* ovf = nullptr;
    double *sv = nullptr, *w = nullptr;
    int rc = FEM_OK;
    int32_t nnz = 0;
    FEM_HIP(hipMemcpyAsync(&nnz, rowptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FEM_HIP(::fem::malloc_async((void**)&width, sizeof(int64_t) * ns, st));
    FEM_HIP(::fem::malloc_async((void**)&slice_ptr, sizeof(int64_t) * (ns + 1), st));
    FEM_HIP(::fem::malloc_async((void**)&work, sizeof(int64_t) * (fem_scan_work_len(ns) + 1), st));
    if ((rc = fem_sell_widths(rowptr, n, width, stream))) return rc;
    if ((rc = fem_scan_i64(width, ns, slice_ptr, work, stream))) return rc;
    int64_t ent = 0;
    FEM_HIP(hipMemcpyAsync(&ent, slice_ptr + ns, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    FEM_HIP(hipStreamSynchronize(st));
    FEM_HIP(::fem::malloc_async((void**)&cols, sizeof(int32_t) * (ent > 0 ? ent : 1), st));
    FEM_HIP(::fem::malloc_async((void**)&csr2sell, sizeof(int64_t) * (nnz > 0 ? nnz : 1), st));
    FEM_HIP(::fem::malloc_async((void**)&sv, sizeof(double) * (ent > 0 ? ent : 1), st));
    FEM_HIP(::fem::malloc_async((void**)&d16, sizeof(int16_t) * (ent > 0 ? ent : 1), st));
    FEM_HIP(::fem::malloc_async((void**)&ovf, sizeof(int32_t), st));
    FEM_HIP(::fem::malloc_async((void**)&w, sizeof(double) * n, st));
    FEM_HIP(hipMemsetAsync(sv, 0, sizeof(double) * (ent > 0 ? ent : 1), st));
    FEM_HIP(hipMemsetAsync(ovf, 0, sizeof(int32_t), st));
    if ((rc = fem_sell_fill(rowptr, colidx, n, slice_ptr, cols, csr2sell, stream))) return rc;
    hipLaunchKernelGGL(k_scatter_vals, dim3(stream_grid(nnz, 256)), dim3(256), 0, st, vals, csr2sell, (int64_t)nnz, sv);
    hipLaunchKernelGGL(k_pcg_weights, dim3(stream_grid(n, 256)), dim3(256), 0, st,
                       mode == FEM_MODE_PCG ? dinv : (const double*)nullptr, fixed_mask, n, w);
    FEM_LAUNCHED();
    if ((rc = fem_sell_delta16(cols, n, slice_ptr, d16, ovf, stream))) return rc;
    int32_t h_ovf = 0;
    FEM_HIP(hipMemcpyAsync(&h_ovf, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    FEM_HIP(hipStreamSynchronize(st));
    fem_pcg* s = nullptr;
    rc = fem_pcg_create(n, 1, slice_ptr, cols, sv, b, x, w, mode, tol, eps, res_hist_out,
                        res_hist_out ? max_iter : 0, stream, &s);
    if (!rc && !h_ovf) rc = fem_pcg_set_cols16(s, d16);
    int it = 0, stt = 0;
    double rz = 0.0;
    if (!rc) rc = fem_pcg_solve(s, max_iter, 32, &it, &stt, &rz);
    if (s) fem_pcg_destroy(s);
    if (iters_out) *iters_out = it;
    if (status_out) *status_out = stt;
    (void)hipFreeAsync(width, st);
    (void)hipFreeAsync(slice_ptr, st);
    (void)hipFreeAsync(work, st);
    (void)hipFreeAsync(cols, st);
    (void)hipFreeAsync(csr2sell, st);
    (void)hipFreeAsync(sv, st);
    (void)hipFreeAsync(d16, st);
    (void)hipFreeAsync(ovf, st);
    (void)hipFreeAsync(w, st);
    (void)hipStreamSynchronize(st);
    return rc;
}

}  // extern "C"
