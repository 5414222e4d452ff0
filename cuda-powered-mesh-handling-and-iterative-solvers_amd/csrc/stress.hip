// Stress recovery (post-solve) on gfx950.
//
// Per element and quadrature point: strain = B u_e (Voigt xx, yy, zz, xy, yz, xz with engineering shear),
// stress = D strain with the reference's isotropic D (`solver/element.py:282-306`), the symmetric 3x3 tensor
// (`compute_stress_tensor`, `:308-330`) and von Mises (`compute_von_mises_stress`, `:332-353`). The c3d4 path is
// `compute_c3d4_element_stress` (`:905-937`, closed-form P1 gradients); the isoparametric path covers
// `compute_c3d8_element_stress` (`:1696-1752`), `compute_c3d6_element_stress` (`:2570-2629`) and
// `compute_c3d10_element_stress` (`:1127-1189`) from host-evaluated natural derivative tables, returning either
// the weight-summed tensor / von Mises (single=True) or one per point.
//
// Bandwidth-bound: per element the connectivity, npe coordinates and npe displacements are read (gathers of
// 24 B rows) and 10 doubles per output point are written; no B matrix is materialised.
#include "element.hpp"

namespace fem {

struct Dmat {
    double d0, d1, g;   // D[0][0] = c(1-nu), D[0][1] = c nu, D[3][3] = c (1-2nu)/2
};

__host__ __device__ inline Dmat dmat(double E, double nu) {
    const double c = E / ((1.0 + nu) * (1.0 - 2.0 * nu));
    return Dmat{c * (1.0 - nu), c * nu, c * ((1.0 - 2.0 * nu) / 2.0)};
}

// strain from gradients g[a][k] and displacements u[a][k] -> stress (6) -> von Mises
template <int NPE>
__device__ __forceinline__ double point_stress(const double g[NPE][3], const double u[NPE][3], const Dmat& D,
                                               double s[6]) {
    double e[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < NPE; ++a) {
        e[0] += g[a][0] * u[a][0];
        e[1] += g[a][1] * u[a][1];
        e[2] += g[a][2] * u[a][2];
        e[3] += g[a][1] * u[a][0] + g[a][0] * u[a][1];
        e[4] += g[a][2] * u[a][1] + g[a][1] * u[a][2];
        e[5] += g[a][2] * u[a][0] + g[a][0] * u[a][2];
    }
    s[0] = D.d0 * e[0] + D.d1 * e[1] + D.d1 * e[2];
    s[1] = D.d1 * e[0] + D.d0 * e[1] + D.d1 * e[2];
    s[2] = D.d1 * e[0] + D.d1 * e[1] + D.d0 * e[2];
    s[3] = D.g * e[3];
    s[4] = D.g * e[4];
    s[5] = D.g * e[5];
    const double a = s[0] - s[1], b = s[1] - s[2], c = s[2] - s[0];
    return sqrt((a * a + b * b + c * c + 6.0 * (s[3] * s[3] + s[4] * s[4] + s[5] * s[5])) / 2.0);
}

// symmetric tensor rows (xx xy xz / xy yy yz / xz yz zz) with Voigt (xx, yy, zz, xy, yz, xz)
__device__ __forceinline__ void store_tensor(double* __restrict__ out, const double s[6]) {
    out[0] = s[0];
    out[1] = s[3];
    out[2] = s[5];
    out[3] = s[3];
    out[4] = s[1];
    out[5] = s[4];
    out[6] = s[5];
    out[7] = s[4];
    out[8] = s[2];
}

template <int NPE>
__device__ __forceinline__ void load_element(const double* __restrict__ X, const double* __restrict__ U,
                                             const int64_t* __restrict__ c, double x[NPE][3], double u[NPE][3]) {
#pragma unroll
    for (int a = 0; a < NPE; ++a) {
        const int64_t n = c[a];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            x[a][k] = X[3 * n + k];
            u[a][k] = U[3 * n + k];
        }
    }
}

// c3d4: one point, thread per element, 256-element tiles: the tile's connectivity is loaded coalesced through
// LDS and its [256,3,3] tensor block (18 KB, contiguous in the output) is staged in LDS and written coalesced
// (a thread-per-element store of 9 doubles would stride the wave's stores by 72 B).
constexpr int ST_TILE = 256;

__device__ __forceinline__ void write_tile(double* __restrict__ dst, const double* __restrict__ lds, int64_t nval) {
    for (int t = threadIdx.x; t < nval; t += ST_TILE) dst[t] = lds[t];
}

__global__ void __launch_bounds__(ST_TILE) k_tet4_stress(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                         int64_t M, const double* __restrict__ U, Dmat D,
                                                         double* __restrict__ sig, double* __restrict__ vm,
                                                         int64_t* __restrict__ bad) {
    __shared__ int64_t c_s[ST_TILE * 4];
    __shared__ double s_s[ST_TILE * 9];
    const int64_t ntiles = (M + ST_TILE - 1) / ST_TILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t e0 = tile * ST_TILE;
        const int nt = (int)min((int64_t)ST_TILE, M - e0);
        for (int t = threadIdx.x; t < 4 * nt; t += ST_TILE) c_s[t] = conn[4 * e0 + t];
        __syncthreads();
        if ((int)threadIdx.x < nt) {
            const int64_t e = e0 + threadIdx.x;
            const int64_t* c = c_s + 4 * threadIdx.x;
            double g[4][3], u[4][3];
            const double det = tet4_grads(X, c, g);
            // the reference forms B through compute_c3d4_B_matrix, which raises on |det| < 1e-12 (`:857-858`)
            if (bad && fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) u[a][k] = U[3 * c[a] + k];
            double s[6];
            const double v = point_stress<4>(g, u, D, s);
            store_tensor(s_s + 9 * threadIdx.x, s);
            if (vm) vm[e] = v;
        }
        __syncthreads();
        if (sig) write_tile(sig + 9 * e0, s_s, 9 * (int64_t)nt);
        __syncthreads();
    }
}

// isoparametric: thread per element, all points; dN [n_ip][NPE][3] and w [n_ip] staged in LDS.
// layout 0: single (weighted sums) [M,3,3] / [M]; 1: point-minor [M,n_ip,3,3] / [M,n_ip];
// 2: point-major [n_ip,M,3,3] / [n_ip,M] (the c3d10 stack, `:1183-1186`)
constexpr int STRESS_MAX_IP = 32;

template <int NPE>
__global__ void __launch_bounds__(256) k_iso_stress(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                    int64_t M, const double* __restrict__ U, Dmat D,
                                                    const double* __restrict__ dN, const double* __restrict__ w,
                                                    int n_ip, int layout, double* __restrict__ sig,
                                                    double* __restrict__ vm) {
    __shared__ double dn_s[STRESS_MAX_IP * NPE * 3];
    __shared__ double w_s[STRESS_MAX_IP];
    for (int t = threadIdx.x; t < n_ip * NPE * 3; t += blockDim.x) dn_s[t] = dN[t];
    for (int t = threadIdx.x; t < n_ip; t += blockDim.x) w_s[t] = w ? w[t] : 0.0;
    __syncthreads();
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        double x[NPE][3], u[NPE][3];
        load_element<NPE>(X, U, conn + (int64_t)NPE * e, x, u);
        double acc[6] = {0, 0, 0, 0, 0, 0}, vacc = 0.0;
        for (int q = 0; q < n_ip; ++q) {
            const double* dq = dn_s + q * NPE * 3;
            double J[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // J[i][k] = sum_j dN[j][i] x[j][k]
#pragma unroll
            for (int j = 0; j < NPE; ++j)
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) J[3 * i + k] += dq[j * 3 + i] * x[j][k];
            double Ji[9];
            inv3(J, Ji);
            double g[NPE][3];
#pragma unroll
            for (int n = 0; n < NPE; ++n)
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    g[n][i] = Ji[3 * i] * dq[n * 3] + Ji[3 * i + 1] * dq[n * 3 + 1] + Ji[3 * i + 2] * dq[n * 3 + 2];
            double s[6];
            const double v = point_stress<NPE>(g, u, D, s);
            if (layout == 0) {
#pragma unroll
                for (int t = 0; t < 6; ++t) acc[t] += w_s[q] * s[t];
                vacc += w_s[q] * v;
            } else {
                const int64_t slot = layout == 1 ? e * n_ip + q : (int64_t)q * M + e;
                if (sig) store_tensor(sig + 9 * slot, s);
                if (vm) vm[slot] = v;
            }
        }
        if (layout == 0) {
            if (sig) store_tensor(sig + 9 * e, acc);
            if (vm) vm[e] = vacc;
        }
    }
}

// node average of an element field over the sorted incidence (`compute_node_vm_stress`, `:466-504`): the sum runs
// in ascending element order like the reference's sequential index_add; count = incidence length
__global__ void __launch_bounds__(256) k_node_average(const double* __restrict__ ev, int npe,
                                                      const int32_t* __restrict__ inc_ptr,
                                                      const int32_t* __restrict__ inc, int64_t N,
                                                      double* __restrict__ out) {
    constexpr int CH = 8;   // independent loads in flight per chunk; the adds stay in incidence order
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
        const int b = inc_ptr[n], e = inc_ptr[n + 1];
        double s = 0.0;
        for (int i0 = b; i0 < e; i0 += CH) {
            int id[CH];
            double v[CH];
#pragma unroll
            for (int j = 0; j < CH; ++j) id[j] = (i0 + j < e) ? inc[i0 + j] : -1;
#pragma unroll
            for (int j = 0; j < CH; ++j) v[j] = id[j] >= 0 ? ev[id[j] / npe] : 0.0;
#pragma unroll
            for (int j = 0; j < CH; ++j)
                if (id[j] >= 0) s += v[j];
        }
        out[n] = e > b ? s / (double)(e - b) : 0.0;
    }
}

// face traction sigma_e n_ef (`compute_c3d4_surface_forces`, `:3343-3362`): normals [M,F,3], stress [M,3,3]
__global__ void k_face_forces(const double* __restrict__ nrm, const double* __restrict__ sig, int64_t M, int F,
                              double* __restrict__ out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < M * F; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = t / F;
        const double* s = sig + 9 * e;
        const double* v = nrm + 3 * t;
#pragma unroll
        for (int i = 0; i < 3; ++i) out[3 * t + i] = s[3 * i] * v[0] + s[3 * i + 1] * v[1] + s[3 * i + 2] * v[2];
    }
}

// f[e0, f0] + f[e1, f1] per shared face (`compute_c3d4_shared_face_forces_sum`, `:3364-3382`); idx [S,2,2]
__global__ void k_shared_face_sum(const int64_t* __restrict__ idx, const double* __restrict__ ff, int F, int64_t S,
                                  double* __restrict__ out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < S; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = idx[4 * t] * F + idx[4 * t + 1];
        const int64_t b = idx[4 * t + 2] * F + idx[4 * t + 3];
#pragma unroll
        for (int i = 0; i < 3; ++i) out[3 * t + i] = ff[3 * a + i] + ff[3 * b + i];
    }
}

// Voigt [M,6] -> symmetric tensor [M,3,3] (`compute_stress_tensor`, `:308-330`)
__global__ void k_voigt_to_tensor(const double* __restrict__ v, int64_t M, double* __restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        double s[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) s[t] = v[6 * e + t];
        store_tensor(out + 9 * e, s);
    }
}

// tensor [M,3,3] -> von Mises [M] (`compute_von_mises_stress`, `:332-353`; reads the upper triangle like it)
__global__ void k_von_mises(const double* __restrict__ t, int64_t M, double* __restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        const double* s = t + 9 * e;
        const double a = s[0] - s[4], b = s[4] - s[8], c = s[8] - s[0];
        out[e] = sqrt((a * a + b * b + c * c + 6.0 * (s[1] * s[1] + s[5] * s[5] + s[2] * s[2])) / 2.0);
    }
}

}  // namespace fem

using namespace fem;

extern "C" {

int fem_tet4_stress(const double* coords, const int64_t* conn, int64_t M, const double* u, double E, double nu,
                    double* sig, double* vm, int64_t* bad_idx, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_tet4_stress, dim3(stream_grid(M, 256)), dim3(256), 0, S(stream), coords, conn, M, u,
                       dmat(E, nu), sig, vm, bad_idx);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_iso_stress(const double* coords, const int64_t* conn, int64_t M, int npe, const double* u, double E, double nu,
                   const double* dN, const double* w, int n_ip, int layout, double* sig, double* vm,
                   fem_stream_t stream) {
    if (n_ip < 1 || n_ip > STRESS_MAX_IP || layout < 0 || layout > 2 || (layout == 0 && !w)) {
        set_error("fem_iso_stress: n_ip must be in [1, %d], layout in {0,1,2} (0 needs weights)", STRESS_MAX_IP);
        return FEM_EARG;
    }
    if (M <= 0) return FEM_OK;
    const dim3 g(stream_grid(M, 256)), b(256);
    const Dmat D = dmat(E, nu);
    switch (npe) {
        case 6: hipLaunchKernelGGL(k_iso_stress<6>, g, b, 0, S(stream), coords, conn, M, u, D, dN, w, n_ip, layout, sig, vm); break;
        case 8: hipLaunchKernelGGL(k_iso_stress<8>, g, b, 0, S(stream), coords, conn, M, u, D, dN, w, n_ip, layout, sig, vm); break;
        case 10: hipLaunchKernelGGL(k_iso_stress<10>, g, b, 0, S(stream), coords, conn, M, u, D, dN, w, n_ip, layout, sig, vm); break;
        default:
            set_error("fem_iso_stress: npe %d not supported (6, 8, 10)", npe);
            return FEM_EBADTYPE;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_voigt_to_tensor(const double* voigt, int64_t M, double* tensor, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_voigt_to_tensor, dim3(stream_grid(M, 256)), dim3(256), 0, S(stream), voigt, M, tensor);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_von_mises(const double* tensor, int64_t M, double* vm, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_von_mises, dim3(stream_grid(M, 256)), dim3(256), 0, S(stream), tensor, M, vm);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_node_average(const double* ev, int npe, const int32_t* inc_ptr, const int32_t* inc, int64_t N, double* out,
                     fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_node_average, dim3(stream_grid(N, 256)), dim3(256), 0, S(stream), ev, npe, inc_ptr, inc, N,
                       out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_face_forces(const double* normals, const double* sig, int64_t M, int F, double* out, fem_stream_t stream) {
    if (M * F <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_face_forces, dim3(stream_grid(M * F, 256)), dim3(256), 0, S(stream), normals, sig, M, F, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_shared_face_sum(const int64_t* idx, const double* face_forces, int F, int64_t S_, double* out,
                        fem_stream_t stream) {
    if (S_ <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_shared_face_sum, dim3(stream_grid(S_, 256)), dim3(256), 0, S(stream), idx, face_forces, F, S_,
                       out);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // extern "C"
