// Element stiffness quadrature (L1) and deterministic global assembly (row-gather) on gfx950.
//
// P1 tets use the closed form of the reference's B^T D B V (`solver/element.py:835-903`): with the
// gradients g_a of the 4 barycentric shape functions and Lame constants
//   lambda = E nu / ((1+nu)(1-2nu)),  mu = E / (2(1+nu))   (the D of `solver/element.py:282-306`),
// block (a,b) of K_e is V (lambda g_a g_b^T + mu g_b g_a^T + mu (g_a.g_b) I). Isoparametric solids use
// the same block formula per quadrature point with signed detJ (Q2), which is exactly B^T D B for the
// isotropic D; only the rounding order differs from the reference's dense einsums.
#include <algorithm>

#include "common.hpp"
#include "element.hpp"

namespace fem {

// ---------------------------------------------------------------- c3d4 element matrices
// 64 elements per 256-thread block: 64 lanes form gradients into LDS, then all 256 threads write the
// block's contiguous output (64 * d * d values) coalesced.
template <int KIND>
__global__ void __launch_bounds__(256) k_tet4_ke(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                 int64_t M, double E, double nu, double* __restrict__ Ke,
                                                 int64_t* __restrict__ bad) {
    constexpr int D = (KIND == FEM_KIND_POISSON) ? 4 : 12;
    __shared__ double g_s[64][4][3];
    __shared__ double v_s[64];
    const int64_t e0 = (int64_t)blockIdx.x * 64;
    if (threadIdx.x < 64) {
        int64_t e = e0 + threadIdx.x;
        if (e < M) {
            double g[4][3];
            double det = tet4_grads(X, conn + 4 * e, g);
            if (fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) g_s[threadIdx.x][a][k] = g[a][k];
            v_s[threadIdx.x] = fabs(det) / 6.0;
        }
    }
    __syncthreads();
    const Lame L = lame(E, nu);
    const int64_t nval = min((int64_t)64, M - e0) * D * D;
    double* out = Ke + e0 * D * D;
    for (int64_t t = threadIdx.x; t < nval; t += 256) {
        const int le = (int)(t / (D * D));
        const int ij = (int)(t - (int64_t)le * D * D);
        const int i = ij / D, j = ij - (ij / D) * D;
        const double V = v_s[le];
        double val;
        if (KIND == FEM_KIND_ELASTIC) {
            const int a = i / 3, ci = i - 3 * (i / 3), b = j / 3, cj = j - 3 * (j / 3);
            const double* ga = g_s[le][a];
            const double* gb = g_s[le][b];
            double s = L.lam * ga[ci] * gb[cj] + L.mu * ga[cj] * gb[ci];
            if (ci == cj) s += L.mu * (ga[0] * gb[0] + ga[1] * gb[1] + ga[2] * gb[2]);
            val = s * V;
        } else if (KIND == FEM_KIND_POISSON) {
            const double* ga = g_s[le][i];
            const double* gb = g_s[le][j];
            val = E * (ga[0] * gb[0] + ga[1] * gb[1] + ga[2] * gb[2]) * V;
        } else {  // consistent P1 mass, rho V (1 + delta_ab) / 20 per component (E carries rho)
            const int a = i / 3, ci = i - 3 * (i / 3), b = j / 3, cj = j - 3 * (j / 3);
            val = (ci == cj) ? E * V * ((a == b) ? 2.0 : 1.0) / 20.0 : 0.0;
        }
        out[t] = val;
    }
}

// volumes / gradients / B of c3d4 (`compute_tetrahedral_volumes` `solver/element.py:514-541`,
// `compute_c3d4_B_matrix` `:835-881`); any output pointer may be null.
__global__ void __launch_bounds__(256) k_tet4_geom(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                   int64_t M, double* __restrict__ vol, double* __restrict__ grads,
                                                   double* __restrict__ B, int64_t* __restrict__ bad) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        double g[4][3];
        const double det = tet4_grads(X, conn + 4 * e, g);
        if (bad && fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
        if (vol) vol[e] = fabs(det) / 6.0;
        if (grads)
            for (int a = 0; a < 4; ++a)
                for (int k = 0; k < 3; ++k) grads[e * 12 + a * 3 + k] = g[a][k];
        if (B) {
            double* b = B + e * 72;
            for (int t = 0; t < 72; ++t) b[t] = 0.0;
            for (int a = 0; a < 4; ++a) {
                const double gx = g[a][0], gy = g[a][1], gz = g[a][2];
                b[0 * 12 + 3 * a] = gx;
                b[1 * 12 + 3 * a + 1] = gy;
                b[2 * 12 + 3 * a + 2] = gz;
                b[3 * 12 + 3 * a] = gy;
                b[3 * 12 + 3 * a + 1] = gx;
                b[4 * 12 + 3 * a + 1] = gz;
                b[4 * 12 + 3 * a + 2] = gy;
                b[5 * 12 + 3 * a] = gz;
                b[5 * 12 + 3 * a + 2] = gx;
            }
        }
    }
}

// Jacobian / global gradients / B of an isoparametric element at ONE point (dN [npe,3] natural derivatives):
// compute_c3d8_Jacobian `solver/element.py:1601-1632`, _shape_gradients `:1634-1664`, _B_matrix `:1666-1694`
// (and the c3d6 `:2482-2568` / c3d10 `:1026-1125` equivalents). Thread per element; outputs may be null.
__global__ void __launch_bounds__(256) k_iso_geom(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                  int64_t M, int npe, const double* __restrict__ dN,
                                                  double* __restrict__ Jout, double* __restrict__ Gout,
                                                  double* __restrict__ Bout) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x) {
        double J[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int j = 0; j < npe; ++j) {
            const int64_t n = conn[e * npe + j];
            const double x0 = X[3 * n], x1 = X[3 * n + 1], x2 = X[3 * n + 2];
            for (int i = 0; i < 3; ++i) {
                const double d = dN[j * 3 + i];
                J[3 * i] += d * x0;
                J[3 * i + 1] += d * x1;
                J[3 * i + 2] += d * x2;
            }
        }
        if (Jout)
            for (int t = 0; t < 9; ++t) Jout[e * 9 + t] = J[t];
        if (!Gout && !Bout) continue;
        const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8], c02 = J[3] * J[7] - J[4] * J[6];
        const double id = 1.0 / (J[0] * c00 + J[1] * c01 + J[2] * c02);
        const double Ji[9] = {c00 * id, (J[2] * J[7] - J[1] * J[8]) * id, (J[1] * J[5] - J[2] * J[4]) * id,
                              c01 * id, (J[0] * J[8] - J[2] * J[6]) * id, (J[2] * J[3] - J[0] * J[5]) * id,
                              c02 * id, (J[1] * J[6] - J[0] * J[7]) * id, (J[0] * J[4] - J[1] * J[3]) * id};
        const int d3 = 3 * npe;
        if (Bout)
            for (int t = 0; t < 6 * d3; ++t) Bout[e * 6 * d3 + t] = 0.0;
        for (int n = 0; n < npe; ++n) {
            double g[3];
            for (int i = 0; i < 3; ++i)
                g[i] = Ji[3 * i] * dN[n * 3] + Ji[3 * i + 1] * dN[n * 3 + 1] + Ji[3 * i + 2] * dN[n * 3 + 2];
            if (Gout)
                for (int i = 0; i < 3; ++i) Gout[(e * npe + n) * 3 + i] = g[i];
            if (Bout) {
                double* b = Bout + e * 6 * d3;
                b[0 * d3 + 3 * n] = g[0];
                b[1 * d3 + 3 * n + 1] = g[1];
                b[2 * d3 + 3 * n + 2] = g[2];
                b[3 * d3 + 3 * n] = g[1];
                b[3 * d3 + 3 * n + 1] = g[0];
                b[4 * d3 + 3 * n + 1] = g[2];
                b[4 * d3 + 3 * n + 2] = g[1];
                b[5 * d3 + 3 * n] = g[2];
                b[5 * d3 + 3 * n + 2] = g[0];
            }
        }
    }
}

// ---------------------------------------------------------------- packed symmetric element matrices (bs = 3)
// K_e = sum_q B_q^T D B_q is symmetric: the internal assembly path stores only its upper 3x3 blocks (a <= b), row-major
// over the upper triangle (block index ke_sym_blk(a, b)), 9 doubles each, padded to an even count per element
// (16-byte aligned elements): c3d10 496 doubles instead of 900, c3d8 324 of 576, c3d6 190 of 324, c3d4 78 of 144.
__host__ __device__ constexpr int ke_sym_nb(int npe) { return npe * (npe + 1) / 2; }
__host__ __device__ constexpr int ke_sym_stride(int npe) { return (9 * ke_sym_nb(npe) + 1) & ~1; }
__host__ __device__ constexpr int ke_sym_blk(int npe, int a, int b) { return a * npe - a * (a - 1) / 2 + (b - a); }

// ---------------------------------------------------------------- isoparametric solids (wave per element)
constexpr int ISO_MAX_IP = 32;
constexpr int ISO_IPC = 16;   // points whose geometry is staged in LDS at once

// LDS hand-off between the lanes of one wave (program order for the compiler; a wave's LDS operations run in order)
__device__ __forceinline__ void iso_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int NPE, bool MASS, bool SC = false, bool PK = false>
__global__ void __launch_bounds__(256) k_iso_ke(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                int64_t M, double E, double nu, const double* __restrict__ dN,
                                                const double* __restrict__ w, int n_ip, int mode,
                                                double* __restrict__ Ke, const double* __restrict__ Nv = nullptr) {
    // Wave per element, 4 per block. Per chunk of up to ISO_IPC points, lane q of a wave forms the Jacobian,
    // detJ and the global gradients of point q (`einsum("ji,mjk->mik")`, `einsum("mij,nj->mni")`) into LDS —
    // all points of the chunk at once, one barrier — then lane (a,b), a <= b, adds the 3x3 block of every point
    // in point order. c3d10 (100 blocks > 64 lanes): only a <= b, block (b,a) written as its transpose (K_e =
    // sum B^T D B is symmetric; mirrored entries equal the directly formed ones up to the order of two products),
    // 55 blocks, one per lane. c3d8 / c3d6 (<= 64 blocks): every block formed directly.
    // mode FEM_ISO_MASS (E = rho, Nv = shape values [n_ip][NPE]): block (a,b) = rho sum_q w_q |detJ_q| N_a N_b I3.
    // Every wave walks its elements (grid-stride; the grid is the resident one) with wave-level LDS hand-offs only:
    // no workgroup barrier after the rule tables are staged, the next element's coordinates and the one after's node
    // ids are loaded while the current element is formed.
    constexpr int D = 3 * NPE;
    // PK (stiffness only): the packed symmetric form -- lanes form the upper blocks a <= b only, written as
    // ke_sym_stride(NPE) doubles per element (ke_row3's packed read mirrors the lower ones)
    static_assert(!PK || !MASS, "packed K_e: stiffness only");
    constexpr bool SYM = NPE * NPE > 64 || PK;
    constexpr int NS = SYM ? NPE * (NPE + 1) / 2 : NPE * NPE;
    static_assert(NS <= 64, "one block per lane");
    // rule tables in dynamic LDS sized to the rule (n_ip NPE 3 natural derivatives, then n_ip NPE shape values)
    extern __shared__ double iso_dyn[];
    double* dn_s = iso_dyn;
    double* nv_s = iso_dyn + n_ip * NPE * 3;
    __shared__ double x_s[4][NPE][3];
    // point gradients of the current chunk; after the last chunk the same space stages the element matrix so
    // that the wave writes it out as contiguous 16-byte stores
    constexpr int GK = (ISO_IPC * NPE * 3 > D * D) ? ISO_IPC * NPE * 3 : D * D;
    __shared__ double gk_s[4][GK];
    __shared__ double c_s[4][ISO_IPC];
    constexpr bool mass = MASS;   // mode == FEM_ISO_MASS
    for (int t = threadIdx.x; t < n_ip * NPE * 3; t += 256) dn_s[t] = dN[t];
    if (mass)
        for (int t = threadIdx.x; t < n_ip * NPE; t += 256) nv_s[t] = Nv[t];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();   // rule tables staged (the only workgroup barrier)
    const int64_t step = (int64_t)gridDim.x * 4;
    const bool xl = lane < NPE * 3;   // lane (node a, coordinate k) of the coordinate loads
    const int xa = lane / 3, xk = lane - 3 * (lane / 3);
    int64_t e = (int64_t)blockIdx.x * 4 + wid;
    int64_t cn = (xl && e < M) ? conn[e * NPE + xa] : 0;
    double xr = (xl && e < M) ? X[3 * cn + xk] : 0.0;
    int64_t e1 = e + step;
    int64_t cn1 = (xl && e1 < M) ? conn[e1 * NPE + xa] : 0;
    const Lame L = lame(E, nu);
    int ba = 0, bb = 0;   // this lane's block (SYM: ba <= bb), lane < NS
    if (SYM) {
        int t = lane;
        while (ba < NPE && t >= NPE - ba) {
            t -= NPE - ba;
            ++ba;
        }
        bb = ba + t;
    } else {
        ba = lane / NPE;
        bb = lane - NPE * (lane / NPE);
    }
    const bool mirror = SYM && ba != bb;
    const bool blk_lane = lane < NS;
  for (; e < M; e += step) {
    iso_wave_sync();   // the previous element's LDS reads are done
    if (xl) x_s[wid][xa][xk] = xr;
    const int64_t e2 = e1 + step;
    const double xr1 = (xl && e1 < M) ? X[3 * cn1 + xk] : 0.0;
    const int64_t cn2 = (xl && e2 < M) ? conn[e2 * NPE + xa] : 0;
    iso_wave_sync();
    const bool active = true;
    double acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = 0.0;

    double vol = 0.0;
    if (mode == FEM_ISO_VOLUME) {  // wedge volume: 3 sub-tets (`solver/element.py:2198-2232`)
        const int T[3][4] = {{0, 1, 2, 3}, {1, 2, 4, 3}, {2, 4, 5, 3}};
        for (int s = 0; s < 3; ++s) {
            double u[3], v[3], d[3];
            for (int k = 0; k < 3; ++k) {
                u[k] = x_s[wid][T[s][1]][k] - x_s[wid][T[s][0]][k];
                v[k] = x_s[wid][T[s][2]][k] - x_s[wid][T[s][0]][k];
                d[k] = x_s[wid][T[s][3]][k] - x_s[wid][T[s][0]][k];
            }
            double cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2], cz = u[0] * v[1] - u[1] * v[0];
            vol += fabs(cx * d[0] + cy * d[1] + cz * d[2]) / 6.0;
        }
    }

    for (int q0 = 0; q0 < n_ip; q0 += ISO_IPC) {
        const int nq = min(ISO_IPC, n_ip - q0);
        if (lane < nq) {
            const int q = q0 + lane;
            const double* dq = dn_s + q * NPE * 3;
            double J[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
            for (int j = 0; j < NPE; ++j) {   // node order j ascending for every entry, as the einsum loop
                const double d[3] = {dq[j * 3], dq[j * 3 + 1], dq[j * 3 + 2]};
                const double xx[3] = {x_s[wid][j][0], x_s[wid][j][1], x_s[wid][j][2]};
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) J[3 * i + k] += d[i] * xx[k];
            }
            const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8],
                         c02 = J[3] * J[7] - J[4] * J[6];
            const double det = J[0] * c00 + J[1] * c01 + J[2] * c02;
            const double id = 1.0 / det;
            const double Ji[9] = {c00 * id, (J[2] * J[7] - J[1] * J[8]) * id, (J[1] * J[5] - J[2] * J[4]) * id,
                                  c01 * id, (J[0] * J[8] - J[2] * J[6]) * id, (J[2] * J[3] - J[0] * J[5]) * id,
                                  c02 * id, (J[1] * J[6] - J[0] * J[7]) * id, (J[0] * J[4] - J[1] * J[3]) * id};
#pragma unroll 1
            for (int n = 0; n < NPE; ++n)
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    gk_s[wid][(lane * NPE + n) * 3 + i] =
                        Ji[3 * i] * dq[n * 3] + Ji[3 * i + 1] * dq[n * 3 + 1] + Ji[3 * i + 2] * dq[n * 3 + 2];
            c_s[wid][lane] = mass ? fabs(det) * w[q] * E
                                  : (mode == FEM_ISO_SUM) ? det * w[q] : (mode == FEM_ISO_STACK ? det : vol);
        }
        iso_wave_sync();
        for (int ql = 0; ql < nq; ++ql) {
            const double coef = c_s[wid][ql];
            if (mass) {
                if (blk_lane) {
                    const double s = nv_s[(q0 + ql) * NPE + ba] * nv_s[(q0 + ql) * NPE + bb] * coef;
                    acc[0] += s;
                    acc[4] += s;
                    acc[8] += s;
                }
            } else if (blk_lane) {
                const double* ga = &gk_s[wid][(ql * NPE + ba) * 3];
                const double* gb = &gk_s[wid][(ql * NPE + bb) * 3];
                const double dot = ga[0] * gb[0] + ga[1] * gb[1] + ga[2] * gb[2];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        double s = L.lam * ga[i] * gb[k] + L.mu * ga[k] * gb[i];
                        if (i == k) s += L.mu * dot;
                        if (mode == FEM_ISO_STACK) acc[3 * i + k] = s * coef;
                        else acc[3 * i + k] += s * coef;
                    }
            }
            if (mode == FEM_ISO_STACK && active && blk_lane) {
                double* out = Ke + ((int64_t)(q0 + ql) * M + e) * D * D;
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        out[(3 * ba + i) * D + 3 * bb + k] = acc[3 * i + k];
                        if (mirror) out[(3 * bb + k) * D + 3 * ba + i] = acc[3 * i + k];
                    }
            }
        }
        iso_wave_sync();
    }
    if (SC && active) {   // scalar mass (MASS only): the NPE x NPE factor of M_e = M_s (x) I3, acc[0] of each block
        double* ks = gk_s[wid];
        if (blk_lane) {
            ks[ba * NPE + bb] = acc[0];
            if (mirror) ks[bb * NPE + ba] = acc[0];
        }
        __builtin_amdgcn_wave_barrier();
        double2* out2 = reinterpret_cast<double2*>(Ke + e * NPE * NPE);   // NPE^2 even: 16-byte aligned rows
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < NPE * NPE / 2; t += 64) out2[t] = ks2[t];
    } else if (PK && mode != FEM_ISO_STACK && active) {   // packed upper blocks, lane = packed block index
        double* ks = gk_s[wid];
        constexpr int PKS = ke_sym_stride(NPE);
        if (blk_lane) {
#pragma unroll
            for (int t = 0; t < 9; ++t) ks[lane * 9 + t] = acc[t];
        }
        if (lane == 0 && PKS > 9 * NS) ks[9 * NS] = 0.0;   // the padding double of an odd 9 NS
        __builtin_amdgcn_wave_barrier();
        double2* out2 = reinterpret_cast<double2*>(Ke + e * PKS);   // PKS even: 16-byte aligned elements
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < PKS / 2; t += 64) out2[t] = ks2[t];
    } else if (mode != FEM_ISO_STACK && active) {   // (the loop above ended on a wave sync: gk_s is free)
        double* ks = gk_s[wid];
        if (blk_lane) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ks[(3 * ba + i) * D + 3 * bb + k] = acc[3 * i + k];
                    if (mirror) ks[(3 * bb + k) * D + 3 * ba + i] = acc[3 * i + k];
                }
        }
        __builtin_amdgcn_wave_barrier();
        // D*D is even for every NPE here, and e * D * D * 8 bytes is 16-byte aligned
        double2* out2 = reinterpret_cast<double2*>(Ke + e * D * D);
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < D * D / 2; t += 64) out2[t] = ks2[t];
    }
    xr = xr1;
    cn1 = cn2;
    e1 = e2;
  }
}

template <int NPE, bool MASS, bool SC = false, bool PK = false>
__global__ void __launch_bounds__(256) k_iso_ke1(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                int64_t M, double E, double nu, const double* __restrict__ dN,
                                                const double* __restrict__ w, int n_ip, int mode,
                                                double* __restrict__ Ke, const double* __restrict__ Nv = nullptr) {
    // (the one-element-per-wave form: c3d8 / c3d6, whose cheaper elements ran 5-7 % slower in the walking k_iso_ke)
    // Wave per element, 4 per block. Per chunk of up to ISO_IPC points, lane q of a wave forms the Jacobian,
    // detJ and the global gradients of point q (`einsum("ji,mjk->mik")`, `einsum("mij,nj->mni")`) into LDS —
    // all points of the chunk at once, one barrier — then lane (a,b), a <= b, adds the 3x3 block of every point
    // in point order. c3d10 (100 blocks > 64 lanes): only a <= b, block (b,a) written as its transpose (K_e =
    // sum B^T D B is symmetric; mirrored entries equal the directly formed ones up to the order of two products),
    // 55 blocks, one per lane. c3d8 / c3d6 (<= 64 blocks): every block formed directly.
    // mode FEM_ISO_MASS (E = rho, Nv = shape values [n_ip][NPE]): block (a,b) = rho sum_q w_q |detJ_q| N_a N_b I3.
    constexpr int D = 3 * NPE;
    // PK (stiffness only): the packed symmetric form -- lanes form the upper blocks a <= b only, written as
    // ke_sym_stride(NPE) doubles per element (ke_row3's packed read mirrors the lower ones)
    static_assert(!PK || !MASS, "packed K_e: stiffness only");
    constexpr bool SYM = NPE * NPE > 64 || PK;
    constexpr int NS = SYM ? NPE * (NPE + 1) / 2 : NPE * NPE;
    static_assert(NS <= 64, "one block per lane");
    // rule tables in dynamic LDS sized to the rule (n_ip NPE 3 natural derivatives, then n_ip NPE shape values)
    extern __shared__ double iso_dyn[];
    double* dn_s = iso_dyn;
    double* nv_s = iso_dyn + n_ip * NPE * 3;
    __shared__ double x_s[4][NPE][3];
    // point gradients of the current chunk; after the last chunk the same space stages the element matrix so
    // that the wave writes it out as contiguous 16-byte stores
    constexpr int GK = (ISO_IPC * NPE * 3 > D * D) ? ISO_IPC * NPE * 3 : D * D;
    __shared__ double gk_s[4][GK];
    __shared__ double c_s[4][ISO_IPC];
    constexpr bool mass = MASS;   // mode == FEM_ISO_MASS
    for (int t = threadIdx.x; t < n_ip * NPE * 3; t += 256) dn_s[t] = dN[t];
    if (mass)
        for (int t = threadIdx.x; t < n_ip * NPE; t += 256) nv_s[t] = Nv[t];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t e = (int64_t)blockIdx.x * 4 + wid;
    const bool active = e < M;
    if (active && lane < NPE * 3) {
        int a = lane / 3, k = lane - 3 * (lane / 3);
        x_s[wid][a][k] = X[3 * conn[e * NPE + a] + k];
    }
    __syncthreads();
    const Lame L = lame(E, nu);
    int ba = 0, bb = 0;   // this lane's block (SYM: ba <= bb), lane < NS
    if (SYM) {
        int t = lane;
        while (ba < NPE && t >= NPE - ba) {
            t -= NPE - ba;
            ++ba;
        }
        bb = ba + t;
    } else {
        ba = lane / NPE;
        bb = lane - NPE * (lane / NPE);
    }
    const bool mirror = SYM && ba != bb;
    const bool blk_lane = lane < NS;
    double acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = 0.0;

    double vol = 0.0;
    if (mode == FEM_ISO_VOLUME) {  // wedge volume: 3 sub-tets (`solver/element.py:2198-2232`)
        const int T[3][4] = {{0, 1, 2, 3}, {1, 2, 4, 3}, {2, 4, 5, 3}};
        for (int s = 0; s < 3; ++s) {
            double u[3], v[3], d[3];
            for (int k = 0; k < 3; ++k) {
                u[k] = x_s[wid][T[s][1]][k] - x_s[wid][T[s][0]][k];
                v[k] = x_s[wid][T[s][2]][k] - x_s[wid][T[s][0]][k];
                d[k] = x_s[wid][T[s][3]][k] - x_s[wid][T[s][0]][k];
            }
            double cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2], cz = u[0] * v[1] - u[1] * v[0];
            vol += fabs(cx * d[0] + cy * d[1] + cz * d[2]) / 6.0;
        }
    }

    for (int q0 = 0; q0 < n_ip; q0 += ISO_IPC) {
        const int nq = min(ISO_IPC, n_ip - q0);
        if (lane < nq) {
            const int q = q0 + lane;
            const double* dq = dn_s + q * NPE * 3;
            double J[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
            for (int j = 0; j < NPE; ++j) {   // node order j ascending for every entry, as the einsum loop
                const double d[3] = {dq[j * 3], dq[j * 3 + 1], dq[j * 3 + 2]};
                const double xx[3] = {x_s[wid][j][0], x_s[wid][j][1], x_s[wid][j][2]};
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) J[3 * i + k] += d[i] * xx[k];
            }
            const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8],
                         c02 = J[3] * J[7] - J[4] * J[6];
            const double det = J[0] * c00 + J[1] * c01 + J[2] * c02;
            const double id = 1.0 / det;
            const double Ji[9] = {c00 * id, (J[2] * J[7] - J[1] * J[8]) * id, (J[1] * J[5] - J[2] * J[4]) * id,
                                  c01 * id, (J[0] * J[8] - J[2] * J[6]) * id, (J[2] * J[3] - J[0] * J[5]) * id,
                                  c02 * id, (J[1] * J[6] - J[0] * J[7]) * id, (J[0] * J[4] - J[1] * J[3]) * id};
#pragma unroll 1
            for (int n = 0; n < NPE; ++n)
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    gk_s[wid][(lane * NPE + n) * 3 + i] =
                        Ji[3 * i] * dq[n * 3] + Ji[3 * i + 1] * dq[n * 3 + 1] + Ji[3 * i + 2] * dq[n * 3 + 2];
            c_s[wid][lane] = mass ? fabs(det) * w[q] * E
                                  : (mode == FEM_ISO_SUM) ? det * w[q] : (mode == FEM_ISO_STACK ? det : vol);
        }
        __syncthreads();
        for (int ql = 0; ql < nq; ++ql) {
            const double coef = c_s[wid][ql];
            if (mass) {
                if (blk_lane) {
                    const double s = nv_s[(q0 + ql) * NPE + ba] * nv_s[(q0 + ql) * NPE + bb] * coef;
                    acc[0] += s;
                    acc[4] += s;
                    acc[8] += s;
                }
            } else if (blk_lane) {
                const double* ga = &gk_s[wid][(ql * NPE + ba) * 3];
                const double* gb = &gk_s[wid][(ql * NPE + bb) * 3];
                const double dot = ga[0] * gb[0] + ga[1] * gb[1] + ga[2] * gb[2];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        double s = L.lam * ga[i] * gb[k] + L.mu * ga[k] * gb[i];
                        if (i == k) s += L.mu * dot;
                        if (mode == FEM_ISO_STACK) acc[3 * i + k] = s * coef;
                        else acc[3 * i + k] += s * coef;
                    }
            }
            if (mode == FEM_ISO_STACK && active && blk_lane) {
                double* out = Ke + ((int64_t)(q0 + ql) * M + e) * D * D;
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        out[(3 * ba + i) * D + 3 * bb + k] = acc[3 * i + k];
                        if (mirror) out[(3 * bb + k) * D + 3 * ba + i] = acc[3 * i + k];
                    }
            }
        }
        __syncthreads();
    }
    if (SC && active) {   // scalar mass: as k_iso_ke
        double* ks = gk_s[wid];
        if (blk_lane) {
            ks[ba * NPE + bb] = acc[0];
            if (mirror) ks[bb * NPE + ba] = acc[0];
        }
        __builtin_amdgcn_wave_barrier();
        double2* out2 = reinterpret_cast<double2*>(Ke + e * NPE * NPE);
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < NPE * NPE / 2; t += 64) out2[t] = ks2[t];
    } else if (PK && mode != FEM_ISO_STACK && active) {   // packed upper blocks (as k_iso_ke)
        double* ks = gk_s[wid];
        constexpr int PKS = ke_sym_stride(NPE);
        if (blk_lane) {
#pragma unroll
            for (int t = 0; t < 9; ++t) ks[lane * 9 + t] = acc[t];
        }
        if (lane == 0 && PKS > 9 * NS) ks[9 * NS] = 0.0;
        __builtin_amdgcn_wave_barrier();
        double2* out2 = reinterpret_cast<double2*>(Ke + e * PKS);
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < PKS / 2; t += 64) out2[t] = ks2[t];
    } else if (mode != FEM_ISO_STACK && active) {   // (the loop above ended on a barrier: gk_s is free)
        double* ks = gk_s[wid];
        if (blk_lane) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ks[(3 * ba + i) * D + 3 * bb + k] = acc[3 * i + k];
                    if (mirror) ks[(3 * bb + k) * D + 3 * ba + i] = acc[3 * i + k];
                }
        }
        __builtin_amdgcn_wave_barrier();
        // D*D is even for every NPE here, and e * D * D * 8 bytes is 16-byte aligned
        double2* out2 = reinterpret_cast<double2*>(Ke + e * D * D);
        const double2* ks2 = reinterpret_cast<const double2*>(ks);
        for (int t = lane; t < D * D / 2; t += 64) out2[t] = ks2[t];
    }
}

// Scalar consistent mass (fem_iso_mass_scalar): Ms_e[a][b] = rho sum_q w_q |detJ_q| N_a(q) N_b(q) -- the factor of
// M_e = Ms_e (x) I3. The element's only per-point quantity is c_q = rho w_q |detJ_q|, so one THREAD forms an element:
// its NPE nodes in registers, per point J (the einsum order of k_iso_ke: node j ascending), detJ and c_q, then the
// NPE (NPE + 1) / 2 upper-triangle sums in point order (s = (N_a N_b) c_q, the additions and order of k_iso_ke's mass
// lanes: the same values), written out as the full symmetric NPE x NPE block with 16-byte stores. The wave-per-element
// form spent its time in per-point lane hand-offs (c3d8 0.9 ms for 681k elements; this form is arithmetic + one
// contiguous 8 NPE^2-byte store per element).
template <int NPE>
__global__ void __launch_bounds__(256) k_iso_mass_s(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                    int64_t M, double rho, const double* __restrict__ dN,
                                                    const double* __restrict__ Nv, const double* __restrict__ w,
                                                    int n_ip, double* __restrict__ Ms) {
    extern __shared__ double mtab[];   // dN [n_ip][NPE][3], Nv [n_ip][NPE], w [n_ip]
    double* dn_s = mtab;
    double* nv_s = mtab + n_ip * NPE * 3;
    double* w_s = nv_s + n_ip * NPE;
    for (int t = threadIdx.x; t < n_ip * NPE * 3; t += 256) dn_s[t] = dN[t];
    for (int t = threadIdx.x; t < n_ip * NPE; t += 256) nv_s[t] = Nv[t];
    for (int t = threadIdx.x; t < n_ip; t += 256) w_s[t] = w[t];
    __syncthreads();
    constexpr int NS = NPE * (NPE + 1) / 2;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < M; e += (int64_t)gridDim.x * 256) {
        double x[NPE][3];
#pragma unroll
        for (int j = 0; j < NPE; ++j) {
            const int64_t c = conn[e * NPE + j];
#pragma unroll
            for (int k = 0; k < 3; ++k) x[j][k] = X[3 * c + k];
        }
        double m[NS];
#pragma unroll
        for (int t = 0; t < NS; ++t) m[t] = 0.0;
#pragma unroll 1
        for (int q = 0; q < n_ip; ++q) {
            const double* dq = dn_s + q * NPE * 3;
            double J[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NPE; ++j) {
                const double d[3] = {dq[j * 3], dq[j * 3 + 1], dq[j * 3 + 2]};
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int k = 0; k < 3; ++k) J[3 * i + k] += d[i] * x[j][k];
            }
            const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8],
                         c02 = J[3] * J[7] - J[4] * J[6];
            const double det = J[0] * c00 + J[1] * c01 + J[2] * c02;
            const double coef = fabs(det) * w_s[q] * rho;
            const double* nq = nv_s + q * NPE;
            int t = 0;
#pragma unroll
            for (int a = 0; a < NPE; ++a)
#pragma unroll
                for (int b = a; b < NPE; ++b) m[t++] += nq[a] * nq[b] * coef;
        }
        double2* out = reinterpret_cast<double2*>(Ms + e * NPE * NPE);   // NPE^2 even: 16-byte aligned blocks
#pragma unroll
        for (int p = 0; p < NPE * NPE / 2; ++p) {
            double v2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 2 * p + h, a = i / NPE, b = i - NPE * (i / NPE);
                const int lo = a < b ? a : b, hi = a < b ? b : a;
                v2[h] = m[lo * NPE - lo * (lo - 1) / 2 + (hi - lo)];
            }
            out[p] = make_double2(v2[0], v2[1]);
        }
    }
}

// ---------------------------------------------------------------- SELL value addressing
// entry index E = slice_ptr[s] + 64 k + lane  ->  value index of block entry rc (row-major in the block)
__device__ __forceinline__ int64_t sell_val(int64_t E, int bs2, int rc) {
    const int64_t lane = E & 63;
    return (E - lane) * bs2 + (int64_t)rc * 64 + lane;
}

__device__ __forceinline__ int find_col(const int32_t* __restrict__ colidx, int lo, int hi, int j) {
    // binary search of column j in the sorted row [lo, hi)
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (colidx[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------- row-gather assembly from element matrices
template <int BS>
__global__ void __launch_bounds__(256) k_assemble_from_ke(const double* __restrict__ Ke, const int64_t* __restrict__ conn,
                                                          int npe, const int32_t* __restrict__ inc_ptr,
                                                          const int32_t* __restrict__ inc, int64_t N,
                                                          const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ colidx,
                                                          const int64_t* __restrict__ csr2sell,
                                                          double* __restrict__ vals) {
    const int d = npe * BS;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        const int lo = rowptr[i], hi = rowptr[i + 1];
        for (int t = inc_ptr[i]; t < inc_ptr[i + 1]; ++t) {
            const int ea = inc[t];
            const int64_t e = ea / npe;
            const int a = ea - (int)e * npe;
            const double* Krow = Ke + e * d * d + (int64_t)(a * BS) * d;
            for (int b = 0; b < npe; ++b) {
                const int j = (int)conn[e * npe + b];
                const int p = find_col(colidx, lo, hi, j);
                const int64_t E = csr2sell[p];
#pragma unroll
                for (int r = 0; r < BS; ++r)
#pragma unroll
                    for (int c = 0; c < BS; ++c) vals[sell_val(E, BS * BS, r * BS + c)] += Krow[r * d + b * BS + c];
            }
        }
    }
}

// XCD-aware row walk of the wave-per-row assembly kernels: SELL slice c (64 rows) belongs to XCD c % 8
// (blockIdx % 8 under the observed round-robin placement), whose blocks take its slices in order. All 64 rows of a
// slice are then written through ONE L2, where their partial value lines merge instead of reaching HBM from eight
// L2s, and heavy row ranges (c3d10 corner nodes, numbered first) stay spread over all XCDs.
// Needs gridDim.x % 8 == 0 (grid_multiple_of_xcd).
struct RowWalk {
    int64_t k, step;
    int xcd;
    __device__ __forceinline__ int64_t row(int64_t kk) const { return ((kk >> 6) * NXCD + xcd) * 64 + (kk & 63); }
};

__device__ __forceinline__ RowWalk row_walk(int waves, int rows_per_wave = 1, int sub = 0) {
    const int xcd = blockIdx.x % NXCD;
    const int64_t lb = blockIdx.x / NXCD, nlb = gridDim.x / NXCD;
    return RowWalk{(lb * waves + (threadIdx.x >> 6)) * rows_per_wave + sub, nlb * waves * rows_per_wave, xcd};
}

// Wave-per-row version of k_assemble_from_ke. The chunk's element nodes are staged in LDS; each owner lane
// (column, block row) builds, per incident element, the bit mask of element-local nodes equal to its column by
// broadcast compares, then issues the element-row loads KU elements at a time (independent, all in flight) before
// adding them in ascending (incidence, b) order onto the stored value — the additions and order of the
// thread-per-row kernel (bit-identical). Repeated nodes inside one element (degenerate input) take the exact
// extra-bit loop.
constexpr int AW_WAVES = 4;   // waves per 256-thread block of the wave-per-row assembly kernels
#ifndef FEM_P1_LPR
#define FEM_P1_LPR 16   // P1 assembly: lanes per row (four rows per wave; 64: 2.95 ms, 32: 1.52, 16: 1.11 on 10M tets)
#endif
#ifndef FEM_KE_KU
#define FEM_KE_KU 8     // bs = 3 / bs = 1 assembly from K_e: incident elements whose loads are in flight per batch
#endif
#ifndef FEM_KE_RPL3
#define FEM_KE_RPL3 1   // bs = 3 assembly from K_e: block rows per lane (3, one lane per column: c3d8 4.2 -> 5.1 ms)
#endif

// CSRW: the row sums (from zero) go to out in row-contiguous block-CSR order (block j of row i at
// (rowptr[i] + j) BS^2, row-major) -- every wave writes a contiguous range -- and k_csr_add_sell adds them into the SELL
// planes slice by slice; otherwise each owner lane read-modify-writes its SELL entry in place.
template <int BS, int NPE, int RPL, bool CSRW = false>
__global__ void __launch_bounds__(256) k_assemble_ke_w(const double* __restrict__ Ke, const int64_t* __restrict__ conn,
                                                       const int32_t* __restrict__ inc_ptr,
                                                       const int32_t* __restrict__ inc, int64_t N,
                                                       const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ colidx,
                                                       const int64_t* __restrict__ csr2sell,
                                                       double* __restrict__ vals) {
    // RPL block rows per lane: BS / RPL lanes per column, 64 RPL / BS columns per group
    constexpr int LPC = BS / RPL;
    constexpr int JG = 64 / LPC;
    constexpr int D = NPE * BS;
    constexpr int KU = (RPL == 1) ? FEM_KE_KU : 4;
    __shared__ int node_s[AW_WAVES][64 * NPE];
    __shared__ int64_t krow_s[AW_WAVES][64];   // offset of the element's block row a in Ke
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int jl = lane / LPC, r0 = (lane - LPC * (lane / LPC)) * RPL;
    const RowWalk rw = row_walk(AW_WAVES);
    for (int64_t k = rw.k, i; (i = rw.row(k)) < N; k += rw.step) {
        const int lo = rowptr[i], len = rowptr[i + 1] - lo;
        const int t0 = inc_ptr[i], C = inc_ptr[i + 1] - t0;
        for (int j0 = 0; j0 < len; j0 += JG) {
            const int nj = min(JG, len - j0);
            const bool owner = jl < nj;
            int myj = -1;
            int64_t Ei = 0;
            double acc[RPL][BS];
            if (owner) {
                myj = colidx[lo + j0 + jl];
                if constexpr (CSRW) {
#pragma unroll
                    for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                        for (int c = 0; c < BS; ++c) acc[rr][c] = 0.0;
                } else {
                    Ei = csr2sell[lo + j0 + jl];
#pragma unroll
                    for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                        for (int c = 0; c < BS; ++c)
                            acc[rr][c] = vals[BS == 1 ? Ei : sell_val(Ei, BS * BS, (r0 + rr) * BS + c)];
                }
            }
            for (int k0 = 0; k0 < C; k0 += 64) {
                const int nk = min(64, C - k0);
                if (j0 == 0 || C > 64) {   // one chunk: staged once per row, reused by every column group
                    __builtin_amdgcn_wave_barrier();
                    if (lane < nk) {
                        const int ea = inc[t0 + k0 + lane];
                        const int e = ea / NPE;
                        krow_s[wid][lane] = (int64_t)e * D * D + (int64_t)((ea - e * NPE) * BS) * D;
                    }
                    for (int q = lane; q < nk * NPE; q += 64) {
                        const int k = q / NPE;
                        const int e = inc[t0 + k0 + k] / NPE;
                        node_s[wid][q] = (int)conn[(int64_t)e * NPE + (q - k * NPE)];
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                if (owner) {
                    for (int kk = 0; kk < nk; kk += KU) {
                        unsigned m[KU];
                        double v[KU][RPL][BS];
#pragma unroll
                        for (int u = 0; u < KU; ++u) {
                            const int k = min(kk + u, nk - 1);
                            unsigned mm = 0;
#pragma unroll
                            for (int b = 0; b < NPE; ++b) mm |= (unsigned)(node_s[wid][k * NPE + b] == myj) << b;
                            m[u] = (kk + u < nk) ? mm : 0u;
                            const double* p =
                                Ke + krow_s[wid][k] + (int64_t)r0 * D + (m[u] ? __builtin_ctz(m[u]) : 0) * BS;
#pragma unroll
                            for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                                for (int c = 0; c < BS; ++c) v[u][rr][c] = m[u] ? p[rr * D + c] : 0.0;
                        }
#pragma unroll
                        for (int u = 0; u < KU; ++u) {
                            if (!m[u]) continue;
#pragma unroll
                            for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                                for (int c = 0; c < BS; ++c) acc[rr][c] += v[u][rr][c];
                            unsigned rest = m[u] & (m[u] - 1);
                            while (rest) {   // the same node twice in one element
                                const double* p =
                                    Ke + krow_s[wid][kk + u] + (int64_t)r0 * D + __builtin_ctz(rest) * BS;
#pragma unroll
                                for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                                    for (int c = 0; c < BS; ++c) acc[rr][c] += p[rr * D + c];
                                rest &= rest - 1;
                            }
                        }
                    }
                }
            }
            if (owner) {
#pragma unroll
                for (int rr = 0; rr < RPL; ++rr)
#pragma unroll
                    for (int c = 0; c < BS; ++c) {
                        if constexpr (CSRW)
                            vals[(int64_t)(lo + j0 + jl) * BS * BS + (r0 + rr) * BS + c] = acc[rr][c];
                        else
                            vals[BS == 1 ? Ei : sell_val(Ei, BS * BS, (r0 + rr) * BS + c)] = acc[rr][c];
                    }
            }
        }
    }
}

// Element-row form of the bs = 3 block-CSR row sums (default for fem_assemble_from_ke): wave per row, and per
// incident element the wave loads that element's whole block row a of K_e -- 3 D contiguous doubles (rows 3a..3a+2
// of the row-major K_e), one coalesced segment, lane = value -- as soon as the incidence entry is known (no wait for
// the element's nodes); lanes (u, b) meanwhile look up the slot of node b of incidence u in the row's sorted column
// list (LDS binary search), and the values are added into LDS accumulators [slot][r][c] one incidence after the
// other. Every slot therefore sums its contributions in ascending (incidence, b) order from +0.0, exactly as
// k_assemble_ke_w<..., CSRW>: the row sums are bit-identical. Columns are taken KR_LMAX at a time (wider rows: one
// more pass over the incidences per window); an element listing one node twice adds its b's in ascending order.
// SELLW: the row sums go straight into the SELL planes of a fresh matrix (stored, the row's padding entries zeroed;
// 8-byte stores whose 16 rows per 128-byte line are written by the workgroups of one XCD at about the same time),
// instead of the block-CSR buffer + k_csr_add_sell pass (FEM355_KE_SELLW A/B).
constexpr int KR_LMAX = 64;

// per-lane constants of the element-row form: for the lane's NL loaded values, element node b of the value's column
// and the offset r*3 + c inside the 3x3 block
template <int NPE>
struct KeRowLane {
    static constexpr int BS = 3, D = NPE * BS, RV = BS * D, NL = (RV + 63) / 64, KU = 64 / NPE;
    int vb[NL], vo[NL];
    bool vv[NL];
    __device__ __forceinline__ explicit KeRowLane(int lane) {
#pragma unroll
        for (int m = 0; m < NL; ++m) {
            const int idx = lane + 64 * m;
            vv[m] = idx < RV;
            const int r = idx / D, col = idx - D * (idx / D);
            vb[m] = col / BS;
            vo[m] = r * BS + (col - BS * (col / BS));
        }
    }
};

// One wave, one row i, one column window [j0, j0 + nj) of it (cs = those columns, staged by the caller): acc[slot *
// 9 + r * 3 + c] += the row's K_e block rows over its incidences in ascending (incidence, b) order (acc zeroed by the
// caller). Scratch: slot_s / koff_s / eid_s [64] of this wave.
// PK: Ke holds the packed upper blocks (ke_sym_stride(NPE) doubles per element): block (a, b) of the row's element
// node a is read from block ke_sym_blk(a, b) for a <= b and as the transpose of block ke_sym_blk(b, a) otherwise --
// the same values in the same (incidence, b) order, so the sums equal the full-K_e sums whenever the full K_e's lower
// blocks are the transposes of its upper ones (c3d10: mirrored by k_iso_ke, bit-identical)
// An element listing one node twice, seen by the lanes (u, b) = u NPE + b holding node b of incidence u: 1 in the lane
// when one of the lanes (u, b2 < b) holds the same node. Cross-lane reads of the nodes the lanes already hold (NPE - 1
// independent ds_bpermute, the whole wave active) instead of reloading the element's first b nodes from memory one
// after the other (a loop of up to NPE - 1 dependent global loads per incidence pass). Lanes without an incidence
// pass a distinct negative node (-1 - lane): never a match. FEM_KE_DUPLOAD = 1: the reload loop (A/B).
#ifndef FEM_KE_DUPLOAD
#define FEM_KE_DUPLOAD 0
#endif
// ke_row3 (bs = 3) takes the cross-lane check from 8 nodes per element on: c3d6's stiffness measured slower with it
// (0.83 vs 0.66 ms; c3d10 1.87 vs 2.19, c3d8 1.67 vs 1.69; profiles/r06zg_dup_check_ab.txt); ke_row1 for every NPE
// FEM_KE_ATOM1 = 1 (default): ke_row1's adds as LDS atomics (ds_add_f64, no return) -- one incidence per step, so the
// lanes of a step hit distinct slots, and a wave's LDS operations complete in issue order: the same sums, bit for bit.
// bs = 1 stored-matrix assembly 2-4 % faster (profiles/r06zg_dup_check_ab.txt); 0: read-modify-write
#ifndef FEM_KE_ATOM1
#define FEM_KE_ATOM1 1
#endif
// FEM_KE_PIPE1 = 1 (A/B): ke_row1's passes software-pipelined (loads one / two passes ahead); 0 (default): one pass at a time
#ifndef FEM_KE_PIPE1
#define FEM_KE_PIPE1 0
#endif
template <int NPE>
constexpr bool ke_dup_shfl3() { return !FEM_KE_DUPLOAD && NPE >= 8; }
template <int NPE>
__device__ __forceinline__ int ke_dup_in_incidence(int node, int b, int lane) {
    int dup = 0;
#pragma unroll
    for (int d = 1; d < NPE; ++d) {
        const int o = __shfl(node, lane >= d ? lane - d : lane, 64);
        dup |= (b >= d && o == node) ? 1 : 0;
    }
    return dup;
}

// FEM_KE_ATOM = 1 (A/B; measured no faster, profiles/r06ze_ke_atom_fused_ab.txt): each add is one LDS add (ds_add_f64, no return) instead of a read, a wait and a write --
// the lanes of one step hit distinct accumulators (distinct (b, r, c); distinct slots per b, or one b per step in the
// repeated-node branch) and a wave's LDS operations complete in issue order, so every accumulator still sums in
// ascending (incidence, b) order, bit for bit; 0 (default): the read-modify-write form
#ifndef FEM_KE_ATOM
#define FEM_KE_ATOM 0
#endif
__device__ __forceinline__ void ke_lds_add(double* p, double v) {
#if FEM_KE_ATOM
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
    *p += v;
#endif
}

// MS: also the scalar element matrices Me [M, NPE, NPE] (e.g. the consistent-mass factor M_s of M = M_s (x) I3) of the
// same elements, into accm[slot]: the lane holding value (r, c) = (0, 0) of column b (lane 3 b of the first value
// group) adds Me's (a, b) in the same step as its K value -- per slot ascending (incidence, b) from the caller's start
// value, the order of ke_row1 (bit-identical to k_assemble_ke_tile1), with no column search of its own
template <int NPE, bool PK = false, bool MS = false>
__device__ __forceinline__ void ke_row3(const KeRowLane<NPE>& L, const double* __restrict__ Ke,
                                        const int64_t* __restrict__ conn, const int32_t* __restrict__ inc, int t0,
                                        int C, const int* cs, int nj, double* acc, int* slot_s, int64_t* koff_s,
                                        int* eid_s, int lane, const double* __restrict__ Me = nullptr,
                                        double* accm = nullptr) {
    constexpr int B2 = 9, D = KeRowLane<NPE>::D, RV = KeRowLane<NPE>::RV, NL = KeRowLane<NPE>::NL;
    constexpr int KU = KeRowLane<NPE>::KU;
    constexpr int PKS = ke_sym_stride(NPE);
    int vt[NL];   // PK: offset of the value inside the transposed block (c * 3 + r for vo = r * 3 + c)
#pragma unroll
    for (int m = 0; m < NL; ++m) vt[m] = (L.vo[m] % 3) * 3 + L.vo[m] / 3;
    static_assert(!MS || !PK, "ke_row3: the fused scalar matrix takes the full K_e");
    const bool mlane = MS && L.vv[0] && L.vo[0] == 0;   // value (0, 0) of column L.vb[0] in group 0 (lane 3 b)
    for (int k0 = 0; k0 < C; k0 += 64) {
        const int nk = min(64, C - k0);
        __builtin_amdgcn_wave_barrier();
        if (lane < nk) {
            const int ea = inc[t0 + k0 + lane];
            const int e = ea / NPE;
            // PK: the element's packed base, times 16, plus its node a (< 16)
            koff_s[lane] = PK ? (int64_t)e * PKS * 16 + (ea - e * NPE)
                              : (int64_t)e * D * D + (int64_t)(ea - e * NPE) * RV;
            eid_s[lane] = e;
        }
        __builtin_amdgcn_wave_barrier();
        for (int kb = 0; kb < nk; kb += KU) {
            const int nu = min(KU, nk - kb);
            double v[KU][NL];
            double mv[MS ? KU : 1];
#pragma unroll
            for (int u = 0; u < KU; ++u) {
                const int64_t ko = koff_s[kb + (u < nu ? u : 0)];
                if constexpr (PK) {
                    const int a = (int)(ko & 15);
                    const int64_t base = ko >> 4;
#pragma unroll
                    for (int m = 0; m < NL; ++m) {
                        const int b = L.vb[m];
                        const int off = a <= b ? ke_sym_blk(NPE, a, b) * 9 + L.vo[m] : ke_sym_blk(NPE, b, a) * 9 + vt[m];
                        v[u][m] = (u < nu && L.vv[m]) ? Ke[base + off] : 0.0;
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < NL; ++m) v[u][m] = (u < nu && L.vv[m]) ? Ke[ko + lane + 64 * m] : 0.0;
                }
                if constexpr (MS) {   // Me row a of the incidence's element, value b = lane / 3 (lanes 3 b)
                    const int e = eid_s[kb + (u < nu ? u : 0)];
                    const int a = (int)((ko - (int64_t)e * D * D) / RV);
                    mv[u] = (u < nu && mlane) ? Me[((int64_t)e * NPE + a) * NPE + lane / 3] : 0.0;
                }
            }
            int dup = 0;
            int node = -1 - lane;
            if (lane < nu * NPE) {   // slot of node b of incidence u in this column window (-1: outside)
                const int u = lane / NPE, b = lane - NPE * (lane / NPE);
                const int64_t eb = (int64_t)eid_s[kb + u] * NPE;
                node = (int)conn[eb + b];
                int l = 0, h = nj;
                while (l < h) {
                    const int mid = (l + h) >> 1;
                    if (cs[mid] < node) l = mid + 1;
                    else h = mid;
                }
                slot_s[lane] = (l < nj && cs[l] == node) ? l : -1;
                if constexpr (!ke_dup_shfl3<NPE>())
                    for (int b2 = 0; b2 < b; ++b2) dup |= (int)conn[eb + b2] == node;
            }
            if constexpr (ke_dup_shfl3<NPE>()) dup = ke_dup_in_incidence<NPE>(node, lane - NPE * (lane / NPE), lane);
            __builtin_amdgcn_wave_barrier();
            if (!__any(dup)) {
#pragma unroll
                for (int u = 0; u < KU; ++u) {
                    if (u >= nu) break;
#pragma unroll
                    for (int m = 0; m < NL; ++m) {
                        if (!L.vv[m]) continue;
                        const int s = slot_s[u * NPE + L.vb[m]];
                        if (s >= 0) ke_lds_add(&acc[s * B2 + L.vo[m]], v[u][m]);
                        if constexpr (MS)
                            if (m == 0 && mlane && s >= 0) ke_lds_add(&accm[s], mv[u]);
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            } else {   // an element lists a node twice: its b's one after the other
                for (int u = 0; u < nu; ++u)
                    for (int bb = 0; bb < NPE; ++bb) {
#pragma unroll
                        for (int m = 0; m < NL; ++m) {
                            if (!L.vv[m] || L.vb[m] != bb) continue;
                            const int s = slot_s[u * NPE + bb];
                            if (s >= 0) ke_lds_add(&acc[s * B2 + L.vo[m]], v[u][m]);
                            if constexpr (MS)
                                if (m == 0 && mlane && s >= 0) ke_lds_add(&accm[s], mv[u]);
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <int NPE, bool SELLW = false>
__global__ void __launch_bounds__(256) k_assemble_ke_rows3(const double* __restrict__ Ke, const int64_t* __restrict__ conn,
                                                           const int32_t* __restrict__ inc_ptr,
                                                           const int32_t* __restrict__ inc, int64_t N,
                                                           const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ colidx, double* __restrict__ out,
                                                           const int64_t* __restrict__ slice_ptr = nullptr) {
    constexpr int B2 = 9;
    __shared__ int cols_s[AW_WAVES][KR_LMAX];
    __shared__ double acc_s[AW_WAVES][KR_LMAX * B2];
    __shared__ int slot_s[AW_WAVES][64];
    __shared__ int64_t koff_s[AW_WAVES][64];
    __shared__ int eid_s[AW_WAVES][64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const KeRowLane<NPE> L(lane);
    int* cs = cols_s[wid];
    double* acc = acc_s[wid];
    const RowWalk rw = row_walk(AW_WAVES);
    for (int64_t kk = rw.k, i; (i = rw.row(kk)) < N; kk += rw.step) {
        const int lo = rowptr[i], len = rowptr[i + 1] - lo;
        const int t0 = inc_ptr[i], C = inc_ptr[i + 1] - t0;
        for (int j0 = 0; j0 < len; j0 += KR_LMAX) {
            const int nj = min(KR_LMAX, len - j0);
            __builtin_amdgcn_wave_barrier();
            if (lane < nj) cs[lane] = colidx[lo + j0 + lane];
            for (int t = lane; t < nj * B2; t += 64) acc[t] = 0.0;
            ke_row3<NPE>(L, Ke, conn, inc, t0, C, cs, nj, acc, slot_s[wid], koff_s[wid], eid_s[wid], lane);
            if constexpr (SELLW) {
                const int64_t p0 = slice_ptr[i >> 6];
                double* o = out + B2 * p0 + (i & 63);
                for (int t = lane; t < nj * B2; t += 64) {
                    const int sl = t / B2, rc = t - B2 * (t / B2);
                    o[(int64_t)64 * (B2 * (j0 + sl) + rc)] = acc[t];
                }
            } else {
                double* o = out + (int64_t)(lo + j0) * B2;
                for (int t = lane; t < nj * B2; t += 64) o[t] = acc[t];
            }
        }
        if constexpr (SELLW) {   // the row's padding entries of its slice
            const int64_t p0 = slice_ptr[i >> 6];
            const int w = (int)((slice_ptr[(i >> 6) + 1] - p0) >> 6);
            double* o = out + B2 * p0 + (i & 63);
            for (int t = len * B2 + lane; t < w * B2; t += 64) o[(int64_t)64 * t] = 0.0;
        }
    }
}

// Tile form (default for fem_assemble_from_ke_ex2, bs = 3): R consecutive rows of one SELL slice per workgroup, a
// wave per row running the element-row sums above (the same additions in the same order: bit-identical), the R
// rows' sums of a column window kept in LDS together ([R][Wc * 9 + 1], Wc = min(widest slice, 64) columns: dynamic
// LDS sized to the pattern), then written straight into the SELL planes -- per (entry, block value) R contiguous
// doubles (R = 16: one whole 128-byte line) -- padding entries and lanes past the last row zeroed in store mode.
// No block-CSR buffer, no k_csr_add_sell pass (c3d10: 1.85 GB written once instead of written, read and written).
// Tiles of a slice run on one XCD, so its lines are completed in one L2.
// MS: the same pass also assembles the scalar element matrices Me of the same elements into the plain bs = 1 SELL
// values mvals of the same pattern (the mass factor beside the stiffness: one column search, one incidence walk, one
// launch), their window sums in LDS after the K sums ([R][Wc + 1]) and written out like k_assemble_ke_tile1's
// (bit-identical to it, store or add)
template <int NPE, int R, bool STORE, bool LA = false, bool PK = false, bool MS = false>
__global__ void __launch_bounds__(R * 64) k_assemble_ke_tile3(const double* __restrict__ Ke,
                                                               const int64_t* __restrict__ conn,
                                                               const int32_t* __restrict__ inc_ptr,
                                                               const int32_t* __restrict__ inc, int64_t N,
                                                               const int32_t* __restrict__ rowptr,
                                                               const int32_t* __restrict__ colidx,
                                                               const int64_t* __restrict__ slice_ptr,
                                                               double* __restrict__ vals, int Wc, int64_t ntiles,
                                                               const double* __restrict__ Me = nullptr,
                                                               double* __restrict__ mvals = nullptr) {
    constexpr int B2 = 9;
    extern __shared__ double tacc[];          // [R][Wc * 9 + 1] (MS: then [R][Wc + 1])
    __shared__ int cols_s[R][KR_LMAX];
    __shared__ int slot_s[R][64];
    __shared__ int64_t koff_s[R][64];
    __shared__ int eid_s[R][64];
    __shared__ int len_s[R];
    // slice s on XCD s % 8 (its R-row tiles consecutive there: a slice's plane lines complete in one L2), slices
    // interleaved over the XCDs (heavy rows numbered together, e.g. c3d10 corner nodes, spread over all of them)
    constexpr int T = 64 / R;
    const int64_t kx = blockIdx.x / NXCD;
    const int64_t tile = ((kx / T) * NXCD + blockIdx.x % NXCD) * T + kx % T;
    if (tile >= ntiles) return;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r0 = tile * R, i = r0 + wid;
    const int64_t p0 = slice_ptr[r0 >> 6];
    const int W = (int)((slice_ptr[(r0 >> 6) + 1] - p0) >> 6);
    const int l0 = (int)(r0 & 63);
    const int rs = Wc * B2 + 1;              // row stride (odd: the write-out's R rows fall into different banks)
    const KeRowLane<NPE> L(lane);
    int lo = 0, len = 0, t0 = 0, C = 0;
    if (i < N) {
        lo = rowptr[i];
        len = rowptr[i + 1] - lo;
        t0 = inc_ptr[i];
        C = inc_ptr[i + 1] - t0;
    }
    if (lane == 0) len_s[wid] = len;
    double* acc = tacc + wid * rs;
    const int rsm = Wc + 1;
    double* taccm = tacc + R * rs;             // MS
    double* accm = taccm + wid * rsm;
    for (int j0 = 0; j0 < W; j0 += Wc) {
        const int nw = min(Wc, W - j0);              // entries of this window (slice-wide)
        const int nj = max(0, min(Wc, len - j0));    // of them real columns of this row
        __syncthreads();                             // the previous window written out
        if (lane < nj) cols_s[wid][lane] = colidx[lo + j0 + lane];
        for (int t = lane; t < nw * B2; t += 64) acc[t] = 0.0;
        if constexpr (MS)   // adding: the mass sums start from the stored values (k_assemble_ke_tile1's order)
            for (int t = lane; t < nw; t += 64)
                accm[t] = (!STORE && t < nj) ? mvals[p0 + (int64_t)64 * (j0 + t) + l0 + wid] : 0.0;
        __builtin_amdgcn_wave_barrier();
        if (nj > 0) ke_row3<NPE, PK, MS>(L, Ke, conn, inc, t0, C, cols_s[wid], nj, acc, slot_s[wid], koff_s[wid],
                                         eid_s[wid], lane, Me, accm);
        __syncthreads();
        if constexpr (MS) {
            for (int q = threadIdx.x; q < nw * R; q += R * 64) {
                const int r = q % R, k = q / R;
                const double v = taccm[r * rsm + k];
                double* d = mvals + p0 + (int64_t)64 * (j0 + k) + l0 + r;
                if (STORE || j0 + k < len_s[r]) *d = v;   // adding: padding stays as stored
            }
        }
        double* dst = vals + B2 * p0 + (int64_t)64 * B2 * j0 + l0;
        for (int q = threadIdx.x; q < nw * B2 * R; q += R * 64) {
            const int r = q % R, pl = q / R, k = pl / B2, rc = pl - B2 * (pl / B2);
            const double v = tacc[r * rs + k * B2 + rc];
            // LA: the plane-paired layout A (the solver layout of bs = 3), else the plain planes
            double* d = LA ? vals + sell_val_a(p0 + (int64_t)64 * (j0 + k) + l0 + r, rc)
                           : dst + (int64_t)64 * (k * B2 + rc) + r;
            if constexpr (STORE) *d = v;                          // padding / missing rows: zero sums
            else if (j0 + k < len_s[r]) *d += v;                  // adding: padding stays as stored
        }
    }
}

// bs = 1 stored-K_e rows (scalar systems from stored element matrices, e.g. the consistent-mass factor M_s of
// M = M_s (x) I3): per incidence of the row the element's row a of K_e (NPE contiguous doubles), lanes (incidence u,
// element node b) for 64 / NPE incidences at once; every slot sums in ascending (incidence, b) order from +0.0, the
// order of k_assemble_ke_w<1, NPE> (bit-identical). acc: the window's nj sums in LDS (zeroed by the caller).
template <int NPE>
__device__ __forceinline__ void ke_row1(const double* __restrict__ Ke, const int64_t* __restrict__ conn,
                                        const int32_t* __restrict__ inc, int t0, int C, const int* cs, int nj,
                                        double* acc, int lane) {
    constexpr int KU = 64 / NPE;
    const int u = lane / NPE, b = lane - NPE * (lane / NPE);
#if FEM_KE_PIPE1
    // software pipeline over the row's passes of KU incidences: the incidence entries two passes ahead and the node
    // ids / values one pass ahead are in flight while a pass searches and adds. Every load is unconditional (indices
    // clamped into the row; validity kept apart), so the waits stay partial; the same adds in the same order
    if (C <= 0) return;
    const auto ld_inc = [&](int kk) { return inc[t0 + min(kk + u, C - 1)]; };
    int eaB = ld_inc(0);
    int eaC = ld_inc(KU);
    int nodeB, nodeC = 0;
    double vB, vC = 0.0;
    {
        const int e = eaB / NPE;
        nodeB = (int)conn[(int64_t)e * NPE + b];
        vB = Ke[(int64_t)e * NPE * NPE + (eaB - e * NPE) * NPE + b];
    }
    for (int k0 = 0; k0 < C; k0 += KU) {
        const int nu = min(KU, C - k0);
        const int eaD = ld_inc(k0 + 2 * KU);
        {
            const int e = eaC / NPE;
            nodeC = (int)conn[(int64_t)e * NPE + b];
            vC = Ke[(int64_t)e * NPE * NPE + (eaC - e * NPE) * NPE + b];
        }
        const bool on = u < nu;
        const int node = on ? nodeB : -1 - lane;
        const double v = vB;
        int s = -1;
        if (on) {
            int l = 0, h = nj;
            while (l < h) {
                const int mid = (l + h) >> 1;
                if (cs[mid] < node) l = mid + 1;
                else h = mid;
            }
            s = (l < nj && cs[l] == node) ? l : -1;
        }
        const int dup = ke_dup_in_incidence<NPE>(node, b, lane);
        __builtin_amdgcn_wave_barrier();
        if (!__any(dup)) {
            for (int uu = 0; uu < nu; ++uu) {   // one incidence at a time: its NPE slots are distinct
#if FEM_KE_ATOM1
                if (u == uu && s >= 0) __hip_atomic_fetch_add(&acc[s], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
                if (u == uu && s >= 0) acc[s] += v;
#endif
                __builtin_amdgcn_wave_barrier();
            }
        } else {   // an element lists a node twice: its b's one after the other
            for (int uu = 0; uu < nu; ++uu)
                for (int bb = 0; bb < NPE; ++bb) {
                    if (u == uu && b == bb && s >= 0) acc[s] += v;
                    __builtin_amdgcn_wave_barrier();
                }
        }
        eaC = eaD;
        nodeB = nodeC;
        vB = vC;
    }
    __builtin_amdgcn_wave_barrier();
    return;
#endif
    for (int k0 = 0; k0 < C; k0 += KU) {
        const int nu = min(KU, C - k0);
        double v = 0.0;
        int s = -1, dup = 0, node = -1 - lane;
        if (u < nu) {
            const int ea = inc[t0 + k0 + u];
            const int e = ea / NPE;
            const int64_t eb = (int64_t)e * NPE;
            node = (int)conn[eb + b];   // (issued before the value: the search waits for it alone)
            v = Ke[(int64_t)e * NPE * NPE + (ea - e * NPE) * NPE + b];
            int l = 0, h = nj;
            while (l < h) {
                const int mid = (l + h) >> 1;
                if (cs[mid] < node) l = mid + 1;
                else h = mid;
            }
            s = (l < nj && cs[l] == node) ? l : -1;
#if FEM_KE_DUPLOAD
            for (int b2 = 0; b2 < b; ++b2) dup |= (int)conn[eb + b2] == node;
#endif
        }
#if !FEM_KE_DUPLOAD
        dup = ke_dup_in_incidence<NPE>(node, b, lane);
#endif
        __builtin_amdgcn_wave_barrier();
        if (!__any(dup)) {
            for (int uu = 0; uu < nu; ++uu) {   // one incidence at a time: its NPE slots are distinct
#if FEM_KE_ATOM1
                if (u == uu && s >= 0) __hip_atomic_fetch_add(&acc[s], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
                if (u == uu && s >= 0) acc[s] += v;
#endif
                __builtin_amdgcn_wave_barrier();
            }
        } else {   // an element lists a node twice: its b's one after the other
            for (int uu = 0; uu < nu; ++uu)
                for (int bb = 0; bb < NPE; ++bb) {
                    if (u == uu && b == bb && s >= 0) acc[s] += v;
                    __builtin_amdgcn_wave_barrier();
                }
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Tile form of the bs = 1 stored-K_e assembly: k_assemble_ke_tile3's geometry with one value per entry -- R rows of a
// slice per workgroup, a wave per row (ke_row1), the window's sums in LDS, then written straight into the SELL values
// (R contiguous doubles per entry), padding entries and lanes past the last row zeroed in store mode. No csr2sell, no
// memset, no read of the old values when storing; adding reads each value once and sums onto it in k_assemble_ke_w's
// order.
template <int NPE, int R, bool STORE>
__global__ void __launch_bounds__(R * 64) k_assemble_ke_tile1(const double* __restrict__ Ke,
                                                               const int64_t* __restrict__ conn,
                                                               const int32_t* __restrict__ inc_ptr,
                                                               const int32_t* __restrict__ inc, int64_t N,
                                                               const int32_t* __restrict__ rowptr,
                                                               const int32_t* __restrict__ colidx,
                                                               const int64_t* __restrict__ slice_ptr,
                                                               double* __restrict__ vals, int Wc, int64_t ntiles) {
    extern __shared__ double tacc1[];         // [R][Wc + 1]
    __shared__ int cols_s[R][KR_LMAX];
    __shared__ int len_s[R];
    constexpr int T = 64 / R;
    const int64_t kx = blockIdx.x / NXCD;
    const int64_t tile = ((kx / T) * NXCD + blockIdx.x % NXCD) * T + kx % T;
    if (tile >= ntiles) return;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r0 = tile * R, i = r0 + wid;
    const int64_t p0 = slice_ptr[r0 >> 6];
    const int W = (int)((slice_ptr[(r0 >> 6) + 1] - p0) >> 6);
    const int l0 = (int)(r0 & 63);
    const int rs = Wc + 1;
    int lo = 0, len = 0, t0 = 0, C = 0;
    if (i < N) {
        lo = rowptr[i];
        len = rowptr[i + 1] - lo;
        t0 = inc_ptr[i];
        C = inc_ptr[i + 1] - t0;
    }
    if (lane == 0) len_s[wid] = len;
    double* acc = tacc1 + wid * rs;
    for (int j0 = 0; j0 < W; j0 += Wc) {
        const int nw = min(Wc, W - j0);
        const int nj = max(0, min(Wc, len - j0));
        __syncthreads();   // the previous window written out
        if (lane < nj) cols_s[wid][lane] = colidx[lo + j0 + lane];
        // adding: the sums start from the stored values (k_assemble_ke_w<1>'s ((v + c_1) + c_2) ...: the same bits)
        for (int t = lane; t < nw; t += 64)
            acc[t] = (!STORE && t < nj) ? vals[p0 + (int64_t)64 * (j0 + t) + l0 + wid] : 0.0;
        __builtin_amdgcn_wave_barrier();
        if (nj > 0) ke_row1<NPE>(Ke, conn, inc, t0, C, cols_s[wid], nj, acc, lane);
        __syncthreads();
        for (int q = threadIdx.x; q < nw * R; q += R * 64) {
            const int r = q % R, k = q / R;
            const double v = tacc1[r * rs + k];
            double* d = vals + p0 + (int64_t)64 * (j0 + k) + l0 + r;
            if (STORE || j0 + k < len_s[r]) *d = v;   // adding: padding stays as stored
        }
    }
}

// zero the lanes past the last row (N % 64 .. 63) of the last slice, every entry and plane (store paths that write
// rows only)
__global__ void k_sell_tail_zero(const int64_t* __restrict__ slice_ptr, int64_t N, int B2, double* __restrict__ vals) {
    const int64_t s = (N - 1) >> 6;
    const int64_t p0 = slice_ptr[s];
    const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
    const int l0 = (int)(N & 63);
    for (int t = threadIdx.x; t < w * B2 * 64; t += blockDim.x)
        if ((t & 63) >= l0) vals[B2 * p0 + t] = 0.0;
}

// SELL planes += block-CSR row sums (k_assemble_ke_w<..., CSRW>): wave per slice, lane = row; for every (entry k,
// block value rc) the 64 rows of the slice write one contiguous 512-byte plane segment, and each lane reads its own
// row's blocks in order (row-contiguous in the block-CSR buffer). Padding entries are left untouched.
// STORE: the SELL values were never written (fresh matrix): the row sums are stored (0 + s == s bit for bit: the
// sums start from +0.0, so none is -0.0) and the padding entries zeroed -- no memset of the matrix, no read of it.
template <int BS, bool STORE = false>
__global__ void __launch_bounds__(256) k_csr_add_sell(const double* __restrict__ csr, const int32_t* __restrict__ rowptr,
                                                      int64_t N, int64_t nslices, const int64_t* __restrict__ slice_ptr,
                                                      double* __restrict__ vals) {
    constexpr int B2 = BS * BS;
    const int lane = threadIdx.x & 63;
    for (int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < nslices;
         s += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t row = s * 64 + lane;
        const int64_t p0 = slice_ptr[s];
        int len = 0, rp = 0;
        if (row < N) {
            rp = rowptr[row];
            len = rowptr[row + 1] - rp;
        }
        const double* src = csr + (int64_t)rp * B2;
        double* dst = vals + p0 * B2 + lane;
        for (int k = 0; k < len; ++k) {
            double v[B2];
#pragma unroll
            for (int rc = 0; rc < B2; ++rc) v[rc] = src[(int64_t)k * B2 + rc];
#pragma unroll
            for (int rc = 0; rc < B2; ++rc) {
                if constexpr (STORE) dst[((int64_t)k * B2 + rc) * 64] = v[rc];
                else dst[((int64_t)k * B2 + rc) * 64] += v[rc];
            }
        }
        if constexpr (STORE) {
            const int w = (int)((slice_ptr[s + 1] - p0) >> 6);
            for (int k = len; k < w; ++k)
#pragma unroll
                for (int rc = 0; rc < B2; ++rc) dst[((int64_t)k * B2 + rc) * 64] = 0.0;
        }
    }
}

// ---------------------------------------------------------------- fused c3d4 assembly (K_e never stored)
// Straight into SELL (addresses from the slice pointer, no csr2sell reads; a fresh matrix is stored whole, padding
// zeroed, without a memset), with the additions and order of the wave-per-row kernels below (k_assemble_p1w /
// k_assemble_el3w, FEM355_ASM_ROWS; bit for bit, tests/test_gpu_parity.py): the accumulator form k_asm_tet4_acc.
// (An owner form -- one thread per (row, column) output scanning the row's incidences -- measured 3.85 ms for the
// 10M elastic cube, 3.7 ms with the element blocks formed once per incidence: its owners test every (incidence,
// node) pair of the row and 3/4 of a wave's lanes idle at each, VALU-bound; the accumulator form 2.55 ms.)

// a + b never fused with the product that formed b (the row kernels store the product to LDS before adding it)
__device__ __forceinline__ double add_nc(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}

// Elastic blocks by sums (both assembly forms, bit for bit): per incident element the row node a contributes the
// products M_ab[r][c] += (V g_a[r]) g_b[c] and P_ab += (V g_a) . g_b for every element node b (V g_a formed once per
// element and row); the block is K_ab = lambda M_ab + mu M_ab^T + mu P_ab I, formed once from the sums when the
// row is written -- the element formula V (lambda g_a g_b^T + mu g_b g_a^T + mu (g_a . g_b) I) summed in another
// order (rounding-level difference; the oracle checks stay at 1e-12). Per product one multiply and one add instead
// of the element formula's eight operations per entry.
__device__ __forceinline__ double el_pdot(const double* vga, const double* gb) {
#pragma clang fp contract(off)
    return vga[0] * gb[0] + vga[1] * gb[1] + vga[2] * gb[2];
}
__device__ __forceinline__ double el_combine(const Lame& L, double m_rc, double m_cr, double p, bool diag) {
#pragma clang fp contract(off)
    double s = L.lam * m_rc + L.mu * m_cr;
    if (diag) s += L.mu * p;
    return s;
}

#ifndef FEM_ACC_POSREP
#define FEM_ACC_POSREP 0   // bs = 3: the repeated-node flag in the position fields (no a_s read; without the
                           // atomics' per-step check, FEM_ACC_ATOM, nothing reads the flag)
#endif
// the accumulator kernel's column positions are 16-bit fields (bs = 3: 15-bit beside the flag), all-ones = absent
constexpr int acc_max_cols(int bs) { return FEM_ACC_POSREP && bs == 3 ? 0x7fff : 0xffff; }

// lane L of every quad (four consecutive lanes) to all four lanes of it (DPP quad_perm, no LDS)
template <int L>
__device__ __forceinline__ double quad_bcast(double x) {
    constexpr int ctrl = L | (L << 2) | (L << 4) | (L << 6);
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ double p1_value(const double ga[3], const double gb[3], double kappa, double V) {
    const double dot = ga[0] * gb[0] + ga[1] * gb[1] + ga[2] * gb[2];
    return kappa * dot * V;
}

// position of j in the ascending cs[0, n) (0xffff: absent): branch-free halving whose step count depends on n only
// (rows of one wave share it), every read inside [0, n)
__device__ __forceinline__ uint32_t sorted_pos(const int32_t* cs, int n, int j) {
    if (n <= 0) return 0xffffu;
    int b = 0;
    for (int len = n; len > 1;) {
        const int half = len >> 1;
        b = cs[b + half] < j ? b + half : b;
        len -= half;
    }
    b += cs[b] < j;
    return (b < n && cs[b] == j) ? (uint32_t)b : 0xffffu;
}

// sorted_pos of four keys in one lockstep search (the same halving steps and result per key): the four probes of a
// step are independent LDS reads in flight together instead of four searches one after another
__device__ __forceinline__ void sorted_pos4(const int32_t* cs, int n, const int j[4], uint32_t p[4]) {
    if (n <= 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = 0xffffu;
        return;
    }
    int b[4] = {0, 0, 0, 0};
    for (int len = n; len > 1;) {
        const int half = len >> 1;
        int v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = cs[b[q] + half];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = v[q] < j[q] ? b[q] + half : b[q];
        len -= half;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        b[q] += cs[b[q]] < j[q];
        p[q] = (b[q] < n && cs[b[q]] == j[q]) ? (uint32_t)b[q] : 0xffffu;
    }
}

// zero the SELL values of slices [0, ns) (slice_ptr on the device)
__global__ void k_sell_zero(const int64_t* __restrict__ slice_ptr, int64_t ns, int bs2, double* __restrict__ vals) {
    const int64_t n = slice_ptr[ns] * bs2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        vals[i] = 0.0;
}

// Accumulator form (default): one workgroup per R rows of a slice, the rows' block values accumulated in LDS.
// Items = (row, j-th incident element of the row); per batch the j0..j0+J-1 items of every row are formed by one
// thread each (gradients, volume, the column slots of the element's nodes in the row) and staged in LDS; then
// every row is swept by its own lanes in lockstep -- lane (row, b[, rr]) takes the row's items in ascending order
// and adds element node b's contribution (block row rr) into the accumulator of b's column: within one step the
// row's lanes hit distinct columns (an element lists a node once; elements that do not are swept node by node), so
// every accumulator receives its contributions in ascending incidence order -- the sums of k_assemble_p1w /
// k_assemble_el3w bit for bit, without their owner loops (whose lanes stepped through every item to find their
// few matches). The rows' accumulators are written out whole slice columns at a time (coalesced SELL stores).
// Columns past ACC_W per row: the accumulators cover the row's columns in windows of ACC_W, one sweep per window.
// LDS strides padded (R + 1, NI + 1): a row's lanes update accumulators of different columns and read staged
// values of different element nodes at once, which power-of-two strides put into one bank (bs = 3: 5.8 -> 3.0 ms).
template <int R_, int J_, int LPR_, int W_, int SEG_, bool XP_ = false, bool XS_ = false>
struct AccCfg {
    static constexpr int R = R_, J = J_, LPR = LPR_, W = W_, SEG = SEG_;
    // XP: the next batch's vertex coordinates loaded during the current batch's sweep (a third pipeline stage, 24
    // more VGPRs: for bs = 3, whose occupancy LDS caps anyway)
    static constexpr bool XP = XP_;
    // XS: the coordinates of the tile's CSR column segment staged in LDS once (every node of an element incident to a
    // row is a column of that row, found by the item's column search anyway): no coordinate gathers per batch
    static constexpr bool XS = XS_;
};
// bs = 1: lanes (row, b), 64 rows (a slice), 4 items per row per batch, 32 accumulated columns per row (10M cube:
// 0.86 ms; 16 columns 0.79 ms but two sweeps for rows past 16 columns, 8 items per row 1.16 ms at 3 waves per SIMD).
// bs = 3: lanes (row, b, rr), 16 rows, 8 items per row per batch, 16 accumulated columns (10M cube: 2.55 ms; 16
// items per row 2.95, 12 items 2.83, 4 items 2.66 ms; with the M / P sums since round 4: 2.45 ms. The coordinates of
// the tile's columns staged in LDS instead of the per-batch prefetch (XS): 3.0 ms at 8 items per row, 2.96 / 3.37 /
// 3.12 ms at 5 / 6 / 4 -- the staging's gathers at the tile start are exposed, and 3 instead of 4 tiles per CU).
// Round 6, the sweep's LDS operations per (row, item) step cut from 13 to 6 (profiles/r06o_acc_sweep_ab.txt,
// r06r_acc_sweep_step2_ab.txt; 10M cube, bit-identical): the adds as LDS atomics (FEM_ACC_ATOM: 2277 -> 2248 us;
// P1 649 -> 641 us), the P sum from the quad's products over DPP (FEM_ACC_PDPP), g_b read once per quad
// (FEM_ACC_GDPP), and no per-step repeated-node check under the atomics: 1952 us; P1 618 us.
#ifndef FEM_P1_CFG
#define FEM_P1_CFG 64, 4, 4, 32, 1024
#endif
using AccP1 = AccCfg<FEM_P1_CFG>;
#ifndef FEM_P1W16_CFG
#define FEM_P1W16_CFG 64, 4, 4, 16, 1024
#endif
// patterns of at most 16 columns per row (10M cube: 0.67 vs 0.74 ms); with the coordinate prefetch (XP) 0.83 ms:
// 107 VGPRs, 4 instead of 6 waves per SIMD
using AccP1w16 = AccCfg<FEM_P1W16_CFG>;
#ifndef FEM_EL3_CFG
#define FEM_EL3_CFG 16, 8, 16, 16, 256, true, false
#endif
using AccEl = AccCfg<FEM_EL3_CFG>;

// SL: the values go into the solver layout -- bs = 1 (whole-slice tiles): lane-paired entries of the pattern's
// k_sell_sl_pattern, and in a slice-uniform slice (uoff[s] >= 0) the accumulators are indexed by the slice's delta
// list (the column search looks up node - row in it), so a row's missing offsets hold zeros there; bs = 3: the
// plane-paired layout A (sell_val_a). The same additions in the same order as the plain layout: only positions differ.
template <int BS, class Cfg, bool STORE, bool SL = false>
__global__ void __launch_bounds__(256) k_asm_tet4_acc(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                      double E, double nu, const int32_t* __restrict__ inc_ptr,
                                                      const int32_t* __restrict__ inc, int64_t N,
                                                      const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ colidx,
                                                      const int64_t* __restrict__ slice_ptr,
                                                      double* __restrict__ vals, int64_t* __restrict__ bad,
                                                      int64_t ntiles, const int32_t* __restrict__ uoff = nullptr,
                                                      const int16_t* __restrict__ ucol = nullptr) {
    static_assert(!SL || BS == 3 || Cfg::R == 64, "solver layout, bs = 1: one slice per tile");
    constexpr int R = Cfg::R, J = Cfg::J, LPR = Cfg::LPR, AW = Cfg::W, SEG = Cfg::SEG;
    constexpr int B2 = BS * BS;
    constexpr int NI = R * J;
    constexpr int NT = R * LPR;                        // threads of the workgroup
    constexpr int RPL = (BS == 3 && LPR == 4) ? 3 : 1;   // block rows per sweep lane (bs = 3: lanes (row, b) or
                                                         // (row, b, rr))
    constexpr int ND = BS == 1 ? 4 : 15;                // staged per item: P1 values / (V g_a, g_0 .. g_3)
    constexpr int AV = BS == 1 ? 1 : 10;                // accumulated per column: the value / M (9) and P
    static_assert(NI <= NT, "one item per thread per batch");
    static_assert(64 % R == 0 && NT <= 256 && NT % 64 == 0 && 64 % LPR == 0, "tile geometry");
    static_assert(BS == 1 || LPR == 4 || LPR == 16, "bs = 3 lanes: (row, b) or (row, b, rr)");
    static_assert(!(Cfg::XP && Cfg::XS), "coordinates either prefetched per batch or staged per tile");
    __shared__ int ip_s[R + 1];
    __shared__ int rp_s[R + 1];
    __shared__ int col_s[SEG];
    // FEM_ASM_HASH (bs = 1, slice-uniform tiles): the slice's delta list also in a 64-slot open-addressing table
    // (delta -> list position), so an element node's column is one LDS read (rarely two) instead of a binary search
    // whose reads depend on each other. A timing build without any column search (FEM_ASM_NOSEARCH, wrong values)
    // ran the 10M P1 value kernel in 544 instead of 724 us.
#ifndef FEM_ASM_HASH
#define FEM_ASM_HASH 1
#endif
#ifndef FEM_ASM_NOSEARCH
#define FEM_ASM_NOSEARCH 0
#endif
#ifndef FEM_ASM_SEARCH4
#define FEM_ASM_SEARCH4 1   // the other tiles: the four binary searches of an item in lockstep (sorted_pos4)
#endif
    constexpr bool HT = FEM_ASM_HASH && SL && BS == 1;
    // FEM_ASM_HASH3 (bs = 3): the tile's longest row (the first of them) is the reference; its deltas (column - row)
    // go into the same 64-slot table, and every row whose deltas equal them (all of a Kuhn cube's interior tiles)
    // looks its element nodes' positions up there -- the same positions as the binary search, one LDS read each
    // instead of ~5 dependent ones. Other rows keep the lockstep search.
#ifndef FEM_ASM_HASH3
#define FEM_ASM_HASH3 0   // measured slower (profiles/r06u_acc_negative_ab.txt): off
#endif
    constexpr bool HT3 = FEM_ASM_HASH3 && BS == 3;
    constexpr int HTN = 64;
    __shared__ int2 ht_s[(HT || HT3) ? HTN : 1];
    __shared__ int hrow_s[HT3 ? R : 1];   // HT3: row r's deltas are the reference row's
    __shared__ double xs_s[Cfg::XS ? SEG : 1][3];
    // padded strides: the sweep's lanes of one row read dat_s rows of different element nodes and update
    // accumulators of different columns -- with power-of-two strides those all fall into one LDS bank
    __shared__ double dat_s[ND][NI + 1];
    __shared__ uint2 pos_s[NI];
    __shared__ uint8_t a_s[NI];             // local index of the row's node; bit 7: the element repeats a node
    // accumulators of (column slot i = k AV + value, row r): [i][r] with a padded row stride (default), or
    // FEM_ACC_T = 1 (bs = 3, A/B): [r][i] with row stride AW AV + FEM_ACC_PAD -- the sweep's 16 lanes of one row then
    // hit consecutive slots of their columns, the 4 rows of a wave offset by the padded stride
#ifndef FEM_ACC_T
#define FEM_ACC_T 0
#endif
#ifndef FEM_ACC_PAD
#define FEM_ACC_PAD 1
#endif
    // bs = 3: positions of 15 bits, the repeated-node flag in bit 15 of every field (no a_s read in the sweep)
    constexpr bool POSREP = FEM_ACC_POSREP && BS == 3;
#ifndef FEM_ACC_PROBE
#define FEM_ACC_PROBE 0   // timing builds (wrong values): 1 no gradients, 2 no sweep, with FEM_ASM_NOSEARCH no search
#endif
#ifndef FEM_ACC_PF2
#define FEM_ACC_PF2 0   // loads a whole phase ahead (measured slower, profiles/r06u_acc_negative_ab.txt)
#endif
#ifndef FEM_ACC_ATOM
#define FEM_ACC_ATOM 1   // sweep adds as LDS atomics
#endif
#ifndef FEM_ACC_GDPP
#define FEM_ACC_GDPP 1   // bs = 3 (with PDPP): g_b read once per quad and shared over DPP
#endif
#ifndef FEM_ACC_PDPP
#define FEM_ACC_PDPP 1   // bs = 3: the P sum from the quad's products (DPP) instead of three more LDS reads
#endif
    constexpr bool ACT = FEM_ACC_T && BS == 3;
    constexpr int ARS = ACT ? AW * AV + FEM_ACC_PAD : R + 1;   // stride of the outer index
    __shared__ double acc_flat[ACT ? R * ARS : AW * AV * ARS];
    auto ACC = [&](int i, int r) -> double& { return ACT ? acc_flat[r * ARS + i] : acc_flat[i * ARS + r]; };
    __shared__ int maxc_s;
    const int tid = threadIdx.x;
    const int64_t per = (ntiles + NXCD - 1) / NXCD;
    const int64_t tile = (int64_t)(blockIdx.x % NXCD) * per + blockIdx.x / NXCD;
    if (tile >= ntiles) return;
    const int64_t r0 = tile * R;
    const int l0 = (int)(r0 & 63);
    const int64_t e0 = slice_ptr[r0 >> 6];
    const int W = (int)((slice_ptr[(r0 >> 6) + 1] - e0) >> 6);
    if (tid == 0) maxc_s = 0;
    __syncthreads();
    if (tid <= R) {
        const int64_t r = r0 + tid < N ? r0 + tid : N;
        ip_s[tid] = inc_ptr[r];
        rp_s[tid] = rowptr[r];
        if (tid < R) {
            const int64_t r1 = r0 + tid + 1 < N ? r0 + tid + 1 : N;
            atomicMax(&maxc_s, inc_ptr[r1] - ip_s[tid]);
        }
    }
    __syncthreads();
    const int seg0 = rp_s[0], segn = rp_s[R] - seg0;
    // SL: a slice-uniform slice searches its delta list (W entries) instead of the rows' CSR columns
    const int uo = (SL && BS == 1) ? uoff[r0 >> 6] : -1;   // bs = 3: layout A, per-lane columns
    const bool staged = SL && uo >= 0 ? true : segn <= SEG;
    const bool use_ht = HT && uo >= 0 && W <= HTN / 2;
    if (SL && uo >= 0) {
        for (int q = tid; q < W; q += NT) col_s[q] = ucol[uo + q];
        if (use_ht) {   // empty the table, then every list entry claims a slot (linear probing, compare-and-swap)
            for (int q = tid; q < HTN; q += NT) ht_s[q] = make_int2(INT_MIN, 0);
            __syncthreads();
            if (tid < W) {
                const int d = ucol[uo + tid];
                unsigned h = ((unsigned)d * 2654435761u) >> 26;
                while (atomicCAS(&ht_s[h].x, INT_MIN, d) != INT_MIN) h = (h + 1) & (HTN - 1);
                ht_s[h].y = tid;
            }
        }
    } else if (staged)
        for (int q = tid; q < segn; q += NT) {
            const int cq = colidx[seg0 + q];
            col_s[q] = cq;
            if constexpr (Cfg::XS) {
                xs_s[q][0] = X[3 * (int64_t)cq];
                xs_s[q][1] = X[3 * (int64_t)cq + 1];
                xs_s[q][2] = X[3 * (int64_t)cq + 2];
            }
        }
    bool use_ht3 = false;
    if constexpr (HT3) {
        int rref = 0, lref = rp_s[1] - rp_s[0];   // (every thread: the same reference row)
        for (int r = 1; r < R; ++r) {
            const int len = rp_s[r + 1] - rp_s[r];
            if (len > lref) {
                lref = len;
                rref = r;
            }
        }
        use_ht3 = staged && lref > 0 && lref <= HTN / 2;
        if (use_ht3) {
            for (int q = tid; q < HTN; q += NT) ht_s[q] = make_int2(INT_MIN, 0);
            if (tid < R) hrow_s[tid] = (rp_s[tid + 1] - rp_s[tid]) == lref;
            __syncthreads();   // col_s staged, table empty
            const int cref = rp_s[rref] - seg0;
            const int64_t gref = r0 + rref;
            if (tid < lref) {
                const int d = (int)(col_s[cref + tid] - gref);
                unsigned h = ((unsigned)d * 2654435761u) >> 26;
                while (atomicCAS(&ht_s[h].x, INT_MIN, d) != INT_MIN) h = (h + 1) & (HTN - 1);
                ht_s[h].y = tid;
            }
            for (int q = tid; q < R * lref; q += NT) {   // a row of another delta list: back to the search
                const int r = q / lref, k = q - r * lref;
                if (hrow_s[r] && col_s[rp_s[r] - seg0 + k] - (r0 + r) != col_s[cref + k] - gref) hrow_s[r] = 0;
            }
        }
    }
    const int maxc = maxc_s;
    const Lame L = lame(E, nu);
    // phase-2 lane: row lr, element node lb, block rows lrr .. lrr + RPL - 1
    const int lr = tid / LPR, lb = (BS == 1 || LPR == 4) ? tid % LPR : (tid % LPR) / 4;
    const int lrr = (BS == 1 || LPR == 4) ? 0 : tid % 4;   // bs = 3, LPR = 16: rr = 3 is the P lane
    constexpr bool PDPP = FEM_ACC_PDPP && BS == 3 && LPR == 16;
    constexpr bool REPCHK = !FEM_ACC_ATOM;
    constexpr int ISTR = ACT ? 1 : ARS;   // accumulator stride between a column's consecutive slots
    // PDPP: the lane's first slot (block row lrr: 3 lrr, P lane: 9) and its accumulator address at column 0
    double* const abase = PDPP ? &ACC(lrr < 3 ? 3 * lrr : 9, lr) : nullptr;
    for (int c0 = 0; c0 < W; c0 += AW) {
        const int cw = min(AW, W - c0);
        __syncthreads();
        for (int q = tid; q < AW * AV * R; q += NT) {
            const int r = q % R, kc = q / R, k = kc / AV;
            double v = 0.0;   // bs = 3: the sums start from zero, stored values are added when the row is written
            if (BS == 1 && !STORE && k < cw && ((SL && uo >= 0) || c0 + k < rp_s[r + 1] - rp_s[r]))
                v = vals[SL ? e0 + pair_pos(c0 + k, W, l0 + r) : e0 + (int64_t)(c0 + k) * 64 + l0 + r];
            ACC(kc, r) = v;
        }
        // software pipeline over the batches: a thread's next incidence entry is loaded before the current batch
        // is swept and its element's node ids right after, so a batch waits only for its coordinates
        const int ir = tid / J, ij = tid - (tid / J) * J;   // this thread's item: row ir, j-th element of the batch
        int ea_n = 0;
        bool v_n = false;
        int64_t cn_n[4] = {0, 0, 0, 0};
        double xn[Cfg::XP ? 4 : 1][3];
        if (tid < NI) {
            const int t = ip_s[ir] + ij;
            v_n = t < ip_s[ir + 1];
            if (v_n) ea_n = inc[t];
        }
        if (v_n) {
#pragma unroll
            for (int b = 0; b < 4; ++b) cn_n[b] = conn[4 * (int64_t)(ea_n >> 2) + b];
            if constexpr (Cfg::XP) {
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int q = 0; q < 3; ++q) xn[b][q] = X[3 * cn_n[b] + q];
            }
        }
        // PF2 (XP): incidence entries two batches ahead, node ids one batch ahead loaded as a batch starts (under
        // its phase 1), coordinates one batch ahead as its sweep starts -- each load a whole phase before its use
        constexpr bool PF2 = FEM_ACC_PF2 && Cfg::XP;
        int ea_nn = 0;
        bool v_nn = false;
        if (PF2 && tid < NI && J < maxc) {
            const int t = ip_s[ir] + J + ij;
            v_nn = t < ip_s[ir + 1];
            if (v_nn) ea_nn = inc[t];
        }
        for (int j0 = 0; j0 < maxc; j0 += J) {
            __syncthreads();   // accumulators initialised / previous batch swept
            const bool vcur = v_n;
            const int eacur = ea_n;
            const int64_t cncur[4] = {cn_n[0], cn_n[1], cn_n[2], cn_n[3]};
            double xc[Cfg::XP ? 4 : 1][3];
            if constexpr (Cfg::XP) {
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int q = 0; q < 3; ++q) xc[b][q] = xn[b][q];
            }
            if constexpr (PF2) {
                v_n = v_nn;
                ea_n = ea_nn;
                if (v_n) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) cn_n[b] = conn[4 * (int64_t)(ea_n >> 2) + b];
                }
                v_nn = false;
                if (tid < NI && j0 + 2 * J < maxc) {
                    const int t = ip_s[ir] + j0 + 2 * J + ij;
                    v_nn = t < ip_s[ir + 1];
                    if (v_nn) ea_nn = inc[t];
                }
            } else {
                v_n = false;
                if (tid < NI && j0 + J < maxc) {
                    const int t = ip_s[ir] + j0 + J + ij;
                    v_n = t < ip_s[ir + 1];
                    if (v_n) ea_n = inc[t];
                }
            }
            {
                const int it0 = tid;
                const int r = ir;
                uint32_t pk[2] = {0xffffffffu, 0xffffffffu};
                uint8_t aflag = 0;
                if (tid < NI && vcur) {
                    const int ea = eacur;
                    const int64_t e = ea >> 2;
                    const int a = ea & 3;
                    const int64_t* c = cncur;
                    const bool ulist = SL && uo >= 0;
                    const int cl = ulist ? 0 : rp_s[r] - seg0, cn = ulist ? W : rp_s[r + 1] - rp_s[r];
                    const int kshift = ulist ? (int)(r0 + r) : 0;   // list entries are deltas node - row
                    int nodes[4];
                    uint32_t pp[4];
                    pk[0] = pk[1] = 0u;
                    // a table row: positions from the hash of the deltas node - row (hshift)
                    const bool hrow = use_ht || (HT3 && use_ht3 && hrow_s[r]);
                    const int hshift = use_ht ? kshift : (int)(r0 + r);
#if !FEM_ASM_NOSEARCH
                    int2 hfirst[4];   // HT3 table rows: the four keys' first probes, read together
                    if (HT3 && hrow && !use_ht) {
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) {
                            const int jd = (int)c[bb] - hshift;
                            hfirst[bb] = ht_s[((unsigned)jd * 2654435761u) >> 26];
                        }
                    }
                    if (!hrow && FEM_ASM_SEARCH4) {   // the four nodes' binary searches in lockstep
                        int jj4[4];
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) jj4[bb] = (int)c[bb] - kshift;
                        if (staged) sorted_pos4(col_s + cl, cn, jj4, pp);
                        else sorted_pos4(colidx + seg0 + cl, cn, jj4, pp);
                    }
#endif
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb) {
                        nodes[bb] = (int)c[bb];
                        const int j = nodes[bb] - kshift;
                        // the tile-uniform branch keeps the LDS search on ds_read (one pointer for both would
                        // make every probe a flat load)
#if FEM_ASM_NOSEARCH   // timing builds only (wrong values): no column search, a fixed in-range slot
                        pp[bb] = (uint32_t)(bb < cn ? bb : 0);
                        (void)j;
#else
                        if (HT3 && hrow && !use_ht && hfirst[bb].x == nodes[bb] - hshift) {
                            pp[bb] = (uint32_t)hfirst[bb].y;   // (the usual case: no collision on the first probe)
                        } else if (hrow) {   // deltas are unique: the first matching key, or an empty slot = absent
                            const int jd = nodes[bb] - hshift;
                            unsigned h = ((unsigned)jd * 2654435761u) >> 26;
                            uint32_t q = 0xffffu;
                            for (int probe = 0; probe < HTN; ++probe) {
                                const int2 e = ht_s[h];
                                if (e.x == jd) {
                                    q = (uint32_t)e.y;
                                    break;
                                }
                                if (e.x == INT_MIN) break;
                                h = (h + 1) & (HTN - 1);
                            }
                            pp[bb] = q;
                        } else if (!FEM_ASM_SEARCH4) {
                            pp[bb] = staged ? sorted_pos(col_s + cl, cn, j) : sorted_pos(colidx + seg0 + cl, cn, j);
                        }
#endif
                        pk[bb >> 1] |= (POSREP ? pp[bb] & 0x7fffu : pp[bb]) << (16 * (bb & 1));
                    }
                    double g[4][3];
                    double det;
                    if constexpr (Cfg::XS) {
                        if (staged) {   // every element node is a column of the row: its coordinates are in LDS
                            double xq[4][3];
#pragma unroll
                            for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                                for (int q = 0; q < 3; ++q) xq[bb][q] = xs_s[cl + (int)pp[bb]][q];
                            det = tet4_grads_p(xq, g);
                        } else {
                            det = tet4_grads_n(X, cncur, g);
                        }
                    } else if constexpr (Cfg::XP) {
#if FEM_ACC_PROBE & 1   // timing builds only (wrong values): no gradients (the coordinates stand in), det = 1
                        det = 1.0;
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                            for (int q = 0; q < 3; ++q) g[bb][q] = xc[bb][q];
#else
                        det = tet4_grads_p(xc, g);
#endif
                    } else {
                        det = tet4_grads_n(X, cncur, g);
                    }
                    if (c0 == 0 && fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
                    const double V = fabs(det) / 6.0;
                    if constexpr (BS == 1) {
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) dat_s[bb][it0] = p1_value(g[a], g[bb], E, V);
                    }
                    if constexpr (REPCHK || POSREP) {   // (nothing reads the flag otherwise)
                        const bool rep = nodes[0] == nodes[1] || nodes[0] == nodes[2] || nodes[0] == nodes[3] ||
                                         nodes[1] == nodes[2] || nodes[1] == nodes[3] || nodes[2] == nodes[3];
                        aflag = (uint8_t)(a | (rep ? 0x80 : 0));
                    }
                    if constexpr (BS == 3) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) {
                            const double gaq = a == 0 ? g[0][q] : a == 1 ? g[1][q] : a == 2 ? g[2][q] : g[3][q];
                            dat_s[q][it0] = V * gaq;
                        }
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                            for (int q = 0; q < 3; ++q) dat_s[3 + 3 * bb + q][it0] = g[bb][q];
                    }
                }
                if (tid < NI) {
                    if (POSREP && (aflag & 0x80)) {   // bit 15 of every field: the element repeats a node
                        pk[0] |= 0x80008000u;
                        pk[1] |= 0x80008000u;
                    }
                    pos_s[it0] = make_uint2(pk[0], pk[1]);
                    if constexpr (REPCHK) a_s[it0] = aflag;
                }
            }
            __syncthreads();
            if (!PF2 && v_n) {   // the next batch's element node ids (its incidence entry was loaded above)
#pragma unroll
                for (int b = 0; b < 4; ++b) cn_n[b] = conn[4 * (int64_t)(ea_n >> 2) + b];
            }
            // sweep: lanes of one row are consecutive lanes of one wave, in lockstep
#pragma unroll
            for (int jj = 0; jj < ((FEM_ACC_PROBE & 2) ? 0 : J); ++jj) {   // (probe 2: no sweep, timing only)
                if constexpr (Cfg::XP) {
                    if (jj == (PF2 ? 0 : J / 2) && v_n) {   // the next batch's coordinates, under the sweep
#pragma unroll
                        for (int b = 0; b < 4; ++b)
#pragma unroll
                            for (int q = 0; q < 3; ++q) xn[b][q] = X[3 * cn_n[b] + q];
                    }
                }
                const int it = lr * J + jj;
                const uint2 pp = pos_s[it];
                const uint32_t fld = ((lb < 2 ? pp.x : pp.y) >> (16 * (lb & 1))) & 0xffffu;
                constexpr uint32_t NOPOS = POSREP ? 0x7fffu : 0xffffu;
                const uint32_t praw = fld & NOPOS;
                const int k = (int)praw - c0;
                const bool hit = praw != NOPOS && k >= 0 && k < cw;
                const uint8_t af = POSREP ? (uint8_t)((fld >> 15) << 7) : a_s[it];
                // bs = 3: NV products M[r][c] = (V g_a[r]) g_b[c] of the lane's block rows, then (P lane / LPR = 4)
                // P = (V g_a) . g_b; every value lands in its own accumulator slot of column k
                constexpr int NV = BS == 1 ? 1 : (LPR == 4 ? 10 : 3);
                double v[NV];
                int slot0 = 0;        // first accumulator slot of the lane's values (consecutive)
                int nv = 0;           // values of this lane
                if constexpr (PDPP) {
                    // lanes (row, b, rr) of one quad share the item and node b: lane rr < 3 forms block row rr, and
                    // the P lane takes the three products (V g_a[q]) g_b[q] it needs from lanes q = 0, 1, 2 of its
                    // quad (DPP broadcasts) -- el_pdot's rounded products summed in its order, without its three
                    // LDS reads. Unconditional (every lane active for the DPP); the values of a miss are not used.
#if FEM_ACC_GDPP   // lane rr < 3 of the quad reads g_b[rr] alone, the quad shares the three over DPP
                    const double gmine = dat_s[3 + 3 * lb + (lrr < 3 ? lrr : 2)][it];
                    const double gb[3] = {quad_bcast<0>(gmine), quad_bcast<1>(gmine), quad_bcast<2>(gmine)};
#else
                    const double gb[3] = {dat_s[3 + 3 * lb][it], dat_s[4 + 3 * lb][it], dat_s[5 + 3 * lb][it]};
#endif
                    const double vr = dat_s[lrr < 3 ? lrr : 2][it];
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) v[cc] = vr * gb[cc];
                    const double p0 = quad_bcast<0>(v[0]), p1 = quad_bcast<1>(v[1]), p2 = quad_bcast<2>(v[2]);
                    if (lrr == 3) v[0] = add_nc(add_nc(p0, p1), p2);
                    slot0 = lrr < 3 ? 3 * lrr : 9;
                    nv = hit ? (lrr == 3 ? 1 : 3) : 0;
                } else if (hit) {
                    if constexpr (BS == 1) {
                        v[0] = dat_s[lb][it];
                        nv = 1;
                    } else {
                        const double gb[3] = {dat_s[3 + 3 * lb][it], dat_s[4 + 3 * lb][it], dat_s[5 + 3 * lb][it]};
                        if (LPR == 4) {
                            const double vga[3] = {dat_s[0][it], dat_s[1][it], dat_s[2][it]};
#pragma unroll
                            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                                for (int cc = 0; cc < 3; ++cc) v[rr * 3 + cc] = vga[rr] * gb[cc];
                            v[NV - 1] = el_pdot(vga, gb);
                            nv = 10;
                        } else if (lrr < 3) {
                            const double vr = dat_s[lrr][it];
#pragma unroll
                            for (int cc = 0; cc < 3; ++cc) v[cc] = vr * gb[cc];
                            slot0 = lrr * 3;
                            nv = 3;
                        } else {
                            const double vga[3] = {dat_s[0][it], dat_s[1][it], dat_s[2][it]};
                            v[0] = el_pdot(vga, gb);
                            slot0 = 9;
                            nv = 1;
                        }
                    }
                }
                // REPCHK (plain read-modify-writes): an element repeating a node would give two lanes of one step
                // the same accumulator, so such a step goes node by node. With LDS atomics both adds land, and such an
                // element has a determinant of exactly 0 (two equal columns, or a zero one): it is reported by `bad`
                // (check_singular raises) and its NaN / inf values are never a result -- no per-step check.
                const bool any_rep = REPCHK && __ballot(hit && (af & 0x80)) != 0;
                if (!any_rep) {
                    if (hit) {
#pragma unroll
                        for (int cc = 0; cc < NV; ++cc) {
                            if (cc < nv) {
                                // PDPP: the lane's slot base is loop-invariant (abase), one multiply per address
                                double* ap = PDPP ? abase + (k * AV + cc) * ISTR : &ACC(k * AV + slot0 + cc, lr);
#if FEM_ACC_ATOM
                                // one LDS add (ds_add_f64, no return) instead of a read, a wait and a write: the
                                // row's lanes of one step hit distinct slots and a wave's LDS operations complete
                                // in issue order, so every slot still sums in ascending incidence order
                                __hip_atomic_fetch_add(ap, v[cc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
                                *ap = add_nc(*ap, v[cc]);
#endif
                            }
                        }
                    }
                } else {   // an element repeating a node: its nodes' contributions one after the other (b order)
                    for (int b = 0; b < 4; ++b) {
                        if (hit && lb == b) {
#pragma unroll
                            for (int cc = 0; cc < NV; ++cc) {
                                if (cc < nv) {
                                    double* ap = &ACC(k * AV + slot0 + cc, lr);
                                    *ap = add_nc(*ap, v[cc]);
                                }
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    }
                }
            }
        }
        __syncthreads();
        if constexpr (BS == 1 && SL && STORE) {
            // solver layout, storing: lane-paired entries (2k, 2k + 1) of a row are adjacent, so a thread stores both
            // as one 16-byte value and a wave one contiguous 1 KB segment (per-entry 8-byte stores left every other
            // 8 bytes of each segment to the next instruction); the unpaired last entry of an odd-width slice after
            static_assert(AW % 2 == 0, "windows start at even entries");
            const int np = W >> 1;
            const int kp0 = c0 >> 1, kp1 = min((c0 + cw) >> 1, np);
            for (int q = tid; q < (kp1 - kp0) * R; q += NT) {
                const int r = q % R, kp = kp0 + q / R, k = 2 * kp - c0;
                *reinterpret_cast<double2*>(vals + e0 + (int64_t)kp * 128 + 2 * (l0 + r)) =
                    make_double2(ACC(k, r), ACC(k + 1, r));
            }
            if ((W & 1) && c0 + cw == W)
                for (int r = tid; r < R; r += NT) vals[e0 + (int64_t)np * 128 + l0 + r] = ACC(W - 1 - c0, r);
            continue;
        }
        for (int q = tid; q < cw * B2 * R; q += NT) {
            const int r = q % R, kc = q / R, k = kc / B2, c = kc - k * B2;
            if (!STORE && !(SL && uo >= 0) && c0 + k >= rp_s[r + 1] - rp_s[r]) continue;   // adding: padding stays
            const int64_t Ei = e0 + (int64_t)(c0 + k) * 64 + l0 + r;
            if constexpr (BS == 1) {
                vals[SL ? e0 + pair_pos(c0 + k, W, l0 + r) : Ei] = ACC(kc, r);
            } else {
                const int rr = c / 3, cc = c - 3 * (c / 3);
                double kv = el_combine(L, ACC(k * AV + c, r), ACC(k * AV + cc * 3 + rr, r), ACC(k * AV + 9, r),
                                       rr == cc);
                double* dst = &vals[SL ? sell_val_a(Ei, c) : sell_val(Ei, B2, c)];
                if constexpr (!STORE) kv = add_nc(*dst, kv);
                *dst = kv;
            }
        }
    }
}

// bs = 1 (P1 Poisson): each element lane forms its 4 scalar contributions E (g_a . g_b) V itself and finds the 4
// column slots by binary search in the row's LDS column list; an owner lane per column then adds the (at most one)
// contribution of every element in ascending incidence order — 2 LDS reads per element instead of ~20.
// LPR lanes per row (64 or 32): with 32, each half-wave assembles its own row — P1 rows (~15 columns, ~24
// incident tets) fill half a wave, so two rows' dependent loads are in flight per wave. Chunk loops cover longer rows.
template <int LPR>
__global__ void __launch_bounds__(256) k_assemble_p1w(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                      double kappa, const int32_t* __restrict__ inc_ptr,
                                                      const int32_t* __restrict__ inc, int64_t N,
                                                      const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ colidx,
                                                      const int64_t* __restrict__ csr2sell, double* __restrict__ vals,
                                                      int64_t* __restrict__ bad) {
    constexpr int RPW = 64 / LPR;
    __shared__ double c_s[AW_WAVES][64][4];
    __shared__ uint32_t pos_s[AW_WAVES][64];    // 4 column slots (bytes), 0xff = outside this column group
    __shared__ int col_s[AW_WAVES][64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sub = lane / LPR, sl = lane - LPR * sub, base = LPR * sub;
    const RowWalk rw = row_walk(AW_WAVES, RPW, sub);
    for (int64_t k = rw.k, i; (i = rw.row(k)) < N; k += rw.step) {
        const int lo = rowptr[i], len = rowptr[i + 1] - lo;
        const int t0 = inc_ptr[i], C = inc_ptr[i + 1] - t0;
        for (int j0 = 0; j0 < len; j0 += LPR) {
            const int nj = min(LPR, len - j0);
            if (sl < nj) col_s[wid][base + sl] = colidx[lo + j0 + sl];
            const bool owner = sl < nj;
            int64_t Ei = 0;
            double acc = 0.0;
            if (owner) {
                Ei = csr2sell[lo + j0 + sl];
                acc = vals[Ei];
            }
            for (int k0 = 0; k0 < C; k0 += LPR) {
                const int nk = min(LPR, C - k0);
                __builtin_amdgcn_wave_barrier();
                if (sl < nk) {
                    const int ea = inc[t0 + k0 + sl];
                    const int64_t e = ea >> 2;
                    const int a = ea & 3;
                    const int64_t* c = conn + 4 * e;
                    double g[4][3];
                    const double det = tet4_grads(X, c, g);
                    if (j0 == 0 && fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
                    const double V = fabs(det) / 6.0;
                    uint32_t packed = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const double dot = g[a][0] * g[b][0] + g[a][1] * g[b][1] + g[a][2] * g[b][2];
                        c_s[wid][base + sl][b] = kappa * dot * V;
                        const int j = (int)c[b];
                        int l = 0, h = nj;   // binary search of j among the group's sorted columns
                        while (l < h) {
                            const int m = (l + h) >> 1;
                            if (col_s[wid][base + m] < j) l = m + 1;
                            else h = m;
                        }
                        const uint32_t p = (l < nj && col_s[wid][base + l] == j) ? (uint32_t)l : 0xffu;
                        packed |= p << (8 * b);
                    }
                    pos_s[wid][base + sl] = packed;
                }
                __builtin_amdgcn_wave_barrier();
                if (owner) {
                    for (int kk = 0; kk < nk; ++kk) {
                        const uint32_t pk = pos_s[wid][base + kk];
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            if (((pk >> (8 * b)) & 0xffu) == (uint32_t)sl) acc += c_s[wid][base + kk][b];
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (owner) vals[Ei] = acc;
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// bs = 3 (c3d4 elasticity), same scheme with 3x3 blocks: element lanes (chunks of 32 elements) form the 4 blocks of
// their element row V (lambda g_a g_b^T + mu g_b g_a^T + mu (g_a . g_b) I) in LDS; owner lanes (column, block row)
// add their block row of every element in ascending incidence order.
constexpr int AE_K = 32;

__global__ void __launch_bounds__(256) k_assemble_el3w(const double* __restrict__ X, const int64_t* __restrict__ conn,
                                                       double E, double nu, const int32_t* __restrict__ inc_ptr,
                                                       const int32_t* __restrict__ inc, int64_t N,
                                                       const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ colidx,
                                                       const int64_t* __restrict__ csr2sell, double* __restrict__ vals,
                                                       int64_t* __restrict__ bad) {
    __shared__ double blk_s[AW_WAVES][AE_K][4][10];   // per (element, b): M_ab (9) and P_ab
    __shared__ uint32_t pos_s[AW_WAVES][AE_K];
    __shared__ int col_s[AW_WAVES][21];
    constexpr int JG = 21;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const Lame L = lame(E, nu);
    const RowWalk rw = row_walk(AW_WAVES);
    for (int64_t k = rw.k, i; (i = rw.row(k)) < N; k += rw.step) {
        const int lo = rowptr[i], len = rowptr[i + 1] - lo;
        const int t0 = inc_ptr[i], C = inc_ptr[i + 1] - t0;
        for (int j0 = 0; j0 < len; j0 += JG) {
            const int nj = min(JG, len - j0);
            if (lane < nj) col_s[wid][lane] = colidx[lo + j0 + lane];
            const int jl = lane / 3, r = lane - 3 * (lane / 3);
            const bool owner = lane < nj * 3;
            int64_t Ei = 0;
            // owner (column jl, block row r): M row r and M column r of the block, P; stored values added at the end
            double mr[3] = {0.0, 0.0, 0.0}, mc[3] = {0.0, 0.0, 0.0}, pp = 0.0;
            if (owner) Ei = csr2sell[lo + j0 + jl];
            for (int k0 = 0; k0 < C; k0 += AE_K) {
                const int nk = min(AE_K, C - k0);
                __builtin_amdgcn_wave_barrier();
                if (lane < nk) {
                    const int ea = inc[t0 + k0 + lane];
                    const int64_t e = ea >> 2;
                    const int a = ea & 3;
                    const int64_t* c = conn + 4 * e;
                    double g[4][3];
                    const double det = tet4_grads(X, c, g);
                    if (j0 == 0 && fabs(det) < 1e-12) atomicMin((unsigned long long*)bad, (unsigned long long)e);
                    const double V = fabs(det) / 6.0;
                    double vga[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        vga[q] = V * (a == 0 ? g[0][q] : a == 1 ? g[1][q] : a == 2 ? g[2][q] : g[3][q]);
                    uint32_t packed = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
#pragma unroll
                        for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                            for (int kk = 0; kk < 3; ++kk) blk_s[wid][lane][b][rr * 3 + kk] = vga[rr] * g[b][kk];
                        blk_s[wid][lane][b][9] = el_pdot(vga, g[b]);
                        const int j = (int)c[b];
                        int l = 0, h = nj;
                        while (l < h) {
                            const int m = (l + h) >> 1;
                            if (col_s[wid][m] < j) l = m + 1;
                            else h = m;
                        }
                        const uint32_t p = (l < nj && col_s[wid][l] == j) ? (uint32_t)l : 0xffu;
                        packed |= p << (8 * b);
                    }
                    pos_s[wid][lane] = packed;
                }
                __builtin_amdgcn_wave_barrier();
                if (owner) {
                    for (int k = 0; k < nk; ++k) {
                        const uint32_t pk = pos_s[wid][k];
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            if (((pk >> (8 * b)) & 0xffu) == (uint32_t)jl) {
                                const double* br = blk_s[wid][k][b];
#pragma unroll
                                for (int c = 0; c < 3; ++c) {
                                    mr[c] += br[r * 3 + c];
                                    mc[c] += br[c * 3 + r];
                                }
                                pp += br[9];
                            }
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (owner) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    double* dst = &vals[sell_val(Ei, 9, r * 3 + c)];
                    *dst = add_nc(*dst, el_combine(L, mr[c], mc[c], pp, r == c));
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int BS>
__global__ void k_sell_to_csr(const double* __restrict__ vals, const int32_t* __restrict__ rowptr, int64_t nrows,
                              const int64_t* __restrict__ csr2sell, double* __restrict__ out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x)
        for (int p = rowptr[r]; p < rowptr[r + 1]; ++p) {
            const int64_t E = csr2sell[p];
#pragma unroll
            for (int rc = 0; rc < BS * BS; ++rc) out[(int64_t)p * BS * BS + rc] = vals[sell_val(E, BS * BS, rc)];
        }
}

// csr2sell == nullptr: the SELL entry of the diagonal from the slice pointer (slot dp - rowptr[node] of the row)
__global__ void k_jacobi(const double* __restrict__ vals, int bs, const int32_t* __restrict__ rowptr,
                         const int32_t* __restrict__ diagpos, const int64_t* __restrict__ csr2sell,
                         const int64_t* __restrict__ slice_ptr, int64_t nrows, const uint8_t* __restrict__ mask,
                         double* __restrict__ w) {
    const int64_t n = nrows * bs;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t node = i / bs;
        const int r = (int)(i - node * bs);
        // diagpos < 0: a node no element touches (diagonal 0 -> 1/0 = inf -> 0, `solver/solver.py:828-831`)
        const int32_t dp = diagpos[node];
        const int64_t E = dp < 0 ? 0
                          : csr2sell ? csr2sell[dp]
                                     : slice_ptr[node >> 6] + (int64_t)(dp - rowptr[node]) * 64 + (node & 63);
        const double dg = dp < 0 ? 0.0 : vals[sell_val(E, bs * bs, r * bs + r)];
        double v = 1.0 / dg;
        if (v == INFINITY) v = 0.0;  // `solver/solver.py:831` (only +inf)
        if (mask && mask[i]) v = 0.0;
        w[i] = v;
    }
}

// Jacobi weights of a bs = 1 matrix in the solver layout (k_sell_sl_pattern): the diagonal at the paired position of
// the row's diagonal entry -- the list position of delta 0 in a slice-uniform slice, its CSR index otherwise
template <int BS>
__global__ void k_jacobi_sl(const double* __restrict__ svals, const int32_t* __restrict__ rowptr,
                            const int32_t* __restrict__ diagpos, const int64_t* __restrict__ slice_ptr,
                            const int32_t* __restrict__ uoff, const int16_t* __restrict__ ucol, int64_t nrows,
                            const uint8_t* __restrict__ mask, double* __restrict__ w) {
    // wave-uniform trip count (the ballot below needs every lane): lanes past the end work on the last dof, unstored
    const int64_t nd = nrows * BS;
    for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); t0 < nd;
         t0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tl = t0 + (threadIdx.x & 63);
        const bool act = tl < nd;
        const int64_t t = act ? tl : nd - 1;
        const int64_t i = t / BS;
        const int r = (int)(t - i * BS);
        const int64_t s = i >> 6;
        const int l = (int)(i & 63);
        const int64_t p0 = slice_ptr[s];
        const int wd = (int)((slice_ptr[s + 1] - p0) >> 6);
        const int32_t dp = diagpos[i];
        const int uo = BS == 1 ? uoff[s] : -1;
        int k = -1;
        if (BS == 1 && uo >= 0) {
            // slice-uniform: the wave's 64 rows are this slice (the grid stride is a multiple of 64), so the list
            // position of delta 0 is found by one compare per lane and a ballot -- not a walk of dependent loads
            const int lane = threadIdx.x & 63;
            for (int u0 = 0; u0 < wd; u0 += 64) {
                const bool z = u0 + lane < wd && ucol[uo + u0 + lane] == 0;
                const unsigned long long m = __ballot(z);
                if (m) {
                    k = u0 + __ffsll((long long)m) - 1;
                    break;
                }
            }
            if (dp < 0) k = -1;
        } else if (dp >= 0) {
            k = dp - rowptr[i];
        }
        const double dg = k < 0 ? 0.0
                          : BS == 1 ? svals[p0 + pair_pos(k, wd, l)]
                                    : svals[sell_val_a(p0 + 64 * (int64_t)k + l, r * 3 + r)];
        const int64_t i_ = t;   // the dof
        double v = 1.0 / dg;
        if (v == INFINITY) v = 0.0;  // `solver/solver.py:831` (only +inf)
        if (mask && mask[i_]) v = 0.0;
        if (act) w[i_] = v;
    }
}

__global__ void k_sell_diag(const double* __restrict__ vals, int bs, const int32_t* __restrict__ diagpos,
                            const int64_t* __restrict__ csr2sell, int64_t nrows, double* __restrict__ out) {
    const int64_t n = nrows * bs;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t node = i / bs;
        const int r = (int)(i - node * bs);
        const int32_t dp = diagpos[node];   // < 0: no diagonal entry (unused node)
        out[i] = dp < 0 ? 0.0 : vals[sell_val(csr2sell[dp], bs * bs, r * bs + r)];
    }
}

__global__ void k_jacobi_from_diag(const double* __restrict__ d, int64_t n, const uint8_t* __restrict__ mask,
                                   double* __restrict__ w) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double v = 1.0 / d[i];
        if (v == INFINITY) v = 0.0;
        if (mask && mask[i]) v = 0.0;
        w[i] = v;
    }
}

// ---------------------------------------------------------------- element-by-element operator
template <int DPN>
__global__ void __launch_bounds__(256) k_ebe_apply(const double* __restrict__ Ke, const int64_t* __restrict__ conn,
                                                   int npe, const int32_t* __restrict__ inc_ptr,
                                                   const int32_t* __restrict__ inc, int64_t N,
                                                   const double* __restrict__ u, double* __restrict__ y) {
    const int d = npe * DPN;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        double acc[DPN];
#pragma unroll
        for (int r = 0; r < DPN; ++r) acc[r] = 0.0;
        for (int t = inc_ptr[i]; t < inc_ptr[i + 1]; ++t) {
            const int ea = inc[t];
            const int64_t e = ea / npe;
            const int a = ea - (int)e * npe;
            const double* Krow = Ke + e * d * d + (int64_t)(a * DPN) * d;
            double f[DPN];
#pragma unroll
            for (int r = 0; r < DPN; ++r) f[r] = 0.0;
            for (int b = 0; b < npe; ++b) {
                const int64_t j = conn[e * npe + b];
#pragma unroll
                for (int c = 0; c < DPN; ++c) {
                    const double uj = u[j * DPN + c];
#pragma unroll
                    for (int r = 0; r < DPN; ++r) f[r] += Krow[r * d + b * DPN + c] * uj;
                }
            }
#pragma unroll
            for (int r = 0; r < DPN; ++r) acc[r] += f[r];
        }
#pragma unroll
        for (int r = 0; r < DPN; ++r) y[i * DPN + r] = acc[r];
    }
}

template <int DPN>
__global__ void k_ebe_diag(const double* __restrict__ Ke, int npe, const int32_t* __restrict__ inc_ptr,
                           const int32_t* __restrict__ inc, int64_t N, int colzero, double* __restrict__ diag) {
    const int d = npe * DPN;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        double acc[DPN];
#pragma unroll
        for (int r = 0; r < DPN; ++r) acc[r] = 0.0;
        for (int t = inc_ptr[i]; t < inc_ptr[i + 1]; ++t) {
            const int ea = inc[t];
            const int64_t e = ea / npe;
            const int a = ea - (int)e * npe;
#pragma unroll
            for (int r = 0; r < DPN; ++r) {
                const int row = a * DPN + r;
                acc[r] += Ke[e * d * d + (int64_t)row * d + (colzero ? 0 : row)];
            }
        }
#pragma unroll
        for (int r = 0; r < DPN; ++r) diag[i * DPN + r] = acc[r];
    }
}

__global__ void k_invert(const double* __restrict__ in, int64_t n, double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double v = 1.0 / in[i];
        out[i] = (v == INFINITY) ? 0.0 : v;
    }
}

}  // namespace fem

using namespace fem;

extern "C" {

int fem_tet4_ke(const double* coords, const int64_t* conn, int64_t M, double E, double nu, int kind, double* Ke,
                int64_t* bad_idx, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    dim3 g((unsigned)cdiv(M, 64));
    if (kind == FEM_KIND_ELASTIC)
        hipLaunchKernelGGL(k_tet4_ke<FEM_KIND_ELASTIC>, g, dim3(256), 0, S(stream), coords, conn, M, E, nu, Ke, bad_idx);
    else if (kind == FEM_KIND_POISSON)
        hipLaunchKernelGGL(k_tet4_ke<FEM_KIND_POISSON>, g, dim3(256), 0, S(stream), coords, conn, M, E, nu, Ke, bad_idx);
    else if (kind == FEM_KIND_MASS)
        hipLaunchKernelGGL(k_tet4_ke<FEM_KIND_MASS>, g, dim3(256), 0, S(stream), coords, conn, M, E, nu, Ke, bad_idx);
    else {
        set_error("fem_tet4_ke: unknown kind %d", kind);
        return FEM_EARG;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_tet4_geom(const double* coords, const int64_t* conn, int64_t M, double* vol, double* grads, double* B,
                  int64_t* bad_idx, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    hipLaunchKernelGGL(k_tet4_geom, dim3(stream_grid(M, 256)), dim3(256), 0, S(stream), coords, conn, M, vol, grads, B,
                       bad_idx);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_iso_geom(const double* coords, const int64_t* conn, int64_t M, int npe, const double* dN, double* J,
                 double* grads, double* B, fem_stream_t stream) {
    if (M <= 0) return FEM_OK;
    if (npe != 6 && npe != 8 && npe != 10) {
        set_error("fem_iso_geom: unsupported nodes per element %d", npe);
        return FEM_EBADTYPE;
    }
    hipLaunchKernelGGL(k_iso_geom, dim3(stream_grid(M, 256)), dim3(256), 0, S(stream), coords, conn, M, npe, dN, J,
                       grads, B);
    FEM_LAUNCHED();
    return FEM_OK;
}

// grid of the element-walking k_iso_ke: the resident workgroups (occupancy with the rule tables' dynamic LDS), at most
// one element per wave
static unsigned iso_grid(const void* fn, size_t lds, int64_t M) {
    int dev = 0, ncu = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, lds) != hipSuccess || nb < 1)
        nb = 1, ncu = 256;
    int64_t g = (int64_t)ncu * nb;
    const int64_t want = cdiv(M, 4);
    if (want < g) g = want;
    return (unsigned)(g < 1 ? 1 : g);
}
// the walking grid pays for c3d10 (K_e 2.0 -> 1.9 ms, M_e 1.5 -> 1.3 ms on the configs[4] set); the cheaper c3d8 /
// c3d6 elements ran 5-7 % slower walking than with a wave per element (1.45 -> 1.55, 1.01 -> 1.08 ms for c3d8)
static unsigned iso_grid_npe(const void* fn, size_t lds, int64_t M, int npe) {
    return npe == 10 ? iso_grid(fn, lds, M) : (unsigned)cdiv(M, 4);
}

int fem_iso_ke(const double* coords, const int64_t* conn, int64_t M, int npe, double E, double nu, const double* dN,
               const double* w, int n_ip, int mode, double* Ke, fem_stream_t stream) {
    if (mode != FEM_ISO_SUM && mode != FEM_ISO_STACK && mode != FEM_ISO_VOLUME) {
        set_error("fem_iso_ke: unknown mode %d", mode);
        return FEM_EARG;
    }
    if (M <= 0) return FEM_OK;
    if (n_ip < 1 || n_ip > ISO_MAX_IP) {
        set_error("fem_iso_ke: n_ip = %d out of range [1, %d]", n_ip, ISO_MAX_IP);
        return FEM_EARG;
    }
    const size_t lds = sizeof(double) * (size_t)n_ip * npe * 3;
    const void* fn = (const void*)k_iso_ke<10, false>;   // the walking grid (c3d10 only, iso_grid_npe)
    const dim3 g(iso_grid_npe(fn, lds, M, npe));
    switch (npe) {
        case 6: hipLaunchKernelGGL((k_iso_ke1<6, false>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Ke); break;
        case 8: hipLaunchKernelGGL((k_iso_ke1<8, false>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Ke); break;
        case 10: hipLaunchKernelGGL((k_iso_ke<10, false>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Ke); break;
        default: set_error("fem_iso_ke: unsupported nodes per element %d", npe); return FEM_EBADTYPE;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_ke_sym_stride(int npe) { return (npe >= 1 && npe <= 15) ? ke_sym_stride(npe) : -1; }

int fem_iso_ke_sym(const double* coords, const int64_t* conn, int64_t M, int npe, double E, double nu,
                   const double* dN, const double* w, int n_ip, int mode, double* Kp, fem_stream_t stream) {
    if (mode != FEM_ISO_SUM && mode != FEM_ISO_VOLUME) {
        set_error("fem_iso_ke_sym: mode %d (the packed form takes FEM_ISO_SUM / FEM_ISO_VOLUME)", mode);
        return FEM_EARG;
    }
    if (M <= 0) return FEM_OK;
    if (n_ip < 1 || n_ip > ISO_MAX_IP) {
        set_error("fem_iso_ke_sym: n_ip = %d out of range [1, %d]", n_ip, ISO_MAX_IP);
        return FEM_EARG;
    }
    const size_t lds = sizeof(double) * (size_t)n_ip * npe * 3;
    const void* fn = (const void*)k_iso_ke<10, false, false, true>;
    const dim3 g(iso_grid_npe(fn, lds, M, npe));
    switch (npe) {
        case 6: hipLaunchKernelGGL((k_iso_ke1<6, false, false, true>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Kp); break;
        case 8: hipLaunchKernelGGL((k_iso_ke1<8, false, false, true>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Kp); break;
        case 10: hipLaunchKernelGGL((k_iso_ke<10, false, false, true>), g, dim3(256), lds, S(stream), coords, conn, M, E, nu, dN, w, n_ip, mode, Kp); break;
        default: set_error("fem_iso_ke_sym: unsupported nodes per element %d", npe); return FEM_EBADTYPE;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

static int iso_mass(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                    const double* dN, const double* w, int n_ip, double* Me, bool scalar, hipStream_t st);

int fem_iso_mass(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                 const double* dN, const double* w, int n_ip, double* Me, fem_stream_t stream) {
    return iso_mass(coords, conn, M, npe, rho, Nv, dN, w, n_ip, Me, false, S(stream));
}

int fem_iso_mass_scalar(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                        const double* dN, const double* w, int n_ip, double* Ms, fem_stream_t stream) {
    return iso_mass(coords, conn, M, npe, rho, Nv, dN, w, n_ip, Ms, true, S(stream));
}

static int iso_mass(const double* coords, const int64_t* conn, int64_t M, int npe, double rho, const double* Nv,
                    const double* dN, const double* w, int n_ip, double* Me, bool scalar, hipStream_t st) {
    if (M <= 0) return FEM_OK;
    if (n_ip < 1 || n_ip > ISO_MAX_IP) {
        set_error("fem_iso_mass: n_ip = %d out of range [1, %d]", n_ip, ISO_MAX_IP);
        return FEM_EARG;
    }
    const int mode = FEM_ISO_MASS;
    const size_t lds = sizeof(double) * (size_t)n_ip * npe * 4;
    const void* fn = (const void*)k_iso_ke<10, true>;   // the walking grid (c3d10 only, iso_grid_npe)
    const dim3 g(iso_grid_npe(fn, lds, M, npe));
    if (scalar && getenv("FEM355_MASS_WAVE") == nullptr) {   // thread per element (k_iso_mass_s)
        const size_t tl = sizeof(double) * (size_t)n_ip * (npe * 4 + 1);
        const dim3 gs((unsigned)std::min<int64_t>(cdiv(M, 256), 65536));
        switch (npe) {
            case 6: hipLaunchKernelGGL(k_iso_mass_s<6>, gs, dim3(256), tl, st, coords, conn, M, rho, dN, Nv, w, n_ip, Me); break;
            case 8: hipLaunchKernelGGL(k_iso_mass_s<8>, gs, dim3(256), tl, st, coords, conn, M, rho, dN, Nv, w, n_ip, Me); break;
            case 10: hipLaunchKernelGGL(k_iso_mass_s<10>, gs, dim3(256), tl, st, coords, conn, M, rho, dN, Nv, w, n_ip, Me); break;
            default: set_error("fem_iso_mass: unsupported nodes per element %d", npe); return FEM_EBADTYPE;
        }
        FEM_LAUNCHED();
        return FEM_OK;
    }
#define FEM_IM(K, P, SC_) hipLaunchKernelGGL((K<P, true, SC_>), g, dim3(256), lds, st, coords, conn, M, rho, 0.0, dN, w, \
                                             n_ip, mode, Me, Nv)
    switch (npe) {
        case 6: if (scalar) FEM_IM(k_iso_ke1, 6, true); else FEM_IM(k_iso_ke1, 6, false); break;
        case 8: if (scalar) FEM_IM(k_iso_ke1, 8, true); else FEM_IM(k_iso_ke1, 8, false); break;
        case 10: if (scalar) FEM_IM(k_iso_ke, 10, true); else FEM_IM(k_iso_ke, 10, false); break;
        default: set_error("fem_iso_mass: unsupported nodes per element %d", npe); return FEM_EBADTYPE;
    }
#undef FEM_IM
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_assemble_from_ke(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                         const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                         const int64_t* csr2sell, const int64_t* slice_ptr, double* vals, fem_stream_t stream) {
    return fem_assemble_from_ke_ex(Ke, conn, npe, bs, inc_ptr, inc, N, rowptr, colidx, csr2sell, slice_ptr, -1, -1, 0,
                                   vals, stream);
}

// tile form of the bs = 3 stored-K_e assembly (k_assemble_ke_tile3): R = 16 rows per tile while the LDS allows
// (whole 128-byte plane lines), else 8; false when the pattern's width is unknown or the form is switched off
static int ke_tile_launch(const double* Ke, const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc,
                          int64_t N, const int32_t* rowptr, const int32_t* colidx, const int64_t* slice_ptr, int store,
                          int max_width, double* vals, hipStream_t st, bool* done, bool la = false, bool pk = false) {
    *done = false;
    if (max_width <= 0) return FEM_OK;
    if (!la && !pk && (getenv("FEM355_KE_ROWS") != nullptr || getenv("FEM355_KE_COLS") != nullptr)) return FEM_OK;
    const int Wc = max_width < KR_LMAX ? max_width : KR_LMAX;
    const int R = (16 * (Wc * 9 + 1) * 8 + 16 * 1280 <= 65536) ? 16 : 8;
    const size_t dyn = sizeof(double) * (size_t)R * (Wc * 9 + 1);
    const int64_t ntiles = cdiv(N, 64) * (64 / R);   // whole slices: lanes past the last row are zeroed too
    const dim3 g((unsigned)(cdiv(cdiv(N, 64), NXCD) * NXCD * (64 / R)));
#define FEM_KT(P, RR, ST, LA_, PK_)                                                                                \
    if (npe == P && R == RR && (store != 0) == ST && la == LA_ && pk == PK_)                                       \
        hipLaunchKernelGGL((k_assemble_ke_tile3<P, RR, ST, LA_, PK_>), g, dim3(RR * 64), dyn, st, Ke, conn, inc_ptr,\
                           inc, N, rowptr, colidx, slice_ptr, vals, Wc, ntiles);
#define FEM_KT_LA(P, PK_) FEM_KT(P, 16, true, false, PK_) FEM_KT(P, 16, false, false, PK_)                          \
    FEM_KT(P, 8, true, false, PK_) FEM_KT(P, 8, false, false, PK_) FEM_KT(P, 16, true, true, PK_)                    \
    FEM_KT(P, 16, false, true, PK_) FEM_KT(P, 8, true, true, PK_) FEM_KT(P, 8, false, true, PK_)
#define FEM_KT_ALL(P) FEM_KT_LA(P, false) FEM_KT_LA(P, true)
    FEM_KT_ALL(4) FEM_KT_ALL(6) FEM_KT_ALL(8) FEM_KT_ALL(10)
#undef FEM_KT_ALL
#undef FEM_KT_LA
#undef FEM_KT
    FEM_LAUNCHED();
    *done = true;
    return FEM_OK;
}

static int assemble_from_ke(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                            const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                            const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                            int max_width, double* vals, fem_stream_t stream);

// the fused stiffness + scalar (mass) form of the tile assembly (k_assemble_ke_tile3<..., LA, MS>): K into the solver
// layout A of the bs = 3 values, Me into the plain bs = 1 values of the same pattern
static int ke_tile_launch_ms(const double* Ke, const double* Me, const int64_t* conn, int npe, const int32_t* inc_ptr,
                             const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                             const int64_t* slice_ptr, int store, int max_width, double* svals, double* mvals,
                             hipStream_t st) {
    const int Wc = max_width < KR_LMAX ? max_width : KR_LMAX;
    const int R = (16 * (Wc * 10 + 2) * 8 + 16 * 1280 <= 65536) ? 16 : 8;
    const size_t dyn = sizeof(double) * (size_t)R * (Wc * 10 + 2);
    const int64_t ntiles = cdiv(N, 64) * (64 / R);
    const dim3 g((unsigned)(cdiv(cdiv(N, 64), NXCD) * NXCD * (64 / R)));
#define FEM_KTM(P, RR, ST)                                                                                          \
    if (npe == P && R == RR && (store != 0) == ST)                                                                  \
        hipLaunchKernelGGL((k_assemble_ke_tile3<P, RR, ST, true, false, true>), g, dim3(RR * 64), dyn, st, Ke, conn,\
                           inc_ptr, inc, N, rowptr, colidx, slice_ptr, svals, Wc, ntiles, Me, mvals);
#define FEM_KTM_ALL(P) FEM_KTM(P, 16, true) FEM_KTM(P, 16, false) FEM_KTM(P, 8, true) FEM_KTM(P, 8, false)
    FEM_KTM_ALL(4) FEM_KTM_ALL(6) FEM_KTM_ALL(8) FEM_KTM_ALL(10)
#undef FEM_KTM_ALL
#undef FEM_KTM
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_assemble_from_ke_ex(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                            const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                            const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                            double* vals, fem_stream_t stream) {
    return assemble_from_ke(Ke, conn, npe, bs, inc_ptr, inc, N, rowptr, colidx, csr2sell, slice_ptr, nnz, ent, store,
                            0, vals, stream);
}

int fem_assemble_from_ke_ex2(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                             const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                             const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                             int max_width, double* vals, fem_stream_t stream) {
    return assemble_from_ke(Ke, conn, npe, bs, inc_ptr, inc, N, rowptr, colidx, csr2sell, slice_ptr, nnz, ent, store,
                            max_width, vals, stream);
}

static int assemble_from_ke(const double* Ke, const int64_t* conn, int npe, int bs, const int32_t* inc_ptr,
                            const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                            const int64_t* csr2sell, const int64_t* slice_ptr, int64_t nnz, int64_t ent, int store,
                            int max_width, double* vals, fem_stream_t stream) {
    if (store && ent < 0) {
        set_error("fem_assemble_from_ke_ex: store mode needs the SELL entry count");
        return FEM_EARG;
    }
    const bool csrw = bs == 3 && getenv("FEM355_KE_DIRECT") == nullptr && N > 0 &&
                      (npe == 4 || npe == 6 || npe == 8 || npe == 10);
    // bs = 1 with the pattern's widest slice known: the tile form (k_assemble_ke_tile1; FEM355_KE_ROWS: wave per row)
    const bool tile1 = bs == 1 && max_width > 0 && N > 0 && (npe == 4 || npe == 6 || npe == 8 || npe == 10) &&
                       getenv("FEM355_KE_ROWS") == nullptr;
    if (tile1) {
        const int Wc = max_width < KR_LMAX ? max_width : KR_LMAX;
#ifndef FEM_KE_R1
#define FEM_KE_R1 16
#endif
        constexpr int R1 = FEM_KE_R1;   // rows per tile (FEM_KE_R1: A/B of the tile height)
        const size_t dyn = sizeof(double) * (size_t)R1 * (Wc + 1);
        const int64_t ntiles = cdiv(N, 64) * (64 / R1);
        const dim3 g((unsigned)(cdiv(cdiv(N, 64), NXCD) * NXCD * (64 / R1)));
#define FEM_KT1(P)                                                                                                 \
    if (npe == P) {                                                                                                \
        if (store) hipLaunchKernelGGL((k_assemble_ke_tile1<P, R1, true>), g, dim3(R1 * 64), dyn, S(stream), Ke, conn, \
                                      inc_ptr, inc, N, rowptr, colidx, slice_ptr, vals, Wc, ntiles);             \
        else hipLaunchKernelGGL((k_assemble_ke_tile1<P, R1, false>), g, dim3(R1 * 64), dyn, S(stream), Ke, conn,    \
                                inc_ptr, inc, N, rowptr, colidx, slice_ptr, vals, Wc, ntiles);                   \
    }
        FEM_KT1(4) FEM_KT1(6) FEM_KT1(8) FEM_KT1(10)
#undef FEM_KT1
        FEM_LAUNCHED();
        return FEM_OK;
    }
    // store mode on the paths that add in place: zero the matrix first (the block-CSR path stores every entry)
    if (store && !csrw && ent > 0) FEM_HIP(hipMemsetAsync(vals, 0, sizeof(double) * bs * bs * (size_t)ent, S(stream)));
    if ((bs == 1 || bs == 3) && (npe == 4 || npe == 6 || npe == 8 || npe == 10)) {   // wave per row
        const dim3 g((unsigned)grid_multiple_of_xcd(cdiv(N, AW_WAVES), 8192));
        // bs = 3: row sums to a block-CSR buffer with contiguous per-wave writes, then one slice-coalesced add into
        // the SELL planes (the in-place variant's scattered 8-byte plane updates measured 4.6x their bytes in
        // WRITE_SIZE on c3d10); FEM355_KE_DIRECT=1 keeps the in-place kernel
        if (csrw) {
            bool tiled = false;
            const int trc = ke_tile_launch(Ke, conn, npe, inc_ptr, inc, N, rowptr, colidx, slice_ptr, store, max_width,
                                           vals, S(stream), &tiled);
            if (trc != FEM_OK || tiled) return trc;
            if (nnz < 0) {   // not given: one device-to-host read of rowptr[N]
                nnz = 0;
                FEM_HIP(hipMemcpyAsync(&nnz, rowptr + N, sizeof(int32_t), hipMemcpyDeviceToHost, S(stream)));
                FEM_HIP(hipStreamSynchronize(S(stream)));
                nnz &= 0xffffffffLL;
            }
            // FEM355_KE_COLS set: the column-owner form (k_assemble_ke_w) instead of the element-row form (read per
            // call: the parity test compares both in one process)
            const bool colform = getenv("FEM355_KE_COLS") != nullptr;
            if (store && !colform && getenv("FEM355_KE_SELLW") != nullptr) {   // straight into the SELL planes
#define FEM_KE_S(P)                                                                                             \
    if (npe == P)                                                                                               \
        hipLaunchKernelGGL((k_assemble_ke_rows3<P, true>), g, dim3(256), 0, S(stream), Ke, conn, inc_ptr, inc, N, \
                           rowptr, colidx, vals, slice_ptr);
                FEM_KE_S(4) FEM_KE_S(6) FEM_KE_S(8) FEM_KE_S(10)
#undef FEM_KE_S
                FEM_LAUNCHED();
                if (N & 63) {
                    hipLaunchKernelGGL(k_sell_tail_zero, dim3(1), dim3(256), 0, S(stream), slice_ptr, N, 9, vals);
                    FEM_LAUNCHED();
                }
                return FEM_OK;
            }
            double* tmp = nullptr;
            FEM_HIP(::fem::malloc_async((void**)&tmp, sizeof(double) * 9 * (size_t)(nnz > 0 ? nnz : 1), S(stream)));
#define FEM_KE_C(P)                                                                                             \
    if (npe == P && colform)                                                                                    \
        hipLaunchKernelGGL((k_assemble_ke_w<3, P, FEM_KE_RPL3, true>), g, dim3(256), 0, S(stream), Ke, conn,     \
                           inc_ptr, inc, N, rowptr, colidx, csr2sell, tmp);                                     \
    else if (npe == P)                                                                                          \
        hipLaunchKernelGGL(k_assemble_ke_rows3<P>, g, dim3(256), 0, S(stream), Ke, conn, inc_ptr, inc, N,       \
                           rowptr, colidx, tmp);
            FEM_KE_C(4) FEM_KE_C(6) FEM_KE_C(8) FEM_KE_C(10)
#undef FEM_KE_C
            FEM_LAUNCHED();
            const int64_t ns = cdiv(N, 64);
            if (store)
                hipLaunchKernelGGL((k_csr_add_sell<3, true>), dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)),
                                   dim3(256), 0, S(stream), tmp, rowptr, N, ns, slice_ptr, vals);
            else
                hipLaunchKernelGGL(k_csr_add_sell<3>, dim3((unsigned)std::min<int64_t>(cdiv(ns, 4), 16384)), dim3(256),
                                   0, S(stream), tmp, rowptr, N, ns, slice_ptr, vals);
            FEM_LAUNCHED();
            FEM_HIP(hipFreeAsync(tmp, S(stream)));
            return FEM_OK;
        }
#define FEM_KE_W(B, P)                                                                                          \
    if (bs == B && npe == P)                                                                                    \
        hipLaunchKernelGGL((k_assemble_ke_w<B, P, (B == 3 ? FEM_KE_RPL3 : 1)>), g, dim3(256), 0, S(stream), Ke,  \
                           conn, inc_ptr, inc, N, rowptr, colidx, csr2sell, vals);
        FEM_KE_W(1, 4) FEM_KE_W(1, 6) FEM_KE_W(1, 8) FEM_KE_W(1, 10)
        FEM_KE_W(3, 4) FEM_KE_W(3, 6) FEM_KE_W(3, 8) FEM_KE_W(3, 10)
#undef FEM_KE_W
        FEM_LAUNCHED();
        return FEM_OK;
    }
    dim3 g(stream_grid(N, 256));
    if (bs == 1)
        hipLaunchKernelGGL(k_assemble_from_ke<1>, g, dim3(256), 0, S(stream), Ke, conn, npe, inc_ptr, inc, N, rowptr, colidx, csr2sell, vals);
    else if (bs == 3)
        hipLaunchKernelGGL(k_assemble_from_ke<3>, g, dim3(256), 0, S(stream), Ke, conn, npe, inc_ptr, inc, N, rowptr, colidx, csr2sell, vals);
    else {
        set_error("fem_assemble_from_ke: block size %d unsupported", bs);
        return FEM_EARG;
    }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_assemble_tet4_ex2(const double* coords, const int64_t* conn, double E, double nu, int bs,
                          const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                          const int32_t* colidx, const int64_t* csr2sell, const int64_t* slice_ptr, int store,
                          int max_width, double* vals, int64_t* bad_idx, fem_stream_t stream) {
    if (bs != 1 && bs != 3) {
        set_error("fem_assemble_tet4: block size %d unsupported", bs);
        return FEM_EARG;
    }
    if (N <= 0) return FEM_OK;
    if (max_width >= acc_max_cols(bs)) {
        set_error("fem_assemble_tet4: a row of %d columns exceeds the value kernel's %d", max_width,
                  acc_max_cols(bs) - 1);
        return FEM_EARG;
    }
    hipStream_t st = S(stream);
    if (getenv("FEM355_ASM_ROWS") != nullptr) {
        if (!csr2sell) {
            set_error("fem_assemble_tet4: the row kernels (FEM355_ASM_ROWS) need csr2sell");
            return FEM_EARG;
        }
        // wave per row (k_assemble_p1w / k_assemble_el3w, CSR-addressed through csr2sell; k_asm_tet4_acc's bits):
        // kept as the reference formulation of the accumulator kernel's summation order
        if (store) {
            hipLaunchKernelGGL(k_sell_zero, dim3(2048), dim3(256), 0, st, slice_ptr, cdiv(N, 64), bs * bs, vals);
            FEM_LAUNCHED();
        }
        const dim3 g((unsigned)grid_multiple_of_xcd(cdiv(N, AW_WAVES), 8192));
        if (bs == 1)
            hipLaunchKernelGGL(k_assemble_p1w<FEM_P1_LPR>, g, dim3(256), 0, st, coords, conn, E, inc_ptr, inc, N, rowptr, colidx, csr2sell, vals, bad_idx);
        else
            hipLaunchKernelGGL(k_assemble_el3w, g, dim3(256), 0, st, coords, conn, E, nu, inc_ptr, inc, N, rowptr, colidx, csr2sell, vals, bad_idx);
        FEM_LAUNCHED();
        return FEM_OK;
    }
    if (bs == 1) {
#define AA_LAUNCH(BS_, CFG_, ST_)                                                                                   \
    do {                                                                                                            \
        const int64_t nt = cdiv(N, 64) * (64 / CFG_::R);                                                            \
        hipLaunchKernelGGL((k_asm_tet4_acc<BS_, CFG_, ST_>), dim3((unsigned)(cdiv(nt, NXCD) * NXCD)),               \
                           dim3(CFG_::R * CFG_::LPR), 0,                                                             \
                           st, coords, conn, E, nu, inc_ptr, inc, N, rowptr, colidx, slice_ptr, vals, bad_idx, nt); \
    } while (0)
        if (max_width > 0 && max_width <= AccP1w16::W) {
            if (store) AA_LAUNCH(1, AccP1w16, true);
            else AA_LAUNCH(1, AccP1w16, false);
        } else {
            if (store) AA_LAUNCH(1, AccP1, true);
            else AA_LAUNCH(1, AccP1, false);
        }
        FEM_LAUNCHED();
        return FEM_OK;
    }
    if (store) AA_LAUNCH(3, AccEl, true);
    else AA_LAUNCH(3, AccEl, false);
#undef AA_LAUNCH
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_assemble_tet4_sl(const double* coords, const int64_t* conn, double E, double nu, int bs,
                         const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                         const int32_t* colidx, const int64_t* slice_ptr, const int32_t* uoff, const int16_t* ucol,
                         int store, int max_width, double* svals, int64_t* bad_idx, fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    if (bs == 1 && (!uoff || !ucol)) {
        set_error("fem_assemble_tet4_sl: the solver-layout pattern (fem_sell_sl_pattern) is required");
        return FEM_EARG;
    }
    if (bs != 1 && bs != 3) {
        set_error("fem_assemble_tet4_sl: block size %d unsupported", bs);
        return FEM_EARG;
    }
    if (max_width >= acc_max_cols(bs)) {
        set_error("fem_assemble_tet4_sl: a row of %d columns exceeds the value kernel's %d", max_width,
                  acc_max_cols(bs) - 1);
        return FEM_EARG;
    }
    hipStream_t st = S(stream);
#define AS_LAUNCH(BS_, CFG_, ST_)                                                                                   \
    do {                                                                                                            \
        const int64_t nt = cdiv(N, 64) * (64 / CFG_::R);                                                            \
        hipLaunchKernelGGL((k_asm_tet4_acc<BS_, CFG_, ST_, true>), dim3((unsigned)(cdiv(nt, NXCD) * NXCD)),         \
                           dim3(CFG_::R * CFG_::LPR), 0, st, coords, conn, E, nu, inc_ptr, inc, N, rowptr, colidx,   \
                           slice_ptr, svals, bad_idx, nt, uoff, ucol);                                               \
    } while (0)
    if (bs == 3) {
        if (store) AS_LAUNCH(3, AccEl, true);
        else AS_LAUNCH(3, AccEl, false);
    } else if (max_width > 0 && max_width <= AccP1w16::W) {
        if (store) AS_LAUNCH(1, AccP1w16, true);
        else AS_LAUNCH(1, AccP1w16, false);
    } else {
        if (store) AS_LAUNCH(1, AccP1, true);
        else AS_LAUNCH(1, AccP1, false);
    }
#undef AS_LAUNCH
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_assemble_from_ke_sl(const double* Ke, const int64_t* conn, int npe, const int32_t* inc_ptr, const int32_t* inc,
                            int64_t N, const int32_t* rowptr, const int32_t* colidx, const int64_t* slice_ptr,
                            int store, int max_width, double* svals, fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    if (!(npe == 4 || npe == 6 || npe == 8 || npe == 10) || max_width <= 0) {
        set_error("fem_assemble_from_ke_sl: npe 4/6/8/10 and the pattern width required");
        return FEM_EARG;
    }
    bool done = false;
    const int rc = ke_tile_launch(Ke, conn, npe, inc_ptr, inc, N, rowptr, colidx, slice_ptr, store, max_width, svals,
                                  S(stream), &done, true);
    if (rc == FEM_OK && !done) {
        set_error("fem_assemble_from_ke_sl: tile form not launched");
        return FEM_EARG;
    }
    return rc;
}

int fem_assemble_from_ke_mass_sl(const double* Ke, const double* Me, const int64_t* conn, int npe,
                                 const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                                 const int32_t* colidx, const int64_t* slice_ptr, int store, int max_width,
                                 double* svals, double* mvals, fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    if (!(npe == 4 || npe == 6 || npe == 8 || npe == 10) || max_width <= 0 || !Ke || !Me || !svals || !mvals) {
        set_error("fem_assemble_from_ke_mass_sl: npe 4/6/8/10, the pattern width and all four arrays required");
        return FEM_EARG;
    }
    return ke_tile_launch_ms(Ke, Me, conn, npe, inc_ptr, inc, N, rowptr, colidx, slice_ptr, store, max_width, svals,
                             mvals, S(stream));
}

int fem_assemble_from_ke_sym(const double* Kp, const int64_t* conn, int npe, const int32_t* inc_ptr,
                             const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                             const int64_t* slice_ptr, int store, int max_width, int layout_a, double* vals,
                             fem_stream_t stream) {
    if (N <= 0) return FEM_OK;
    if (!(npe == 4 || npe == 6 || npe == 8 || npe == 10) || max_width <= 0) {
        set_error("fem_assemble_from_ke_sym: npe 4/6/8/10 and the pattern width required");
        return FEM_EARG;
    }
    bool done = false;
    const int rc = ke_tile_launch(Kp, conn, npe, inc_ptr, inc, N, rowptr, colidx, slice_ptr, store, max_width, vals,
                                  S(stream), &done, layout_a != 0, true);
    if (rc == FEM_OK && !done) {
        set_error("fem_assemble_from_ke_sym: tile form not launched");
        return FEM_EARG;
    }
    return rc;
}

int fem_assemble_tet4_ex(const double* coords, const int64_t* conn, double E, double nu, int bs,
                         const int32_t* inc_ptr, const int32_t* inc, int64_t N, const int32_t* rowptr,
                         const int32_t* colidx, const int64_t* csr2sell, const int64_t* slice_ptr, int store,
                         double* vals, int64_t* bad_idx, fem_stream_t stream) {
    return fem_assemble_tet4_ex2(coords, conn, E, nu, bs, inc_ptr, inc, N, rowptr, colidx, csr2sell, slice_ptr, store,
                                 0, vals, bad_idx, stream);
}

int fem_assemble_tet4(const double* coords, const int64_t* conn, double E, double nu, int bs, const int32_t* inc_ptr,
                      const int32_t* inc, int64_t N, const int32_t* rowptr, const int32_t* colidx,
                      const int64_t* csr2sell, const int64_t* slice_ptr, double* vals, int64_t* bad_idx,
                      fem_stream_t stream) {
    return fem_assemble_tet4_ex(coords, conn, E, nu, bs, inc_ptr, inc, N, rowptr, colidx, csr2sell, slice_ptr, 0,
                                vals, bad_idx, stream);
}

int fem_sell_to_csr_vals(const double* vals, int bs, const int32_t* rowptr, int64_t nrows, const int64_t* csr2sell,
                         const int64_t* slice_ptr, double* csr_vals, fem_stream_t stream) {
    (void)slice_ptr;
    dim3 g(stream_grid(nrows, 256));
    if (bs == 1) hipLaunchKernelGGL(k_sell_to_csr<1>, g, dim3(256), 0, S(stream), vals, rowptr, nrows, csr2sell, csr_vals);
    else if (bs == 3) hipLaunchKernelGGL(k_sell_to_csr<3>, g, dim3(256), 0, S(stream), vals, rowptr, nrows, csr2sell, csr_vals);
    else { set_error("fem_sell_to_csr_vals: block size %d unsupported", bs); return FEM_EARG; }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_jacobi(const double* vals, int bs, const int32_t* rowptr, const int32_t* diagpos, const int64_t* csr2sell,
               const int64_t* slice_ptr, int64_t nrows, const uint8_t* mask, double* w, fem_stream_t stream) {
    hipLaunchKernelGGL(k_jacobi, dim3(stream_grid(nrows * bs, 256)), dim3(256), 0, S(stream), vals, bs, rowptr,
                       diagpos, csr2sell, slice_ptr, nrows, mask, w);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_jacobi_sl(const double* svals, int bs, const int32_t* rowptr, const int32_t* diagpos,
                  const int64_t* slice_ptr, const int32_t* uoff, const int16_t* ucol, int64_t nrows,
                  const uint8_t* mask, double* w, fem_stream_t stream) {
    if (nrows <= 0) return FEM_OK;
    if (bs == 1)
        hipLaunchKernelGGL(k_jacobi_sl<1>, dim3(stream_grid(nrows, 256)), dim3(256), 0, S(stream), svals, rowptr,
                           diagpos, slice_ptr, uoff, ucol, nrows, mask, w);
    else
        hipLaunchKernelGGL(k_jacobi_sl<3>, dim3(stream_grid(nrows * 3, 256)), dim3(256), 0, S(stream), svals, rowptr,
                           diagpos, slice_ptr, uoff, ucol, nrows, mask, w);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_sell_diag(const double* vals, int bs, const int32_t* diagpos, const int64_t* csr2sell, int64_t nrows,
                  double* diag, fem_stream_t stream) {
    hipLaunchKernelGGL(k_sell_diag, dim3(stream_grid(nrows * bs, 256)), dim3(256), 0, S(stream), vals, bs, diagpos,
                       csr2sell, nrows, diag);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_jacobi_from_diag(const double* diag, int64_t n, const uint8_t* mask, double* w, fem_stream_t stream) {
    hipLaunchKernelGGL(k_jacobi_from_diag, dim3(stream_grid(n, 256)), dim3(256), 0, S(stream), diag, n, mask, w);
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_ebe_apply(const double* Ke, const int64_t* conn, int npe, int dpn, const int32_t* inc_ptr, const int32_t* inc,
                  int64_t N, const double* u, double* y, fem_stream_t stream) {
    dim3 g(stream_grid(N, 256));
    if (dpn == 1) hipLaunchKernelGGL(k_ebe_apply<1>, g, dim3(256), 0, S(stream), Ke, conn, npe, inc_ptr, inc, N, u, y);
    else if (dpn == 3) hipLaunchKernelGGL(k_ebe_apply<3>, g, dim3(256), 0, S(stream), Ke, conn, npe, inc_ptr, inc, N, u, y);
    else { set_error("fem_ebe_apply: dofs per node %d unsupported", dpn); return FEM_EARG; }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_ebe_diag(const double* Ke, const int64_t* conn, int npe, int dpn, const int32_t* inc_ptr, const int32_t* inc,
                 int64_t N, int colzero, double* diag, fem_stream_t stream) {
    (void)conn;
    dim3 g(stream_grid(N, 256));
    if (dpn == 1) hipLaunchKernelGGL(k_ebe_diag<1>, g, dim3(256), 0, S(stream), Ke, npe, inc_ptr, inc, N, colzero, diag);
    else if (dpn == 3) hipLaunchKernelGGL(k_ebe_diag<3>, g, dim3(256), 0, S(stream), Ke, npe, inc_ptr, inc, N, colzero, diag);
    else { set_error("fem_ebe_diag: dofs per node %d unsupported", dpn); return FEM_EARG; }
    FEM_LAUNCHED();
    return FEM_OK;
}

int fem_invert_diag(const double* in, int64_t n, double* out, fem_stream_t stream) {
    hipLaunchKernelGGL(k_invert, dim3(stream_grid(n, 256)), dim3(256), 0, S(stream), in, n, out);
    FEM_LAUNCHED();
    return FEM_OK;
}

}  // extern "C"
