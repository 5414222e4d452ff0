// Per-element geometry shared by the quadrature (assemble.hip) and stress recovery (stress.hip) kernels.
#pragma once
#include "common.hpp"

namespace fem {

struct Lame {
    double lam, mu;
};

__host__ __device__ inline Lame lame(double E, double nu) {
    // same coefficient the reference forms: coef = E/((1+nu)(1-2nu)); D33 = coef*(1-2nu)/2
    double c = E / ((1.0 + nu) * (1.0 - 2.0 * nu));
    return Lame{c * nu, c * ((1.0 - 2.0 * nu) / 2.0)};
}

// gradients of the P1 shape functions (rows of inv([1 x y z]) 1..3) and signed det of the edge matrix, from the
// element's node ids (already loaded)
// gradients and det from the 4 vertices' coordinates
__device__ __forceinline__ double tet4_grads_p(const double p[4][3], double g[4][3]) {
    double e1[3], e2[3], e3[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        e1[k] = p[1][k] - p[0][k];
        e2[k] = p[2][k] - p[0][k];
        e3[k] = p[3][k] - p[0][k];
    }
    double c23[3] = {e2[1] * e3[2] - e2[2] * e3[1], e2[2] * e3[0] - e2[0] * e3[2], e2[0] * e3[1] - e2[1] * e3[0]};
    double c31[3] = {e3[1] * e1[2] - e3[2] * e1[1], e3[2] * e1[0] - e3[0] * e1[2], e3[0] * e1[1] - e3[1] * e1[0]};
    double c12[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    double det = e1[0] * c23[0] + e1[1] * c23[1] + e1[2] * c23[2];
    double inv = 1.0 / det;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g[1][k] = c23[k] * inv;
        g[2][k] = c31[k] * inv;
        g[3][k] = c12[k] * inv;
        g[0][k] = -(g[1][k] + g[2][k] + g[3][k]);
    }
    return det;
}

__device__ __forceinline__ double tet4_grads_n(const double* __restrict__ X, const int64_t c[4], double g[4][3]) {
    double p[4][3];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int64_t n = c[a];
#pragma unroll
        for (int k = 0; k < 3; ++k) p[a][k] = X[3 * n + k];
    }
    return tet4_grads_p(p, g);
}

__device__ __forceinline__ double tet4_grads(const double* __restrict__ X, const int64_t* __restrict__ c,
                                             double g[4][3]) {
    const int64_t n[4] = {c[0], c[1], c[2], c[3]};
    return tet4_grads_n(X, n, g);
}

// inverse of a row-major 3x3 Jacobian (cofactors), returns det
__device__ __forceinline__ double inv3(const double J[9], double Ji[9]) {
    const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8], c02 = J[3] * J[7] - J[4] * J[6];
    const double det = J[0] * c00 + J[1] * c01 + J[2] * c02;
    const double id = 1.0 / det;
    Ji[0] = c00 * id;
    Ji[1] = (J[2] * J[7] - J[1] * J[8]) * id;
    Ji[2] = (J[1] * J[5] - J[2] * J[4]) * id;
    Ji[3] = c01 * id;
    Ji[4] = (J[0] * J[8] - J[2] * J[6]) * id;
    Ji[5] = (J[2] * J[3] - J[0] * J[5]) * id;
    Ji[6] = c02 * id;
    Ji[7] = (J[1] * J[6] - J[0] * J[7]) * id;
    Ji[8] = (J[0] * J[4] - J[1] * J[3]) * id;
    return det;
}

}  // namespace fem
