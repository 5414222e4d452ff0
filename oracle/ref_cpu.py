"""ORACLE — test infrastructure only. CPU restatement of the reference's hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module, and
only as the checker / CPU baseline. The product path (the HIP library behind
`cuda-powered-mesh-handling-and-iterative-solvers_amd/`) never imports or calls it.

Every function restates one reference function of sml2004/CUDA-powered-mesh-handling-and-Iterative-solvers
(reference @ 2025-04-18, paths relative to its root) with the same batched torch-CPU op sequence, so it is
both the numerical oracle and a faithful timing stand-in for the reference's CPU path.
Quirks are kept on purpose (SURVEY.md §8(a) quirk register Q1-Q6).

Pinning: `tests/test_oracle_golden.py` checks every function here against `tests/golden/*.npz`, which
`tools/gen_golden.py` produced by importing the reference itself in the build container.
"""
from __future__ import annotations

import math

import torch

F64 = torch.float64


# ----------------------------------------------------------------------------- material / element algebra
def elasticity_matrix(E, nu, dtype=F64):
    """Isotropic 6x6 D, Voigt (xx,yy,zz,xy,yz,xz), engineering shear. `solver/element.py:282-306`."""
    c = E / ((1.0 + nu) * (1.0 - 2.0 * nu))
    g = (1.0 - 2.0 * nu) / 2.0
    D = torch.zeros((6, 6), dtype=dtype)
    D[:3, :3] = nu
    D[0, 0] = D[1, 1] = D[2, 2] = 1.0 - nu
    D[3, 3] = D[4, 4] = D[5, 5] = g
    return c * D


def _voigt_B(grads):
    """[M, n, 3] global shape gradients -> B [M, 6, 3n]; rows xx, yy, zz, xy, yz, xz
    (the strided fill of `solver/element.py:868-879`, `:1114-1123`, `:1683-1692`, `:2557-2566`)."""
    M, n, _ = grads.shape
    gx, gy, gz = grads[..., 0], grads[..., 1], grads[..., 2]
    B = torch.zeros((M, 6, n, 3), dtype=grads.dtype)
    B[:, 0, :, 0] = gx
    B[:, 1, :, 1] = gy
    B[:, 2, :, 2] = gz
    B[:, 3, :, 0] = gy
    B[:, 3, :, 1] = gx
    B[:, 4, :, 1] = gz
    B[:, 4, :, 2] = gy
    B[:, 5, :, 0] = gz
    B[:, 5, :, 2] = gx
    return B.reshape(M, 6, 3 * n)


# ----------------------------------------------------------------------------- c3d4
def tet_volumes(coords, elements):
    """|det[p1-p0, p2-p0, p3-p0]| / 6. `solver/element.py:514-541`."""
    p = coords[elements]
    edges = torch.stack([p[:, 1] - p[:, 0], p[:, 2] - p[:, 0], p[:, 3] - p[:, 0]], dim=1)
    return torch.det(edges).abs() / 6.0


def tet4_gradients(coords, elements):
    """Gradients of the 4 P1 shape functions: rows 1..3 of inv([1 x y z]). `solver/element.py:851-866`.
    Raises ValueError on |det| < 1e-12 exactly like `:857-858`. Returns [M, 4, 3] (node, xyz)."""
    p = coords[elements]
    A = torch.cat([torch.ones((p.shape[0], 4, 1), dtype=p.dtype), p], dim=2)
    if bool((torch.det(A).abs() < 1e-12).any()):
        raise ValueError("Singular matrix encountered while computing B matrix.")
    return torch.inverse(A)[:, 1:, :].transpose(1, 2)


def tet4_B(coords, elements):
    """`compute_c3d4_B_matrix`, `solver/element.py:835-881` -> [M, 6, 12]."""
    return _voigt_B(tet4_gradients(coords, elements))


def tet4_K(coords, elements, E, nu):
    """`compute_c3d4_K_matrix`, `solver/element.py:883-903`: K = B^T (D B) V -> [M, 12, 12]."""
    B = tet4_B(coords, elements)
    D = elasticity_matrix(E, nu, B.dtype)
    K = torch.matmul(B.transpose(1, 2), torch.matmul(D, B))
    return K * tet_volumes(coords, elements).view(-1, 1, 1)


def tet4_poisson_K(coords, elements, kappa=1.0):
    """Scalar P1 Laplacian K^P = kappa V G G^T -> [M, 4, 4]. No reference function exists;
    derived from the reference's own P1 gradients (`:851-866`) and volumes (`:514-541`)."""
    G = tet4_gradients(coords, elements)
    return kappa * torch.matmul(G, G.transpose(1, 2)) * tet_volumes(coords, elements).view(-1, 1, 1)


# ----------------------------------------------------------------------------- isoparametric solids
def hex8_points(dtype=F64):
    """2x2x2 Gauss, w = 1. `solver/element.py:1583-1599` (points ordered xi-major)."""
    a = 1.0 / math.sqrt(3.0)
    pts = torch.tensor([[sx * a, sy * a, sz * a] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)], dtype=dtype)
    return pts, torch.ones(8, dtype=dtype)


def hex8_dN(xi, eta, zeta, dtype=F64):
    """[8, 3] natural derivatives of the trilinear shape functions. `solver/element.py:1617-1626`."""
    s = ((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (-1, -1, 1), (1, -1, 1), (1, 1, 1), (-1, 1, 1))
    rows = []
    for (a, b, c) in s:
        rows.append([0.125 * a * (1 + b * eta) * (1 + c * zeta),
                     0.125 * b * (1 + a * xi) * (1 + c * zeta),
                     0.125 * c * (1 + a * xi) * (1 + b * eta)])
    return torch.tensor(rows, dtype=dtype)


def wedge6_points(dtype=F64):
    """3 triangle x 2 line points, w_tri = 1/3 (Q3: sums to 2). `solver/element.py:2448-2480`.
    The line points are formed from a float32 sqrt(3) in the reference, so they carry float32 rounding."""
    tri = [(1 / 6, 1 / 6), (2 / 3, 1 / 6), (1 / 6, 2 / 3)]
    r3 = float(1.0 / torch.sqrt(torch.tensor(3.0)))  # float32 value, as in the reference
    pts, w = [], []
    for (r, s) in tri:
        for t in (-r3, r3):
            pts.append([r, s, t])
            w.append(1.0 / 3.0)
    return torch.tensor(pts, dtype=dtype), torch.tensor(w, dtype=dtype)


def wedge6_dN(r, s, t, dtype=F64):
    """[6, 3] natural derivatives of the linear prism. `solver/element.py:2498-2505`."""
    return torch.tensor([
        [-0.5 * (1 - t), -0.5 * (1 - t), -0.5 * (1 - r - s)],
        [0.5 * (1 - t), 0.0, -0.5 * r],
        [0.0, 0.5 * (1 - t), -0.5 * s],
        [-0.5 * (1 + t), -0.5 * (1 + t), 0.5 * (1 - r - s)],
        [0.5 * (1 + t), 0.0, 0.5 * r],
        [0.0, 0.5 * (1 + t), 0.5 * s]], dtype=dtype)


def tet10_points(dtype=F64):
    """The reference's 11-point rule (weights sum to 0.45, Q2). `solver/element.py:995-1024`."""
    pts = [[0.25, 0.25, 0.25], [0.1, 0.1, 0.1], [0.1, 0.1, 0.7], [0.1, 0.7, 0.1], [0.7, 0.1, 0.1],
           [0.1, 0.4, 0.4], [0.4, 0.1, 0.4], [0.4, 0.4, 0.1], [0.3, 0.3, 0.3], [0.2, 0.2, 0.6], [0.2, 0.6, 0.2]]
    w = [0.1, 0.05, 0.05, 0.05, 0.05, 0.03, 0.03, 0.03, 0.02, 0.02, 0.02]
    return torch.tensor(pts, dtype=dtype), torch.tensor(w, dtype=dtype)


def tet10_dN(xi, eta, zeta, dtype=F64):
    """[10, 3] natural derivatives, reference node convention. `solver/element.py:1043-1054`."""
    L = 1 - xi - eta - zeta
    return torch.tensor([
        [4 * xi - 1, 0, 0], [0, 4 * eta - 1, 0], [0, 0, 4 * zeta - 1],
        [-4 * L + 1, -4 * L + 1, -4 * L + 1],
        [4 * eta, 4 * xi, 0], [0, 4 * zeta, 4 * eta], [4 * zeta, 0, 4 * xi],
        [4 * (1 - 2 * xi - eta - zeta), -4 * xi, -4 * xi],
        [-4 * eta, 4 * (1 - xi - 2 * eta - zeta), -4 * eta],
        [-4 * zeta, -4 * zeta, 4 * (1 - xi - eta - 2 * zeta)]], dtype=dtype)


DN = {"c3d8": hex8_dN, "c3d6": wedge6_dN, "c3d10": tet10_dN}
POINTS = {"c3d8": hex8_points, "c3d6": wedge6_points, "c3d10": tet10_points}


def iso_jacobian(coords, elements, dN):
    """J[m, i, k] = sum_j dN[j, i] x[m, j, k] (`einsum("ji,mjk->mik")`, e.g. `solver/element.py:1628`)."""
    return torch.einsum("ji,mjk->mik", dN, coords[elements])


def iso_gradients(coords, elements, dN):
    """Global gradients J^-1 dN (`einsum("mij,nj->mni")`, e.g. `solver/element.py:1660-1662`) -> [M, n, 3]."""
    Jinv = torch.inverse(iso_jacobian(coords, elements, dN))
    return torch.einsum("mij,nj->mni", Jinv, dN)


def wedge_volumes(coords, elements):
    """Sum of 3 sub-tet |volumes|. `solver/element.py:2198-2232`."""
    p = coords[elements]

    def vol(a, b, c, d):
        return torch.einsum("ij,ij->i", torch.cross(b - a, c - a, dim=1), d - a).abs() / 6.0
    return vol(p[:, 0], p[:, 1], p[:, 2], p[:, 3]) + vol(p[:, 1], p[:, 2], p[:, 4], p[:, 3]) + \
        vol(p[:, 2], p[:, 4], p[:, 5], p[:, 3])


def hex_volumes(coords, elements):
    """Sum of 6 sub-tet |det| / 6, in the reference's order. `solver/element.py:1248-1291`."""
    p = coords[elements]

    def vol(a, b, c, d):
        return torch.abs(torch.det(torch.stack([b - a, c - a, d - a], dim=1))) / 6.0
    return (vol(p[:, 0], p[:, 1], p[:, 3], p[:, 4]) + vol(p[:, 1], p[:, 2], p[:, 3], p[:, 6]) +
            vol(p[:, 1], p[:, 3], p[:, 4], p[:, 5]) + vol(p[:, 3], p[:, 4], p[:, 5], p[:, 7]) +
            vol(p[:, 3], p[:, 5], p[:, 6], p[:, 7]) + vol(p[:, 3], p[:, 5], p[:, 6], p[:, 1]))


def iso_K(coords, elements, etype, E, nu, points=None, weights=None, single=True):
    """`compute_c3d8_K_matrix` (`solver/element.py:1754-1803`), `compute_c3d10_K_matrix` (`:1191-1239`) and
    `compute_c3d6_K_matrix` (`:2631-2676`) in one restatement: sum_ip w * signed detJ * B^T D B.

    single=False returns the per-ip stack [n_ip, M, d, d] *without* weights for c3d8/c3d10 (Q6) and the
    weighted sum for c3d6 (whose `single` flag only selects the one-point rule).
    c3d6 single=True: B at (1/3, 1/3, 0) times the wedge volume (`:2656-2659`)."""
    D = elasticity_matrix(E, nu)
    if etype == "c3d6" and single:
        dN = wedge6_dN(1.0 / 3.0, 1.0 / 3.0, 0.0)
        B = _voigt_B(iso_gradients(coords, elements, dN))
        return torch.einsum("mji,jk,mkq->miq", B, D, B) * wedge_volumes(coords, elements).view(-1, 1, 1)
    if points is None:
        points, weights = POINTS[etype]()
    out = []
    K = None
    for q in range(points.shape[0]):
        dN = DN[etype](*[float(v) for v in points[q]])
        B = _voigt_B(iso_gradients(coords, elements, dN))
        detJ = torch.det(iso_jacobian(coords, elements, dN))
        if etype == "c3d8":      # contraction order of `solver/element.py:1793-1794`
            Kq = torch.einsum("mji,mjk->mik", B, torch.einsum("mji,kj->mki", B, D))
        elif etype == "c3d10":   # `solver/element.py:1229-1230`
            Kq = torch.einsum("mik,mkj->mij", torch.einsum("mji,jk->mik", B, D), B)
        else:                    # `solver/element.py:2672`
            Kq = torch.einsum("mji,jk,mkq->miq", B, D, B)
        Kq = Kq * detJ.view(-1, 1, 1)
        if etype == "c3d6" or single:
            Kq = Kq * float(weights[q])
            K = Kq if K is None else K + Kq
        else:
            out.append(Kq)
    return K if K is not None else torch.stack(out, 0)


def iso_mass(coords, elements, shape_values, shape_derivs, points, weights, rho):
    """Consistent mass of an isoparametric element family (no reference function: parity unpinned; the GPU kernel's
    specification restated): M_e = rho sum_q w_q |detJ_q| (N N^T)(q) (x) I3 -> [M, 3 npe, 3 npe]. shape_values /
    shape_derivs: callables (xi, eta, zeta) -> N [npe] / dN [npe, 3] in the element's node order."""
    M, npe = elements.shape
    m = torch.zeros((M, npe, npe), dtype=F64)
    for q in range(points.shape[0]):
        pq = [float(v) for v in points[q]]
        Nq = torch.tensor(shape_values(*pq), dtype=F64)
        dN = torch.as_tensor(shape_derivs(*pq), dtype=F64)
        detJ = torch.det(iso_jacobian(coords, elements, dN)).abs()
        m = m + (float(weights[q]) * rho) * detJ.view(-1, 1, 1) * torch.outer(Nq, Nq).view(1, npe, npe)
    return torch.kron(m, torch.eye(3, dtype=F64).view(1, 3, 3))


# ----------------------------------------------------------------------------- stress recovery
def stress_tensor(v):
    """Voigt [M,6] (xx, yy, zz, xy, yz, xz) -> [M,3,3]. `solver/element.py:308-330`."""
    t = torch.zeros((v.shape[0], 3, 3), dtype=v.dtype)
    for (i, j), k in (((0, 0), 0), ((1, 1), 1), ((2, 2), 2), ((0, 1), 3), ((1, 0), 3), ((0, 2), 5), ((2, 0), 5),
                      ((1, 2), 4), ((2, 1), 4)):
        t[:, i, j] = v[:, k]
    return t


def von_mises(t):
    """`solver/element.py:332-353` (upper-triangle shears)."""
    sxx, syy, szz = t[:, 0, 0], t[:, 1, 1], t[:, 2, 2]
    sxy, sxz, syz = t[:, 0, 1], t[:, 0, 2], t[:, 1, 2]
    return torch.sqrt(((sxx - syy) ** 2 + (syy - szz) ** 2 + (szz - sxx) ** 2 + 6 * (sxy ** 2 + syz ** 2 + sxz ** 2)) / 2)


def _point_stress(B, ue, D):
    strain = torch.bmm(B, ue.unsqueeze(2)).squeeze(2)     # [M,6]
    s = stress_tensor(torch.matmul(strain, D.t()))
    return s, von_mises(s)


def tet4_stress(coords, elements, u, E, nu):
    """`compute_c3d4_element_stress`, `solver/element.py:905-937` -> ([M,3,3], [M])."""
    ue = u[elements].reshape(elements.shape[0], -1)
    return _point_stress(tet4_B(coords, elements), ue, elasticity_matrix(E, nu))


def iso_stress(coords, elements, u, etype, E, nu, points=None, weights=None, single=True):
    """`compute_c3d8_element_stress` (`:1696-1752`), `compute_c3d6_element_stress` (`:2570-2629`): stack per point,
    single -> einsum("i,mijk->mjk") weights; `compute_c3d10_element_stress` (`:1127-1189`): single -> running
    `+= tensor * w` in point order, else a point-major stack."""
    if points is None:
        points, weights = POINTS[etype]()
    D = elasticity_matrix(E, nu)
    ue = u[elements].reshape(elements.shape[0], -1)
    M, n = elements.shape[0], points.shape[0]
    sig, vm = [], []
    acc_s, acc_v = torch.zeros((M, 3, 3), dtype=F64), torch.zeros(M, dtype=F64)
    for q in range(n):
        dN = DN[etype](*[float(v) for v in points[q]])
        s, v = _point_stress(_voigt_B(iso_gradients(coords, elements, dN)), ue, D)
        if etype == "c3d10" and single:
            acc_s += s * weights[q]
            acc_v += v * weights[q]
        sig.append(s)
        vm.append(v)
    if etype == "c3d10":
        return (acc_s, acc_v) if single else (torch.stack(sig, 0), torch.stack(vm, 0))
    S, V = torch.stack(sig, 1), torch.stack(vm, 1)     # [M,n,3,3], [M,n]
    if single:
        return torch.einsum("i,mijk->mjk", weights, S), torch.einsum("i,mi->m", weights, V)
    return S, V


def node_average(elements, ev, N):
    """`compute_node_vm_stress`, `solver/element.py:466-504`: index_add sums / counts, 0 where unused."""
    idx = elements.reshape(-1)
    vals = ev.repeat_interleave(elements.shape[1])
    s = torch.zeros(N, dtype=ev.dtype).index_add(0, idx, vals)
    c = torch.zeros(N, dtype=ev.dtype).index_add(0, idx, torch.ones_like(vals))
    return torch.where(c > 0, s / c, torch.zeros_like(s))


def face_forces(normals, sig):
    """`compute_c3d4_surface_forces`, `solver/element.py:3343-3362`."""
    return torch.matmul(sig.unsqueeze(1), normals.unsqueeze(-1)).squeeze(-1)


def shared_face_sum(idx, ff):
    """`compute_c3d4_shared_face_forces_sum`, `solver/element.py:3364-3382`."""
    return ff[idx[:, 0, 0], idx[:, 0, 1], :] + ff[idx[:, 1, 0], idx[:, 1, 1], :]


# ----------------------------------------------------------------------------- operator / preconditioner
def dof_map(elements, dpn):
    """dof = dpn*node + comp, element-major (`solver/element.py:451-452`)."""
    return (elements.unsqueeze(-1) * dpn + torch.arange(dpn).view(1, 1, dpn)).reshape(elements.shape[0], -1)


def nodal_forces(K, elements, u):
    """EBE y = sum_e P_e^T K_e P_e u. `compute_nodal_forces`, `solver/element.py:429-464`.
    dpn is K.shape[-1] / nodes-per-element (3 in the reference; 1 for the scalar Poisson system)."""
    M, d = K.shape[0], K.shape[-1]
    dpn = d // elements.shape[1]
    dofs = dof_map(elements, dpn)
    ue = u.reshape(-1)[dofs]
    fe = torch.bmm(K, ue.unsqueeze(-1)).squeeze(-1)
    y = torch.zeros(u.numel(), dtype=K.dtype).index_add(0, dofs.reshape(-1), fe.reshape(-1))
    return y.view(u.shape)


# ----------------------------------------------------------------------------- element product without K_e
def _lame(E, nu):
    c = E / ((1.0 + nu) * (1.0 - 2.0 * nu))
    return c * nu, c * ((1.0 - 2.0 * nu) / 2.0)


def tet4_cofactors(coords, elements):
    """Cofactor vectors c [M,4,3] (c_1 = e_2 x e_3, c_2 = e_3 x e_1, c_3 = e_1 x e_2, c_0 = -(c_1 + c_2 + c_3), with
    e_b = x_b - x_0) and det [M]: the P1 gradients are c_b / det and V = |det| / 6 (`solver/element.py:835-881`,
    `:514-541` restated without the 4x4 inverse)."""
    x = coords[elements]
    e = x[:, 1:, :] - x[:, :1, :]
    c1 = torch.cross(e[:, 1], e[:, 2], dim=1)
    c2 = torch.cross(e[:, 2], e[:, 0], dim=1)
    c3 = torch.cross(e[:, 0], e[:, 1], dim=1)
    return torch.stack([-(c1 + c2 + c3), c1, c2, c3], 1), (e[:, 0] * c1).sum(1)


def tet4_element_forces(coords, elements, u, kind="elastic", E=1.0, nu=0.0):
    """Element vectors f_e = K_e u_e [M,4,dpn] of the c3d4 stiffness (`compute_c3d4_K_matrix`, `solver/element.py:
    883-903`) or the P1 Laplacian (kappa = E), formed in closed form from the cofactors -- what the element-chunk
    operator (csrc/matfree.hpp mf_element) evaluates: f_a = s sigma(H) c_a with H = sum_b (u_b - u_0) c_b^T,
    sigma(H) = lambda tr(H) I + mu (H + H^T), s = 1 / (6 |det|); Poisson f_a = kappa s c_a . sum_b c_b (u_b - u_0).
    Equal to the K_e product up to rounding (tests/test_matfree_cpu.py pins it to tet4_K / tet4_poisson_K)."""
    c, det = tet4_cofactors(coords, elements)
    s = 1.0 / (6.0 * det.abs())
    if kind == "poisson":
        ue = u.reshape(-1)[elements]
        gu = torch.einsum("mbk,mb->mk", c[:, 1:, :], ue[:, 1:] - ue[:, :1])
        return (E * s)[:, None, None] * torch.einsum("mak,mk->ma", c, gu).unsqueeze(-1)
    lam, mu = _lame(E, nu)
    ue = u.reshape(-1, 3)[elements]
    d = ue[:, 1:, :] - ue[:, :1, :]
    H = torch.einsum("mbi,mbj->mij", d, c[:, 1:, :])
    tr = H.diagonal(dim1=1, dim2=2).sum(1)
    sig = lam * tr[:, None, None] * torch.eye(3, dtype=F64) + mu * (H + H.transpose(1, 2))
    return torch.einsum("mij,maj->mai", sig * s[:, None, None], c)


def tet4_forces_matfree(coords, elements, u, kind="elastic", E=1.0, nu=0.0):
    """y = sum_e P_e^T f_e: the reference's element-by-element product (`solver/element.py:429-464`: gather, local
    product, index_add) with the closed-form element vectors instead of a stored K_e. u [N*dpn] -> y [N*dpn]."""
    dpn = 1 if kind == "poisson" else 3
    f = tet4_element_forces(coords, elements, u, kind, E, nu)
    y = torch.zeros(coords.shape[0] * dpn, dtype=F64)
    return y.index_add_(0, dof_map(elements, dpn).reshape(-1), f.reshape(-1))


def tet4_diag_matfree(coords, elements, kind="elastic", E=1.0, nu=0.0):
    """The exact diagonal of the same operator from the cofactors: (K_aa)_qq = s ((lambda + mu) c_aq^2 + mu |c_a|^2),
    Poisson kappa s |c_a|^2 (csrc/matfree.hpp MF_DIAG). [N*dpn]."""
    c, det = tet4_cofactors(coords, elements)
    s = 1.0 / (6.0 * det.abs())
    cc = (c * c).sum(2)
    if kind == "poisson":
        dv, dpn = (E * s)[:, None] * cc, 1
    else:
        lam, mu = _lame(E, nu)
        dv, dpn = s[:, None, None] * ((lam + mu) * c * c + mu * cc[:, :, None]), 3
    y = torch.zeros(coords.shape[0] * dpn, dtype=F64)
    return y.index_add_(0, dof_map(elements, dpn).reshape(-1), dv.reshape(-1))


def diag_preconditioner(K, elements, N, dpn=3, compat_colzero=False):
    """`compute_diagonal_preconditioner`, `solver/solver.py:814-833`.
    compat_colzero=True reproduces the reference slice bug (Q1: column 0 of every element row, `:828`);
    the default returns 1/diag(K) with inf -> 0, the function's documented intent."""
    d = K.shape[-1]
    dofs = dof_map(elements, dpn).reshape(-1)
    if compat_colzero:
        entries = K.reshape(-1, d)[:, ::d + 1].reshape(-1)
    else:
        entries = torch.diagonal(K, dim1=1, dim2=2).reshape(-1)
    diag = torch.zeros(N * dpn, dtype=K.dtype).index_add_(0, dofs, entries)
    Minv = 1.0 / diag
    Minv[Minv == float("inf")] = 0.0
    return Minv.view(N, dpn)


# ----------------------------------------------------------------------------- solvers
def stable_cg(K, elements, F, fixed, u_init=None, tol=1e-10, max_iter=1000, eps=1e-30, history=None,
              verbose=False):
    """`stable_conjugate_gradient_solver`, `solver/solver.py:144-229`. Returns (u, iterations, status)
    with status in {"converged", "max_iter", "breakdown_pAp", "alpha_nan", "beta_nan"}.
    `history` (a list) receives ||r_k|| after every iteration (the reference does not return it)."""
    u = torch.zeros_like(F) if u_init is None else u_init.clone().to(F.dtype)
    u[fixed] = 0.0
    r = F - nodal_forces(K, elements, u)
    r[fixed] = 0.0
    p = r.clone()
    rs_old = torch.sum(r * r)
    for i in range(max_iter):
        Ap = nodal_forces(K, elements, p)
        pAp = torch.sum(p * Ap)
        if pAp.abs() < eps or pAp < 0.0:
            return u, i + 1, "breakdown_pAp"
        alpha = rs_old / (pAp + eps)
        if torch.isnan(alpha) or torch.isinf(alpha):
            return u, i + 1, "alpha_nan"
        u += alpha * p
        u[fixed] = 0.0
        r -= alpha * Ap
        r[fixed] = 0.0
        rs_new = torch.sum(r * r)
        if history is not None:
            history.append(float(torch.sqrt(rs_new)))
        if torch.sqrt(rs_new) < tol:
            if verbose:
                print(f"Converged after {i+1} iterations. Residual norm: {rs_new.item():.3e}")
            return u, i + 1, "converged"
        beta = rs_new / (rs_old + eps)
        if torch.isnan(beta) or torch.isinf(beta):
            return u, i + 1, "beta_nan"
        p = r + beta * p
        p[fixed] = 0.0
        rs_old = rs_new
    return u, max_iter, "max_iter"


def pcg(K, elements, F, M_inv, u_init=None, tol=1e-8, max_iter=1000, history=None, matvec=None):
    """`preconditioned_conjugate_gradient_solver`, `solver/solver.py:766-812` (no eps, no guards,
    stop on sqrt(r.z) < tol). `matvec` overrides the EBE operator (used for CSR timing)."""
    A = matvec or (lambda v: nodal_forces(K, elements, v))
    u = torch.zeros_like(F) if u_init is None else u_init.clone().to(F.dtype)
    r = F - A(u)
    z = M_inv * r
    p = z.clone()
    rs_old = torch.sum(r * z)
    for i in range(max_iter):
        Ap = A(p)
        alpha = rs_old / torch.sum(p * Ap)
        u += alpha * p
        r -= alpha * Ap
        z = M_inv * r
        rs_new = torch.sum(r * z)
        if history is not None:
            history.append(float(torch.sqrt(rs_new)))
        if torch.sqrt(rs_new) < tol:
            return u, i + 1, "converged"
        p = z + (rs_new / rs_old) * p
        rs_old = rs_new
    return u, max_iter, "max_iter"


# ---------------------------------------------------------------- constraints (`solver/solver.py:394-759`)
def enforce(u, r, rbe2_list, spc_list, rbe3_list=None):
    """`enforce_constraints` (:478-510, rbe3_list None: RBE2 then SPC) or `new_enforce_constraints`
    (:665-700: SPC, RBE2, then every RBE3 per distinct dof in ascending order). u, r: [N, dpn], in place."""
    # flattened in the order of `parse_rbe2_list` (:437-476: rbe2 -> slave -> dof) / `parse_spc_list` (:396-435)
    rbe2 = [(sl, c["master"], d) for c in rbe2_list for sl in c["slaves"] for d in c["dofs"]]
    spc = [(c["node"], d, float(c["value"])) for c in spc_list for d in c["dofs"]]

    def _rbe2():
        if rbe2:
            s, m, d = (torch.tensor(v) for v in zip(*rbe2))
            u[s, d] = u[m, d]
            r[s, d] = 0.0

    def _spc():
        if spc:
            n, d, v = zip(*spc)
            n, d = torch.tensor(n), torch.tensor(d)
            u[n, d] = torch.tensor(v, dtype=u.dtype)
            r[n, d] = 0.0

    if rbe3_list is None:
        _rbe2()
        _spc()
        return
    _spc()
    _rbe2()
    for c in rbe3_list:
        w = torch.tensor([float(x) for x in c["weights"]], dtype=u.dtype)
        w_sum = torch.tensor(float(sum(c["weights"])), dtype=u.dtype)
        slaves = torch.tensor(c["slaves"])
        for d in sorted(set(c["dofs"])):
            u[c["master"], d] = torch.sum(w * u[slaves, d]) / (w_sum + 1e-30)


def constrained_cg(K, elements, F, rbe2_list, spc_list, rbe3_list=None, u_init=None, tol=1e-10, max_iter=1000,
                   eps=1e-30, history=None):
    """`constrained_conjugate_gradient_solver` (:512-600; rbe3_list None) and the loop of
    `new_constrained_conjugate_gradient_solver` (:702-759; rbe3_list given, F already built by the loads).
    r0 = F - K u0 is formed BEFORE the first projection, as in the reference. Returns (u, iterations, status)."""
    u = torch.zeros_like(F) if u_init is None else u_init.clone().to(F.dtype)
    r = F - nodal_forces(K, elements, u)
    enforce(u, r, rbe2_list, spc_list, rbe3_list)
    p = r.clone()
    rs_old = torch.sum(r * r)
    for i in range(max_iter):
        Ap = nodal_forces(K, elements, p)
        pAp = torch.sum(p * Ap)
        if pAp.abs() < eps or pAp < 0.0:
            return u, i + 1, "breakdown_pAp"
        alpha = rs_old / (pAp + eps)
        if torch.isnan(alpha) or torch.isinf(alpha):
            return u, i + 1, "alpha_nan"
        u += alpha * p
        r -= alpha * Ap
        enforce(u, r, rbe2_list, spc_list, rbe3_list)
        rs_new = torch.sum(r * r)
        if history is not None:
            history.append(float(torch.sqrt(rs_new)))
        if torch.sqrt(rs_new) < tol:
            return u, i + 1, "converged"
        beta = rs_new / (rs_old + eps)
        if torch.isnan(beta) or torch.isinf(beta):
            return u, i + 1, "beta_nan"
        p = r + beta * p
        rs_old = rs_new
    return u, max_iter, "max_iter"


def loads_to_F(N, load_list, dtype=F64):
    """`apply_loads_to_F` (:653-663) into a fresh [N, 3] array."""
    F = torch.zeros((N, 3), dtype=dtype)
    for ld in load_list:
        for d in range(3):
            F[ld["node"], d] += ld["force"][d]
    return F


def static_structure(coords, force, fixed, blocks, E, nu, u_init=None, tol=1e-10, max_iter=1000, eps=1e-30):
    """`static_structure_solver`, `solver/solver.py:11-135`, solid families only (shells are out of scope).
    `blocks` = {"c3d4": elems, "c3d8": elems, "c3d6": elems}; c3d8 uses the 8-point rule, c3d6 single=True.
    Returns (u [N,6], iterations, status)."""
    Ks = []
    for et in ("c3d4", "c3d8", "c3d6"):      # the reference's family order, `solver/solver.py:61-72`
        el = blocks.get(et)
        if el is None:
            continue
        Ke = tet4_K(coords, el, E, nu) if et == "c3d4" else iso_K(coords, el, et, E, nu)
        Ks.append((Ke, el))
    N = coords.shape[0]
    u = torch.zeros((N, 6), dtype=F64) if u_init is None else u_init.clone().to(F64)
    u[fixed] = 0.0

    def apply(v):
        out = torch.zeros((N, 6), dtype=F64)
        for Ke, el in Ks:
            out[:, :3] += nodal_forces(Ke, el, v[:, :3].contiguous())
        return out
    r = force - apply(u)
    r[fixed] = 0.0
    p = r.clone()
    rs_old = torch.sum(r * r)
    for i in range(max_iter):
        Ap = apply(p)
        pAp = torch.sum(p * Ap)
        if pAp.abs() < eps or pAp < 0.0:
            return u, i + 1, "breakdown_pAp"
        alpha = rs_old / (pAp + eps)
        if torch.isnan(alpha) or torch.isinf(alpha):
            return u, i + 1, "alpha_nan"
        u += alpha * p
        u[fixed] = 0.0
        r -= alpha * Ap
        r[fixed] = 0.0
        rs_new = torch.sum(r * r)
        if torch.sqrt(rs_new) < tol:
            return u, i + 1, "converged"
        beta = rs_new / (rs_old + eps)
        if torch.isnan(beta) or torch.isinf(beta):
            return u, i + 1, "beta_nan"
        p = r + beta * p
        p[fixed] = 0.0
        rs_old = rs_new
    return u, max_iter, "max_iter"


# ----------------------------------------------------------------------------- global assembly
def coo_to_csr(K, elements, dpn):
    """Global matrix = coalesce(COO) of `subdivision.ipynb:118-139` (rows = dof_i repeated, cols = dof_j
    tiled, values = K.view(-1)); returned as CSR (rowptr int64, colidx int64, vals) with sorted columns
    and duplicates summed. Also the pattern oracle for the HIP pattern builder (bit-exact)."""
    M, d = K.shape[0], K.shape[-1]
    dofs = dof_map(elements, dpn)
    rows = dofs.unsqueeze(2).expand(M, d, d).reshape(-1)
    cols = dofs.unsqueeze(1).expand(M, d, d).reshape(-1)
    n = int(elements.max()) + 1
    S = torch.sparse_coo_tensor(torch.stack([rows, cols]), K.reshape(-1), (n * dpn, n * dpn)).coalesce()
    idx = S.indices()
    counts = torch.bincount(idx[0], minlength=n * dpn)
    rowptr = torch.zeros(n * dpn + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(counts, 0)
    return rowptr, idx[1].clone(), S.values().clone()


def node_pattern(elements, n_nodes):
    """Scalar node-graph pattern (the block pattern of every dpn): sorted unique (i, j) over all element
    node pairs. Returns (rowptr int64 [N+1], colidx int64)."""
    npe = elements.shape[1]
    r = elements.unsqueeze(2).expand(-1, npe, npe).reshape(-1)
    c = elements.unsqueeze(1).expand(-1, npe, npe).reshape(-1)
    key = torch.unique(r * n_nodes + c)
    rows, cols = key // n_nodes, key % n_nodes
    rowptr = torch.zeros(n_nodes + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n_nodes), 0)
    return rowptr, cols


def csr_matvec(rowptr, colidx, vals, x):
    """y = A x for a CSR matrix (row-sequential sums)."""
    rows = torch.repeat_interleave(torch.arange(rowptr.numel() - 1), rowptr[1:] - rowptr[:-1])
    return torch.zeros(rowptr.numel() - 1, dtype=vals.dtype).index_add_(0, rows, vals * x[colidx])


def partition_local_maps(elements, element_ids):
    """Global->local node map of one element group: `torch.unique` of its nodes, `subdivision.ipynb:254-259`.
    Returns (global node ids sorted, local connectivity)."""
    elems = elements[element_ids]
    g, inv = torch.unique(elems, return_inverse=True)
    return g, inv.reshape(elems.shape)


# ----------------------------------------------------------------------------- mesh topology
def boundary_faces(elements, table, extra):
    """`compute_tetrahedral_surface_faces_with_fourth_node` (`solver/element.py:543-579`) and the hex / wedge
    variants (`:1293-1334`, `:2234-2283`): faces seen once, face-major order, plus their extra node."""
    faces = torch.cat([elements[:, list(r)] for r in table], 0)
    xs = torch.cat([elements[:, x] for x in extra], 0)
    _, inv, cnt = torch.unique(torch.sort(faces, dim=1)[0], dim=0, return_inverse=True, return_counts=True)
    m = cnt[inv] == 1
    return faces[m], xs[m]


def shared_faces(elements, table):
    """`identify_tetrahedral_shared_faces` (`:707-762`) / `identify_hexahedral_shared_faces` (`:1474-1532`)."""
    M, F = elements.shape[0], len(table)
    flat = torch.sort(elements[:, torch.tensor(table)], dim=2)[0].reshape(-1, len(table[0]))
    eid = torch.arange(M).repeat_interleave(F)
    fid = torch.tile(torch.arange(F), (M,))
    _, inv, cnt = torch.unique(flat, return_inverse=True, return_counts=True, dim=0)
    ids = torch.nonzero(cnt == 2, as_tuple=True)[0]
    if ids.numel() == 0:
        return torch.empty((0, 2, 2), dtype=torch.long)
    sinv, order = torch.sort(inv)
    pos = torch.searchsorted(sinv, ids)
    e, f = eid[order], fid[order]
    return torch.stack([torch.stack([e[pos], f[pos]], 1), torch.stack([e[pos + 1], f[pos + 1]], 1)], 1)


def surface_normals(coords, faces, extra, v2):
    """`compute_tetrahdral_surface_normals` (`:581-619`), hex (`:1336-1374`), wedge (`:2285-2338`)."""
    p = coords[faces]
    n = torch.cross(p[:, 1] - p[:, 0], p[:, v2] - p[:, 0], dim=1)
    n = n / torch.norm(n, dim=1, keepdim=True)
    t = coords[extra] - p.mean(dim=1)
    t = t / torch.norm(t, dim=1, keepdim=True)
    d = (n * t).sum(dim=1)
    n[d > 0] = -n[d > 0]
    return n


def element_face_normals(coords, elements, table, edge_rows, extra=None, scale=1.0, unit=False):
    """`compute_tetrahedral_normals_and_area` (`:652-705`, scale 1/2), hex (`:1418-1472`), wedge (`:2377-2422`,
    unit, no orientation): (p[r1]-p[r0]) x (p[r2]-p[r0]) per face row."""
    ce = coords[elements]
    outs = []
    for f, (a0, a1, a2) in enumerate(edge_rows):
        n = torch.cross(ce[:, a1] - ce[:, a0], ce[:, a2] - ce[:, a0], dim=1)
        if scale != 1.0:
            n = n / (1.0 / scale)
        outs.append(n)
    n = torch.stack(outs, 1)
    if unit:
        n = n / torch.norm(n, dim=2, keepdim=True)
    if extra is not None:
        cen = torch.stack([ce[:, list(r)].mean(dim=1) for r in table], 1)
        d = torch.sum(n * (coords[elements[:, list(extra)]] - cen), dim=2)
        n[d > 0] = -n[d > 0]
    return n


def unique_edges(elements, edges):
    """`element_to_edge`, `:2687-2713`."""
    e = torch.sort(elements[:, torch.tensor(edges)].view(-1, 2), dim=1)[0]
    return torch.unique(e, dim=0).t()


def split_elements(elements, table):
    """`c3d8_to_c3d4` (`:1555-1581`), `c3d6_to_c3d4` (`:2424-2446`), `c3d10_to_c3d4` (`:963-993`)."""
    return elements[:, torch.tensor(table)].reshape(-1, len(table[0]))
