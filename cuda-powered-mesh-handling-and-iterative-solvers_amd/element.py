"""Reference-compatible element API (`solver/element.py` of sml2004/CUDA-powered-mesh-handling-and-Iterative-
solvers @ 2025-04-18), executed by the fem355 HIP kernels.

Same function names, arguments, defaults (device="cuda:0") and return shapes as the reference, so its
notebook call sites work unchanged. Differences, all deliberate:
  * arithmetic is always fp64 on the MI355X; `dtype` only selects the dtype of the returned tensor;
  * a `device="cpu"` request is computed on the current HIP device and the result is returned on the CPU
    (there is no CPU code path in this package: see `_capi.lib()`);
  * integration-point tables are evaluated on the host exactly as the reference evaluates them (including its
    quirks: c3d10 weights summing to 0.45, the float32-rounded line points of c3d6), then handed to the kernels.
Out of scope: shells, topology, visualisation, c3d20/c3d15.
"""
from __future__ import annotations

import ctypes
import math
import os
import warnings
from collections import OrderedDict

import torch

try:  # package import (fem355.element) or the reference's flat import (`from element import *`)
    from . import _capi as C
    from . import system as _sys
except ImportError:  # pragma: no cover - exercised by the notebook-style loader test
    import _capi as C  # type: ignore
    import system as _sys  # type: ignore

F64 = torch.float64
LONG = torch.long

__all__ = [
    "human_readable_number", "vtk_loader_to_torch", "read_vtk", "compute_elasticity_matrix", "integral_points",
    "compute_Jacobian", "compute_shape_gradients", "compute_B_matrix", "compute_K_matrix", "compute_nodal_forces",
    "compute_tetrahedral_volumes", "compute_c3d4_B_matrix", "compute_c3d4_K_matrix", "compute_L_matrix",
    "compute_c3d4_M_matrix", "compute_c3d4_poisson_K_matrix",
    "c3d8_integration_points", "compute_c3d8_Jacobian", "compute_c3d8_shape_gradients", "compute_c3d8_B_matrix",
    "compute_c3d8_K_matrix",
    "c3d6_integration_points", "compute_c3d6_Jacobian", "compute_c3d6_shape_gradients", "compute_c3d6_B_matrix",
    "compute_c3d6_K_matrix", "compute_wedge_volumes",
    "c3d10_integration_points", "compute_c3d10_Jacobian", "compute_c3d10_shape_gradients", "compute_c3d10_B_matrix",
    "compute_c3d10_K_matrix",
    "mass_integration_points", "compute_c3d8_M_matrix", "compute_c3d6_M_matrix", "compute_c3d10_M_matrix",
    "compute_M_matrix",
]


# ============================================================================ utilities
def human_readable_number(num):
    """`solver/element.py:23-37` (used by the CG progress print)."""
    for lim, suf in ((1e18, "Quint"), (1e15, "Quad"), (1e12, "T"), (1e9, "B"), (1e6, "M"), (1e3, "K")):
        if abs(num) >= lim:
            return f"{num / lim:.1f}{suf}"
    return f"{num:.1f}"


_VTK_NPE = {"c3d4": 4, "c3d10": 10, "c3d8": 8, "c3d20": 20, "c3d6": 6, "c3d15": 15, "s3": 3, "s6": 6, "s4": 4,
            "s8": 8}
_VTK_CODE = {10: "c3d4", 24: "c3d10", 12: "c3d8", 25: "c3d20", 13: "c3d6", 26: "c3d15", 5: "s3", 22: "s6", 9: "s4",
             23: "s8"}


def read_vtk(file_path):
    """Parse a legacy VTK unstructured grid with the native reader (`csrc/vtk.cpp`, host only) ->
    (points [N,3] float64 numpy, count-prefixed cell array int64 numpy, cell types int64 numpy)."""
    import numpy as np
    lib = C.load_library()
    path = os.fspath(file_path)
    if not os.path.exists(path):
        raise FileNotFoundError(f"File '{path}' does not exist.")
    h = ctypes.c_void_p()
    C.check(lib.fem_vtk_read(path.encode(), ctypes.byref(h)), "fem_vtk_read")
    try:
        n = [ctypes.c_int64() for _ in range(4)]
        lib.fem_vtk_sizes(h, *[ctypes.byref(v) for v in n])
        npts, _, clen, ntyp = (v.value for v in n)
        pts = np.empty((npts, 3), dtype=np.float64)
        cells = np.empty(clen, dtype=np.int64)
        types = np.empty(ntyp, dtype=np.int64)
        lib.fem_vtk_copy(h, pts.ctypes.data_as(ctypes.c_void_p), cells.ctypes.data_as(ctypes.c_void_p),
                         types.ctypes.data_as(ctypes.c_void_p))
    finally:
        lib.fem_vtk_free(h)
    return pts, cells, types


def infer_vtk_element_type(cell_types):
    """Element type name of a homogeneous VTK cell-type array (VTK codes: 10 tetra, 24 quadratic tetra, 12
    hexahedron, 25 quadratic hexahedron, 13 wedge, 26 quadratic wedge, 5 triangle, 22 quadratic triangle, 9 quad,
    23 quadratic quad). ValueError for an empty, mixed or unsupported cell set."""
    import numpy as np
    kinds = np.unique(np.asarray(cell_types, dtype=np.int64))
    if kinds.size != 1:
        raise ValueError("Cannot infer the element type: the file holds "
                         + ("no cells." if kinds.size == 0 else f"mixed VTK cell types {kinds.tolist()}."))
    code = int(kinds[0])
    if code not in _VTK_CODE:
        raise ValueError(f"Cannot infer the element type: unsupported VTK cell type {code}.")
    return _VTK_CODE[code]


def vtk_loader_to_torch(file_path, element_type=None, device="cuda:0", dtype=torch.float32):
    """(points [N,3], connectivity [M,npe]) from a VTK file: the count-prefixed cell array reshaped to
    [-1, npe+1] with the count column dropped, exactly as `solver/element.py:39-90` does with pyvista's
    mesh.cells (so mixed cell sizes fail the same way). ValueError("Invalid element type.") for other types.
    `element_type=None` (the one-argument call of `solver_example.ipynb:82`, written against an older
    reference API) takes the type from the file's homogeneous cell types (`infer_vtk_element_type`)."""
    pts, cells, types = read_vtk(file_path)
    if element_type is None:
        element_type = infer_vtk_element_type(types)
    points = torch.tensor(pts, device=device, dtype=dtype)
    if element_type not in _VTK_NPE:
        raise ValueError("Invalid element type.")
    npe = _VTK_NPE[element_type]
    element = torch.tensor(cells.reshape(-1, npe + 1)[:, 1:], device=device, dtype=torch.long)
    return points, element


def _dev(device):
    return C.compute_device(device)


def _prep(coords, elements, device):
    dev = _dev(device)
    coords = coords.to(device=dev, dtype=F64).contiguous()
    elements = elements.to(device=dev, dtype=LONG).contiguous()
    _sys.check_connectivity(elements, coords.shape[0])
    return dev, coords, elements


def _out(t, device, dtype):
    return t.to(device=torch.device(device), dtype=dtype)


def compute_elasticity_matrix(E, nu, device="cuda:0", dtype=torch.float32):
    """Isotropic 6x6 D, Voigt (xx,yy,zz,xy,yz,xz), engineering shear. `solver/element.py:282-306`."""
    coef = E / ((1 + nu) * (1 - 2 * nu))
    g = (1 - 2 * nu) / 2
    rows = [[1 - nu, nu, nu, 0, 0, 0], [nu, 1 - nu, nu, 0, 0, 0], [nu, nu, 1 - nu, 0, 0, 0],
            [0, 0, 0, g, 0, 0], [0, 0, 0, 0, g, 0], [0, 0, 0, 0, 0, g]]
    return coef * torch.tensor(rows, device=device, dtype=dtype)


# ============================================================================ c3d4
def _bad_scalar(dev, M):
    return torch.full((1,), M, dtype=torch.int64, device=dev)


def _raise_if_singular(bad, M):
    if int(bad.item()) < M:
        raise ValueError("Singular matrix encountered while computing B matrix.")


def _tet4_geom(coords, elements, device, want_vol=False, want_B=False, check=True):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    M = elements.shape[0]
    vol = torch.empty(M, dtype=F64, device=dev) if want_vol else None
    B = torch.empty((M, 6, 12), dtype=F64, device=dev) if want_B else None
    bad = _bad_scalar(dev, M) if check else None
    C.check(lib.fem_tet4_geom(C.ptr(coords), C.ptr(elements), M, C.ptr(vol), None, C.ptr(B), C.ptr(bad),
                              C.stream(dev)), "fem_tet4_geom")
    if check:
        _raise_if_singular(bad, M)
    return vol, B


def compute_tetrahedral_volumes(coords, elements, device="cuda:0", dtype=torch.float32):
    """|det[p1-p0, p2-p0, p3-p0]|/6 -> [M]. `solver/element.py:514-541`."""
    vol, _ = _tet4_geom(coords, elements, device, want_vol=True, check=False)
    return _out(vol, device, dtype)


def compute_c3d4_B_matrix(coords, elements, device="cuda:0", dtype=torch.float32):
    """Strain-displacement matrix [M,6,12]; ValueError on |det| < 1e-12. `solver/element.py:835-881`."""
    _, B = _tet4_geom(coords, elements, device, want_B=True)
    return _out(B, device, dtype)


def _tet4_ke(coords, elements, a, b, kind, device, dtype):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    M = elements.shape[0]
    d = 4 if kind == C.KIND_POISSON else 12
    K = torch.empty((M, d, d), dtype=F64, device=dev)
    bad = _bad_scalar(dev, M)
    C.check(lib.fem_tet4_ke(C.ptr(coords), C.ptr(elements), M, float(a), float(b), kind, C.ptr(K), C.ptr(bad),
                            C.stream(dev)), "fem_tet4_ke")
    if kind != C.KIND_MASS:
        _raise_if_singular(bad, M)
    return _out(K, device, dtype)


def compute_c3d4_K_matrix(coords, elements, E, nu, device="cuda:0", dtype=torch.float32):
    """K_e = B^T D B V -> [M,12,12]. `solver/element.py:883-903`."""
    return _tet4_ke(coords, elements, E, nu, C.KIND_ELASTIC, device, dtype)


def compute_L_matrix(coords, elements, E, nu, device="cuda:0", dtype=torch.float32):
    """Name used by `solver_example.ipynb:96` for the c3d4 stiffness (stale API of the reference)."""
    return compute_c3d4_K_matrix(coords, elements, E, nu, device=device, dtype=dtype)


def compute_c3d4_M_matrix(coords, elements, rho, device="cuda:0", dtype=torch.float32):
    """Consistent P1 mass [M,12,12] = rho V (1 + delta_ab)/20 per component. Called at
    `solver_example.ipynb:221` but defined nowhere in the reference: parity unpinned."""
    return _tet4_ke(coords, elements, rho, 0.0, C.KIND_MASS, device, dtype)


def compute_c3d4_poisson_K_matrix(coords, elements, kappa=1.0, device="cuda:0", dtype=torch.float32):
    """Scalar P1 Laplacian kappa V G G^T -> [M,4,4] (no reference function: derived from the reference's
    c3d4 gradients and volumes). Used with dofs-per-node 1 everywhere below."""
    return _tet4_ke(coords, elements, kappa, 0.0, C.KIND_POISSON, device, dtype)


# ============================================================================ isoparametric solids
def c3d8_integration_points(device="cuda:0", dtype=torch.float32):
    """2x2x2 Gauss, w=1, xi-major order. `solver/element.py:1583-1599`."""
    a = 1.0 / torch.sqrt(torch.tensor(3.0, dtype=dtype, device=device))
    s = [(-1, -1, -1), (-1, -1, 1), (-1, 1, -1), (-1, 1, 1), (1, -1, -1), (1, -1, 1), (1, 1, -1), (1, 1, 1)]
    pts = torch.stack([torch.stack([u * a, v * a, w * a]) for (u, v, w) in s])
    return pts, torch.ones(8, dtype=dtype, device=device)


def c3d6_integration_points(device="cuda:0", dtype=torch.float32):
    """3 triangle points x 2 line points, triangle weight 1/3 (weights sum to 2, quirk Q3); the line points come
    from a float32 sqrt(3) exactly as in `solver/element.py:2448-2480`."""
    tri = [(1 / 6, 1 / 6), (2 / 3, 1 / 6), (1 / 6, 2 / 3)]
    t = float(1.0 / torch.sqrt(torch.tensor(3.0)))
    pts = [[r, s, z] for (r, s) in tri for z in (-t, t)]
    return (torch.tensor(pts, dtype=dtype, device=device),
            torch.tensor([1 / 3] * 6, dtype=dtype, device=device))


def c3d10_integration_points(device="cuda:0", dtype=torch.float32):
    """The reference's 11-point tet rule (weights sum to 0.45, quirk Q2). `solver/element.py:995-1024`."""
    pts = [[0.25, 0.25, 0.25], [0.1, 0.1, 0.1], [0.1, 0.1, 0.7], [0.1, 0.7, 0.1], [0.7, 0.1, 0.1],
           [0.1, 0.4, 0.4], [0.4, 0.1, 0.4], [0.4, 0.4, 0.1], [0.3, 0.3, 0.3], [0.2, 0.2, 0.6], [0.2, 0.6, 0.2]]
    w = [0.1, 0.05, 0.05, 0.05, 0.05, 0.03, 0.03, 0.03, 0.02, 0.02, 0.02]
    return torch.tensor(pts, dtype=dtype).to(device), torch.tensor(w, dtype=dtype).to(device)


def _dn_c3d8(xi, eta, zeta):
    # natural derivatives, `solver/element.py:1617-1626`
    out = []
    for (a, b, c) in ((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (-1, -1, 1), (1, -1, 1), (1, 1, 1), (-1, 1, 1)):
        out.append([0.125 * a * (1 + b * eta) * (1 + c * zeta), 0.125 * b * (1 + a * xi) * (1 + c * zeta),
                    0.125 * c * (1 + a * xi) * (1 + b * eta)])
    return out


def _dn_c3d6(r, s, t):
    # `solver/element.py:2498-2505`
    return [[-0.5 * (1 - t), -0.5 * (1 - t), -0.5 * (1 - r - s)], [0.5 * (1 - t), 0.0, -0.5 * r],
            [0.0, 0.5 * (1 - t), -0.5 * s], [-0.5 * (1 + t), -0.5 * (1 + t), 0.5 * (1 - r - s)],
            [0.5 * (1 + t), 0.0, 0.5 * r], [0.0, 0.5 * (1 + t), 0.5 * s]]


def _dn_c3d10(xi, eta, zeta):
    # `solver/element.py:1043-1054`
    L = 1 - xi - eta - zeta
    return [[4 * xi - 1, 0, 0], [0, 4 * eta - 1, 0], [0, 0, 4 * zeta - 1], [-4 * L + 1, -4 * L + 1, -4 * L + 1],
            [4 * eta, 4 * xi, 0], [0, 4 * zeta, 4 * eta], [4 * zeta, 0, 4 * xi],
            [4 * (1 - 2 * xi - eta - zeta), -4 * xi, -4 * xi], [-4 * eta, 4 * (1 - xi - 2 * eta - zeta), -4 * eta],
            [-4 * zeta, -4 * zeta, 4 * (1 - xi - eta - 2 * zeta)]]


def _n_c3d8(xi, eta, zeta):
    # shape values matching _dn_c3d8's node order
    return [0.125 * (1 + a * xi) * (1 + b * eta) * (1 + c * zeta)
            for (a, b, c) in ((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1), (-1, -1, 1), (1, -1, 1), (1, 1, 1),
                              (-1, 1, 1))]


def _n_c3d6(r, s, t):
    # shape values matching _dn_c3d6
    L = 1 - r - s
    return [0.5 * L * (1 - t), 0.5 * r * (1 - t), 0.5 * s * (1 - t), 0.5 * L * (1 + t), 0.5 * r * (1 + t),
            0.5 * s * (1 + t)]


def _n_c3d10(xi, eta, zeta):
    # shape values matching _dn_c3d10 (corners xi, eta, zeta, L; mid-edges (0,1), (1,2), (2,0), (0,3), (1,3), (2,3))
    L = 1 - xi - eta - zeta
    return [xi * (2 * xi - 1), eta * (2 * eta - 1), zeta * (2 * zeta - 1), L * (2 * L - 1), 4 * xi * eta,
            4 * eta * zeta, 4 * zeta * xi, 4 * xi * L, 4 * eta * L, 4 * zeta * L]


def mass_integration_points(element_type, dtype=F64):
    """Quadrature of the consistent mass (no reference: parity unpinned), exact for N_a N_b on affine elements:
    c3d8 the 2x2x2 Gauss rule (w = 1, volume 8); c3d6 the degree-2 triangle rule (1/6, 1/6), (2/3, 1/6), (1/6, 2/3)
    with weight 1/6 (sum = the triangle's 1/2, not the stiffness rule's 1/3 each, Q3) times 2-point Gauss in t;
    c3d10 the 14-point degree-5 tetrahedron rule (weights sum to 1/6). Returns (points [n,3], weights [n])."""
    et = element_type.lower()
    if et == "c3d8":
        return c3d8_integration_points(device="cpu", dtype=dtype)
    if et == "c3d6":
        g = 1.0 / 3.0 ** 0.5
        tri = [(1 / 6, 1 / 6), (2 / 3, 1 / 6), (1 / 6, 2 / 3)]
        pts = [(r, s_, t) for t in (-g, g) for (r, s_) in tri]
        return torch.tensor(pts, dtype=dtype), torch.full((6,), 1.0 / 6.0, dtype=dtype)
    if et == "c3d10":
        a, b, c = 0.0927352503108912, 0.3108859192633006, 0.0455037041256496
        wa, wb, wc = 0.0734930431163619 / 6, 0.1126879257180159 / 6, 0.0425460207770815 / 6
        pts, ws = [], []
        for x, wx in ((a, wa), (b, wb)):
            for k in range(4):
                bary = [x] * 4
                bary[k] = 1 - 3 * x
                pts.append(bary[:3])
                ws.append(wx)
        for i in range(4):
            for j in range(i + 1, 4):
                bary = [c] * 4
                bary[i] = bary[j] = 0.5 - c
                pts.append(bary[:3])
                ws.append(wc)
        return torch.tensor(pts, dtype=dtype), torch.tensor(ws, dtype=dtype)
    _unsupported(element_type)


_ISO = {"c3d8": (8, _dn_c3d8, c3d8_integration_points), "c3d6": (6, _dn_c3d6, c3d6_integration_points),
        "c3d10": (10, _dn_c3d10, c3d10_integration_points)}
_N = {"c3d8": _n_c3d8, "c3d6": _n_c3d6, "c3d10": _n_c3d10}


def _points_weights(etype, integral_point):
    """(points [n,3] fp64 host, weights [n]) — default rule, or the caller's [n,4] (xi, eta, zeta, w) table."""
    if integral_point is None:
        p, w = _ISO[etype][2](device="cpu", dtype=F64)
    else:
        ip = integral_point.detach().to("cpu", F64)
        p, w = ip[:, :3], ip[:, -1]
    return p, w


_CONST = OrderedDict()   # device copies of the per-rule tables (natural derivatives, shape values, weights)


def _dev_const(key, make, dev):
    """Cached device copy of a small host table: forming the tables by Python polynomial evaluation and copying them
    host-to-device on every call cost more host time than the c3d6 / c3d8 element kernels themselves."""
    k = key + (str(dev),)
    t = _CONST.get(k)
    if t is None:
        t = make().to(dev).contiguous()
        _CONST[k] = t
        if len(_CONST) > 64:
            _CONST.popitem(last=False)
    return t


def _dn_table(etype, points, dev):
    fn = _ISO[etype][1]
    pts = points.detach().to("cpu", F64).contiguous()
    return _dev_const((etype, "dN", pts.numpy().tobytes()),
                      lambda: torch.tensor([fn(*[float(v) for v in pts[q]]) for q in range(pts.shape[0])],
                                           dtype=F64), dev)   # [n_ip, npe, 3]


def _iso_ke(coords, elements, etype, E, nu, points, weights, mode, device, dtype):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    npe = _ISO[etype][0]
    if elements.shape[1] != npe:
        raise ValueError(f"{etype} expects {npe} nodes per element, got {elements.shape[1]}")
    M = elements.shape[0]
    dN = _dn_table(etype, points, dev)
    wh = weights.detach().to("cpu", F64).contiguous()
    w = _dev_const(("w", wh.numpy().tobytes()), lambda: wh, dev)
    n_ip = dN.shape[0]
    d = 3 * npe
    shape = (n_ip, M, d, d) if mode == C.ISO_STACK else (M, d, d)
    K = torch.empty(shape, dtype=F64, device=dev)
    C.check(lib.fem_iso_ke(C.ptr(coords), C.ptr(elements), M, npe, float(E), float(nu), C.ptr(dN), C.ptr(w), n_ip,
                           mode, C.ptr(K), C.stream(dev)), "fem_iso_ke")
    return _out(K, device, dtype)


def _solid_ke_sym(coords, elements, element_type, E, nu, device="cuda:0"):
    """Internal assembly path of configs[4]: `compute_K_matrix(..., single=True)` of c3d6 / c3d8 / c3d10 (default
    rules; `solver/element.py:1754-1803`, `:2631-2676`, `:1191-1239`) in the packed symmetric form -- only the upper
    3x3 blocks, [M, fem_ke_sym_stride(npe)] fp64 on the device (include/fem355.h fem_iso_ke_sym), for
    `system.SellMatrix.add_element_matrices_sym`. The upper blocks are compute_K_matrix's bit for bit."""
    et = element_type.lower()
    if et not in ("c3d6", "c3d8", "c3d10"):
        _unsupported(element_type)
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    npe = _ISO[et][0]
    if elements.shape[1] != npe:
        raise ValueError(f"{et} expects {npe} nodes per element, got {elements.shape[1]}")
    if et == "c3d6":   # single=True: B at (1/3, 1/3, 0) times the wedge volume (`solver/element.py:2656-2659`)
        p, w, mode = torch.tensor([[1 / 3, 1 / 3, 0.0]], dtype=F64), torch.ones(1, dtype=F64), C.ISO_VOLUME
    else:
        (p, w), mode = _points_weights(et, None), C.ISO_SUM
    dN = _dn_table(et, p, dev)
    wh = w.detach().to("cpu", F64).contiguous()
    wd = _dev_const(("w", wh.numpy().tobytes()), lambda: wh, dev)
    M = elements.shape[0]
    Kp = torch.empty((M, int(lib.fem_ke_sym_stride(npe))), dtype=F64, device=dev)
    C.check(lib.fem_iso_ke_sym(C.ptr(coords), C.ptr(elements), M, npe, float(E), float(nu), C.ptr(dN), C.ptr(wd),
                               dN.shape[0], mode, C.ptr(Kp), C.stream(dev)), "fem_iso_ke_sym")
    return Kp


def _iso_mass(coords, elements, etype, rho, device, dtype, scalar=False):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    npe = _ISO[etype][0]
    if elements.shape[1] != npe:
        raise ValueError(f"{etype} expects {npe} nodes per element, got {elements.shape[1]}")
    M = elements.shape[0]
    p, w = mass_integration_points(etype)
    dN = _dn_table(etype, p, dev)
    Nv = _dev_const((etype, "N", p.numpy().tobytes()),
                    lambda: torch.tensor([_N[etype](*[float(v) for v in p[q]]) for q in range(p.shape[0])], dtype=F64),
                    dev)
    w = _dev_const(("w", w.to("cpu", F64).contiguous().numpy().tobytes()), lambda: w.to("cpu", F64), dev)
    d = npe if scalar else 3 * npe
    Me = torch.empty((M, d, d), dtype=F64, device=dev)
    fn = lib.fem_iso_mass_scalar if scalar else lib.fem_iso_mass
    C.check(fn(C.ptr(coords), C.ptr(elements), M, npe, float(rho), C.ptr(Nv.contiguous()), C.ptr(dN), C.ptr(w),
               p.shape[0], C.ptr(Me), C.stream(dev)), "fem_iso_mass")
    return _out(Me, device, dtype)


def compute_c3d8_M_matrix(coords, elements, rho, device="cuda:0", dtype=torch.float32):
    """Consistent hex mass [M,24,24] = rho sum_q w_q |detJ_q| N_a N_b (x) I3, 2x2x2 Gauss. No reference function
    (the notebook's `compute_c3d4_M_matrix`, `solver_example.ipynb:221`, is the only mass call): parity unpinned."""
    return _iso_mass(coords, elements, "c3d8", rho, device, dtype)


def compute_c3d6_M_matrix(coords, elements, rho, device="cuda:0", dtype=torch.float32):
    """Consistent wedge mass [M,18,18] (3-point triangle x 2-point Gauss, mass_integration_points). Parity
    unpinned."""
    return _iso_mass(coords, elements, "c3d6", rho, device, dtype)


def compute_c3d10_M_matrix(coords, elements, rho, device="cuda:0", dtype=torch.float32):
    """Consistent P2 tet mass [M,30,30] (14-point degree-5 rule, |detJ|: the reference's node convention makes
    detJ negative on VTK-positive tets, Q2). Parity unpinned."""
    return _iso_mass(coords, elements, "c3d10", rho, device, dtype)


def compute_M_matrix(coords, elements, element_type, rho, device="cuda:0", dtype=torch.float32, scalar=False):
    """Consistent mass dispatch over c3d4 / c3d6 / c3d8 / c3d10 (ValueError otherwise, like compute_K_matrix).
    scalar=True (c3d6 / c3d8 / c3d10): the scalar factor Ms [M, npe, npe] of M_e = Ms (x) I3 instead of the
    [M, 3 npe, 3 npe] matrix -- the same values, 1/9 of the bytes; assembled as a bs = 1 matrix on the node pattern
    it is the global factor of M = M_s (x) I3. Parity unpinned (no reference function)."""
    et = element_type.lower()
    if et == "c3d4":
        if scalar:
            raise ValueError("scalar=True: c3d6 / c3d8 / c3d10 (the c3d4 mass is compute_c3d4_M_matrix)")
        return compute_c3d4_M_matrix(coords, elements, rho, device=device, dtype=dtype)
    if et in _N:
        return _iso_mass(coords, elements, et, rho, device, dtype, scalar)
    _unsupported(element_type)


def _iso_geom(coords, elements, etype, integral_point, what, device, dtype):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    npe = _ISO[etype][0]
    M = elements.shape[0]
    ip = torch.as_tensor(integral_point).detach().to("cpu", F64).reshape(-1)[:3]
    dN = _dn_table(etype, ip.view(1, 3), dev)[0].contiguous()
    J = torch.empty((M, 3, 3), dtype=F64, device=dev) if what == "J" else None
    G = torch.empty((M, npe, 3), dtype=F64, device=dev) if what == "G" else None
    B = torch.empty((M, 6, 3 * npe), dtype=F64, device=dev) if what == "B" else None
    C.check(lib.fem_iso_geom(C.ptr(coords), C.ptr(elements), M, npe, C.ptr(dN), C.ptr(J), C.ptr(G), C.ptr(B),
                             C.stream(dev)), "fem_iso_geom")
    return _out({"J": J, "G": G, "B": B}[what], device, dtype)


def compute_c3d8_Jacobian(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1601-1632` -> [M,3,3]."""
    return _iso_geom(coords, elements, "c3d8", integral_point, "J", device, dtype)


def compute_c3d8_shape_gradients(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1634-1664` -> [M,8,3]."""
    return _iso_geom(coords, elements, "c3d8", integral_point, "G", device, dtype)


def compute_c3d8_B_matrix(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1666-1694` -> [M,6,24]."""
    return _iso_geom(coords, elements, "c3d8", integral_point, "B", device, dtype)


def compute_c3d8_K_matrix(coords, elements, E, nu, integral_point=None, single=True, device="cuda:0",
                          dtype=torch.float32):
    """sum_ip w detJ B^T D B -> [M,24,24]; single=False -> [n_ip,M,24,24] without weights (Q6).
    `solver/element.py:1754-1803`."""
    p, w = _points_weights("c3d8", integral_point)
    return _iso_ke(coords, elements, "c3d8", E, nu, p, w, C.ISO_SUM if single else C.ISO_STACK, device, dtype)


def compute_c3d6_Jacobian(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:2482-2509`."""
    return _iso_geom(coords, elements, "c3d6", integral_point, "J", device, dtype)


def compute_c3d6_shape_gradients(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:2511-2539`."""
    return _iso_geom(coords, elements, "c3d6", integral_point, "G", device, dtype)


def compute_c3d6_B_matrix(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:2541-2568`."""
    return _iso_geom(coords, elements, "c3d6", integral_point, "B", device, dtype)


def compute_wedge_volumes(coords, elements, device="cuda:0", dtype=torch.float32):
    """Sum of the 3 sub-tet |volumes| (p0,p1,p2,p3), (p1,p2,p4,p3), (p2,p4,p5,p3). `solver/element.py:2198-2232`
    (the sub-tet volumes come from the c3d4 geometry kernel)."""
    el = torch.as_tensor(elements).to(LONG)
    subs = torch.stack([el[:, [0, 1, 2, 3]], el[:, [1, 2, 4, 3]], el[:, [2, 4, 5, 3]]], 1).reshape(-1, 4)
    v = compute_tetrahedral_volumes(coords, subs, device=device, dtype=F64).view(-1, 3)
    return _out(v[:, 0] + v[:, 1] + v[:, 2], device, dtype)


def compute_hexahedral_volumes(coords, elements, device="cuda:0", dtype=torch.float32):
    """Sum of the 6 sub-tet |volumes| (p0,p1,p3,p4), (p1,p2,p3,p6), (p1,p3,p4,p5), (p3,p4,p5,p7), (p3,p5,p6,p7),
    (p3,p5,p6,p1), added in that order -> [M]. `solver/element.py:1248-1291` (the sub-tet volumes come from the c3d4
    geometry kernel, |det| / 6 as the reference's inner `v`)."""
    el = torch.as_tensor(elements).to(LONG)
    subs = torch.stack([el[:, [0, 1, 3, 4]], el[:, [1, 2, 3, 6]], el[:, [1, 3, 4, 5]], el[:, [3, 4, 5, 7]],
                        el[:, [3, 5, 6, 7]], el[:, [3, 5, 6, 1]]], 1).reshape(-1, 4)
    v = compute_tetrahedral_volumes(coords, subs, device=device, dtype=F64).view(-1, 6)
    return _out(v[:, 0] + v[:, 1] + v[:, 2] + v[:, 3] + v[:, 4] + v[:, 5], device, dtype)


def compute_c3d6_K_matrix(coords, elements, E, nu, integral_point=None, single=True, device="cuda:0",
                          dtype=torch.float32):
    """single=True: B at (1/3,1/3,0) times the wedge volume; single=False: sum_ip w detJ B^T D B with the
    reference's 6-point rule (weights sum to 2, Q3). Always [M,18,18]. `solver/element.py:2631-2676`."""
    if single:
        p = torch.tensor([[1 / 3, 1 / 3, 0.0]], dtype=F64)
        return _iso_ke(coords, elements, "c3d6", E, nu, p, torch.ones(1, dtype=F64), C.ISO_VOLUME, device, dtype)
    p, w = _points_weights("c3d6", integral_point)
    return _iso_ke(coords, elements, "c3d6", E, nu, p, w, C.ISO_SUM, device, dtype)


def compute_c3d10_Jacobian(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1026-1060`."""
    return _iso_geom(coords, elements, "c3d10", integral_point, "J", device, dtype)


def compute_c3d10_shape_gradients(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1062-1095`."""
    return _iso_geom(coords, elements, "c3d10", integral_point, "G", device, dtype)


def compute_c3d10_B_matrix(coords, elements, integral_point, device="cuda:0", dtype=torch.float32):
    """`solver/element.py:1097-1125`."""
    return _iso_geom(coords, elements, "c3d10", integral_point, "B", device, dtype)


def compute_c3d10_K_matrix(coords, elements, E, nu, integral_point=None, single=True, device="cuda:0",
                           dtype=torch.float32):
    """sum_ip w signed-detJ B^T D B (11-point rule, Q2) -> [M,30,30]; single=False -> [n_ip,M,30,30] unweighted.
    `solver/element.py:1191-1239`."""
    p, w = _points_weights("c3d10", integral_point)
    return _iso_ke(coords, elements, "c3d10", E, nu, p, w, C.ISO_SUM if single else C.ISO_STACK, device, dtype)


# ============================================================================ dispatch (`solver/element.py:371-427`)
def _unsupported(element_type):
    raise ValueError(f"Unsupported element type: {element_type}")


def integral_points(element_type, device="cuda:0"):
    et = element_type.lower()
    if et in ("c3d8", "c3d10", "c3d6"):
        return _ISO[et][2](device=device)
    _unsupported(et)


def compute_Jacobian(coords, elements, element_type, integral_point=None, device="cuda:0"):
    et = element_type.lower()
    et = "c3d8" if et == "c3d8i" else et
    if et in _ISO:
        return _iso_geom(coords, elements, et, integral_point, "J", device, torch.float32)
    _unsupported(et)


def compute_shape_gradients(coords, elements, element_type, integral_point=None, device="cuda:0"):
    et = element_type.lower()
    if et in _ISO:
        return _iso_geom(coords, elements, et, integral_point, "G", device, torch.float32)
    _unsupported(et)


def compute_B_matrix(coords, elements, integral_point, element_type, device="cuda:0", dtype=torch.float32):
    et = element_type.lower()
    if et == "c3d4":
        return compute_c3d4_B_matrix(coords, elements, device, dtype)
    if et in _ISO:
        return _iso_geom(coords, elements, et, integral_point, "B", device, dtype)
    _unsupported(et)


def compute_K_matrix(coords, elements, element_type, E, nu, integral_point=None, single=True, device="cuda:0",
                     dtype=torch.float32):
    """String dispatch of `solver/element.py:419-427` (c3d20/c3d15 are broken in the reference: out of scope)."""
    et = element_type.lower()
    if et == "c3d4":
        return compute_c3d4_K_matrix(coords, elements, E, nu, device, dtype)
    if et == "c3d8":
        return compute_c3d8_K_matrix(coords, elements, E, nu, integral_point, single, device, dtype)
    if et == "c3d10":
        return compute_c3d10_K_matrix(coords, elements, E, nu, integral_point, single, device, dtype)
    if et == "c3d6":
        return compute_c3d6_K_matrix(coords, elements, E, nu, integral_point, single, device, dtype)
    _unsupported(et)


# ============================================================================ element-by-element operator
_INC_CACHE: "OrderedDict[tuple, tuple]" = OrderedDict()


def _key(t: torch.Tensor, *extra):
    return (t.data_ptr(), t._version, tuple(t.shape), str(t.device)) + extra


def cached_incidence(elements: torch.Tensor, n_nodes: int):
    k = _key(elements, n_nodes)
    hit = _INC_CACHE.get(k)
    if hit is not None:
        _INC_CACHE.move_to_end(k)
        return hit[1]
    inc = _sys.incidence(elements, n_nodes)
    _INC_CACHE[k] = (elements, inc)   # keep `elements` alive so its pointer is not reused while cached
    while len(_INC_CACHE) > 8:
        _INC_CACHE.popitem(last=False)
    return inc


def compute_nodal_forces(K, elements, displacement, device="cuda:0", dtype=torch.float32):
    """y = sum_e P_e^T K_e P_e u without assembly -> [N, dpn]. `solver/element.py:429-464`.
    dofs per node = K.shape[-1] / nodes per element (3 in the reference; 1 for the scalar Poisson K)."""
    lib = C.lib()
    dev = _dev(device)
    elements = elements.to(device=dev, dtype=LONG).contiguous()
    K = K.to(device=dev, dtype=F64).contiguous()
    u = displacement.to(device=dev, dtype=F64).contiguous()
    M, npe = elements.shape
    dpn = K.shape[-1] // npe
    N = u.shape[0]
    inc_ptr, inc = cached_incidence(elements, N)
    y = torch.empty((N, dpn), dtype=F64, device=dev)
    C.check(lib.fem_ebe_apply(C.ptr(K), C.ptr(elements), npe, dpn, C.ptr(inc_ptr), C.ptr(inc), N, C.ptr(u), C.ptr(y),
                              C.stream(dev)), "fem_ebe_apply")
    return _out(y, device, dtype)


# ============================================================================ stress recovery
def _disp(displacement, dev, N):
    u = displacement.to(device=dev, dtype=F64).contiguous()
    if u.dim() != 2 or u.shape[1] != 3 or u.shape[0] != N:
        raise ValueError(f"displacement must be [N, 3] with N = {N} nodes, got {list(u.shape)}")
    return u


def compute_stress_tensor(stress_vector):
    """Voigt [M,6] (xx, yy, zz, xy, yz, xz) -> symmetric [M,3,3] on the input's device / dtype.
    `solver/element.py:308-330`."""
    lib = C.lib()
    dev = _dev(stress_vector.device)
    v = stress_vector.to(device=dev, dtype=F64).contiguous()
    M = v.shape[0]
    out = torch.empty((M, 3, 3), dtype=F64, device=dev)
    C.check(lib.fem_voigt_to_tensor(C.ptr(v), M, C.ptr(out), C.stream(dev)), "fem_voigt_to_tensor")
    return out.to(device=stress_vector.device, dtype=stress_vector.dtype)


def compute_von_mises_stress(stress_tensor):
    """[M,3,3] -> sqrt(((sxx-syy)^2 + (syy-szz)^2 + (szz-sxx)^2 + 6 (sxy^2 + syz^2 + sxz^2)) / 2) [M], read from
    the upper triangle. `solver/element.py:332-353`."""
    lib = C.lib()
    dev = _dev(stress_tensor.device)
    t = stress_tensor.to(device=dev, dtype=F64).contiguous()
    M = t.shape[0]
    out = torch.empty(M, dtype=F64, device=dev)
    C.check(lib.fem_von_mises(C.ptr(t), M, C.ptr(out), C.stream(dev)), "fem_von_mises")
    return out.to(device=stress_tensor.device, dtype=stress_tensor.dtype)


def compute_c3d4_element_stress(coords, elements, displacement, E, nu, device="cuda:0", dtype=torch.float32):
    """(stress tensor [M,3,3], von Mises [M]) of P1 tets from nodal displacements [N,3]; ValueError on a
    degenerate element like the reference's B matrix. `solver/element.py:905-937`."""
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    u = _disp(displacement, dev, coords.shape[0])
    M = elements.shape[0]
    sig = torch.empty((M, 3, 3), dtype=F64, device=dev)
    vm = torch.empty(M, dtype=F64, device=dev)
    bad = _bad_scalar(dev, M)
    C.check(lib.fem_tet4_stress(C.ptr(coords), C.ptr(elements), M, C.ptr(u), float(E), float(nu), C.ptr(sig),
                                C.ptr(vm), C.ptr(bad), C.stream(dev)), "fem_tet4_stress")
    _raise_if_singular(bad, M)
    return _out(sig, device, dtype), _out(vm, device, dtype)


def _iso_stress(coords, elements, displacement, E, nu, etype, integral_point, single, point_major, device, dtype):
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    npe = _ISO[etype][0]
    if elements.shape[1] != npe:
        raise ValueError(f"{etype} expects {npe} nodes per element, got {elements.shape[1]}")
    u = _disp(displacement, dev, coords.shape[0])
    M = elements.shape[0]
    p, w = _points_weights(etype, integral_point)
    dN = _dn_table(etype, p, dev)
    w = w.to(dev, F64).contiguous()
    n_ip = dN.shape[0]
    if single:
        layout, shape = 0, (M,)
    else:
        layout, shape = (2, (n_ip, M)) if point_major else (1, (M, n_ip))
    sig = torch.empty(shape + (3, 3), dtype=F64, device=dev)
    vm = torch.empty(shape, dtype=F64, device=dev)
    C.check(lib.fem_iso_stress(C.ptr(coords), C.ptr(elements), M, npe, C.ptr(u), float(E), float(nu), C.ptr(dN),
                               C.ptr(w), n_ip, layout, C.ptr(sig), C.ptr(vm), C.stream(dev)), "fem_iso_stress")
    return _out(sig, device, dtype), _out(vm, device, dtype)


def compute_c3d8_element_stress(coords, elements, displacement, E, nu, integral_point=None, single=True,
                                device="cuda:0", dtype=torch.float32):
    """Per 2x2x2 Gauss point stress / von Mises; single=True -> sum_q w_q (tensor, vm) [M,3,3], [M], else
    [M,n_ip,3,3], [M,n_ip]. `solver/element.py:1696-1752`."""
    return _iso_stress(coords, elements, displacement, E, nu, "c3d8", integral_point, single, False, device, dtype)


def compute_c3d6_element_stress(coords, elements, displacement, E, nu, integral_point=None, single=True,
                                device="cuda:0", dtype=torch.float32):
    """Wedge analogue of compute_c3d8_element_stress (6-point rule, weights 1/3: Q3). `solver/element.py:2570-2629`."""
    return _iso_stress(coords, elements, displacement, E, nu, "c3d6", integral_point, single, False, device, dtype)


def compute_c3d10_element_stress(coords, elements, displacement, E, nu, integral_point=None, single=True,
                                 device="cuda:0", dtype=torch.float32):
    """Quadratic tet, 11-point rule (weights sum to 0.45: Q2); single=False stacks point-major [n_ip,M,3,3],
    [n_ip,M] like the reference's list stack. `solver/element.py:1127-1189`."""
    return _iso_stress(coords, elements, displacement, E, nu, "c3d10", integral_point, single, True, device, dtype)


def compute_element_stress(coords, elements, displacement, E, nu, element_type, integral_point=None, single=True,
                           device="cuda:0", dtype=torch.float32):
    """String dispatch of `solver/element.py:409-417` (c3d20 / c3d15 out of scope, as for compute_K_matrix)."""
    et = element_type.lower()
    if et == "c3d4":
        return compute_c3d4_element_stress(coords, elements, displacement, E, nu, device, dtype)
    if et == "c3d8":
        return compute_c3d8_element_stress(coords, elements, displacement, E, nu, integral_point, single, device,
                                           dtype)
    if et == "c3d10":
        return compute_c3d10_element_stress(coords, elements, displacement, E, nu, integral_point, single, device,
                                            dtype)
    if et == "c3d6":
        return compute_c3d6_element_stress(coords, elements, displacement, E, nu, integral_point, single, device,
                                           dtype)
    _unsupported(et)


def compute_node_vm_stress(coords, elements, element_vm_stress, device="cuda:0", dtype=torch.float32):
    """Node value = mean of the element values over the elements touching it (0 for unused nodes), summed in
    ascending element order. `solver/element.py:466-504`."""
    lib = C.lib()
    dev, coords, elements = _prep(coords, elements, device)
    N = coords.shape[0]
    M, npe = elements.shape
    ev = element_vm_stress.to(device=dev, dtype=F64).contiguous().view(-1)
    if ev.numel() != M:
        raise ValueError(f"element_vm_stress must have one value per element ({M}), got {ev.numel()}")
    inc_ptr, inc = cached_incidence(elements, N)
    out = torch.empty(N, dtype=F64, device=dev)
    C.check(lib.fem_node_average(C.ptr(ev), npe, C.ptr(inc_ptr), C.ptr(inc), N, C.ptr(out), C.stream(dev)),
            "fem_node_average")
    return _out(out, device, dtype)


def compute_c3d4_surface_forces(normal_vectors, stress_tensors, device="cuda:0"):
    """Face tractions sigma_e n_ef [M,F,3] from area-weighted face normals [M,F,3] and element stress [M,3,3].
    `solver/element.py:3343-3362`."""
    lib = C.lib()
    dev = _dev(device)
    out_dtype = torch.promote_types(normal_vectors.dtype, stress_tensors.dtype)
    n = normal_vectors.to(device=dev, dtype=F64).contiguous()
    s = stress_tensors.to(device=dev, dtype=F64).contiguous()
    M, F = n.shape[0], n.shape[1]
    if tuple(s.shape) != (M, 3, 3) or n.shape[2] != 3:
        raise ValueError(f"normals [M,F,3] and stress [M,3,3] expected, got {list(n.shape)} / {list(s.shape)}")
    out = torch.empty((M, F, 3), dtype=F64, device=dev)
    C.check(lib.fem_face_forces(C.ptr(n), C.ptr(s), M, F, C.ptr(out), C.stream(dev)), "fem_face_forces")
    return out.to(device=torch.device(device), dtype=out_dtype)


def compute_c3d4_shared_face_forces_sum(shared_face_indices, element_forces, device="cuda:0"):
    """f[e0,f0] + f[e1,f1] for every shared face [S,2,2] -> [S,3] (zero at equilibrium).
    `solver/element.py:3364-3382`."""
    lib = C.lib()
    dev = _dev(device)
    out_dtype = element_forces.dtype
    idx = shared_face_indices.to(device=dev, dtype=LONG).contiguous()
    ff = element_forces.to(device=dev, dtype=F64).contiguous()
    M, F = ff.shape[0], ff.shape[1]
    S = idx.shape[0]
    if S and (int(idx[..., 0].min()) < 0 or int(idx[..., 0].max()) >= M or int(idx[..., 1].min()) < 0
              or int(idx[..., 1].max()) >= F):
        raise IndexError("shared_face_indices out of range of element_forces")
    out = torch.empty((S, 3), dtype=F64, device=dev)
    C.check(lib.fem_shared_face_sum(C.ptr(idx), C.ptr(ff), F, S, C.ptr(out), C.stream(dev)), "fem_shared_face_sum")
    return out.to(device=torch.device(device), dtype=out_dtype)


__all__ += [
    "compute_stress_tensor", "compute_von_mises_stress", "compute_element_stress", "compute_c3d4_element_stress",
    "compute_c3d8_element_stress", "compute_c3d6_element_stress", "compute_c3d10_element_stress",
    "compute_node_vm_stress", "compute_c3d4_surface_forces", "compute_c3d4_shared_face_forces_sum",
]

# every public function runs in the scope of the device its `device` argument names (_capi.on_device)
C.scope_module(globals())

# mesh topology lives in topology.py; re-exported here because the reference keeps it in
# element.py (`solver/element.py:543-762,963-993,1293-1581,2234-2446,2687-2713`)
try:
    from . import topology as _topo
except ImportError:  # pragma: no cover - flat import from the package directory
    import topology as _topo  # type: ignore
from_topology = [n for n in _topo.__all__ if n != "FaceGroups"]
globals().update({n: getattr(_topo, n) for n in from_topology})
__all__ += from_topology
del from_topology
