"""Mesh topology on the device: surface faces, shared faces (the element graph the
reference's region-growing partitioner consumes, `subdivision.ipynb` cells 8-9), unique edges, face normals and
the c3d8/c3d6/c3d10 -> c3d4 splits, with the reference's names and return conventions
(`solver/element.py:543-762,963-993,1293-1581,2234-2446,2687-2713`).

Face grouping runs in one `fem_topo` context (`csrc/topology.hip`): packed sorted-node keys, a stable radix sort,
run detection; the compactions reproduce torch.unique(dim=0) row order and the reference's pairing order.
Node ids must be in [0, N) with N = max id + 1 (IndexError otherwise, like the reference's indexing).
The curvature helpers of the reference (`:621-650`, `:1376-1416`, `:2340-2375`) are not provided: they read an
undefined `face_normals` / call the normals function with a wrong signature and raise in the reference itself.
"""
from __future__ import annotations

import ctypes

import torch

try:
    from . import _capi as C
    from . import system as _sys
except ImportError:  # pragma: no cover - flat import from the package directory
    import _capi as C  # type: ignore
    import system as _sys  # type: ignore

F64 = torch.float64
LONG = torch.long
I32 = torch.int32

# face tables (local node indices) in the reference's row orders
TET_SHARED = [[0, 1, 2], [0, 1, 3], [1, 2, 3], [0, 2, 3]]          # `:723-728`, `:675-680`
TET_SURFACE = [[0, 1, 2], [0, 1, 3], [0, 2, 3], [1, 2, 3]]         # `:557-562`
TET_SURFACE_X = [3, 2, 1, 0]                                        # `:564-569`
TET_SHARED_X = [3, 2, 0, 1]                                         # `:682-687`
HEX = [[0, 1, 5, 4], [1, 2, 6, 5], [2, 3, 7, 6], [0, 4, 7, 3], [0, 3, 2, 1], [4, 5, 6, 7]]   # `:1308-1315`
HEX_SURFACE_X = [2, 0, 0, 1, 4, 0]                                  # `:1317-1324`
HEX_AREA_X = [2, 0, 0, 1, 6, 0]                                     # `:1458`
WEDGE_QUAD = [[0, 1, 4, 3], [1, 2, 5, 4], [2, 0, 3, 5]]             # `:2249-2253`
WEDGE_QUAD_X = [2, 0, 1]
WEDGE_TRI = [[0, 2, 1], [3, 4, 5]]                                  # `:2260-2263`
WEDGE_TRI_X = [3, 0]
EDGES = [[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]]            # `:2700-2704`
SPLIT = {8: [[0, 1, 3, 4], [1, 2, 3, 6], [1, 3, 4, 5], [3, 4, 5, 7], [3, 5, 6, 7], [3, 5, 6, 2]],   # `:1567-1574`
         6: [[0, 1, 2, 3], [1, 2, 3, 5], [1, 3, 4, 5]],                                            # `:2435-2439`
         10: [[0, 4, 6, 7], [4, 1, 5, 8], [6, 5, 2, 9], [7, 8, 9, 3], [4, 6, 7, 5], [6, 7, 9, 5],
              [4, 7, 8, 5], [5, 8, 7, 9]]}                                                        # `:976-985`


def _i32(tab):
    flat = [int(v) for row in tab for v in (row if isinstance(row, (list, tuple)) else [row])]
    return (ctypes.c_int32 * len(flat))(*flat)


def _dev(device):
    C.lib()
    return C.compute_device(device)


def _conn(elements, dev, npe_min):
    el = elements.to(device=dev, dtype=LONG).contiguous()
    if el.dim() != 2 or el.shape[1] < npe_min:
        raise ValueError(f"elements must be [M, >= {npe_min}], got {list(el.shape)}")
    n = int(el.max()) + 1 if el.numel() else 1
    _sys.check_connectivity(el, n)
    return el, n


class FaceGroups:
    """One fem_topo context: the faces of table `ftab` of every element, grouped by node set."""

    def __init__(self, elements, ftab, device):
        self.lib = C.lib()
        self.dev = _dev(device)
        self.el, self.N = _conn(elements, self.dev, max(max(r) for r in ftab) + 1)
        self.M, self.npe = self.el.shape
        self.F, self.fpn = len(ftab), len(ftab[0])
        self.h = ctypes.c_void_p()
        C.check(self.lib.fem_topo_create(C.ptr(self.el), self.M, self.npe, _i32(ftab), self.F, self.fpn, self.N,
                                         C.stream(self.dev), ctypes.byref(self.h)), "fem_topo_create")
        u, s, p = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        C.check(self.lib.fem_topo_counts(self.h, ctypes.byref(u), ctypes.byref(s), ctypes.byref(p)), "fem_topo_counts")
        self.n_unique, self.n_single, self.n_pair = u.value, s.value, p.value

    def pairs(self):
        out = torch.empty((self.n_pair, 2, 2), dtype=LONG, device=self.dev)
        C.check(self.lib.fem_topo_pairs(self.h, C.ptr(out)), "fem_topo_pairs")
        return out

    def unique(self):
        out = torch.empty((self.n_unique, self.fpn), dtype=LONG, device=self.dev)
        C.check(self.lib.fem_topo_unique(self.h, C.ptr(out)), "fem_topo_unique")
        return out

    def boundary(self, stab, smap, xtab=None):
        Fs = len(stab)
        k = ctypes.c_int64()
        C.check(self.lib.fem_topo_boundary(self.h, C.ptr(self.el), Fs, _i32(smap), _i32(stab),
                                           _i32(xtab) if xtab is not None else None, None, None, ctypes.byref(k)),
                "fem_topo_boundary")
        faces = torch.empty((k.value, self.fpn), dtype=LONG, device=self.dev)
        extra = torch.empty(k.value, dtype=LONG, device=self.dev)
        C.check(self.lib.fem_topo_boundary(self.h, C.ptr(self.el), Fs, _i32(smap), _i32(stab),
                                           _i32(xtab) if xtab is not None else None, C.ptr(faces), C.ptr(extra),
                                           ctypes.byref(k)), "fem_topo_boundary")
        return faces, extra

    def close(self):
        if self.h:
            self.lib.fem_topo_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _smap(stab, ftab):
    key = {tuple(sorted(r)): i for i, r in enumerate(ftab)}
    return [key[tuple(sorted(r))] for r in stab]


def _out(t, device):
    return t.to(torch.device(device))


# ---------------------------------------------------------------- surfaces
def compute_tetrahedral_surface_faces_with_fourth_node(elements, device="cuda:0"):
    """Faces of exactly one tet [K,3] (node order of the face table, face-major like the reference's cat) and
    the opposite node [K]. `solver/element.py:543-579`."""
    g = FaceGroups(elements, TET_SHARED, device)
    f, x = g.boundary(TET_SURFACE, _smap(TET_SURFACE, TET_SHARED), TET_SURFACE_X)
    g.close()
    return _out(f, device), _out(x, device)


def compute_hexahedral_surface_faces_with_extra_node(elements, device="cuda:0"):
    """Faces of exactly one hex [K,4] and a node off the face [K]. `solver/element.py:1293-1334`."""
    g = FaceGroups(elements, HEX, device)
    f, x = g.boundary(HEX, list(range(6)), HEX_SURFACE_X)
    g.close()
    return _out(f, device), _out(x, device)


def compute_wedge_surface_faces_with_extra_node(elements, device="cuda:0"):
    """([quad faces [Kq,4], tri faces [Kt,3]], [quad extra [Kq], tri extra [Kt]]); quads and triangles grouped
    separately like the reference. `solver/element.py:2234-2283`."""
    gq = FaceGroups(elements, WEDGE_QUAD, device)
    fq, xq = gq.boundary(WEDGE_QUAD, list(range(3)), WEDGE_QUAD_X)
    gq.close()
    gt = FaceGroups(elements, WEDGE_TRI, device)
    ft, xt = gt.boundary(WEDGE_TRI, list(range(2)), WEDGE_TRI_X)
    gt.close()
    return [_out(fq, device), _out(ft, device)], [_out(xq, device), _out(xt, device)]


def _surface_normals(coords, faces, extra, v2, device, dtype):
    lib = C.lib()
    dev = _dev(device)
    X = coords.to(device=dev, dtype=F64).contiguous()
    f = faces.to(device=dev, dtype=LONG).contiguous()
    x = extra.to(device=dev, dtype=LONG).contiguous()
    K, fpn = f.shape
    out = torch.empty((K, 3), dtype=F64, device=dev)
    C.check(lib.fem_surface_normals(C.ptr(X), C.ptr(f), C.ptr(x), K, fpn, v2, C.ptr(out), C.stream(dev)),
            "fem_surface_normals")
    return out.to(device=torch.device(device), dtype=dtype)


def compute_tetrahdral_surface_normals(coords, elements, device="cuda:0", dtype=torch.float32):
    """Outward unit normals of the tet surface faces [K,3] (the reference's spelling). `solver/element.py:581-619`."""
    f, x = compute_tetrahedral_surface_faces_with_fourth_node(elements, device=_dev(device))
    return _surface_normals(coords, f, x, 2, device, dtype)


compute_tetrahedral_surface_normals = compute_tetrahdral_surface_normals


def compute_hexahedral_surface_normals(coords, elements, device="cuda:0", dtype=torch.float32):
    """Outward unit normals of the hex surface faces [K,3] (edges p2-p1, p3-p1). `solver/element.py:1336-1374`."""
    f, x = compute_hexahedral_surface_faces_with_extra_node(elements, device=_dev(device))
    return _surface_normals(coords, f, x, 2, device, dtype)


def compute_wedge_surface_normals(coords, elements, device="cuda:0", dtype=torch.float32):
    """[quad normals [Kq,3] (edges p2-p1, p4-p1), tri normals [Kt,3]]. `solver/element.py:2285-2338`."""
    (fq, ft), (xq, xt) = compute_wedge_surface_faces_with_extra_node(elements, device=_dev(device))
    return [_surface_normals(coords, fq, xq, 3, device, dtype), _surface_normals(coords, ft, xt, 2, device, dtype)]


# ---------------------------------------------------------------- per-element face normals
def _element_normals(coords, elements, edges, cen, extra, scale, flip, unit, npe_min, device, dtype):
    lib = C.lib()
    dev = _dev(device)
    X = coords.to(device=dev, dtype=F64).contiguous()
    el = elements.to(device=dev, dtype=LONG).contiguous()
    if el.dim() != 2 or el.shape[1] < npe_min:
        raise ValueError(f"elements must be [M, >= {npe_min}], got {list(el.shape)}")
    _sys.check_connectivity(el, X.shape[0])
    M, npe = el.shape
    F = len(edges)
    cen_pad = [list(r) + [0] * (4 - len(r)) for r in cen]
    out = torch.empty((M, F, 3), dtype=F64, device=dev)
    C.check(lib.fem_element_face_normals(C.ptr(X), C.ptr(el), M, npe, _i32(edges), _i32(cen_pad),
                                         _i32([len(r) for r in cen]), _i32(extra), F, float(scale), int(flip),
                                         int(unit), C.ptr(out), C.stream(dev)), "fem_element_face_normals")
    return out.to(device=torch.device(device), dtype=dtype)


def compute_tetrahedral_normals_and_area(coords, elements, device="cuda:0", dtype=torch.float32):
    """Area-weighted outward face normals [M,4,3] (faces 012, 013, 123, 023). `solver/element.py:652-705`."""
    edges = [[r[0], r[1], r[2]] for r in TET_SHARED]
    return _element_normals(coords, elements, edges, TET_SHARED, TET_SHARED_X, 0.5, True, False, 4, device, dtype)


def compute_hexahedral_normals_and_area(coords, elements, device="cuda:0", dtype=torch.float32):
    """Outward face normals (p1-p0) x (p3-p0) [M,6,3]. `solver/element.py:1418-1472`."""
    edges = [[r[0], r[1], r[3]] for r in HEX]
    return _element_normals(coords, elements, edges, HEX, HEX_AREA_X, 1.0, True, False, 8, device, dtype)


def compute_wedge_normals_and_area(coords, elements, device="cuda:0", dtype=torch.float32):
    """Unit face normals [M,5,3], three quads then two triangles, not oriented. `solver/element.py:2377-2422`."""
    edges = [[r[0], r[1], r[3]] for r in WEDGE_QUAD] + [[r[0], r[1], r[2]] for r in WEDGE_TRI]
    return _element_normals(coords, elements, edges, [[0]] * 5, [0] * 5, 1.0, False, True, 6, device, dtype)


# ---------------------------------------------------------------- shared faces / element graph / edges
def identify_tetrahedral_shared_faces(elements, device="cuda:0"):
    """[S,2,2] ((element, face), (element, face)) for every face shared by exactly two tets, in lexicographic
    order of the sorted face nodes (faces 012, 013, 123, 023). `solver/element.py:707-762`. Inside a pair the
    lower (element, face) comes first; the reference leaves that order to an unstable sort (`:748`)."""
    g = FaceGroups(elements, TET_SHARED, device)
    out = g.pairs()
    g.close()
    return _out(out, device)


def identify_hexahedral_shared_faces(elements, device="cuda:0"):
    """Hex analogue of identify_tetrahedral_shared_faces (6 faces). `solver/element.py:1474-1532`."""
    g = FaceGroups(elements, HEX, device)
    out = g.pairs()
    g.close()
    return _out(out, device)


def element_adjacency(elements, device="cuda:0"):
    """Element graph of the shared faces as CSR (rowptr [M+1] int64, cols int64, neighbours ascending): the
    coalesced symmetric adjacency `subdivision.ipynb` builds (`build_adjacency_matrix`, cell 9) for its
    partitioner. Tets (4 nodes) or hexes (8 nodes)."""
    el = elements
    npe = el.shape[1]
    pairs = (identify_tetrahedral_shared_faces if npe in (4, 10) else identify_hexahedral_shared_faces)(
        el, device=_dev(device))
    M = el.shape[0]
    a, b = pairs[:, 0, 0], pairs[:, 1, 0]
    src = torch.cat([a, b])
    dst = torch.cat([b, a])
    key = src * M + dst
    key = torch.unique(key)            # coalesce (sorted)
    rows, cols = key // M, key % M
    rowptr = torch.zeros(M + 1, dtype=LONG, device=key.device)
    rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=M), 0)
    return _out(rowptr, device), _out(cols, device)


def element_to_edge(elements, device="cuda:0"):
    """Unique node edges [2,E] of tets (6 per element), columns in lexicographic order.
    `solver/element.py:2687-2713`."""
    g = FaceGroups(elements, EDGES, device)
    out = g.unique()
    g.close()
    return _out(out.t(), device)


# ---------------------------------------------------------------- element splits
def _split(elements, npe, device):
    lib = C.lib()
    dev = _dev(device)
    el = elements.to(device=dev, dtype=LONG).contiguous()
    if el.dim() != 2 or el.shape[1] != npe:
        raise ValueError(f"expected [M, {npe}] connectivity, got {list(el.shape)}")
    tab = SPLIT[npe]
    M = el.shape[0]
    out = torch.empty((M * len(tab), 4), dtype=LONG, device=dev)
    C.check(lib.fem_sub_elements(C.ptr(el), M, npe, _i32(tab), len(tab), 4, C.ptr(out), C.stream(dev)),
            "fem_sub_elements")
    return _out(out, device)


def c3d8_to_c3d4(c3d8_elements, device="cuda:0"):
    """[6M, 4] tets of every hex. `solver/element.py:1555-1581`."""
    return _split(c3d8_elements, 8, device)


def c3d6_to_c3d4(element, device="cuda:0"):
    """[3M, 4] tets of every wedge. `solver/element.py:2424-2446`."""
    return _split(element, 6, device)


def c3d10_to_c3d4(c3d10_elements, device="cuda:0"):
    """[8M, 4] linear tets of every quadratic tet. `solver/element.py:963-993`."""
    return _split(c3d10_elements, 10, device)


def to_c3d4(elements, device="cuda:0"):
    """Dispatch on nodes per element (`solver/element.py:355-364`; c3d20 out of scope -> None like an
    unmatched width)."""
    n = elements.shape[1]
    if n in SPLIT:
        return _split(elements, n, device)
    return None


__all__ = [
    "compute_tetrahedral_surface_faces_with_fourth_node", "compute_hexahedral_surface_faces_with_extra_node",
    "compute_wedge_surface_faces_with_extra_node", "compute_tetrahdral_surface_normals",
    "compute_tetrahedral_surface_normals", "compute_hexahedral_surface_normals", "compute_wedge_surface_normals",
    "compute_tetrahedral_normals_and_area", "compute_hexahedral_normals_and_area", "compute_wedge_normals_and_area",
    "identify_tetrahedral_shared_faces", "identify_hexahedral_shared_faces", "element_adjacency", "element_to_edge",
    "c3d8_to_c3d4", "c3d6_to_c3d4", "c3d10_to_c3d4", "to_c3d4", "FaceGroups",
]

# every public function runs in the scope of the device its `device` argument names (_capi.on_device)
C.scope_module(globals())
