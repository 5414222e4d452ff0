"""GPU: mesh topology (reference `solver/element.py:543-762,963-993,1293-1581,2234-2446,
2687-2713`) through the C-ABI.

Oracle: `oracle.ref_cpu.{boundary_faces, shared_faces, surface_normals, element_face_normals, unique_edges,
split_elements}`, pinned to the reference by `tests/test_oracle_golden.py::test_topology_oracle_matches_reference`
(fixture `topology`). Index outputs are bit-exact (shared-face pairs up to the order inside a pair, which the reference leaves to an
unstable sort; fem355 puts the lower (element, face) first); normals 1e-14 relative (sqrt / division order). The wedge
normals_and_area function raises inside the reference (`:2409`): its intended result is checked against the
oracle's restatement only (parity unpinned). Full size: the 10M-tet cube's face / edge counts satisfy the closed
forms (12 n^2 boundary triangles, Euler characteristic 1) and sampled pairs really share their nodes.
"""
import pytest
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
F64 = torch.float64


def canon(pairs, F):
    """Pairs with the lower (element, face) first: the reference's within-pair order comes from an unstable
    torch.sort of the inverse indices (`solver/element.py:748`) and is not defined; the pair list order is."""
    a = pairs[:, 0, 0] * F + pairs[:, 0, 1]
    b = pairs[:, 1, 0] * F + pairs[:, 1, 1]
    sw = (a > b).view(-1, 1, 1)
    return torch.where(sw, pairs.flip(1), pairs)


def _mods():
    import fem355  # noqa: F401
    from fem355 import element, mesh, topology
    return element, mesh, topology


def test_tet_topology_vs_reference(gpu):
    el, _, T = _mods()
    g = load_golden("topology")
    c, t = g["tet_coords"], g["tets"]
    f, x = el.compute_tetrahedral_surface_faces_with_fourth_node(t, device=gpu)
    assert torch.equal(f.cpu(), g["tet_surf"]) and torch.equal(x.cpu(), g["tet_surf_x"])
    assert rel(el.compute_tetrahdral_surface_normals(c, t, device=gpu, dtype=F64), g["tet_surf_n"]) < 1e-14
    assert rel(el.compute_tetrahedral_normals_and_area(c, t, device=gpu, dtype=F64), g["tet_area_n"]) < 1e-14
    sh = el.identify_tetrahedral_shared_faces(t, device=gpu).cpu()
    assert torch.equal(sh, canon(sh, 4)) and torch.equal(sh, canon(g["tet_shared"], 4))
    assert torch.equal(el.element_to_edge(t, device=gpu).cpu(), g["tet_edges"])


def test_hex_wedge_topology_vs_reference(gpu):
    el, _, T = _mods()
    g = load_golden("topology")
    ch, h = g["hex_coords"], g["hexes"]
    f, x = el.compute_hexahedral_surface_faces_with_extra_node(h, device=gpu)
    assert torch.equal(f.cpu(), g["hex_surf"]) and torch.equal(x.cpu(), g["hex_surf_x"])
    assert rel(el.compute_hexahedral_surface_normals(ch, h, device=gpu, dtype=F64), g["hex_surf_n"]) < 1e-14
    assert rel(el.compute_hexahedral_normals_and_area(ch, h, device=gpu, dtype=F64), g["hex_area_n"]) < 1e-14
    sh = el.identify_hexahedral_shared_faces(h, device=gpu).cpu()
    assert torch.equal(sh, canon(sh, 6)) and torch.equal(sh, canon(g["hex_shared"], 6))
    assert torch.equal(el.c3d8_to_c3d4(h, device=gpu).cpu(), g["hex_tets"])
    cw, w = g["wedge_coords"], g["wedges"]
    (fq, ft), (xq, xt) = el.compute_wedge_surface_faces_with_extra_node(w, device=gpu)
    assert torch.equal(fq.cpu(), g["wedge_surf_q"]) and torch.equal(ft.cpu(), g["wedge_surf_t"])
    assert torch.equal(xq.cpu(), g["wedge_surf_xq"]) and torch.equal(xt.cpu(), g["wedge_surf_xt"])
    nq, nt = el.compute_wedge_surface_normals(cw, w, device=gpu, dtype=F64)
    assert rel(nq, g["wedge_surf_nq"]) < 1e-14 and rel(nt, g["wedge_surf_nt"]) < 1e-14
    assert torch.equal(el.c3d6_to_c3d4(w, device=gpu).cpu(), g["wedge_tets"])
    assert torch.equal(el.c3d10_to_c3d4(g["tet10"], device=gpu).cpu(), g["tet10_tets"])
    assert torch.equal(el.to_c3d4(h, device=gpu).cpu(), g["hex_tets"])
    # intended result of the (broken) reference wedge normals: unit, quads (p1-p0)x(p3-p0) then triangles
    rows = [[r[0], r[1], r[3]] for r in T.WEDGE_QUAD] + [list(r) for r in T.WEDGE_TRI]
    ref = R.element_face_normals(cw, w, None, rows, unit=True)
    assert rel(el.compute_wedge_normals_and_area(cw, w, device=gpu, dtype=F64), ref) < 1e-14


def test_topology_vs_oracle_medium(gpu):
    """A 12^3 Kuhn cube with 5% of the tets removed (inner surfaces) and shuffled element order."""
    el, mesh, T = _mods()
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    gen = torch.Generator().manual_seed(4)
    keep = torch.randperm(t.shape[0], generator=gen)[: int(0.95 * t.shape[0])]
    t = t[keep]
    f, x = el.compute_tetrahedral_surface_faces_with_fourth_node(t, device=gpu)
    fr, xr = R.boundary_faces(t, T.TET_SURFACE, T.TET_SURFACE_X)
    assert torch.equal(f.cpu(), fr) and torch.equal(x.cpu(), xr)
    assert torch.equal(el.identify_tetrahedral_shared_faces(t, device=gpu).cpu(), canon(R.shared_faces(t, T.TET_SHARED), 4))
    assert torch.equal(el.element_to_edge(t, device=gpu).cpu(), R.unique_edges(t, T.EDGES))
    rowptr, cols = el.element_adjacency(t, device=gpu)
    pairs = R.shared_faces(t, T.TET_SHARED)
    assert int(rowptr[-1]) == 2 * pairs.shape[0]
    deg = torch.bincount(torch.cat([pairs[:, 0, 0], pairs[:, 1, 0]]), minlength=t.shape[0])
    assert torch.equal((rowptr[1:] - rowptr[:-1]).cpu(), deg)


def test_full_size_counts_and_euler(gpu):
    el, mesh, T = _mods()
    n = 119
    c, t = mesh.kuhn_cube(n, device=gpu)
    M, V = t.shape[0], c.shape[0]
    g = T.FaceGroups(t, T.TET_SHARED, gpu)
    assert g.n_single == 12 * n * n and 2 * g.n_pair + g.n_single == 4 * M
    Fu = g.n_unique
    pairs = g.pairs()
    g.close()
    # sampled pairs share exactly their node set
    idx = torch.randint(0, pairs.shape[0], (100000,), device=gpu)
    tab = torch.tensor(T.TET_SHARED, device=gpu)
    p = pairs[idx]
    fa = torch.sort(t[p[:, 0, 0]].gather(1, tab[p[:, 0, 1]]), 1)[0]
    fb = torch.sort(t[p[:, 1, 0]].gather(1, tab[p[:, 1, 1]]), 1)[0]
    assert torch.equal(fa, fb) and bool((p[:, 0, 0] * 4 + p[:, 0, 1] < p[:, 1, 0] * 4 + p[:, 1, 1]).all())
    E = el.element_to_edge(t, device=gpu).shape[1]
    assert V - E + Fu - M == 1          # a ball
    f, x = el.compute_tetrahedral_surface_faces_with_fourth_node(t, device=gpu)
    assert f.shape == (12 * n * n, 3)
    nrm = el.compute_tetrahdral_surface_normals(c, t, device=gpu, dtype=F64)
    # outward normals of the unit cube: one axis-aligned unit vector per face, pointing out
    ctr = c[f].mean(1)
    assert bool(((nrm * (ctr - 0.5)).sum(1) > 0).all()) and float((nrm.abs().max(1)[0] - 1).abs().max()) < 1e-12
