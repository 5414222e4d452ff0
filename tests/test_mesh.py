import torch

from fem355 import mesh
from oracle import ref_cpu as R


def test_kuhn_counts_and_orientation():
    for n in (1, 2, 6):
        c, t = mesh.kuhn_cube(n)
        M, N, nnz = mesh.cube_counts(n)
        assert t.shape == (M, 4) and c.shape == (N, 3)
        rp, ci = R.node_pattern(t, N)
        assert int(rp[-1]) == nnz
        p = c[t]
        det = torch.det(torch.stack([p[:, 1] - p[:, 0], p[:, 2] - p[:, 0], p[:, 3] - p[:, 0]], 1))
        assert bool((det > 0).all())
        assert abs(float(R.tet_volumes(c, t).sum()) - 1.0) < 1e-12


def test_other_families_fill_the_cube():
    c, h = mesh.hex_box(3)
    assert abs(float(R.iso_K(c, h, "c3d8", 1.0, 0.3).shape[0]) - 27) == 0
    c, w = mesh.wedge_box(3)
    assert abs(float(R.wedge_volumes(c, w).sum()) - 1.0) < 1e-12
    c, t10 = mesh.tet10_cube(2)
    assert t10.shape == (48, 10) and c.shape[0] == 27 + 3 * 2 * 9 + 3 * 4 * 3 + 8


def test_mass_rules_and_oracle_mass():
    """Consistent-mass quadrature (no reference function, parity unpinned): the c3d10 rule integrates every monomial of
    degree <= 5 over the unit tet exactly, the wedge rule sums to the reference prism volume 1 (not 2, Q3), and the
    oracle's mass of each family on an unjittered unit box totals rho (sum of entries / 3), symmetric, positive
    definite."""
    import math
    from fem355 import element as el
    p, w = el.mass_integration_points("c3d10")
    for i in range(6):
        for j in range(6 - i):
            for k in range(6 - i - j):
                exact = math.factorial(i) * math.factorial(j) * math.factorial(k) / math.factorial(i + j + k + 3)
                q = float((w * p[:, 0] ** i * p[:, 1] ** j * p[:, 2] ** k).sum())
                assert abs(q - exact) <= 1e-14 * exact
    pw, ww = el.mass_integration_points("c3d6")
    assert abs(float(ww.sum()) - 1.0) < 1e-15 and pw.shape == (6, 3)
    assert abs(float(el.mass_integration_points("c3d8")[1].sum()) - 8.0) < 1e-15
    rho = 4.47e-3
    for etype, gen in (("c3d8", mesh.hex_box), ("c3d6", mesh.wedge_box), ("c3d10", mesh.tet10_cube)):
        c, t = gen(2)
        pts, wts = el.mass_integration_points(etype)
        Me = R.iso_mass(c, t, el._N[etype], el._ISO[etype][1], pts, wts, rho)
        assert abs(float(Me.sum()) / 3 - rho) < 1e-14, etype
        assert float((Me - Me.transpose(1, 2)).abs().max()) == 0.0
        assert float(torch.linalg.eigvalsh(Me[:3]).min()) > 0.0
