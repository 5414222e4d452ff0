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
