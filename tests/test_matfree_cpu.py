"""CPU tier of the element-chunk operator's algebra (csrc/matfree.hpp mf_element): the cofactor form of the c3d4
element force, restated here in torch fp64, against the oracle's element matrices (`oracle/ref_cpu.py` tet4_K /
tet4_poisson_K, pinned to the reference's `compute_c3d4_K_matrix`, `solver/element.py:883-903`) applied to the
element's displacements -- the closed form the GPU kernel evaluates, checked without a GPU."""
import pytest
import torch

from conftest import rel
from oracle import ref_cpu as R

F64 = torch.float64
E, NU = 113.8e9, 0.342


def _mf_elastic(x, u, E, nu):
    """x [M,4,3] element coordinates, u [M,4,3] element displacements -> the oracle's closed-form element vectors."""
    M = x.shape[0]
    t = torch.arange(4 * M).view(M, 4)
    return R.tet4_element_forces(x.reshape(-1, 3), t, u.reshape(-1), "elastic", E, nu)


def _mf_poisson(x, u, kappa):
    M = x.shape[0]
    t = torch.arange(4 * M).view(M, 4)
    return R.tet4_element_forces(x.reshape(-1, 3), t, u.reshape(-1), "poisson", kappa)[..., 0]


@pytest.mark.parametrize("jitter", [0.0, 0.15])
def test_cofactor_form_equals_element_matrices(jitter):
    from fem355 import mesh
    coords, tets = mesh.kuhn_cube(4, jitter=jitter)
    x = coords[tets]                                       # [M,4,3]
    g = torch.Generator().manual_seed(7)
    u = torch.randn(coords.shape[0], 3, dtype=F64, generator=g)
    Ke = R.tet4_K(coords, tets, E, NU)                     # [M,12,12], local dof 3 a + i
    f_ref = torch.einsum("mij,mj->mi", Ke, u[tets].reshape(-1, 12)).reshape(-1, 4, 3)
    assert rel(_mf_elastic(x, u[tets], E, NU), f_ref) < 1e-13
    # reversed orientation (negative det): the |det| of the volume keeps the operator the same
    t2 = tets[:, [0, 2, 1, 3]]
    Ke2 = R.tet4_K(coords, t2, E, NU)
    f2 = torch.einsum("mij,mj->mi", Ke2, u[t2].reshape(-1, 12)).reshape(-1, 4, 3)
    assert rel(_mf_elastic(coords[t2], u[t2], E, NU), f2) < 1e-13
    up = torch.randn(coords.shape[0], dtype=F64, generator=g)
    Kp = R.tet4_poisson_K(coords, tets, kappa=2.5)
    fp_ref = torch.einsum("mij,mj->mi", Kp, up[tets])
    assert rel(_mf_poisson(x, up[tets], 2.5), fp_ref) < 1e-13



@pytest.mark.parametrize("kind", ["elastic", "poisson"])
def test_matfree_product_and_diagonal_vs_element_matrices(kind):
    """The oracle's EBE product without K_e (`tet4_forces_matfree`, the element-chunk operator's algebra) and its exact
    diagonal against the reference op sequence over stored element matrices (`nodal_forces`, `solver/element.py:
    429-464`)."""
    from fem355 import mesh
    coords, tets = mesh.kuhn_cube(5, jitter=0.15)
    N = coords.shape[0]
    dpn, Ek = (3, E) if kind == "elastic" else (1, 2.5)
    K = R.tet4_K(coords, tets, E, NU) if kind == "elastic" else R.tet4_poisson_K(coords, tets, kappa=Ek)
    u = torch.randn(N * dpn, dtype=F64, generator=torch.Generator().manual_seed(3))
    y = R.tet4_forces_matfree(coords, tets, u, kind, Ek, NU)
    assert rel(y, R.nodal_forces(K, tets, u.view(N, dpn)).reshape(-1)) < 1e-13
    d = torch.zeros(N * dpn, dtype=F64).index_add_(0, R.dof_map(tets, dpn).reshape(-1),
                                                    torch.diagonal(K, dim1=1, dim2=2).reshape(-1))
    assert rel(R.tet4_diag_matfree(coords, tets, kind, Ek, NU), d) < 1e-13
