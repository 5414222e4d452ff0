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


def _lame(E, nu):
    c = E / ((1.0 + nu) * (1.0 - 2.0 * nu))
    return c * nu, c * ((1.0 - 2.0 * nu) / 2.0)


def _cofactors(x):
    """x [M,4,3] -> (c [M,4,3] cofactor vectors with c_0 = -(c_1 + c_2 + c_3), det [M])."""
    e = x[:, 1:, :] - x[:, :1, :]
    c1 = torch.cross(e[:, 1], e[:, 2], dim=1)
    c2 = torch.cross(e[:, 2], e[:, 0], dim=1)
    c3 = torch.cross(e[:, 0], e[:, 1], dim=1)
    c = torch.stack([-(c1 + c2 + c3), c1, c2, c3], 1)
    det = (e[:, 0] * c1).sum(1)
    return c, det


def _mf_elastic(x, u, E, nu):
    lam, mu = _lame(E, nu)
    c, det = _cofactors(x)
    s = 1.0 / (6.0 * det.abs())
    d = u[:, 1:, :] - u[:, :1, :]                          # [M,3,3]: (u_b - u_0)[i]
    H = torch.einsum("mbi,mbj->mij", d, c[:, 1:, :])       # sum_b (u_b - u_0) c_b^T
    tr = H.diagonal(dim1=1, dim2=2).sum(1)
    sig = lam * tr[:, None, None] * torch.eye(3, dtype=F64) + mu * (H + H.transpose(1, 2))
    return torch.einsum("mij,maj->mai", sig * s[:, None, None], c)   # f_a = s sigma c_a


def _mf_poisson(x, u, kappa):
    c, det = _cofactors(x)
    s = kappa / (6.0 * det.abs())
    gu = torch.einsum("mbk,mb->mk", c[:, 1:, :], u[:, 1:] - u[:, :1])
    return s[:, None] * torch.einsum("mak,mk->ma", c, gu)


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

