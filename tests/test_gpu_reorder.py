"""Node renumbering on the device (system.rcm_order, csrc/reorder.hip) against the oracle's rule
(oracle/rcm_ref.py): the same permutation exactly, and a solve on the renumbered mesh equal to the oracle's PCG on
the caller's numbering (SURVEY §8(c) contract: u 1e-10, iterations +-2)."""
import numpy as np
import pytest
import torch

from conftest import rel
from oracle import ref_cpu as R
from oracle import rcm_ref

pytestmark = pytest.mark.gpu
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import mesh, solver, system
    return mesh, solver, system


def _permute(c, t, seed):
    perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(seed))
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    return c[perm], inv[t]


def _helix_fan(m):
    th = torch.arange(1, m + 3, dtype=F64) * 0.3
    c = torch.cat([torch.zeros(1, 3, dtype=F64), torch.stack([torch.cos(th), torch.sin(th), 0.05 * th], 1)])
    a = torch.arange(1, m + 1)
    return c, torch.stack([torch.zeros_like(a), a, a + 1, a + 2], 1)


@pytest.mark.parametrize("case", ["permuted", "lexicographic", "components", "fan", "bigfan"])
def test_device_rcm_equals_oracle(gpu, case):
    """bigfan: a 1.1M-tet fan -- a hub row of 1.1M columns (the pattern's bitmap tier) and, from the helix end, a
    BFS level of ~1.1M nodes, wide enough for many rounds of the level-write kernel's 4,096-node scan (the wide-level
    path)."""
    mesh, _, system = _mods()
    if case in ("fan", "bigfan"):
        c, t = _helix_fan(300 if case == "fan" else 1_100_000)
        N = c.shape[0]
    elif case == "components":
        c, t = mesh.kuhn_cube(4)
        N1 = c.shape[0]
        t = torch.cat([_permute(c, t, 1)[1], t + N1 + 7])
        N = 2 * N1 + 11
    else:
        c, t = mesh.kuhn_cube(9)
        if case == "permuted":
            c, t = _permute(c, t, 5)
        N = c.shape[0]
    perm, inv = system.rcm_order(t.to(gpu), N)
    rp, ci = R.node_pattern(t, N)
    operm, oinv = rcm_ref.rcm(rp.numpy(), ci.numpy(), N)
    assert np.array_equal(perm.cpu().numpy(), operm) and np.array_equal(inv.cpu().numpy(), oinv), case
    perm2, _ = system.rcm_order(t.to(gpu), N)
    assert torch.equal(perm, perm2)                      # deterministic


def test_reordered_solve_matches_oracle(gpu):
    """A randomly numbered cube (file order): the RCM-renumbered solve gives the oracle's PCG solution on the
    caller's numbering, and the renumbered operator gets 16-bit columns back."""
    mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    c, t = _permute(c, t, 9)
    f, fixed = mesh.cube_poisson_case(c)
    N = c.shape[0]
    u, res, A = solver.solve_tet4(c, t, f, fixed, kind="poisson", tol=1e-10, device=gpu, reorder="rcm")
    KP = R.tet4_poisson_K(c, t)
    dinv = R.diag_preconditioner(KP, t, N, dpn=1)
    dinv[fixed] = 0.0
    u_ref, it_ref, _ = R.pcg(KP, t, f, dinv, tol=1e-10)
    assert rel(u.cpu().view(-1), u_ref.view(-1)) < 1e-10 and abs(res.iterations - it_ref) <= 2
    assert A.use16
    u0, res0, A0 = solver.solve_tet4(c, t, f, fixed, kind="poisson", tol=1e-10, device=gpu)
    assert not A0.use16 or A0.g.sell_entries >= A.g.sell_entries
    assert rel(u0.cpu().view(-1), u_ref.view(-1)) < 1e-10
