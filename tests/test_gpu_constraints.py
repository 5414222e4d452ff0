"""GPU: constraint-aware CG (reference `solver/solver.py:394-759`) through the C-ABI.

Oracle: `oracle.ref_cpu.constrained_cg` / `enforce`, pinned bit-exact to the reference by
`tests/test_oracle_golden.py::test_constrained_cg_oracle_matches_reference` (fixture `constrained_tet4`).
Tolerances (fp64): projections bit-exact for the copies (SPC / RBE2), 1e-14 relative for RBE3 means (reduction
order); solutions 1e-9 relative with iteration counts within ±2 of the reference; fixed-iteration iterates 1e-10.
"""
import json

import pytest
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import _capi, constraints, mesh, solver, system
    return _capi, constraints, mesh, solver, system


def _fixture():
    g = load_golden("constrained_tet4")
    return g, json.loads(str(g["constraints"]))


def test_constrained_cg_vs_reference(gpu, capsys):
    _, _, _, solver, _ = _mods()
    g, c = _fixture()
    K = R.tet4_K(g["coords"], g["tets"], E, NU)
    tol = float(g["tol"])
    u, res = solver.constrained_conjugate_gradient_solver(K, g["tets"], g["F"], c["rbe2_a"], c["spc"], tol=tol,
                                                          max_iter=3000, device=gpu, return_info=True)
    out = capsys.readouterr().out
    assert res.status == 1 and abs(res.iterations - int(g["n_iter_a"])) <= 2, (res.iterations, int(g["n_iter_a"]))
    assert out.strip().startswith(f"[CG] Converged @ iter {res.iterations}, residual norm = ")
    assert rel(u, g["u_a"]) < 1e-9
    # projections hold exactly on the returned iterate
    m = c["rbe2_a"][0]["master"]
    u = u.cpu()
    assert torch.equal(u[c["rbe2_a"][0]["slaves"]], u[m].expand(len(c["rbe2_a"][0]["slaves"]), 3))
    for s in c["spc"]:
        assert all(float(u[s["node"], d]) == s["value"] for d in s["dofs"])


def test_new_constrained_cg_vs_reference(gpu, capsys):
    _, _, _, solver, _ = _mods()
    g, c = _fixture()
    K = R.tet4_K(g["coords"], g["tets"], E, NU)
    N = g["coords"].shape[0]
    u, res = solver.new_constrained_conjugate_gradient_solver(K, g["tets"], N, c["rbe2_b"], c["rbe3_b"], c["spc"],
                                                              c["loads_b"], tol=float(g["tol"]), max_iter=3000,
                                                              device=gpu, return_info=True)
    out = capsys.readouterr().out
    assert res.status == 1 and abs(res.iterations - int(g["n_iter_b"])) <= 2, (res.iterations, int(g["n_iter_b"]))
    assert out.strip().startswith(f"[CG] Converged @ iter {res.iterations}, residual norm = ")
    assert rel(u, g["u_b"]) < 1e-9
    # RBE3 masters are the weighted means of their slaves (last projection, after SPC and RBE2)
    u = u.cpu()
    for s3 in c["rbe3_b"]:
        w = torch.tensor(s3["weights"], dtype=F64)
        for d in s3["dofs"]:
            mean = torch.sum(w * u[s3["slaves"], d]) / (w.sum() + 1e-30)
            assert abs(float(u[s3["master"], d] - mean)) <= 1e-14 * float(u.abs().max())


@pytest.mark.parametrize("case", ["a", "b"])
def test_constrained_fixed_iterations_vs_oracle(gpu, case, capsys):
    _, _, _, solver, _ = _mods()
    g, c = _fixture()
    K = R.tet4_K(g["coords"], g["tets"], E, NU)
    N = g["coords"].shape[0]
    u0 = torch.randn(N, 3, dtype=F64, generator=torch.Generator().manual_seed(3)) * 1e-6
    if case == "a":
        ref, n, s = R.constrained_cg(K, g["tets"], g["F"], c["rbe2_a"], c["spc"], u_init=u0, tol=0.0, max_iter=15)
        u = solver.constrained_conjugate_gradient_solver(K, g["tets"], g["F"], c["rbe2_a"], c["spc"], u_init=u0,
                                                         tol=0.0, max_iter=15, device=gpu)
    else:
        F = R.loads_to_F(N, c["loads_b"])
        ref, n, s = R.constrained_cg(K, g["tets"], F, c["rbe2_b"], c["spc"], c["rbe3_b"], u_init=u0, tol=0.0,
                                     max_iter=15)
        u = solver.new_constrained_conjugate_gradient_solver(K, g["tets"], N, c["rbe2_b"], c["rbe3_b"], c["spc"],
                                                             c["loads_b"], u_init=u0, tol=0.0, max_iter=15,
                                                             device=gpu)
    assert s == "max_iter" and "[CG] Did not converge within max_iter." in capsys.readouterr().out
    assert rel(u, ref) < 1e-10


def test_enforce_standalone_vs_oracle(gpu):
    _, cons, _, solver, _ = _mods()
    g, c = _fixture()
    N = g["coords"].shape[0]
    gen = torch.Generator().manual_seed(11)
    u = torch.randn(N, 3, dtype=F64, generator=gen)
    r = torch.randn(N, 3, dtype=F64, generator=gen)
    # order 0: pure copies -> bit-exact
    ur, rr = u.clone(), r.clone()
    R.enforce(ur, rr, c["rbe2_a"], c["spc"])
    ud, rd = u.to(gpu), r.to(gpu)
    solver.enforce_constraints(ud, rd, *solver.parse_spc_list(c["spc"], gpu), *solver.parse_rbe2_list(c["rbe2_a"], gpu))
    assert torch.equal(ud.cpu(), ur) and torch.equal(rd.cpu(), rr)
    # order 1 with RBE3, on a host tensor (computed on the device, written back in place)
    ur, rr = u.clone(), r.clone()
    R.enforce(ur, rr, c["rbe2_b"], c["spc"], c["rbe3_b"])
    uh, rh = u.clone(), r.clone()
    solver.new_enforce_constraints(uh, rh, *solver.parse_spc_list(c["spc"], "cpu"),
                                   *solver.parse_rbe2_list(c["rbe2_b"], "cpu"), *solver.parse_rbe3_list(c["rbe3_b"], "cpu"))
    assert rel(uh, ur) < 1e-14 and torch.equal(rh, rr)


def test_large_sets_use_grid_phases(gpu):
    """> 8192 SPC + RBE2 entries switch to the grid-wide gather / scatter / SPC kernels: same result."""
    _, cons, _, _, _ = _mods()
    N = 20000
    gen = torch.Generator().manual_seed(5)
    u = torch.randn(N, 3, dtype=F64, generator=gen)
    r = torch.randn(N, 3, dtype=F64, generator=gen)
    perm = torch.randperm(N, generator=gen).tolist()
    rbe2 = [{"master": perm[i], "slaves": perm[i + 1:i + 4], "dofs": [0, 1, 2]} for i in range(0, 12000, 4)]
    spc = [{"node": perm[i], "dofs": [0, 2], "value": 0.5 * i} for i in range(12000, 16000)]
    spc += [{"node": perm[1], "dofs": [1], "value": -3.0}]   # an RBE2 slave also SPC'd: the later phase wins
    rbe3 = [{"master": perm[16000 + k], "slaves": perm[16100 + 5 * k:16105 + 5 * k], "dofs": [2, 0],
             "weights": [1.0, 2.0, 3.0, 0.5, 0.25]} for k in range(20)]
    for order, r3 in ((0, None), (1, rbe3)):
        ur, rr = u.clone(), r.clone()
        R.enforce(ur, rr, rbe2, spc, r3)
        cs = cons.ConstraintSet(N, 3, gpu, cons.parse_spc_list(spc, "cpu"), cons.parse_rbe2_list(rbe2, "cpu"),
                                cons.parse_rbe3_list(r3, "cpu") if r3 else None, order=order)
        assert cs.rbe2_slave.numel() + cs.spc_dof.numel() > 8192
        ud, rd = u.to(gpu), r.to(gpu)
        cs.enforce(ud, rd)
        assert rel(ud, ur) < 1e-14 and torch.equal(rd.cpu(), rr), order


def test_constraint_errors(gpu):
    C, cons, _, solver, system = _mods()
    g, c = _fixture()
    K = R.tet4_K(g["coords"], g["tets"], E, NU)
    N = g["coords"].shape[0]
    bad = [{"node": N + 3, "dofs": [0], "value": 0.0}]
    with pytest.raises(IndexError):
        solver.constrained_conjugate_gradient_solver(K, g["tets"], g["F"], [], bad, device=gpu)
    with pytest.raises(IndexError):
        solver.constrained_conjugate_gradient_solver(K, g["tets"], g["F"], [], [{"node": 0, "dofs": [3], "value": 0}],
                                                     device=gpu)
    # negative node indices wrap like torch indexing
    u = solver.constrained_conjugate_gradient_solver(K, g["tets"], g["F"], [], [{"node": -1, "dofs": [1],
                                                                                  "value": 2e-6}],
                                                     tol=1e-3, max_iter=5, device=gpu)
    assert float(u[N - 1, 1]) == 2e-6
    # the C-ABI rejects an out-of-range dof and a non-3-kernel schedule
    A = solver.assemble(K, g["tets"], N, gpu)
    cs = cons.ConstraintSet(N, 3, gpu, cons.parse_spc_list(c["spc"], "cpu"), cons.parse_rbe2_list(c["rbe2_a"], "cpu"))
    cs.spc_dof[0] = 3 * N
    b = g["F"].to(gpu).reshape(-1)
    with pytest.raises(C.FemError, match="outside"):
        A.pcg(b, None, w=torch.ones(3 * N, dtype=F64, device=gpu),
              mode=C.MODE_CG_CONSTRAINED, schedule=0, constraints=cs)
    cs.spc_dof[0] = 0
    with pytest.raises(C.FemError, match="3-kernel"):
        A.pcg(b, None, w=torch.ones(3 * N, dtype=F64, device=gpu), mode=C.MODE_CG_CONSTRAINED, schedule=2,
              constraints=cs)
