"""GPU tier at the BASELINE.json configuration sizes: the HIP path against the oracle (`oracle/ref_cpu.py`, the
reference's op sequence on torch-CPU, pinned bit-exactly to the reference's golden vectors by
`tests/test_oracle_golden.py`) on the full benchmark meshes, not on stand-ins. Ordered cheapest first (the driver
runs `pytest -x`).

  * configs[4] (2M-element c3d8 / c3d6 / c3d10 set): `compute_K_matrix` on each whole family mesh, a seeded
    10,000-element sample checked against `R.iso_K` (`solver/element.py:1754-1803`, `:2631-2676`, `:1191-1239`);
  * configs[1] (1M-tet P1 Poisson, n = 55): `solve_tet4` to rtol 1e-8 against `R.pcg` over the oracle's element
    matrices (`solver/solver.py:766-812`): iterations within +-2, u within 1e-10;
  * configs[2] (10M-tet P1 elasticity, n = 119): the assembled SELL operator applied to a seeded vector against the
    oracle's EBE product `R.nodal_forces(R.tet4_K(...))` (`solver/element.py:429-464`, `:883-903`) to 1e-12, and the
    first 5 Jacobi-PCG iterates of the default bs = 3 schedule against `R.pcg` to 1e-10;
  * the metric (10M-tet P1 Poisson): the bench's operator and the exact persistent build it times (7 slots, 26,992
    slice-uniform slices) for 5 iterates against the oracle, the bench's whole DOFs/s solve to rtol 1e-8 (682
    iterations) against the oracle PCG end to end, and the same 5 iterates on the cube renumbered at random and then
    by device RCM (a mesh in file order).
The oracle's element matrices at 10M tets take ~12 GB of host memory and ~10 s on the box's 16 cores."""
import pytest
import torch

from conftest import rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import element, mesh, solver, system
    return element, mesh, solver, system


@pytest.mark.parametrize("etype,n", [("c3d6", 70), ("c3d8", 88), ("c3d10", 48)])
def test_config4_family_stiffness_sample_vs_oracle(gpu, etype, n):
    """BASELINE configs[4]: 686,000 wedges (2 x 70^3), 681,472 hexes (88^3), 663,552 P2 tets (6 x 48^3), jittered."""
    el, mesh, _, _ = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, e = gen(n, jitter=0.1)
    K = el.compute_K_matrix(c, e, etype, E, NU, device=gpu, dtype=F64)
    assert K.shape == (e.shape[0], 3 * e.shape[1], 3 * e.shape[1])
    idx = torch.randperm(e.shape[0], generator=torch.Generator().manual_seed(20250418))[:10000].sort().values
    Ks = K[idx.to(gpu)].cpu()
    del K
    assert rel(Ks, R.iso_K(c, e[idx], etype, E, NU)) < 1e-12


@pytest.mark.parametrize("etype,n", [("c3d6", 70), ("c3d8", 88), ("c3d10", 48)])
def test_config4_family_mass_at_size(gpu, etype, n):
    """BASELINE configs[4]'s mass half at its full size (no reference mass function exists, so
    parity stays unpinned -- these are the size-independent properties): the consistent mass of each whole jittered
    family mesh and its global assembly (the stored-K_e path of the bench) total rho x the unit box volume, the
    assembled matrix is symmetric bit for bit (block (i, j) = block (j, i)^T: both sum the same elements in the same
    ascending order), and on 2,000 sampled rows the assembled operator equals the element-by-element product over the
    oracle's restatement of the rule (`R.iso_mass`) at 1e-13."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    rho = 4.47e-3
    c, e = gen(n, jitter=0.1)
    N = c.shape[0]
    cg, eg = c.to(gpu), e.to(gpu)
    Me = el.compute_M_matrix(cg, eg, etype, rho, device=gpu, dtype=F64)
    assert abs(float(Me.sum()) / 3 / rho - 1.0) < 1e-11
    g = system.build_graph(eg, N)
    A = system.SellMatrix(g, 3).add_element_matrices(Me, eg)
    del Me
    assert abs(float(A.vals.sum()) / 3 / rho - 1.0) < 1e-11
    rp, ci, bv = A.csr()
    rows = torch.repeat_interleave(torch.arange(N, device=gpu), (rp[1:] - rp[:-1]).long())
    key = rows * N + ci.long()
    q = torch.searchsorted(key, ci.long() * N + rows)
    assert torch.equal(key[q], ci.long() * N + rows)          # the pattern is symmetric
    assert torch.equal(bv, bv[q].transpose(1, 2))            # and so are the values, bit for bit
    del rp, ci, bv, rows, key, q
    x = torch.randn(N, 3, dtype=F64, generator=torch.Generator().manual_seed(3))
    y = A.matvec(x.reshape(-1).to(gpu)).view(N, 3).cpu()
    S = torch.randperm(N, generator=torch.Generator().manual_seed(4))[:2000]
    touch = torch.isin(e, S).any(1)
    es = e[touch]
    pts, wts = el.mass_integration_points(etype)
    Ms = R.iso_mass(c, es, el._N[etype], el._ISO[etype][1], pts, wts, rho)
    ys = R.nodal_forces(Ms, es, x)
    assert rel(y[S], ys[S]) < 1e-13


def test_config1_poisson_1m_solve_vs_oracle(gpu):
    """BASELINE configs[1]: 998,250 tets, 175,616 DOFs, Jacobi-PCG to rtol 1e-8 (the bench's DOFs/s solve)."""
    _, mesh, solver, _ = _mods()
    c, t = mesh.kuhn_cube(55)
    f, fixed = mesh.cube_poisson_case(c)
    u, res, _ = solver.solve_tet4(c, t, f, fixed, kind="poisson", rtol=1e-8, device=gpu)
    KP = R.tet4_poisson_K(c, t)
    N = c.shape[0]
    dinv = R.diag_preconditioner(KP, t, N, dpn=1)
    dinv[fixed] = 0.0
    b = f.reshape(N, 1).to(F64)
    tol = 1e-8 * float(torch.sqrt(torch.sum(b * dinv * b)))
    u_ref, it_ref, st = R.pcg(KP, t, b, dinv, tol=tol, max_iter=5000)
    assert st == "converged" and abs(res.iterations - it_ref) <= 2, (res.iterations, it_ref)
    assert rel(u, u_ref) < 1e-10


def test_config2_elasticity_10m_operator_and_iterates_vs_oracle(gpu, cube119):
    """BASELINE configs[2]: 10,110,954 tets, 5,184,000 DOFs. The assembled operator (fused on-the-fly assembly into
    SELL-64 with 16-bit deltas, the bench's) equals the reference's EBE operator over its own element matrices, and
    the default bs = 3 schedule's first 5 PCG iterates equal the reference PCG's."""
    _, mesh, _, system = _mods()
    c, t, N = cube119.c, cube119.t, cube119.N
    assert t.shape[0] == 10_110_954
    f, fixed, dinv = cube119.case("elastic")
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", E, NU)
    assert A.use16
    p, y_ref = cube119.matvec_ref("elastic", 11)
    y = A.matvec(p.reshape(-1).to(gpu)).cpu()
    assert rel(y, y_ref.reshape(-1)) < 1e-12
    mask = torch.zeros((N, 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1)
    res = A.pcg(b, w=w, tol=0.0, max_iter=5)
    assert res.iterations == 5
    assert rel(w.cpu(), dinv.reshape(-1)) < 1e-14
    assert rel(res.x.cpu(), cube119.pcg_ref("elastic", 5).reshape(-1)) < 1e-10


def _poisson_persistent_iterates(system, A, b, w, steps):
    """The bench's fixed-iteration path: a PcgRunner with the default (persistent) schedule, a warm-up launch then a
    timed launch (`bench.py` measure()); returns (runner facts, x after sum(steps) iterations)."""
    run = system.PcgRunner(A, b, w, tol=0.0)
    try:
        run.start()
        facts = {"schedule": run.effective_schedule(), "build": run.persist_build(), "uniform": run.uniform_slices()}
        for k in steps:
            run.profile(k, every=k)
        assert run.poll()[0] == sum(steps)
        return facts, run.x.clone()
    finally:
        run.close()


def test_metric_poisson_10m_persistent_vs_oracle(gpu, cube119):
    """The metric's own system (BASELINE.json: 10M-tet P1 Poisson): the operator assembled by bench.py's path
    against the oracle's EBE product over its element matrices (`solver/element.py:429-464`) at 1e-12, the Jacobi
    weights at 1e-14, and the exact kernel build the bench times -- the 7-slot k_pcg_persist with the packed
    assignment and slice-uniform deltas on 26,992 of 27,000 slices -- for 5 iterations (a 2-step warm-up launch and a
    3-step timed launch, like bench.py) against the oracle PCG's 5th iterate (`solver/solver.py:766-812`) at 1e-10."""
    _, mesh, _, system = _mods()
    c, t, N = cube119.c, cube119.t, cube119.N
    f, fixed, dinv = cube119.case("poisson")
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    assert A.use16 and A.n == 1_728_000
    p, y_ref = cube119.matvec_ref("poisson", 12)
    assert rel(A.matvec(p.reshape(-1).to(gpu)), y_ref.reshape(-1)) < 1e-12
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask)
    assert rel(w, dinv.reshape(-1)) < 1e-14
    facts, x = _poisson_persistent_iterates(system, A, f.reshape(-1), w, (2, 3))
    assert facts["schedule"] == system.SCHED_PERSIST
    assert facts["build"] == (7, 0, 7), facts
    assert facts["uniform"][:2] == (26_992, 27_000), facts
    assert rel(x, cube119.pcg_ref("poisson", 5).reshape(-1)) < 1e-10


def test_metric_poisson_10m_full_solve_vs_oracle(gpu, cube119):
    """The metric's DOFs/s solve end to end: bench.py's assembly, Jacobi weights and Jacobi-PCG
    to rtol 1e-8 on sqrt(r.z) (the persistent kernel, one launch, stopping itself) against `R.pcg`
    (`solver/solver.py:766-812`) over the oracle's element matrices, its operator applied as the COO-coalesced CSR the
    reference assembles (`subdivision.ipynb:118-139`; equal to the EBE product to ~1e-16, and ~25x faster on the host,
    so the 682 oracle iterations take ~30 s). Contract: iterations within +-2, u within 1e-10."""
    _, _, _, system = _mods()
    from fem355 import _capi as C
    c, t, N = cube119.c, cube119.t, cube119.N
    f, fixed, dinv = cube119.case("poisson")
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask.index_fill_(0, fixed.to(gpu), 1)
    w = A.jacobi(mask)
    b = f.reshape(-1).to(gpu)
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    res = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64)
    assert res.status == C.PCG_CONVERGED
    u, iters = res.x.cpu(), res.iterations
    del A, w, res
    K = cube119.K("poisson")
    rows = t.unsqueeze(2).expand(-1, 4, 4).reshape(-1)
    cols = t.unsqueeze(1).expand(-1, 4, 4).reshape(-1)
    Acsr = torch.sparse_coo_tensor(torch.stack([rows, cols]), K.reshape(-1), (N, N)).coalesce().to_sparse_csr()
    del rows, cols
    p, y_ref = cube119.matvec_ref("poisson", 12)
    assert rel(Acsr @ p, y_ref) < 1e-14          # the CSR form is the oracle's EBE operator
    tol_ref = 1e-8 * float(torch.sqrt(torch.sum(f * dinv * f)))
    u_ref, it_ref, st = R.pcg(K, t, f, dinv, tol=tol_ref, max_iter=5000,
                              matvec=lambda v: (Acsr @ v.reshape(-1, 1)).reshape(v.shape))
    assert st == "converged" and abs(iters - it_ref) <= 2, (iters, it_ref)
    assert rel(u, u_ref.reshape(-1)) < 1e-10


def test_metric_poisson_10m_rcm_renumbered_vs_oracle(gpu, cube119):
    """The metric system as a mesh in file order would hand it over: the cube's nodes randomly renumbered (seed 7,
    `bench.py --permute 7`), then device RCM (`bench.py --reorder rcm`). The renumbered operator and the persistent
    schedule's first 5 iterates, mapped back to the cube's numbering, against the same oracle products."""
    _, mesh, _, system = _mods()
    c, t, N = cube119.c, cube119.t, cube119.N
    f, fixed, dinv = cube119.case("poisson")
    perm1 = torch.randperm(N, generator=torch.Generator().manual_seed(7))
    inv1 = torch.empty_like(perm1)
    inv1[perm1] = torch.arange(N)
    cp, tp = c[perm1].to(gpu), inv1[t].to(gpu)
    perm2, inv2 = system.rcm_order(tp, N)
    c2, t2 = system.renumber(cp, tp, perm2, inv2)
    P = perm1[perm2.cpu()]                    # new node j is the cube's node P[j]
    Pinv = torch.empty_like(P)
    Pinv[P] = torch.arange(N)
    A = system.assemble_tet4_system(c2, t2, "poisson")
    assert A.use16                            # RCM brings every |col - row| under 32767
    p, y_ref = cube119.matvec_ref("poisson", 12)
    y = A.matvec(p.reshape(-1)[P].to(gpu)).cpu()
    assert rel(y[Pinv], y_ref.reshape(-1)) < 1e-12
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask[Pinv[fixed].to(gpu)] = 1
    w = A.jacobi(mask)
    assert rel(w.cpu()[Pinv], dinv.reshape(-1)) < 1e-14
    facts, x = _poisson_persistent_iterates(system, A, f.reshape(-1)[P], w, (2, 3))
    assert facts["schedule"] == system.SCHED_PERSIST and facts["build"][1] == 0, facts
    assert rel(x.cpu()[Pinv], cube119.pcg_ref("poisson", 5).reshape(-1)) < 1e-10
