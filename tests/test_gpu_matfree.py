"""GPU tier of the element-chunk (matrix-free) c3d4 operator (`csrc/matfree.hip`, `system.MatFreeOperator`): the
reference's element-by-element product `compute_nodal_forces` (`solver/element.py:429-464`) of the c3d4 stiffness
(`compute_c3d4_K_matrix`, `:883-903`) and of the P1 Laplacian, formed from the coordinates in every application.

Checked against the oracle's EBE product over its element matrices (`oracle/ref_cpu.py` nodal_forces / tet4_K /
tet4_poisson_K) at 1e-12, against the assembled SELL operator, for the exact diagonal, bit-determinism, chunk
splitting (a mesh whose 512-element chunks touch more than 256 nodes), a fan around a hub node, random numbering,
errors, the (P)CG on it against the oracle PCG (`solver/solver.py:766-812`), and at the configs[2] size (10M tets)."""
import pytest
import torch

from conftest import rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import mesh, solver, system
    return mesh, solver, system


def _disjoint_tets(m, seed=3):
    """m tets with 4 private nodes each (every chunk touches 4 nodes per element: the split into pieces)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(m, 1, 3, generator=g, dtype=F64) * 10.0
    ref = torch.tensor([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], dtype=F64)
    c = (base + ref + 0.1 * torch.rand(m, 4, 3, generator=g, dtype=F64)).reshape(-1, 3)
    t = torch.arange(4 * m, dtype=torch.int64).reshape(m, 4)
    return c, t


def _fan(k):
    """k tets around the hub node 0 (a node in every element: one row touching k + 2 nodes)."""
    ang = torch.arange(k + 1, dtype=F64) * (2 * torch.pi / k)
    ring = torch.stack([torch.cos(ang), torch.sin(ang), torch.zeros_like(ang)], 1)
    c = torch.cat([torch.tensor([[0.0, 0.0, 1.0], [0.0, 0.0, -1.0]], dtype=F64), ring[:-1]], 0)
    i = torch.arange(k)
    t = torch.stack([torch.zeros(k, dtype=torch.int64), torch.ones(k, dtype=torch.int64), 2 + i, 2 + (i + 1) % k], 1)
    return c, t


def _meshes():
    mesh, _, _ = _mods()
    out = {}
    out["kuhn6"] = mesh.kuhn_cube(6, jitter=0.15)
    out["kuhn14"] = mesh.kuhn_cube(14, jitter=0.1)
    c, t = mesh.kuhn_cube(10, jitter=0.1)
    g = torch.Generator().manual_seed(5)
    perm = torch.randperm(c.shape[0], generator=g)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    out["permuted"] = (c[perm], inv[t][torch.randperm(t.shape[0], generator=g)])
    out["disjoint"] = _disjoint_tets(1100)
    out["fan"] = _fan(700)
    return out


@pytest.mark.parametrize("name", ["kuhn6", "kuhn14", "permuted", "disjoint", "fan"])
@pytest.mark.parametrize("kind", ["elastic", "poisson"])
def test_operator_vs_oracle_ebe(gpu, name, kind):
    _, _, system = _mods()
    c, t = _meshes()[name]
    N, dpn = c.shape[0], 3 if kind == "elastic" else 1
    Ek = E if kind == "elastic" else 2.5
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), kind, Ek, NU)
    K = R.tet4_K(c, t, E, NU) if kind == "elastic" else R.tet4_poisson_K(c, t, kappa=Ek)
    x = torch.randn(N, dpn, dtype=F64, generator=torch.Generator().manual_seed(1))
    y = A.matvec(x.reshape(-1).to(gpu))
    y_ref = R.nodal_forces(K, t, x).reshape(-1)
    assert rel(y, y_ref) < 1e-12
    # bit-deterministic: a second application gives the same bits
    assert torch.equal(A.matvec(x.reshape(-1).to(gpu)), y)
    # exact diagonal against the oracle's element matrices (the true diagonal, not the Q1 column-0 quirk)
    d_ref = torch.zeros(N * dpn, dtype=F64)
    dm = R.dof_map(t, dpn)
    d_ref.index_add_(0, dm.reshape(-1), torch.diagonal(K, dim1=1, dim2=2).reshape(-1))
    assert rel(A.diag(), d_ref) < 1e-13
    info = A.info()
    assert info["elements"] == t.shape[0] and info["nodes"] == N
    if name == "disjoint":   # chunks touch 4 nodes per element: cut into pieces (<= 64 elements) within the node cap
        assert info["chunks"] >= (t.shape[0] + 63) // 64
        assert info["slots"] == 4 * t.shape[0]


def test_halving_split(gpu):
    """Chunks past the 256-node cap are halved, and halves still past it halved again, down to 64 elements
    (fem_mf_create). A Kuhn cube rotated off the Morton grid with small disjoint tets scattered through it (4 nodes
    of their own each): every chunk is an aligned power-of-two range of 64..512 elements (the last one may be short)
    within the node cap, more than one chunk size occurs, and the operator matches the oracle's EBE product."""
    import math
    mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(16, jitter=0.1)
    k = torch.tensor([1.0, 1.0, 2.0], dtype=F64)
    k = k / k.norm()
    th = math.radians(17.0)
    K3 = torch.tensor([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]], dtype=F64)
    Rm = torch.eye(3, dtype=F64) + math.sin(th) * K3 + (1 - math.cos(th)) * (K3 @ K3)
    c = c @ Rm.T
    g = torch.Generator().manual_seed(11)
    m = 1500
    base = c.min(0).values + torch.rand(m, 1, 3, generator=g, dtype=F64) * (c.max(0).values - c.min(0).values)
    ref = torch.tensor([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]], dtype=F64)
    small = (base + 0.01 * ref).reshape(-1, 3)
    t = torch.cat([t, c.shape[0] + torch.arange(4 * m).view(m, 4)], 0)
    c = torch.cat([c, small], 0).contiguous()
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    _, cp, sb, _ = A.layout()
    cp, sb = cp.cpu().long(), sb.cpu().long()
    M = t.shape[0]
    sizes, nodes = (cp[1:] - cp[:-1]).tolist(), (sb[1:] - sb[:-1]).tolist()
    assert int(cp[0]) == 0 and int(cp[-1]) == M
    assert all(1 <= v <= 256 for v in nodes)
    for a, s in zip(cp[:-1].tolist()[:-1], sizes[:-1]):
        assert s in (64, 128, 256, 512) and a % s == 0, (a, s)
    assert len(set(sizes[:-1])) >= 2, sorted(set(sizes))
    x = torch.randn(c.shape[0], 3, dtype=F64, generator=torch.Generator().manual_seed(2))
    Ke = R.tet4_K(c, t, E, NU)
    assert rel(A.matvec(x.reshape(-1).to(gpu)), R.nodal_forces(Ke, t, x).reshape(-1)) < 1e-12


@pytest.mark.parametrize("nodemajor", ["1", "0"])
def test_chunk_walk_bit_identical(gpu, monkeypatch, nodemajor):
    """Workgroups walking many chunks (the software pipeline's rotation: three chunks in flight) give the same bits as
    one chunk per workgroup: the grid capped at 8 workgroups (FEM355_MF_GRID_CAP) on a 16k-tet cube, both slot
    layouts; and at 1.3M tets (2.5k chunks over the resident grid) the operator equals the assembled one at 1e-13."""
    mesh, _, system = _mods()
    monkeypatch.setenv("FEM355_MF_NODEMAJOR", nodemajor)
    c, t = mesh.kuhn_cube(14, jitter=0.1)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    x = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(3)).to(gpu)
    y, d = A.matvec(x), A.diag()
    monkeypatch.setenv("FEM355_MF_GRID_CAP", "8")
    assert torch.equal(A.matvec(x), y)
    assert torch.equal(A.diag(), d)
    monkeypatch.delenv("FEM355_MF_GRID_CAP")
    c, t = mesh.kuhn_cube(60)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    As = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", E, NU)
    x = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(4)).to(gpu)
    assert A.info()["chunks"] > 1000
    assert rel(A.matvec(x), As.matvec(x)) < 1e-13


def test_layout_invariants(gpu):
    """Morton order is a permutation; every chunk holds <= 512 elements and <= 256 nodes; slot nodes ascend inside a
    chunk and each (chunk, node) pair appears once; every node of an element is a slot of the element's chunk."""
    mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    eo, cp, sb, cn = (v.cpu().long() for v in A.layout())
    assert torch.equal(eo.sort().values, torch.arange(t.shape[0]))
    assert int((cp[1:] - cp[:-1]).max()) <= 512 and int((sb[1:] - sb[:-1]).max()) <= 256
    for ch in range(cp.numel() - 1):
        nodes = cn[sb[ch]:sb[ch + 1]]
        assert torch.all(nodes[1:] > nodes[:-1])
        want = torch.unique(t[eo[cp[ch]:cp[ch + 1]]].reshape(-1))
        assert torch.equal(nodes, want)


def test_errors_and_empty(gpu):
    mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(3)
    bad = t.clone()
    bad[5, 2] = bad[5, 1]          # a repeated node: zero volume
    with pytest.raises(ValueError, match="Singular matrix"):
        system.MatFreeOperator(c.to(gpu), bad.to(gpu), "elastic", E, NU)
    oob = t.clone()
    oob[7, 0] = c.shape[0]
    with pytest.raises(Exception, match="outside"):
        system.MatFreeOperator(c.to(gpu), oob.to(gpu), "elastic", E, NU)
    A = system.MatFreeOperator(c.to(gpu), t[:0].to(gpu), "elastic", E, NU)
    y = A.matvec(torch.ones(c.shape[0] * 3, dtype=F64, device=gpu))
    assert float(y.abs().max()) == 0.0


@pytest.mark.parametrize("kind", ["elastic", "poisson"])
def test_pcg_vs_oracle_and_assembled(gpu, kind):
    """Jacobi-PCG to rtol 1e-8 on the matrix-free operator: u within 1e-10 of the oracle PCG over the reference's
    element matrices, iterations within +-2; the first 20 iterates match the assembled operator's
    3-kernel schedule at 1e-10."""
    mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(8, jitter=0.12)
    N = c.shape[0]
    dpn = 3 if kind == "elastic" else 1
    f, fixed = mesh.cube_elasticity_case(c) if kind == "elastic" else mesh.cube_poisson_case(c)
    u, res, A = solver.solve_tet4(c, t, f, fixed, kind=kind, E=E if kind == "elastic" else 1.0, nu=NU,
                                  rtol=1e-8, device=gpu, operator="matfree")
    assert getattr(A, "is_matfree", False)
    K = R.tet4_K(c, t, E, NU) if kind == "elastic" else R.tet4_poisson_K(c, t)
    dinv = R.diag_preconditioner(K, t, N, dpn=dpn)
    dinv[fixed] = 0.0
    b = f.reshape(N, dpn).to(F64)
    tol = 1e-8 * float(torch.sqrt((b * dinv * b).sum()))
    u_ref, it_ref, _ = R.pcg(K, t, b, dinv, tol=tol, max_iter=5000)
    assert abs(res.iterations - it_ref) <= 2
    assert rel(u.cpu().reshape(N, dpn), u_ref) < 1e-9
    # fixed iterations against the assembled operator's schedule
    As = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, E if kind == "elastic" else 1.0, NU)
    mask = torch.zeros((N, dpn), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = As.jacobi(mask.view(-1))
    w_mf = A.jacobi(mask.view(-1))
    assert rel(w_mf, w) < 1e-14
    r1 = As.pcg(b.reshape(-1), w=w, tol=0.0, max_iter=20, schedule=0)
    r2 = A.pcg(b.reshape(-1), w=w, tol=0.0, max_iter=20)
    assert r1.iterations == r2.iterations == 20
    assert rel(r2.x, r1.x) < 1e-10


def test_runner_chunks_bit_identical(gpu):
    """The bench's fixed-iteration runner on the matrix-free operator: 3 + 4 iterations in two launches give the same
    bits as 7 in one (device state carried between launches)."""
    mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(9, jitter=0.1)
    f, fixed = mesh.cube_elasticity_case(c)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    xs = []
    for steps in ((7,), (3, 4)):
        run = system.PcgRunner(A, f.reshape(-1), w, tol=0.0)
        try:
            run.start()
            for k in steps:
                run.iterate(k)
            assert run.poll()[0] == 7
            xs.append(run.x.clone())
        finally:
            run.close()
    assert torch.equal(xs[0], xs[1])


@pytest.mark.parametrize("kind", ["elastic", "poisson"])
def test_update_fused_q_bit_identical(gpu, kind):
    """The merged update summing each dof's slots itself (default) against the gather launch + stored q
    (FEM_TUNE_MF_GATHER), and with the update's grid capped at 8 workgroups (FEM_TUNE_U2_SMALL: the loop past the
    register-cached elements, and an odd dof count): the same bits after 9 iterations."""
    mesh, _, system = _mods()
    from fem355 import _capi as C
    c, t = mesh.kuhn_cube(7, jitter=0.1)
    if kind == "poisson":   # an odd dof count: the update's scalar tail
        c = torch.cat([c, torch.tensor([[0.5, 0.5, 2.0]], dtype=F64)], 0)
    f, fixed = mesh.cube_elasticity_case(c) if kind == "elastic" else mesh.cube_poisson_case(c)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), kind, E if kind == "elastic" else 1.0, NU)
    mask = torch.zeros((c.shape[0], A.bs), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    xs = []
    for extra in (0, C.TUNE_MF_GATHER, C.TUNE_U2_SMALL, C.TUNE_U2_SMALL | C.TUNE_MF_GATHER):
        run = system.PcgRunner(A, f.reshape(-1), w, tol=0.0)
        try:
            run.set_tuning(C.TUNE_DEFAULT | extra)
            run.start()
            run.iterate(9)
            assert run.poll()[0] == 9
            xs.append(run.x.clone())
        finally:
            run.close()
    assert all(torch.equal(xs[0], v) for v in xs[1:])


def test_update_give_up_is_all_or_nothing(gpu):
    """The merged update on the element-chunk operator shares k_pcg_update2's release protocol (u2_release): with
    workgroup 0 held back past every other workgroup's wait (FEM_TUNE_U2_HOLD) the launch ends with
    FEM_PCG_SYNC_TIMEOUT at give-up site 4 (+ 16 x launch) and no workgroup's x update."""
    import ctypes
    mesh, _, system = _mods()
    from fem355 import _capi as C
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    f, fixed = mesh.cube_elasticity_case(c)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    x0 = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(5)).to(gpu)
    run = system.PcgRunner(A, f.reshape(-1), w, x0=x0, tol=0.0)
    try:
        run.set_tuning(C.TUNE_DEFAULT | C.TUNE_U2_HOLD)
        run.start()
        run.iterate(3)
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        C.check(run.lib.fem_pcg_poll(run.h, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)), "poll")
        site = ctypes.c_int()
        C.check(run.lib.fem_pcg_sync_site(run.h, ctypes.byref(site)), "site")
        assert stt.value == C.PCG_SYNC_TIMEOUT and it.value == 0, (it.value, stt.value)
        assert site.value == 4 + 16 * 1, site.value
        assert torch.equal(run.x, x0)
    finally:
        run.close()


def test_config2_matfree_10m_operator_and_iterates_vs_oracle(gpu, cube119):
    """BASELINE configs[2] (10,110,954 tets, 5,184,000 DOFs) on the matrix-free operator: the operator on a seeded
    vector against the oracle's EBE product over its element matrices at 1e-12, the exact Jacobi weights at 1e-14,
    and the first 5 Jacobi-PCG iterates against the oracle PCG at 1e-10."""
    _, _, system = _mods()
    c, t, N = cube119.c, cube119.t, cube119.N
    f, fixed, dinv = cube119.case("elastic")
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    p, y_ref = cube119.matvec_ref("elastic", 11)
    assert rel(A.matvec(p.reshape(-1).to(gpu)), y_ref.reshape(-1)) < 1e-12
    mask = torch.zeros((N, 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    assert rel(w, dinv.reshape(-1)) < 1e-14
    res = A.pcg(f.reshape(-1), w=w, tol=0.0, max_iter=5)
    assert res.iterations == 5
    assert rel(res.x, cube119.pcg_ref("elastic", 5).reshape(-1)) < 1e-10


def test_refuses_what_it_cannot_run(gpu):
    """a constrained solve on the element-chunk operator used to run as plain CG (constraints dropped).
    Python refuses constraints= / CG_CONSTRAINED / non-default schedules; the C-ABI refuses a CG_CONSTRAINED context
    for the operator and constraints on an operator context."""
    import ctypes
    mesh, _, system = _mods()
    from fem355 import _capi as C
    from fem355 import constraints as CS
    c, t = mesh.kuhn_cube(4)
    A = system.MatFreeOperator(c.to(gpu), t.to(gpu), "elastic", E, NU)
    b = torch.ones(A.n, dtype=F64, device=gpu)
    w = torch.ones(A.n, dtype=F64, device=gpu)
    cons = CS.ConstraintSet(A.n_nodes, 3, gpu, CS.parse_spc_list([{"node": 0, "dofs": [0, 1, 2], "value": 0.0}], "cpu"),
                            CS.parse_rbe2_list([], "cpu"))
    with pytest.raises(ValueError):
        system.PcgRunner(A, b, w, mode=C.MODE_CG_CONSTRAINED, constraints=cons)
    with pytest.raises(ValueError):
        system.PcgRunner(A, b, w, fused=True)
    with pytest.raises(ValueError):
        system.PcgRunner(A, b, w, schedule=3)
    with pytest.raises(ValueError):
        A.pcg(b, w=w, mode=C.MODE_CG_CONSTRAINED)
    lib = C.lib()
    x = torch.zeros_like(b)
    h = ctypes.c_void_p()
    C.check(lib.fem_pcg_create(A.n_nodes, 3, None, None, None, C.ptr(b), C.ptr(x), C.ptr(w), C.MODE_CG_CONSTRAINED,
                               0.0, 1e-30, None, 0, C.stream(torch.device(gpu)), ctypes.byref(h)), "fem_pcg_create")
    try:
        assert lib.fem_pcg_set_operator_mf(h, A.h) == C.FEM_EARG
    finally:
        lib.fem_pcg_destroy(h)
    h = ctypes.c_void_p()
    C.check(lib.fem_pcg_create(A.n_nodes, 3, None, None, None, C.ptr(b), C.ptr(x), C.ptr(w), C.MODE_CG_STABLE,
                               0.0, 1e-30, None, 0, C.stream(torch.device(gpu)), ctypes.byref(h)), "fem_pcg_create")
    try:
        C.check(lib.fem_pcg_set_operator_mf(h, A.h), "fem_pcg_set_operator_mf")
        assert lib.fem_pcg_set_constraints(h, *cons.args()) == C.FEM_EARG
    finally:
        lib.fem_pcg_destroy(h)


def test_concurrent_runners_on_one_operator(gpu):
    """every application used to write the operator's one slot buffer, so two runners on their own
    streams raced. Each (P)CG context now owns its slots: two runners iterating interleaved on their own streams (and
    stand-alone applications on the current stream between them) give the same iterates bit for bit as one runner
    alone."""
    mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(14, jitter=0.1)
    cg, tg = c.to(gpu), t.to(gpu)
    A = system.MatFreeOperator(cg, tg, "elastic", E, NU)
    f, fixed = mesh.cube_elasticity_case(cg)
    mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
    mask[fixed] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1).to(F64)
    solo = system.PcgRunner(A, b, w)
    solo.start()
    solo.iterate(40)
    solo.poll()
    ref = solo.x.clone()
    solo.close()
    r1, r2 = system.PcgRunner(A, b, w), system.PcgRunner(A, b * 2.0, w)
    r1.start()
    r2.start()
    p = torch.randn(A.n, dtype=F64, device=gpu)
    y0 = A.matvec(p)
    for _ in range(8):
        r1.iterate(5)
        r2.iterate(5)
        y = A.matvec(p)
    r1.poll()
    r2.poll()
    assert torch.equal(r1.x, ref)
    assert torch.equal(r2.x, 2.0 * ref)   # a linear solve from x0 = 0: twice the load, twice every iterate (exact)
    assert torch.equal(y, y0)
