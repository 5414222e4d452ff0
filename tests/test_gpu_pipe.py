"""GPU tier: the pipelined persistent Jacobi-PCG (schedule 4, csrc/pcg_pipe.hpp) against the 3-kernel and persistent
schedules and the oracle. It is the same PCG with a = A u carried by recurrence, so rounding differs: the contract is
the survey's: iterations within +-2, solutions within 1e-10 relative, residual history within 1e-8 for
the first iterations; chunk boundaries and geometries change nothing but the partial-sum grouping."""
import pytest
import torch

from conftest import rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
F64 = torch.float64
PIPE_CFGS = (1, 2, 3)   # FEM_TUNE_PIPE_CFG selector (cfg index + 1)
BASE_TUNE = 1 | 2 | 4 | 8


def _mods():
    import fem355  # noqa: F401
    from fem355 import element, mesh, solver, system
    return element, mesh, solver, system


def _poisson_case(system, mesh, n, gpu, jitter=0.0):
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    f, fixed = mesh.cube_poisson_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(A.n, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    return A, f.to(gpu).reshape(-1).to(F64), mask


@pytest.mark.parametrize("n,jitter", [(7, 0.1), (40, 0.0)])
def test_pipe_matches_three_kernel(gpu, n, jitter):
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, n, gpu, jitter)
    w = A.jacobi(mask)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=4)
    run.start()
    assert run.effective_schedule() == 4
    run.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=0, history=True)
    r4 = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=4, history=True)
    assert r0.status == r4.status == 1 and abs(r0.iterations - r4.iterations) <= 2
    assert rel(r4.x, r0.x) < 1e-10
    k = min(20, r0.iterations - 1)
    assert rel(r4.history[:k], r0.history[:k]) < 1e-8
    # CG mode (0/1 weights, masked rows) at fixed iterations
    wm = (mask == 0).to(F64)
    c0 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=0)
    c4 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=4)
    assert c0.iterations == c4.iterations == 25 and c0.status == c4.status == 2 and rel(c4.x, c0.x) < 1e-9


def test_pipe_vs_oracle_reference_semantics(gpu):
    """Poisson solve to the reference's absolute tol against the oracle's PCG (the reference op sequence)."""
    _, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(6, jitter=0.15)
    f, fixed = mesh.cube_poisson_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(A.n, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask)
    res = A.pcg(f.to(gpu).view(-1), w=w, tol=1e-10, max_iter=1000, schedule=4)
    KP = R.tet4_poisson_K(c, t)
    dinv = R.diag_preconditioner(KP, t, c.shape[0], dpn=1)
    dinv[fixed] = 0.0
    u_ref, it_ref, _ = R.pcg(KP, t, f, dinv, tol=1e-10)
    assert res.status == 1 and abs(res.iterations - it_ref) <= 2 and rel(res.x, u_ref.view(-1)) < 1e-10


def test_pipe_initial_guess(gpu):
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 16, gpu, jitter=0.1)
    w = A.jacobi(mask)
    x0 = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(5)).to(gpu)
    x0[mask.bool()] = 0.0
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, x0, w=w, tol=tol, max_iter=3000, schedule=0)
    r4 = A.pcg(b, x0, w=w, tol=tol, max_iter=3000, schedule=4)
    assert r0.status == r4.status == 1 and abs(r0.iterations - r4.iterations) <= 2 and rel(r4.x, r0.x) < 1e-10


def test_pipe_chunks_are_bit_identical_and_geometries_agree(gpu):
    """Chunk boundaries add no arithmetic (one launch of 36 == 4 x 9 == 5 + 31, bit for bit, same poll); the three
    geometries give the same iterates up to the partial-sum grouping."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 24, gpu)
    w = A.jacobi(mask)
    outs = {}
    for cfg in PIPE_CFGS:
        for chunks in ((36,), (9, 9, 9, 9), (5, 31)):
            run = system.PcgRunner(A, b, w, tol=0.0, schedule=4)
            run.set_tuning(BASE_TUNE | (cfg << 6))
            run.start()
            assert run.effective_schedule() == 4
            for k in chunks:
                run.iterate(k)
            outs[(cfg, chunks)] = (run.poll(), run.x.clone())
            run.close()
    for cfg in PIPE_CFGS:
        ref = outs[(cfg, (36,))]
        assert ref[0][0] == 36 and ref[0][1] == 0
        for chunks in ((9, 9, 9, 9), (5, 31)):
            o = outs[(cfg, chunks)]
            assert o[0] == ref[0] and torch.equal(o[1], ref[1])
        assert rel(ref[1], outs[(1, (36,))][1]) < 1e-12


def test_pipe_full_geometry_10m(gpu):
    """The 10M-tet bench system (27,000 slices: every slot of every geometry in use): 50 fixed iterations equal the
    persistent schedule's to 1e-10 and the solve to rtol 1e-8 stops within 2 iterations of it."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 119, gpu)
    w = A.jacobi(mask)
    xs = {}
    for sched, tune in ((3, None), (4, BASE_TUNE | (1 << 6)), (4, BASE_TUNE | (2 << 6))):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
        if tune is not None:
            run.set_tuning(tune)
        run.start()
        assert run.effective_schedule() == sched
        run.iterate(50)
        it, st, rz = run.poll()
        assert it == 50 and st == 0
        xs[(sched, tune)] = (rz, run.x.clone())
        run.close()
    x3 = xs[(3, None)]
    for key, v in xs.items():
        assert rel(v[1], x3[1]) < 1e-10 and abs(v[0] - x3[0]) <= 1e-8 * abs(x3[0]), key
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    r3 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=3)
    r4 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=4)
    assert r3.status == r4.status == 1 and abs(r3.iterations - r4.iterations) <= 2 and rel(r4.x, r3.x) < 1e-10


def test_pipe_guard_stop_and_fallbacks(gpu):
    """CG breakdown on the indefinite c3d10 scalar block: same status and iteration as the 3-kernel schedule; bs = 3
    falls back to the deferred schedule; a mesh past the register capacity to the persistent one."""
    el, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(6)
    Ael = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", 113.8e9, 0.342)
    run = system.PcgRunner(Ael, torch.ones(Ael.n, dtype=F64, device=gpu), Ael.jacobi(None), tol=0.0, schedule=4)
    run.start()
    assert run.effective_schedule() == 2
    run.close()
    c10, t10 = mesh.tet10_cube(1)
    K = el.compute_c3d10_K_matrix(c10, t10, 113.8e9, 0.342, device=gpu, dtype=F64)[:, 0::3, 0::3].contiguous()
    g = system.build_graph(t10.to(gpu), c10.shape[0])
    A = system.SellMatrix(g, 1).add_element_matrices(K, t10.to(gpu))
    F = -torch.ones(A.n, dtype=F64, device=gpu)
    fixed = mesh.face_nodes(c10, 2, 0.0).to(gpu)
    wv = torch.ones(A.n, dtype=F64, device=gpu)
    wv[fixed] = 0.0
    res = [A.pcg(F, w=wv, mode=0, tol=1e-10, max_iter=50, schedule=s) for s in (0, 4)]
    assert res[0].status == res[1].status and res[0].iterations == res[1].iterations
    Ab, bb, maskb = _poisson_case(system, mesh, 130, gpu)
    run = system.PcgRunner(Ab, bb, Ab.jacobi(maskb), tol=0.0, schedule=4)
    run.start()
    assert run.effective_schedule() == 3
    run.close()
