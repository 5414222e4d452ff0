"""GPU tier: the multi-GPU persistent schedule (rows partitioned over ranks, in-kernel hand-offs through the ranks'
comm blocks; dist_persist.py, pcg_persist.hpp DIST build), validated on ONE GPU: the ranks run as contexts of one
process on separate streams, sharing the CUs (EmulatedGroup) -- the same kernel and hand-off code as one process
per GPU, with the comm blocks as plain device pointers instead of IPC mappings. Against the single-GPU persistent
schedule: solutions within 1e-10 and iterations within +-1 (only the grouping of the partial sums differs: rank
sums, then rank order), fixed-iteration iterates within 1e-12, chunk boundaries bit-identical. Two emulated ranks:
each gets a CU-masked stream (a hardware queue and half the CUs of its own); three shares of the 256 CUs did not
always co-schedule on the box (a give-up, not a hang: every spin is bounded)."""
import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import _capi as C, dist_persist as DP, mesh, system
    return C, DP, mesh, system


def _case(mesh, system, n, gpu, jitter=0.0):
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    c, t = c.to(gpu), t.to(gpu)
    f, fixed = mesh.cube_poisson_case(c)
    mask = torch.zeros(c.shape[0], dtype=torch.uint8, device=gpu)
    mask[fixed] = 1
    A = system.assemble_tet4_system(c, t, "poisson")
    w = A.jacobi(mask)
    return c, t, f.reshape(-1).to(F64), mask, A, w


@pytest.mark.parametrize("nranks,n,jitter,fine", [(2, 24, 0.1, False), (2, 40, 0.0, False), (2, 30, 0.05, True)])
def test_dist_persist_solve_matches_single_gpu(gpu, nranks, n, jitter, fine):
    """fine: the comm blocks in fine-grained device memory (bench.py's second attempt on a multi-GPU node)."""
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _case(mesh, system, n, gpu, jitter)
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r3 = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3)
    grp = DP.EmulatedGroup(c, t, nranks, b, fixed_mask=mask, tol=tol, fine=fine)
    try:
        it, stt = grp.solve(max_iter=5000, chunk=97)
        assert stt == C.PCG_CONVERGED and r3.status == C.PCG_CONVERGED
        assert abs(it - r3.iterations) <= 1, (it, r3.iterations)
        assert rel(grp.x(), r3.x) < 1e-10
    finally:
        grp.close()


def test_dist_persist_fixed_iterations_and_chunks(gpu):
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _case(mesh, system, 32, gpu)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    run.iterate(40)
    assert run.poll()[0] == 40   # (syncs the runner's stream)
    x1 = run.x.clone()
    run.close()
    xs = []
    for chunks in ((40,), (10, 10, 20), (1, 39)):
        grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=0.0)
        try:
            grp.start()
            for k in chunks:
                grp.iterate(k)
            it, stt, _ = grp.poll()
            assert it == 40 and stt == C.PCG_RUNNING
            xs.append(grp.x())
        finally:
            grp.close()
    assert rel(xs[0], x1) < 1e-12
    assert torch.equal(xs[0], xs[1]) and torch.equal(xs[0], xs[2])


def test_dist_persist_cg_mode_and_initial_guess(gpu):
    """CG mode (0/1 weights, masked rows) and a non-zero x0: the distributed init forms r0 = b - A x0 in-kernel."""
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _case(mesh, system, 20, gpu, 0.1)
    x0 = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(3)).to(gpu)
    x0[mask.bool()] = 0.0
    wm = (mask == 0).to(F64)
    c3 = A.pcg(b, x0, w=wm, mode=0, tol=0.0, max_iter=30, schedule=3)
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=0.0, mode=0, x0=x0)
    try:
        for rr in grp.ranks:   # CG mode: the weights are the 0/1 free mask
            rr.w.copy_(wm)
        grp.start()
        grp.iterate(30)
        it, stt, _ = grp.poll()
        assert it == 30 and rel(grp.x(), c3.x) < 1e-12
    finally:
        grp.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r3 = A.pcg(b, x0, w=w, tol=tol, max_iter=3000, schedule=3)
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=tol, x0=x0)
    try:
        it, stt = grp.solve(max_iter=3000)
        assert stt == C.PCG_CONVERGED and abs(it - r3.iterations) <= 1 and rel(grp.x(), r3.x) < 1e-10
    finally:
        grp.close()


def test_dist_persist_10m_two_ranks(gpu):
    """The 10M-tet bench system split over 2 emulated ranks (each with half the CUs): 50 fixed iterations within
    1e-12 of the single-GPU persistent schedule."""
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _case(mesh, system, 119, gpu)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    run.iterate(50)
    assert run.poll()[0] == 50
    x1 = run.x.clone()
    run.close()
    del A
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=0.0)
    try:
        grp.start()
        grp.iterate(50)
        it, stt, _ = grp.poll()
        assert it == 50 and stt == C.PCG_RUNNING
        assert rel(grp.x(), x1) < 1e-12
    finally:
        grp.close()


def _elastic_case(mesh, system, n, gpu, jitter=0.0):
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    c, t = c.to(gpu), t.to(gpu)
    f, fixed = mesh.cube_elasticity_case(c)
    mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
    mask[fixed] = 1
    A = system.assemble_tet4_system(c, t, "elastic", 113.8e9, 0.342)
    w = A.jacobi(mask.view(-1))
    return c, t, f.reshape(-1).to(F64), mask.view(-1), A, w


@pytest.mark.parametrize("n,jitter", [(20, 0.1), (36, 0.0)])
def test_dist_persist_elastic_matches_single_gpu(gpu, n, jitter):
    """bs = 3 (k_pcg_persist3 DIST build, three dofs per hand-off row) over 2 emulated ranks: solve to tolerance
    against the single-GPU bs = 3 persistent schedule (iterations +-1, x 1e-10), fixed iterations 1e-12, chunk
    boundaries bit-identical."""
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _elastic_case(mesh, system, n, gpu, jitter)
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r3 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=3)
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, kind="elastic", E=113.8e9, nu=0.342, tol=tol)
    try:
        it, stt = grp.solve(max_iter=20000, chunk=301)
        assert stt == C.PCG_CONVERGED and r3.status == C.PCG_CONVERGED
        assert abs(it - r3.iterations) <= 1, (it, r3.iterations)
        assert rel(grp.x(), r3.x) < 1e-10
    finally:
        grp.close()
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    run.iterate(40)
    assert run.poll()[0] == 40
    x1 = run.x.clone()
    run.close()
    xs = []
    for chunks in ((40,), (15, 25)):
        grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, kind="elastic", E=113.8e9, nu=0.342, tol=0.0)
        try:
            grp.start()
            for k in chunks:
                grp.iterate(k)
            assert grp.poll()[0] == 40
            xs.append(grp.x())
        finally:
            grp.close()
    assert rel(xs[0], x1) < 1e-12 and torch.equal(xs[0], xs[1])
