"""GPU tier: the pipelined persistent Jacobi-PCG (FEM_TUNE_PK_GV, csrc/pcg_persist_gv.hpp) -- the Ghysels-Vanroose
recurrences with the grid reduction posted before the SpMV and waited for after it. Against the single-reduction
persistent schedule, which tests/test_gpu_scale_parity.py pins to the oracle's R.pcg:
  * the first iterates within 1e-10 (the recurrences for M^-1 r and A M^-1 r differ at rounding level);
  * launch boundaries change nothing: 40 iterations in one launch or in chunks are bit-identical;
  * solves to rtol 1e-8 converge in the same iterations +-2, with x within 1e-8 of the single-reduction solution
    and the true residual within 2x of the tolerance (the method's attainable accuracy, not a parity bound);
  * contexts outside its scope (bs = 3, CG mode) keep the single-reduction kernel."""
import pytest
import torch

from conftest import rel

pytestmark = pytest.mark.gpu
F64 = torch.float64


def _mods():
    import fem355  # noqa: F401
    from fem355 import _capi as C, mesh, system
    return C, mesh, system


def _case(mesh, system, n, gpu, jitter=0.0, kind="poisson"):
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    c, t = c.to(gpu), t.to(gpu)
    if kind == "poisson":
        f, fixed = mesh.cube_poisson_case(c)
        mask = torch.zeros(c.shape[0], dtype=torch.uint8, device=gpu)
        mask[fixed] = 1
        A = system.assemble_tet4_system(c, t, "poisson")
    else:
        f, fixed = mesh.cube_elasticity_case(c)
        mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
        mask[fixed] = 1
        mask = mask.view(-1)
        A = system.assemble_tet4_system(c, t, "elastic", 113.8e9, 0.342)
    w = A.jacobi(mask)
    return A, f.reshape(-1).to(F64), w


def _iterate(system, A, b, w, chunks, tune, mode=None):
    kw = {} if mode is None else {"mode": mode}
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3, tune=tune, **kw)
    run.start()
    on = run.pipelined()
    for k in chunks:
        run.iterate(k)
    it, status = run.poll()[:2]
    x = run.x.clone()
    run.close()
    return x, it, status, on


@pytest.mark.parametrize("n,jitter", [(24, 0.1), (40, 0.0)])
def test_pipelined_first_iterates(gpu, n, jitter):
    C, mesh, system = _mods()
    A, b, w = _case(mesh, system, n, gpu, jitter)
    gv = C.TUNE_DEFAULT | C.TUNE_PK_GV
    for k in (1, 2, 5):
        x_gv, it, status, on = _iterate(system, A, b, w, (k,), gv)
        x_sr, it_sr, _, on_sr = _iterate(system, A, b, w, (k,), C.TUNE_DEFAULT)
        assert on and not on_sr
        assert it == it_sr == k and status == C.PCG_RUNNING
        assert rel(x_gv, x_sr) < 1e-10, (k, rel(x_gv, x_sr))


def test_pipelined_launch_boundaries_bit_identical(gpu):
    C, mesh, system = _mods()
    A, b, w = _case(mesh, system, 32, gpu, 0.05)
    gv = C.TUNE_DEFAULT | C.TUNE_PK_GV
    xs = []
    for chunks in ((40,), (10, 10, 20), (1, 39), (1, 1, 1, 37)):
        x, it, status, on = _iterate(system, A, b, w, chunks, gv)
        assert on and it == 40 and status == C.PCG_RUNNING
        xs.append(x)
    for x in xs[1:]:
        assert torch.equal(xs[0], x)


@pytest.mark.parametrize("n,jitter", [(30, 0.1), (55, 0.0)])
def test_pipelined_solve(gpu, n, jitter):
    """n = 55: the 1M-tet configs[1] cube (998,250 tets)."""
    C, mesh, system = _mods()
    A, b, w = _case(mesh, system, n, gpu, jitter)
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    ref = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3)
    gv = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3, tune=C.TUNE_DEFAULT | C.TUNE_PK_GV)
    assert ref.status == C.PCG_CONVERGED and gv.status == C.PCG_CONVERGED
    assert abs(gv.iterations - ref.iterations) <= 2, (gv.iterations, ref.iterations)
    print(f"n={n}: iterations {gv.iterations} vs {ref.iterations}, rel x {rel(gv.x, ref.x):.2e}")
    assert rel(gv.x, ref.x) < 1e-8, rel(gv.x, ref.x)
    # the true preconditioned residual of the pipelined solution against the tolerance it stopped on
    r = b - A.matvec(gv.x)
    fixed = w == 0
    r[fixed] = 0.0
    assert float(torch.sqrt(torch.dot(r, w * r))) < 2 * tol


def test_pipelined_scope(gpu):
    C, mesh, system = _mods()
    gv = C.TUNE_DEFAULT | C.TUNE_PK_GV
    A, b, w = _case(mesh, system, 12, gpu, 0.1, kind="elastic")
    _, it, _, on = _iterate(system, A, b, w, (5,), gv)
    assert not on and it == 5
    A, b, w = _case(mesh, system, 12, gpu, 0.1)
    wcg = (w != 0).to(F64)
    _, it, _, on = _iterate(system, A, b, wcg, (5,), gv, mode=C.MODE_CG_STABLE)
    assert not on and it == 5


def test_pipelined_config1_vs_oracle(gpu):
    """BASELINE configs[1] (998,250 tets) on the pipelined kernel against the oracle's R.pcg over its own element
    matrices: the first 5 iterates within 1e-10; the solve to rtol 1e-8 within +-2 iterations and u within 1e-10, the
    contract of the single-reduction kernel (test_gpu_scale_parity.py). Measured on MI355X: 3.5e-14 after 5 iterates,
    330 = 330 iterations, u 9.9e-11 (deterministic: the same bits every run)."""
    from oracle import ref_cpu as R
    C, mesh, system = _mods()
    c, t = mesh.kuhn_cube(55)
    f, fixed = mesh.cube_poisson_case(c)
    N = c.shape[0]
    KP = R.tet4_poisson_K(c, t)
    dinv = R.diag_preconditioner(KP, t, N, dpn=1)
    dinv[fixed] = 0.0
    bo = f.reshape(N, 1).to(F64)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask)
    b = f.reshape(-1).to(F64).to(gpu)
    gv = C.TUNE_DEFAULT | C.TUNE_PK_GV
    x5, it, _, on = _iterate(system, A, b, w, (5,), gv)
    u5, _, _ = R.pcg(KP, t, bo, dinv, tol=0.0, max_iter=5)
    assert on and it == 5
    assert rel(x5.cpu(), u5.reshape(-1)) < 1e-10
    tol = 1e-8 * float(torch.sqrt(torch.sum(bo * dinv * bo)))
    res = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3, tune=gv)
    u_ref, it_ref, st = R.pcg(KP, t, bo, dinv, tol=tol, max_iter=5000)
    assert st == "converged" and res.status == C.PCG_CONVERGED
    assert abs(res.iterations - it_ref) <= 2, (res.iterations, it_ref)
    print(f"configs[1] pipelined vs oracle: 5 iterates {rel(x5.cpu(), u5.reshape(-1)):.2e}, solve "
          f"{res.iterations} vs {it_ref} iterations, rel u {rel(res.x.cpu(), u_ref.reshape(-1)):.2e}")
    assert rel(res.x.cpu(), u_ref.reshape(-1)) < 1e-10


def test_pipelined_initial_guess_max_iter_and_history(gpu):
    """A non-zero x0 (r0 = b - A x0 formed by the start kernel, w0 = A u0 by the first launch), a solve stopped by
    max_iter (status PCG_MAXITER at exactly max_iter iterations, as the single-reduction kernel), and the residual
    history (sqrt(r.u) per iteration, the reference's printed norms) against the single-reduction kernel's."""
    C, mesh, system = _mods()
    A, b, w = _case(mesh, system, 28, gpu, 0.1)
    gv = C.TUNE_DEFAULT | C.TUNE_PK_GV
    g = torch.Generator(device="cpu").manual_seed(3)
    x0 = (torch.rand(A.n, generator=g, dtype=F64) - 0.5).to(gpu)
    x0[w == 0] = 0.0
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    ref = A.pcg(b, x0=x0, w=w, tol=tol, max_iter=5000, schedule=3, history=True)
    res = A.pcg(b, x0=x0, w=w, tol=tol, max_iter=5000, schedule=3, history=True, tune=gv)
    assert ref.status == res.status == C.PCG_CONVERGED
    assert abs(res.iterations - ref.iterations) <= 2
    assert rel(res.x, ref.x) < 1e-8
    h, hr = res.history, ref.history
    m = min(len(h), len(hr))
    assert m > 10 and rel(torch.as_tensor(h[:m]), torch.as_tensor(hr[:m])) < 1e-6
    ref = A.pcg(b, x0=x0, w=w, tol=tol, max_iter=17, schedule=3)
    res = A.pcg(b, x0=x0, w=w, tol=tol, max_iter=17, schedule=3, tune=gv)
    assert ref.status == res.status == C.PCG_MAXITER and ref.iterations == res.iterations == 17
    assert rel(res.x, ref.x) < 1e-10


@pytest.mark.parametrize("n,jitter", [(24, 0.1), (40, 0.0)])
def test_pipelined_dist_emulated_ranks(gpu, n, jitter):
    """The pipelined DIST build (rows over ranks, in-kernel hand-offs through the comm blocks; the rank exchange of
    gamma / delta announced in the arrival and waited for after the SpMV) on 2 ranks emulated on one GPU
    (dist_persist.EmulatedGroup, tests/test_gpu_dist_persist.py): against the single-GPU pipelined solve, iterations
    +-1 and x within 1e-10 (the partial sums group by rank first); fixed iterations in chunks bit-identical."""
    C, mesh, system = _mods()
    from fem355 import dist_persist as DP
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    c, t = c.to(gpu), t.to(gpu)
    f, fixed = mesh.cube_poisson_case(c)
    mask = torch.zeros(c.shape[0], dtype=torch.uint8, device=gpu)
    mask[fixed] = 1
    A = system.assemble_tet4_system(c, t, "poisson")
    w = A.jacobi(mask)
    b = f.reshape(-1).to(F64)
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    ref = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3, tune=C.TUNE_DEFAULT | C.TUNE_PK_GV)
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=tol, gv=True)
    try:
        it, stt = grp.solve(max_iter=5000, chunk=97)
        assert all(r.pipelined() for r in grp.ranks)
        assert stt == C.PCG_CONVERGED and ref.status == C.PCG_CONVERGED
        assert abs(it - ref.iterations) <= 1, (it, ref.iterations)
        print(f"n={n}: dist pipelined {it} vs {ref.iterations} iterations, rel x {rel(grp.x(), ref.x):.2e}")
        assert rel(grp.x(), ref.x) < 1e-10
    finally:
        grp.close()
    xs = []
    for chunks in ((40,), (10, 10, 20), (1, 39)):
        grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=0.0, gv=True)
        try:
            grp.start()
            for k in chunks:
                grp.iterate(k)
            it, stt, _ = grp.poll()
            assert it == 40 and stt == C.PCG_RUNNING
            xs.append(grp.x())
        finally:
            grp.close()
    assert torch.equal(xs[0], xs[1]) and torch.equal(xs[0], xs[2])
