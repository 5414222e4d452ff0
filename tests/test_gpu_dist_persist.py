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


def test_dist_persist_elastic_rank_share_vs_oracle(gpu):
    """The N = 8 per-rank share of configs[3] (n = 59: 1,232,274 tets, the size one rank of the 10M system holds at
    N = 8) on the DIST k_pcg_persist3 build over 2 emulated ranks, against the ORACLE: 20 fixed iterations equal the
    reference PCG's 20th iterate (`solver/solver.py:766-812`, over the reference's element matrices,
    `solver/element.py:883-903`) at 1e-10, every rank running the persistent schedule with its state on chip."""
    from oracle import ref_cpu as R
    C, DP, mesh, system = _mods()
    E, NU = 113.8e9, 0.342
    c, t = mesh.kuhn_cube(59)
    N = c.shape[0]
    f, fixed = mesh.cube_elasticity_case(c)
    mask = torch.zeros((N, 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    b = f.reshape(-1).to(F64).to(gpu)
    grp = DP.EmulatedGroup(c.to(gpu), t.to(gpu), 2, b, fixed_mask=mask.view(-1), kind="elastic", E=E, nu=NU, tol=0.0)
    try:
        grp.start()
        assert all(rr.effective_schedule() == system.SCHED_PERSIST for rr in grp.ranks)
        grp.iterate(20)
        it, stt, _ = grp.poll()
        assert it == 20 and stt == C.PCG_RUNNING
        x = grp.x().cpu()
    finally:
        grp.close()
    K = R.tet4_K(c, t, E, NU)
    dinv = R.diag_preconditioner(K, t, N, dpn=3)
    dinv[fixed] = 0.0
    u_ref, it_ref, _ = R.pcg(K, t, f.reshape(N, 3).to(F64), dinv, tol=0.0, max_iter=20)
    assert it_ref == 20 and rel(x, u_ref.reshape(-1)) < 1e-10


# ---------------------------------------------------------------------------- the N > 1 failure chain
def test_dist_persist_drop_publish_gives_up(gpu):
    """Fault injection (FEM_TUNE_DIST_DROP on rank 1: it publishes no u row and no flag): every rank's launch ends
    with FEM_PCG_SYNC_TIMEOUT within the bounded waits (2 s per in-GPU wait, 5 s for the rank exchange), each with a
    give-up site -- never a hang."""
    import time
    C, DP, mesh, system = _mods()
    c, t, b, mask, A, w = _case(mesh, system, 24, gpu)
    grp = DP.EmulatedGroup(c, t, 2, b, fixed_mask=mask, tol=1e-12, drop_rank=1)
    try:
        t0 = time.perf_counter()
        grp.start()
        grp.iterate(200)
        dt = time.perf_counter() - t0
        polls = grp.poll_ranks()
        assert all(p[1] == C.PCG_SYNC_TIMEOUT for p in polls), polls
        sites = [rr.sync_site() for rr in grp.ranks]
        assert all(s % 16 in (1, 2, 3) for s in sites), sites
        assert all(0 <= p[0] < 200 for p in polls), polls   # completed iterations, not a site code
        assert dt < 15.0, dt
    finally:
        grp.close()


def _bench_two_ranks(extra_env, n=40, timeout=300, extra_args=()):
    import json
    import os
    import socket
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, FEM355_DIST_SAME_GPU="1", MASTER_ADDR="127.0.0.1", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--cube-n", str(n),
           "--steps", "20", "--warmup", "5", "--elastic", "0", "--no-cpu-baseline", *extra_args]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=timeout)
    dt = time.perf_counter() - t0
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p, lines, dt


def test_bench_two_ranks_same_gpu_prints_one_line(gpu):
    """`bench.py --gpus 2` with both ranks on this GPU (FEM355_DIST_SAME_GPU=1): the persistent multi-GPU schedule
    passes its self-check on the first attempt (fine-grained comm blocks) and rank 0 prints exactly one JSON line
    whose timed launch completed its steps, within the stated budget (120 s on one GPU)."""
    p, lines, dt = _bench_two_ranks({})
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout[-2000:]
    cfg = lines[0]["config"]
    assert lines[0]["value"] > 0 and lines[0]["n_gpus"] == 2
    assert cfg["comm_block"] == "fine-grained" and cfg["attempts"][0]["ok"], cfg
    assert dt < 120.0, dt


def test_bench_two_ranks_same_gpu_pipelined(gpu):
    """`bench.py --gpus 2 --pipelined 1` on this GPU: the pipelined DIST build (a second m region in the IPC-mapped
    comm blocks) passes the self-check against the single-GPU pipelined solve and times its steps."""
    p, lines, dt = _bench_two_ranks({}, extra_args=("--pipelined", "1"))
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout[-2000:]
    line = lines[0]
    assert line["pipelined"] is True and line["value"] > 0 and line["n_gpus"] == 2
    assert line["config"]["attempts"][0]["ok"], line["config"]
    assert dt < 120.0, dt


def test_bench_two_ranks_drop_publish(gpu):
    """The failure chain with rank 1 publishing nothing (FEM355_DIST_DROP_RANK=1): both comm-block attempts fail
    their warm-up solve with a bounded give-up, and -- RCCL refusing two ranks per GPU -- the run ends with the
    documented error instead of a line or a hang, within the stated budget (90 s on one GPU). On a
    multi-GPU node the same chain continues with the RCCL element partition (`tests/test_dist_chain.py`)."""
    p, lines, dt = _bench_two_ranks({"FEM355_DIST_DROP_RANK": "1"})
    assert p.returncode != 0 and not lines
    err = p.stderr
    assert err.count("fine-grained comm blocks: warm-up solve status 6") >= 1, err[-3000:]
    assert err.count("coarse-grained comm blocks: warm-up solve status 6") >= 1, err[-3000:]
    assert "no RCCL fallback possible" in err, err[-3000:]
    assert dt < 90.0, dt
