#!/usr/bin/env python3
"""Constraint-aware CG measurement: the reference's `new_constrained_conjugate_gradient_solver`
workload on the 10M-tet c3d4 elasticity Kuhn cube (n=119 -> 5.18M DOFs).

Constraints: SPC on the z=0 face (all dofs 0), a rigid RBE2 top plate (every z=1 node follows the centre node,
3 dofs), one RBE3 (the node below the centre = weighted mean of a ring of top nodes), load -1e6 N on the centre.
Prints one JSON line:
  * it_per_s: fixed-iteration constrained CG (tol 0) between synchronize brackets, and the same system without
    the projections (stable CG, base fixed) -> overhead of the projection kernels;
  * kernel_ms: hip-event samples of the three CG kernels (+ projections in the third slot);
  * end_to_end: element matrices (compute_c3d4_K_matrix on the GPU) + reference-API solve to tol (assembly +
    device CG), DOFs/s;
  * cpu_baseline: oracle.ref_cpu.constrained_cg (the reference's op sequence on torch-CPU) on a bounded sample.

    python tools/bench_constraints.py [--n 119] [--steps 300] [--cpu-n 40]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, constraints as CS, element, mesh, solver, system  # noqa: E402

E, NU = 113.8e9, 0.342
F64 = torch.float64


def case(coords, n):
    z = coords[:, 2]
    base = torch.nonzero(z < 1e-9).view(-1).tolist()
    top = torch.nonzero(z > 1 - 1e-9).view(-1).tolist()
    h = n // 2
    centre = (h * (n + 1) + h) * (n + 1) + n          # grid node (i, j, k) = (h, h, n)
    below = centre - 1
    slaves = [t for t in top if t != centre]
    ring = [((h + di) * (n + 1) + h + dj) * (n + 1) + n for di, dj in ((1, 0), (-1, 0), (0, 1), (0, -1))]
    spc = [{"node": b, "dofs": [0, 1, 2], "value": 0.0} for b in base]
    rbe2 = [{"master": centre, "slaves": slaves, "dofs": [0, 1, 2]}]
    rbe3 = [{"master": below, "slaves": ring, "dofs": [0, 1, 2], "weights": [1.0, 1.0, 2.0, 2.0]}]
    loads = [{"node": centre, "force": [0.0, 0.0, -1e6]}]
    return spc, rbe2, rbe3, loads, base


def timed_iters(run, warmup, steps):
    run.start()
    run.iterate(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms, cnt = run.profile(steps, every=10)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    it, st, _ = run.poll()
    assert it == warmup + steps, (it, st)
    return steps / dt, [m / max(c, 1) for m, c in zip(ms, cnt)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--cpu-n", type=int, default=40)
    ap.add_argument("--cpu-iters", type=int, default=5)
    ap.add_argument("--rtol", type=float, default=1e-6)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C.lib()
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    N = coords.shape[0]
    spc, rbe2, rbe3, loads, base = case(coords.cpu(), a.n)
    out = {"workload": f"{tets.shape[0]:,}-tet c3d4 elasticity Kuhn cube n={a.n}, {3 * N:,} DOFs; SPC base "
                       f"({3 * len(base)} dofs), RBE2 top plate ({3 * len(rbe2[0]['slaves'])} slave dofs), 1 RBE3"}

    # ---- end to end through the reference API: element matrices + constrained solve to tol
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = element.compute_c3d4_K_matrix(coords, tets, E, NU, device=dev, dtype=F64)
    torch.cuda.synchronize()
    t_ke = time.perf_counter() - t0
    tol = a.rtol * 1e6
    t0 = time.perf_counter()
    u, res = solver.new_constrained_conjugate_gradient_solver(K, tets, N, rbe2, rbe3, spc, loads, tol=tol,
                                                              max_iter=50000, device=dev, return_info=True)
    torch.cuda.synchronize()
    t_solve = time.perf_counter() - t0
    out["end_to_end"] = {"element_K_s": t_ke, "solve_s": t_solve, "iterations": res.iterations, "status": res.status,
                         "tol_abs": tol, "dofs_per_s": 3 * N / (t_ke + t_solve)}
    u = u.view(N, 3)
    out["checks"] = {"rbe2_plate_rigid": bool((u[rbe2[0]["slaves"]] == u[rbe2[0]["master"]]).all()),
                     "spc_exact": bool((u[base] == 0).all())}

    # ---- fixed-iteration rates: constrained vs plain stable CG on the same assembled operator
    A = solver.assemble(K, tets, N, dev)
    del K
    F = torch.zeros((N, 3), dtype=F64)
    CS.apply_loads_to_F(F, loads)
    b = F.to(dev).reshape(-1)
    cs = CS.ConstraintSet(N, 3, dev, CS.parse_spc_list(spc, "cpu"), CS.parse_rbe2_list(rbe2, "cpu"),
                          CS.parse_rbe3_list(rbe3, "cpu"), order=1)
    run = system.PcgRunner(A, b, cs.mask(), mode=C.MODE_CG_CONSTRAINED, schedule=system.SCHED_THREE, constraints=cs)
    r_con, k_con = timed_iters(run, a.warmup, a.steps)
    run.close()
    w = torch.ones((N, 3), dtype=F64, device=dev)
    w[base] = 0.0
    run = system.PcgRunner(A, b, w.view(-1), mode=C.MODE_CG_STABLE, schedule=system.SCHED_THREE)
    r_pl, k_pl = timed_iters(run, a.warmup, a.steps)
    run.close()
    alg = A.algorithmic_bytes_spmv()
    out["it_per_s"] = {"constrained": r_con, "stable_cg": r_pl, "projection_overhead": r_pl / r_con - 1.0}
    out["kernel_ms"] = {"constrained": dict(zip(("spmv_dot", "update", "pupdate+projections"), k_con)),
                        "stable_cg": dict(zip(("spmv_dot", "update", "pupdate"), k_pl))}
    out["spmv_roofline"] = {"algorithmic_bytes": alg, "GBps": alg / (k_con[0] * 1e-3) / 1e9,
                            "frac_of_8TBps": alg / (k_con[0] * 1e-3) / 8e12}
    print(json.dumps(out), flush=True)
    del A, run

    # ---- CPU baseline: the oracle's constrained CG (reference op sequence) on a bounded sample
    from oracle import ref_cpu as R
    cc, ct = mesh.kuhn_cube(a.cpu_n)
    Nc = cc.shape[0]
    spc_c, rbe2_c, rbe3_c, loads_c, _ = case(cc, a.cpu_n)
    Kc = R.tet4_K(cc, ct, E, NU)
    Fc = R.loads_to_F(Nc, loads_c)
    t0 = time.perf_counter()
    R.constrained_cg(Kc, ct, Fc, rbe2_c, spc_c, rbe3_c, tol=0.0, max_iter=a.cpu_iters)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": a.cpu_iters / dt, "unit": "CG iterations/s", "cores": torch.get_num_threads(),
                           "kind": "port", "sample": f"oracle constrained_cg, {ct.shape[0]:,}-tet cube n={a.cpu_n} "
                                                     f"({3 * Nc:,} DOFs), {a.cpu_iters} iterations incl. setup"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
