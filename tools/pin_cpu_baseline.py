#!/usr/bin/env python3
"""Pin the CPU baseline: time the oracle's restatement (oracle/ref_cpu.py — the `cpu_baseline` leg of
bench.py, kind "port") against the REFERENCE itself, imported read-only from /root/reference (build container only),
on the same Kuhn-cube elasticity systems with the same torch thread count. Quantities: element stiffness
(compute_c3d4_K_matrix), one EBE matvec (compute_nodal_forces), and fixed-count Jacobi-PCG iterations
(preconditioned_conjugate_gradient_solver with tol = 0). Writes profiles/cpu_baseline_pin.json.

    python tools/pin_cpu_baseline.py [--n 55 90] [--iters 5] [--threads 8]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fem355  # noqa: E402,F401  (synthetic meshes only)
from fem355 import mesh  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402

E, NU = 113.8e9, 0.342
F64 = torch.float64


def best(fn, reps):
    t = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        t.append(time.perf_counter() - t0)
    return min(t), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[55, 90])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from gen_golden import REF, load_reference
    if not os.path.isdir(REF):
        print("reference absent: nothing to pin")
        return
    torch.set_num_threads(a.threads)
    el, sol = load_reference()
    res = {"threads": a.threads, "cpu": os.cpu_count(), "iters": a.iters, "systems": {}}
    for n in a.n:
        c, t = mesh.kuhn_cube(n)
        N = c.shape[0]
        f, fixed = mesh.cube_elasticity_case(c)
        row = {"tets": int(t.shape[0]), "dofs": 3 * N}
        tk_ref, K_ref = best(lambda: el.compute_c3d4_K_matrix(c, t, E, NU, device="cpu", dtype=F64), a.reps)
        tk_orc, K = best(lambda: R.tet4_K(c, t, E, NU), a.reps)
        row["ke_s"] = {"reference": tk_ref, "oracle": tk_orc, "ratio": tk_orc / tk_ref}
        row["ke_max_rel_diff"] = float((K - K_ref).abs().max() / K_ref.abs().max())
        del K_ref
        u = torch.randn(N, 3, dtype=F64, generator=torch.Generator().manual_seed(5))
        tm_ref, _ = best(lambda: el.compute_nodal_forces(K, t, u, device="cpu", dtype=F64), a.reps)
        tm_orc, _ = best(lambda: R.nodal_forces(K, t, u), a.reps)
        row["matvec_s"] = {"reference": tm_ref, "oracle": tm_orc, "ratio": tm_orc / tm_ref}
        Minv = R.diag_preconditioner(K, t, N)
        Minv[fixed] = 0.0
        with contextlib.redirect_stdout(io.StringIO()):
            tc_ref, _ = best(lambda: sol.preconditioned_conjugate_gradient_solver(
                K, t, f.view(N, 3), Minv, tol=0.0, max_iter=a.iters, device="cpu", dtype=F64), 1)
        tc_orc, _ = best(lambda: R.pcg(K, t, f.view(N, 3), Minv, tol=0.0, max_iter=a.iters), 1)
        row["pcg_it_per_s"] = {"reference": a.iters / tc_ref, "oracle": a.iters / tc_orc, "ratio": tc_ref / tc_orc}
        res["systems"][f"kuhn{n}_elastic"] = row
        print(json.dumps({n: row}), flush=True)
        del K, Minv
    out = os.path.join(ROOT, "profiles", "cpu_baseline_pin.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
