#!/usr/bin/env python3
"""Where the assembly wall time of bench.py's DOFs/s goes (host launches and syncs vs kernels):
python tools/asm_breakdown.py [--n 55] [--kind poisson] [--reps 5]

Times, per repetition, the whole assembly as bench.py does it (pattern + values + Jacobi, one sync at the end) and
each step on its own (sync after each step), host wall clock. Run under rocprofv3 --kernel-trace --stats for the
kernel side."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=55)
    ap.add_argument("--kind", default="poisson", choices=["poisson", "elastic"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--solve", action="store_true", help="also solve after each whole assembly (as bench.py does)")
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    N = coords.shape[0]
    f, fixed = mesh.cube_poisson_case(coords) if a.kind == "poisson" else mesh.cube_elasticity_case(coords)
    E, nu = (1.0, 0.0) if a.kind == "poisson" else (113.8e9, 0.342)
    bs = 1 if a.kind == "poisson" else 3
    sync = torch.cuda.synchronize

    def whole():
        A = system.assemble_tet4_system(coords, tets, a.kind, E, nu)
        mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
        mask.index_fill_(0, fixed, 1)   # a fill kernel: no host-to-device copy (and host wait) of the 1
        w = A.jacobi(mask.view(-1))
        return A, w

    res = {"n": a.n, "kind": a.kind, "tets": int(tets.shape[0]), "whole_ms": [], "steps_ms": []}
    for _ in range(a.reps):
        sync()
        t0 = time.perf_counter()
        A, w = whole()
        sync()
        res["whole_ms"].append((time.perf_counter() - t0) * 1e3)
        if a.solve:
            b = f.reshape(-1).to(torch.float64).contiguous()
            tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
            sync()
            t0 = time.perf_counter()
            r = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64)
            sync()
            res.setdefault("solve_ms", []).append((time.perf_counter() - t0) * 1e3)
            del b, r
        del A, w
        st = {}
        sync()
        t0 = time.perf_counter()
        g = system.build_graph(tets, N, solver_layout=(bs == 1))
        sync()
        st["graph"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        A = system.SellMatrix(g, bs).add_tet4(coords.to(torch.float64).contiguous(), tets.contiguous(), E, nu)
        sync()
        st["values"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
        mask.index_fill_(0, fixed, 1)   # a fill kernel: no host-to-device copy (and host wait) of the 1
        sync()
        st["mask"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        w = A.jacobi(mask.view(-1))
        sync()
        st["jacobi"] = (time.perf_counter() - t0) * 1e3
        res["steps_ms"].append(st)
        del A, w, g
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
