#!/usr/bin/env python3
"""Element-chunk operator against the assembled one on the Kuhn cube: operator and diagonal agreement, and the PCG
solve to rtol on both (iterations, status, solution difference).

    python tools/mf_solve_check.py [--n 119] [--kind elastic] [--rtol 1e-8]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402

E, NU = 113.8e9, 0.342


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--kind", default="elastic")
    ap.add_argument("--rtol", type=float, default=1e-8)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    N = c.shape[0]
    Ek = E if a.kind == "elastic" else 1.0
    A = system.MatFreeOperator(c, t, a.kind, Ek, NU)
    As = system.assemble_tet4_system(c, t, a.kind, Ek, NU)
    x = torch.randn(A.n, dtype=torch.float64, device=dev)
    y, ys = A.matvec(x), As.matvec(x)
    out = {"n": a.n, "kind": a.kind, "info": A.info(),
           "rel_matvec": float((y - ys).abs().max() / ys.abs().max())}
    f, fixed = mesh.cube_elasticity_case(c) if a.kind == "elastic" else mesh.cube_poisson_case(c)
    mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w, ws = A.jacobi(mask.view(-1)), As.jacobi(mask.view(-1))
    out["rel_jacobi"] = float((w - ws).abs().max() / ws.abs().max())
    b = f.reshape(-1).to(torch.float64).contiguous()
    tol = a.rtol * float(torch.sqrt(torch.dot(b, ws * b)))
    r1 = As.pcg(b, None, w=ws, tol=tol, max_iter=20000, chunk=64)
    r2 = A.pcg(b, None, w=ws, tol=tol, max_iter=20000, chunk=64)
    out["assembled"] = {"iters": r1.iterations, "status": r1.status}
    out["matfree"] = {"iters": r2.iterations, "status": r2.status}
    out["rel_x"] = float((r1.x - r2.x).abs().max() / r1.x.abs().max())
    for k in (1, 2, 5, 20):
        q1 = As.pcg(b, None, w=ws, tol=0.0, max_iter=k, schedule=0)
        q2 = A.pcg(b, None, w=ws, tol=0.0, max_iter=k)
        out[f"rel_x_{k}"] = float((q1.x - q2.x).abs().max() / q1.x.abs().max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
