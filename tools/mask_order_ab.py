#!/usr/bin/env python3
"""Whole assembly as bench.py times it, the Dirichlet mask built before vs after the pattern, alternating in one
process: python tools/mask_order_ab.py [--n 119] [--kind poisson] [--reps 8]"""
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
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--kind", default="poisson", choices=["poisson", "elastic"])
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    N = coords.shape[0]
    f, fixed = mesh.cube_poisson_case(coords) if a.kind == "poisson" else mesh.cube_elasticity_case(coords)
    E, nu = (1.0, 0.0) if a.kind == "poisson" else (113.8e9, 0.342)
    bs = 1 if a.kind == "poisson" else 3
    sync = torch.cuda.synchronize

    def before():
        mask = torch.zeros((N, bs), dtype=torch.uint8, device=dev)
        mask[fixed] = 1
        A = system.assemble_tet4_system(coords, tets, a.kind, E, nu)
        return A, A.jacobi(mask.view(-1))

    def after():
        A = system.assemble_tet4_system(coords, tets, a.kind, E, nu)
        mask = torch.zeros((N, bs), dtype=torch.uint8, device=dev)
        mask[fixed] = 1
        return A, A.jacobi(mask.view(-1))

    out = {"before": [], "after": []}
    for i in range(a.reps):
        for name, fn in (("before", before), ("after", after)) if i % 2 == 0 else (("after", after), ("before", before)):
            sync()
            t0 = time.perf_counter()
            A, w = fn()
            sync()
            out[name].append(round((time.perf_counter() - t0) * 1e3, 4))
            del A, w
    out = {k: {"ms": v, "median": sorted(v)[len(v) // 2]} for k, v in out.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
