#!/usr/bin/env python3
"""Fixed-iteration time of the persistent Poisson iteration, single-reduction vs pipelined (FEM_TUNE_PK_GV), on the
Kuhn cube of --n (timing only; FEM355_LIB selects a build, e.g. a FEM_GV_PROBE timing build).

    python tools/gv_probe.py --n 55 --iters 500
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=55)
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    c, t = mesh.kuhn_cube(a.n)
    c, t = c.to(dev), t.to(dev)
    f, fixed = mesh.cube_poisson_case(c)
    mask = torch.zeros(c.shape[0], dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    A = system.assemble_tet4_system(c, t, "poisson")
    w = A.jacobi(mask)
    b = f.reshape(-1).to(torch.float64)
    for name, tune in (("single-reduction", C.TUNE_DEFAULT), ("pipelined", C.TUNE_DEFAULT | C.TUNE_PK_GV)):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=3, tune=tune)
        run.start()
        run.iterate(50)
        run.poll()
        best = None
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.iterate(a.iters)
            run.poll()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print(f"n={a.n} {name:16s} pipelined={run.pipelined()} {best / a.iters * 1e6:.2f} us/iteration")
        run.close()


if __name__ == "__main__":
    main()
