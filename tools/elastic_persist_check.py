#!/usr/bin/env python3
"""bs = 3 persistent PCG (elasticity) on the GPU box against the three-kernel schedule -- fixed-iteration rate and
the solve to rtol 1e-8 (iterations, x) -- with and without FEM_TUNE_PK_WIDE. (A one-slot bs = 3 build with 2 blocks
in flight was measured with this probe, profiles/r02e_elastic_one_slot_probe.txt: "persist" there is that build,
no faster than the two-slot one, so it was not kept; the flag has no effect on bs = 3 now.)

    python tools/elastic_persist_check.py [--n 40 55 59] [--iters 500]
"""
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

DEFAULT_TUNE = 1 | 2 | 4 | 8 | 128   # fem355.h: REVERSE | PAIR | PK_SC1 | PK_PACK | PK_UNI
WIDE = 256                            # FEM_TUNE_PK_WIDE


def case(n, dev):
    coords, tets = mesh.kuhn_cube(n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "elastic", 113.8e9, 0.342)
    f, fixed = mesh.cube_elasticity_case(coords)
    mask = torch.zeros((coords.shape[0], 3), dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1).to(torch.float64).contiguous()
    return A, b, w


def rate(A, b, w, sched, tune, warm, iters):
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
    run.set_tuning(tune)
    run.start()
    eff = run.effective_schedule()
    run.iterate(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.iterate(iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    it, stt, _ = run.poll()
    run.close()
    return {"sched": eff, "us_per_it": dt / iters * 1e6, "iter": it, "status": stt}


def solve(A, b, w, sched, tune, rtol=1e-8):
    tol = rtol * float(torch.sqrt(torch.dot(b, w * b)))
    run = system.PcgRunner(A, b, w, tol=tol, schedule=sched)
    run.set_tuning(tune)
    run.start()
    while True:
        run.iterate(256)
        it, stt, _ = run.poll()
        if stt != C.PCG_RUNNING or it >= 20000:
            break
    x = run.x.clone()
    run.close()
    return it, stt, x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[40, 55, 59])
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--warm", type=int, default=50)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    for n in a.n:
        A, b, w = case(n, dev)
        out = {"n": n, "rows": A.n_rows, "dofs": A.n}
        for name, sched, tune in (("persist", 3, DEFAULT_TUNE), ("persist_wide", 3, DEFAULT_TUNE | WIDE),
                                  ("three_kernel", 0, DEFAULT_TUNE)):
            out[name] = rate(A, b, w, sched, tune, a.warm, a.iters)
        it0, st0, x0 = solve(A, b, w, 3, DEFAULT_TUNE | WIDE)
        it1, st1, x1 = solve(A, b, w, 3, DEFAULT_TUNE)
        out["solve"] = {"wide": [it0, st0], "default": [it1, st1],
                        "x_rel": float((x1 - x0).norm() / x0.norm())}
        print(json.dumps(out), flush=True)
        del A, b, w


if __name__ == "__main__":
    main()
