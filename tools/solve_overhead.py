#!/usr/bin/env python3
"""Where the solve-to-tolerance wall time goes beyond the iterations (10M Poisson, persistent schedule): context
create (vector + paired-copy allocations), schedule setup, the solve launch, destroy.

    python tools/solve_overhead.py [--n 119] [--reps 3]
"""
import argparse
import ctypes
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
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    f, fixed = mesh.cube_poisson_case(coords)
    mask = torch.zeros(coords.shape[0], dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask)
    b = f.reshape(-1).to(torch.float64).contiguous()
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    lib = C.lib()
    s = C.stream(dev)

    def sync():
        torch.cuda.synchronize(dev)
        return time.perf_counter()

    for rep in range(a.reps):
        x = torch.zeros(A.n, dtype=torch.float64, device=dev)
        h = ctypes.c_void_p()
        t = [sync()]
        C.check(lib.fem_pcg_create(A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols), C.ptr(A.vals),
                                   C.ptr(b), C.ptr(x), C.ptr(w), C.MODE_PCG, float(tol), 1e-30, None, 0, s,
                                   ctypes.byref(h)), "create")
        t.append(sync())
        C.check(lib.fem_pcg_set_schedule(h, 3), "sched")
        A.attach_cols16(h)
        t.append(sync())
        C.check(lib.fem_pcg_start(h), "start")
        t.append(sync())
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        C.check(lib.fem_pcg_solve(h, 20000, 64, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)), "solve")
        t.append(sync())
        lib.fem_pcg_destroy(h)
        t.append(sync())
        d = [round((t[i + 1] - t[i]) * 1e3, 3) for i in range(len(t) - 1)]
        print(json.dumps({"rep": rep, "create_ms": d[0], "schedule_ms": d[1], "start_ms": d[2], "solve_ms": d[3],
                          "destroy_ms": d[4], "iters": it.value, "status": stt.value,
                          "us_per_it_in_solve": d[3] * 1e3 / max(it.value, 1)}), flush=True)
    # the product call as bench.py times it
    for rep in range(a.reps):
        t0 = sync()
        r = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64)
        print(json.dumps({"pcg_call_ms": round((sync() - t0) * 1e3, 3), "iters": r.iterations}), flush=True)


if __name__ == "__main__":
    main()
