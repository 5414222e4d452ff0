#!/usr/bin/env python3
"""Stability of the per-workgroup SpMV time of the persistent schedule across launches (GPU box): 8 consecutive
instrumented launches (20 and 100 iterations) of k_pcg_persist on the 10M-tet Poisson bench system; prints the mean
and max over workgroups and the correlation matrix of the per-workgroup times, and writes them to
gpurun_out/wgstab.json.

    python tools/wg_stability_probe.py
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(119, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    f, fixed = mesh.cube_poisson_case(coords)
    mask = torch.zeros(A.n, dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask)
    b = f.reshape(-1).to(torch.float64).contiguous()
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    run.iterate(20)
    G = 256
    rows, iters_used = [], []
    for _ in range(4):
        for iters in (20, 100):
            buf = (ctypes.c_ulonglong * (G * 24))()
            g = ctypes.c_int()
            C.check(run.lib.fem_pcg_persist_profile(run.h, iters, buf, ctypes.byref(g)), "fem_pcg_persist_profile")
            t = torch.tensor(list(buf), dtype=torch.float64)
            rows.append((t[: G * 8].view(G, 8)[:, 1] / 2.4e3 / iters).tolist())   # SpMV phase, us per iteration
            iters_used.append(iters)
    run.close()
    S = torch.tensor(rows)
    print("means", [round(v, 2) for v in S.mean(1).tolist()])
    print("max", [round(v, 2) for v in S.max(1).values.tolist()])
    print("corr matrix:")
    for row in torch.corrcoef(S).tolist():
        print(" ".join("%.2f" % v for v in row))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump({"spmv": rows, "iters": iters_used}, open(os.path.join(ROOT, "gpurun_out", "wgstab.json"), "w"))


if __name__ == "__main__":
    main()
