#!/usr/bin/env python3
"""Assembly-only driver for profiling (tools/profile passes): pattern + c3d4 Poisson/elastic assembly of the Kuhn
cube, timed with events per stage. python tools/assemble_only.py [--n 119] [--kind poisson] [--reps 3]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, mesh, system  # noqa: E402


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--kind", default="poisson")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    bs = 1 if a.kind == "poisson" else 3
    out = []
    import time
    for _ in range(a.reps):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        e0 = ev()
        g = system.build_graph(t, c.shape[0])
        e1 = ev()
        A = system.SellMatrix(g, bs)
        e2 = ev()
        A.add_tet4(c, t, 1.0 if bs == 1 else 113.8e9, 0.0 if bs == 1 else 0.342)
        e3 = ev()
        w = A.jacobi(torch.zeros(A.n, dtype=torch.uint8, device=dev))
        torch.cuda.synchronize()
        bits = int(A.vals.view(torch.int64).sum())
        wall = (time.perf_counter() - h0) * 1e3
        out.append({"graph_ms": e0.elapsed_time(e1), "alloc_ms": e1.elapsed_time(e2), "assemble_ms": e2.elapsed_time(e3),
                    "wall_ms_incl_jacobi": wall, "vals_bits": bits})
        del w
        del A, g
    print(json.dumps(out))


if __name__ == "__main__":
    main()
