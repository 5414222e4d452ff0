#!/usr/bin/env python3
"""Host/device wall time of each step of the pattern build + assembly (system._build_graph, SellMatrix.add_tet4,
jacobi), synchronising after every step, warm (third of three builds). python tools/graph_steps.py [--n 55]"""
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C.lib()
    c, t = mesh.kuhn_cube(a.n, device=dev)
    N = c.shape[0]
    steps = {}
    orig_check = C.check

    def timed_check(rc, what):
        torch.cuda.synchronize()
        now = time.perf_counter()
        steps[what] = steps.get(what, 0.0) + (now - timed_check.last) * 1e3
        timed_check.last = now
        return orig_check(rc, what)

    for rep in range(3):
        steps.clear()
        torch.cuda.synchronize()
        timed_check.last = t0 = time.perf_counter()
        C.check = timed_check
        try:
            A = system.assemble_tet4_system(c, t, "poisson", 1.0, 0.0)
            w = A.jacobi(torch.zeros(N, dtype=torch.uint8, device=dev))
            torch.cuda.synchronize()
        finally:
            C.check = orig_check
        total = (time.perf_counter() - t0) * 1e3
        del A, w
    print(json.dumps({"n": a.n, "total_ms": total, "steps_ms (wall since the previous C call, incl. host work)":
                      {k: round(v, 3) for k, v in steps.items()}}))


if __name__ == "__main__":
    main()
