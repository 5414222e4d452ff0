#!/usr/bin/env python3
"""Device RCM on a randomly numbered cube, timed: python tools/rcm_probe.py [--n 119] [--reps 4] (run under
rocprofv3 --kernel-trace --stats for the per-kernel side)"""
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
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    N = coords.shape[0]
    g = torch.Generator(device="cpu").manual_seed(7)
    perm = torch.randperm(N, generator=g).to(dev)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(N, device=dev)
    tets = inv[tets].contiguous()
    graph = system.build_graph(tets, N, compress=False)
    torch.cuda.synchronize()
    out = {"rcm_ms": [], "graph_plus_rcm_ms": []}
    for _ in range(a.reps):
        t0 = time.perf_counter()
        system.rcm_order(tets, N, graph=graph)
        torch.cuda.synchronize()
        out["rcm_ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
        t0 = time.perf_counter()
        system.rcm_order(tets, N)
        torch.cuda.synchronize()
        out["graph_plus_rcm_ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
