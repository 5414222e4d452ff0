#!/usr/bin/env python3
"""Host timestamps (no synchronisation) at every C-ABI return during one warm 10M Poisson assembly + Jacobi (GPU
box): where the host spends the time after the pattern's size read-back, when the GPU waits for its launches.
    python tools/probes/asm_host_steps.py [--n 119]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=119)
a = ap.parse_args()
C.lib()
dev = torch.device("cuda", 0)
coords, tets = mesh.kuhn_cube(a.n, device=dev)
N = coords.shape[0]
f, fixed = mesh.cube_poisson_case(coords)
marks = []
orig_check = C.check
orig_cpu = torch.Tensor.cpu


def check(rc, what):
    marks.append((what, time.perf_counter()))
    return orig_check(rc, what)


def whole():
    marks.append(("start", time.perf_counter()))
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    marks.append(("assembled", time.perf_counter()))
    mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
    mask.index_fill_(0, fixed, 1)
    marks.append(("mask", time.perf_counter()))
    w = A.jacobi(mask.view(-1))
    marks.append(("jacobi", time.perf_counter()))
    torch.cuda.synchronize()
    marks.append(("synced", time.perf_counter()))
    return A, w


for _ in range(3):
    A, w = whole()
    del A, w
res = []
for rep in range(3):
    marks.clear()
    C.check = check
    try:
        A, w = whole()
    finally:
        C.check = orig_check
    t0 = marks[0][1]
    res.append([(k, round((t - t0) * 1e6, 1)) for k, t in marks])
    del A, w
print(json.dumps(res[-1]))
