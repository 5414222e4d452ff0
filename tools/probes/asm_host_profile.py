#!/usr/bin/env python3
"""Host-side (Python) cost of one warm 10M Poisson assembly + Jacobi (GPU box): cProfile of the call sequence of
tools/asm_breakdown.py's whole(), to see which host work sits on the critical path after the pattern's size sync.
    python tools/probes/asm_host_profile.py [--n 119]"""
import argparse
import cProfile
import os
import pstats
import sys

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


def whole():
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
    mask.index_fill_(0, fixed, 1)
    w = A.jacobi(mask.view(-1))
    return A, w


for _ in range(3):
    A, w = whole()
    torch.cuda.synchronize()
    del A, w
pr = cProfile.Profile()
for _ in range(5):
    torch.cuda.synchronize()
    pr.enable()
    A, w = whole()
    torch.cuda.synchronize()
    pr.disable()
    del A, w
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
