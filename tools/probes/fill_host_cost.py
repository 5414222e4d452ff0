#!/usr/bin/env python3
"""Host cost of the C-ABI calls after the pattern's size read-back (GPU box): each call repeated on a warm 10M
Poisson pattern, host time per call without synchronisation (the launches queue behind each other), and the
SellMatrix / value-kernel / Jacobi Python path. python tools/probes/fill_host_cost.py [--n 119]"""
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
lib = C.lib()
dev = torch.device("cuda", 0)
coords, tets = mesh.kuhn_cube(a.n, device=dev)
N = coords.shape[0]
out = {}
for _ in range(3):
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
torch.cuda.synchronize()
g = A.graph if hasattr(A, "graph") else A.g
sl = g._sl
st = C.stream(dev)
ent = int(g.cols.numel())
tmp = torch.empty(max(int(lib.fem_graph_tmp_len(N)), 1), dtype=torch.int32, device=dev)
tmp.fill_(0)
torch.cuda.synchronize()


def host_time(fn, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / reps * 1e6


out["empty_alloc_us"] = host_time(lambda: (torch.empty(g.colidx.numel(), dtype=torch.int32, device=dev),
                                           torch.empty(N, dtype=torch.int32, device=dev),
                                           torch.empty(ent, dtype=torch.int32, device=dev),
                                           torch.empty(ent, dtype=torch.int16, device=dev)))
out["sl_arrays_us"] = host_time(lambda: system._solver_layout_arrays(dev, ent, N))
tets_c = tets.contiguous()
out["fill_sl_call_us"] = host_time(lambda: lib.fem_graph_sell_fill_sl(
    C.ptr(tets_c), 4, C.ptr(g.inc_ptr), C.ptr(g.inc), N, C.ptr(g.rowptr), C.ptr(tmp), C.ptr(g.slice_ptr),
    C.ptr(g.colidx), C.ptr(g.diagpos), C.ptr(g.cols), C.ptr(g.dcols), sl.G, C.ptr(sl.pcols), C.ptr(sl.ucol),
    C.ptr(sl.uoff), C.ptr(sl.win), st), reps=10)
out["fill_sl_call_nospans_us"] = host_time(lambda: lib.fem_graph_sell_fill_sl(
    C.ptr(tets_c), 4, C.ptr(g.inc_ptr), C.ptr(g.inc), N, C.ptr(g.rowptr), C.ptr(tmp), C.ptr(g.slice_ptr),
    C.ptr(g.colidx), C.ptr(g.diagpos), C.ptr(g.cols), C.ptr(g.dcols), 0, C.ptr(sl.pcols), C.ptr(sl.ucol),
    C.ptr(sl.uoff), None, st), reps=10)
c64 = coords.to(torch.float64).contiguous()
out["sellmatrix_add_tet4_us"] = host_time(lambda: system.SellMatrix(g, 1).add_tet4(c64, tets_c, 1.0, 0.0), reps=5)
print(json.dumps(out))
