#!/usr/bin/env python3
"""bs = 3 SpMV layout lab on the GPU box (sell_pair3.hpp): the 10M-tet elasticity matrix (n = 119, 25.6M 3x3
blocks) in the plain layout (9 eight-byte plane loads per block), the plane-paired layout A (4 sixteen-byte + 1
eight-byte) and the entry-paired layout B (9 sixteen-byte loads per two blocks + one int32 column pair); U blocks
(pairs) in flight, default or nontemporal loads. Prints one JSON object: median ms, GB/s of the algorithmic bytes,
and the max |difference| to the production SpMV (expected 0: same summation order).

    python tools/spmv3_layout.py [--n 119] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, mesh, system  # noqa: E402
import lab as lab_lib  # noqa: E402  (tools/lab: probe kernels, not part of libfem355)


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    lib = C.lib()
    lab = lab_lib.load()
    dev = torch.device("cuda", 0)
    st = C.stream(dev)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "elastic", 113.8e9, 0.342)
    g = A.g
    assert g.dcols is not None
    xp = torch.randn(A.n + 1, dtype=torch.float64, device=dev)
    x = xp[:A.n]
    y = torch.empty_like(x)
    alg = A.algorithmic_bytes_spmv(index_bytes=2)
    ref = A.matvec(x.contiguous()).clone()
    out = {"alg_bytes": alg, "n_dofs": A.n}

    def prod():
        C.check(lib.fem_spmv16(g.n_nodes, 3, C.ptr(g.slice_ptr), C.ptr(g.dcols), C.ptr(A.vals), C.ptr(x), C.ptr(y),
                               st), "spmv16")
    prod()
    out["production_ms"] = timed(prod, a.reps)
    lay = {0: (A.vals, g.dcols)}
    for L in (1, 2):
        v = torch.empty_like(A.vals)
        c = torch.empty_like(g.dcols) if L == 2 else g.dcols
        C.check(lab.fem_lab_sell3_layout(L, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(A.vals), C.ptr(g.dcols), C.ptr(v),
                                         C.ptr(c), st), "layout")
        lay[L] = (v, c)
    torch.cuda.synchronize()
    lay[3] = lay[1]   # layout A, 8 + 16-byte gathers (x padded by one double)
    for L in (0, 1, 2, 3):
        v, c = lay[L]
        for u in (1, 2):
            for nt in (0, 1):
                def run(L=L, u=u, nt=nt, v=v, c=c):
                    C.check(lab.fem_lab_spmv3(L, u, nt, 0, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(c), C.ptr(v),
                                              C.ptr(x), C.ptr(y), st), "spmv3")
                y.zero_()
                run()
                torch.cuda.synchronize()
                key = f"L{L}_u{u}_nt{nt}"
                out[key + "_maxdiff"] = float((y - ref).abs().max())
                out[key + "_ms"] = timed(run, a.reps)
    for k in list(out):
        if k.endswith("_ms"):
            out[k.replace("_ms", "_GBps")] = alg / (out[k] * 1e-3) / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
