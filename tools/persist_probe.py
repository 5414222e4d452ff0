#!/usr/bin/env python3
"""Persistent-geometry SpMV probe (GPU box): how fast is the paired bs = 1 SpMV of the 10M Poisson matrix when each
wave owns a fixed contiguous slice range and occupancy is pinned to one workgroup per CU (the geometry a
register-resident persistent PCG would need), against the production launch (grid-stride, ~5 waves/SIMD)?

    python tools/persist_probe.py [--n 119] [--reps 20]
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


def timed(fn, reps, pre=None):
    ts = []
    for _ in range(reps):
        if pre:
            pre()
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
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    g = A.g
    x = torch.randn(A.n, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    alg = A.algorithmic_bytes_spmv(index_bytes=2)
    vp = torch.empty_like(A.vals)
    cp = torch.empty_like(g.dcols)
    C.check(lab.fem_lab_sell_pair(g.n_nodes, C.ptr(g.slice_ptr), C.ptr(A.vals), C.ptr(g.dcols), C.ptr(vp), C.ptr(cp),
                                  st), "pair")
    pol = torch.empty(140 * (1 << 20) // 8, dtype=torch.float64, device=dev)
    pol2 = torch.empty_like(pol)

    def pollute():
        C.check(lab.fem_lab_copy(16, 0, C.ptr(pol), C.ptr(pol2), pol.numel(), 2048, st), "pollute")

    def base():
        C.check(lab.fem_lab_spmv16_pair(8, 0, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(cp), C.ptr(vp), C.ptr(x), C.ptr(y),
                                        st), "pair spmv")
    base()
    torch.cuda.synchronize()
    ref = y.clone()
    out = {"n_cu": ncu, "alg_bytes": alg, "base_ms": timed(base, a.reps), "base_pol_ms": timed(base, a.reps, pollute)}
    for thr, lds, wgs in ((512, 96 << 10, 1), (1024, 96 << 10, 1), (256, 96 << 10, 1), (256, 64 << 10, 2),
                          (512, 64 << 10, 2)):
        for u in (4, 8):
            def run(thr=thr, lds=lds, u=u, wgs=wgs):
                C.check(lab.fem_lab_spmv_persist(thr, u, ncu * wgs, lds, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(cp),
                                                 C.ptr(vp), C.ptr(x), C.ptr(y), st), "persist")
            y.zero_()
            run()
            torch.cuda.synchronize()
            key = f"t{thr}_wg{wgs}_u{u}"
            out[key + "_equal"] = bool(torch.equal(y, ref))
            out[key + "_ms"] = timed(run, a.reps)
            out[key + "_pol_ms"] = timed(run, a.reps, pollute)
    for k in list(out):
        if k.endswith("_ms"):
            out[k.replace("_ms", "_GBps")] = alg / (out[k] * 1e-3) / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
