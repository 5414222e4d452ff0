#!/usr/bin/env python3
"""SpMV layout lab on the GPU box: why does the in-PCG SpMV (k_pcg_d1) run slower than the stand-alone one, and
does a lane-paired SELL layout (16-byte value loads) help? Prints one JSON object.

  * copy / read probes at 8, 16, 32 bytes per lane on 2 x 1 GiB
  * k_spmv16 (plain layout) vs k_spmv16_pair (paired layout, U = 2, 4, 8) on the 10M Poisson matrix
  * cache state: k_spmv16 alone vs interleaved with a 140 MB stream (the PCG's vector traffic)
  * PCG kernel times (deferred schedule) for reference

    python tools/spmv_layout.py [--n 119] [--reps 20]
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
    """median ms of fn, each launch bracketed by events; pre() runs (untimed) before each launch."""
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
    ap.add_argument("--pcg-only", action="store_true")
    ap.add_argument("--tunes", default="0,1")
    a = ap.parse_args()
    lib = C.lib()
    lab = lab_lib.load()
    dev = torch.device("cuda", 0)
    st = C.stream(dev)
    out = {}
    if a.pcg_only:
        return pcg_tunes(a, lib, dev, out)
    nb = (1 << 30) // 8
    src = torch.randn(nb, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    for w in (8, 16, 32):
        for g in (2048, 8192):
            ms = timed(lambda: C.check(lab.fem_lab_copy(w, 0, C.ptr(src), C.ptr(dst), nb, g, st), "copy"), 5)
            out[f"copy{w}_g{g}_GBps"] = 2 * nb * 8 / (ms * 1e-3) / 1e9
    for w in (8, 16):
        ms = timed(lambda: C.check(lab.fem_lab_copy(w, 1, C.ptr(src), C.ptr(dst), nb, 4096, st), "read"), 5)
        out[f"read{w}_GBps"] = nb * 8 / (ms * 1e-3) / 1e9
    del src, dst
    print(json.dumps(out), flush=True)

    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    g = A.g
    assert g.dcols is not None
    x = torch.randn(A.n, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    alg = A.algorithmic_bytes_spmv(index_bytes=2)
    ref = A.matvec(x).clone()
    vp = torch.empty_like(A.vals)
    cp = torch.empty_like(g.dcols)
    C.check(lab.fem_lab_sell_pair(g.n_nodes, C.ptr(g.slice_ptr), C.ptr(A.vals), C.ptr(g.dcols), C.ptr(vp), C.ptr(cp),
                                  st), "pair")

    def plain():
        C.check(lib.fem_spmv16(g.n_nodes, 1, C.ptr(g.slice_ptr), C.ptr(g.dcols), C.ptr(A.vals), C.ptr(x), C.ptr(y),
                               st), "spmv16")

    res = {"alg_bytes": alg}
    plain()
    ms = timed(plain, a.reps)
    res["plain_ms"] = ms
    for u in (2, 4, 8):
        def pair(u=u):
            C.check(lab.fem_lab_spmv16_pair(u, 0, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(cp), C.ptr(vp), C.ptr(x),
                                            C.ptr(y), st), "pair spmv")
        pair()
        torch.cuda.synchronize()
        err = float((y - ref).abs().max() / ref.abs().max())
        res[f"pair_u{u}_ms"] = timed(pair, a.reps)
        res[f"pair_u{u}_relerr"] = err
    # cache pollution: stream 140 MB (the PCG vector traffic) between launches
    pol = torch.empty(140 * (1 << 20) // 8, dtype=torch.float64, device=dev)
    pol2 = torch.empty_like(pol)

    def pollute():
        C.check(lab.fem_lab_copy(16, 0, C.ptr(pol), C.ptr(pol2), pol.numel(), 2048, st), "pollute")
    res["plain_after_140MB_ms"] = timed(plain, a.reps, pre=pollute)
    bigp = torch.empty(600 * (1 << 20) // 8, dtype=torch.float64, device=dev)
    bigp2 = torch.empty_like(bigp)

    def flush():
        C.check(lab.fem_lab_copy(16, 0, C.ptr(bigp), C.ptr(bigp2), bigp.numel(), 2048, st), "flush")
    res["plain_after_1200MB_ms"] = timed(plain, a.reps, pre=flush)

    def pair4():
        C.check(lab.fem_lab_spmv16_pair(4, 0, g.n_nodes, C.ptr(g.slice_ptr), C.ptr(cp), C.ptr(vp), C.ptr(x),
                                        C.ptr(y), st), "pair spmv")
    res["pair_u4_after_1200MB_ms"] = timed(pair4, a.reps, pre=flush)
    for k in list(res):
        if k.endswith("_ms"):
            res[k.replace("_ms", "_GBps")] = alg / (res[k] * 1e-3) / 1e9
    out["spmv"] = res
    print(json.dumps(out), flush=True)
    del bigp, bigp2

    pcg_tunes(a, lib, dev, out, A, x)


def pcg_tunes(a, lib, dev, out, A=None, x=None):
    import time
    if A is None:
        coords, tets = mesh.kuhn_cube(a.n, device=dev)
        A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
        x = torch.randn(A.n, dtype=torch.float64, device=dev)
    w = torch.ones(A.n, dtype=torch.float64, device=dev)
    tunes = [int(t) for t in a.tunes.split(",")]
    for tune in tunes + tunes:
        run = system.PcgRunner(A, x, w, tol=0.0)
        run.set_tuning(tune)
        run.start()
        run.iterate(20)
        ms, n = run.profile(200, every=1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.iterate(400)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 400 * 1e3
        out.setdefault(f"pcg_tune{tune}", []).append({"kernel_ms": [m / max(c, 1) for m, c in zip(ms, n)],
                                                     "wall_ms_per_it": wall})
        run.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
