#!/usr/bin/env python3
"""SpMV / PCG kernel tuning on the GPU box: interleaved A/B rounds of the SpMV code variants and grid sizes on
the benchmark matrix, the HBM copy ceiling, and the per-kernel PCG times. Prints one JSON object.

    python tools/spmv_tune.py [--n 119] [--kind poisson] [--rounds 5]
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


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--kind", default="poisson")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--grids", default="0,1024,4096,8192")
    a = ap.parse_args()
    lib = C.lib()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, a.kind, 1.0 if a.kind == "poisson" else 113.8e9, 0.342)
    torch.cuda.synchronize()
    x = torch.randn(A.n, dtype=torch.float64, device=dev)
    y = torch.empty_like(x)
    alg = A.algorithmic_bytes_spmv()
    st = C.stream(dev)
    out = {"n": a.n, "kind": a.kind, "nnz_blocks": A.g.nnz, "sell_entries": A.g.sell_entries, "alg_bytes": alg}
    ref = A.matvec(x).clone()
    variants = [int(v) for v in a.variants.split(",")] if A.bs == 1 else [0]
    grids = [int(g) for g in a.grids.split(",")]
    res = {}
    for r in range(a.rounds):
        for v in variants:
            for g in grids:
                def f():
                    C.check(lib.fem_spmv_variant(v, g, A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols),
                                                 C.ptr(A.vals), C.ptr(x), C.ptr(y), st), "variant")
                f()
                t = timed(f, a.reps)
                res.setdefault(f"v{v}_g{g}", []).append(t)
        if r == 0:
            for v in variants:
                C.check(lib.fem_spmv_variant(v, 0, A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols),
                                             C.ptr(A.vals), C.ptr(x), C.ptr(y), st), "variant")
                torch.cuda.synchronize()
                assert float((y - ref).abs().max()) <= 1e-12 * float(ref.abs().max()), v
    print(json.dumps({"stage": "variants"}), flush=True)
    if A.g.dcols is not None:
        t16 = []
        for r in range(a.rounds):
            def f16():
                C.check(lib.fem_spmv16(A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.dcols), C.ptr(A.vals),
                                       C.ptr(x), C.ptr(y), st), "spmv16")
            f16()
            t16.append(timed(f16, a.reps))
        alg16 = A.algorithmic_bytes_spmv(index_bytes=2)
        med = sorted(t16)[len(t16) // 2]
        out["spmv16_ms"] = {"min": min(t16), "med": med, "GBps_med": alg16 / (med * 1e-3) / 1e9, "alg_bytes": alg16}
    out["spmv_ms"] = {k: {"min": min(v), "med": sorted(v)[len(v) // 2],
                          "GBps_med": alg / (sorted(v)[len(v) // 2] * 1e-3) / 1e9} for k, v in res.items()}
    # HBM copy ceiling on 2 x 1 GiB
    nbuf = (1 << 30) // 8
    src = torch.randn(nbuf, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    cc = {}
    for g in (1024, 2048, 4096, 8192):
        def f():
            C.check(lib.fem_stream_copy(C.ptr(src), C.ptr(dst), nbuf, g, st), "copy")
        f()
        t = timed(f, 10)
        cc[g] = 2 * nbuf * 8 / (t * 1e-3) / 1e9
    out["copy_GBps"] = cc
    print(json.dumps(out), flush=True)
    del src, dst
    # PCG kernels, both schedules
    import time
    w = torch.ones(A.n, dtype=torch.float64, device=dev)
    for sched in (0, 1, 2):
        tag = {0: "3k", 1: "fused", 2: "deferred"}[sched]
        run = system.PcgRunner(A, x, w, tol=0.0, schedule=sched)
        run.start()
        run.iterate(20)
        ms, n = run.profile(200, every=1)
        out[f"pcg_kernel_ms_{tag}"] = {"spmv_dot": ms[0] / n[0], "update": ms[1] / n[1], "pupdate": ms[2] / n[2]}
        torch.cuda.synchronize()
        for rnd in range(3):
            t0 = time.perf_counter()
            run.iterate(200)
            torch.cuda.synchronize()
            out.setdefault(f"pcg_ms_per_iter_plain_{tag}", []).append((time.perf_counter() - t0) / 200 * 1e3)
        try:
            run.use_graph(20)
            run.iterate(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run.iterate(200)
            torch.cuda.synchronize()
            out[f"pcg_ms_per_iter_graph_{tag}"] = (time.perf_counter() - t0) / 200 * 1e3
        except Exception as e:  # report and continue
            out["graph_error"] = str(e)
        run.close()
        print(json.dumps(out), flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
