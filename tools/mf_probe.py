#!/usr/bin/env python3
"""Element-chunk (matrix-free) operator probe on the Kuhn cube: build time, application time against the assembled
SELL operator's SpMV, agreement with it, and the PCG iteration split (K1 = chunk kernel + gather, merged update).

    python tools/mf_probe.py [--n 119] [--kind elastic] [--iters 50]
"""
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

E, NU = 113.8e9, 0.342


def ev(fn, reps=1):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--kind", default="elastic")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-assembled", action="store_true")
    ap.add_argument("--rotate", type=float, default=0.0,
                    help="rotate the cube by this many degrees about (1,1,2) (Morton cells no longer on its hexes)")
    ap.add_argument("--graph", type=int, default=0, help="also time the iterations replayed from a hipGraph of k")
    ap.add_argument("--tune-extra", type=int, default=int(os.environ.get("FEM355_PROBE_TUNE", "0")),
                    help="FEM_TUNE_* flags added to the library default (e.g. 8192: q by a gather launch)")
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    c0 = c   # the load case on the cube's own faces
    if a.rotate:
        import math
        k = torch.tensor([1.0, 1.0, 2.0], dtype=torch.float64, device=dev)
        k = k / k.norm()
        th = math.radians(a.rotate)
        K = torch.tensor([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]], dtype=torch.float64, device=dev)
        Rm = torch.eye(3, dtype=torch.float64, device=dev) + math.sin(th) * K + (1 - math.cos(th)) * (K @ K)
        c = (c @ Rm.T).contiguous()
    N = c.shape[0]
    Ek = E if a.kind == "elastic" else 1.0
    out = {"n": a.n, "kind": a.kind, "tets": t.shape[0], "nodes": N, "rotate_deg": a.rotate}
    for _ in range(2):
        ms, A = ev(lambda: system.MatFreeOperator(c, t, a.kind, Ek, NU))
    out["mf_build_ms"] = ms
    out["mf_info"] = A.info()
    x = torch.randn(A.n, dtype=torch.float64, device=dev)
    y = A.matvec(x)
    ms, _ = ev(lambda: A.matvec(x, y), reps=20)
    out["mf_apply_ms"] = ms
    if not a.no_assembled:
        ms, As = ev(lambda: system.assemble_tet4_system(c, t, a.kind, Ek, NU))
        out["asm_ms"] = ms
        ys = As.matvec(x)
        out["rel_vs_assembled"] = float((y - ys).abs().max() / ys.abs().max())
        out["max_abs"] = [float(y.abs().max()), float(ys.abs().max()), float((y - ys).abs().max())]
        out["bitwise_equal_frac"] = float((y == ys).double().mean())
        ms, _ = ev(lambda: As.matvec(x, ys), reps=20)
        out["sell_spmv_ms"] = ms
        del As
    f, fixed = mesh.cube_elasticity_case(c0) if a.kind == "elastic" else mesh.cube_poisson_case(c0)
    dpn = A.bs
    mask = torch.zeros((N, dpn), dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask.view(-1))
    run = system.PcgRunner(A, f.reshape(-1), w, tol=0.0)
    if a.tune_extra:
        run.set_tuning(C.TUNE_DEFAULT | a.tune_extra)
    run.start()
    run.profile(5, every=1)
    ms, n = run.profile(a.iters, every=1)
    out["k1_ms"] = ms[0] / n[0]
    out["update_ms"] = ms[1] / n[1]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.iterate(a.iters)
    run.poll()
    dt = (time.perf_counter() - t0) / a.iters
    out["iter_ms"] = dt * 1e3
    out["it_per_s"] = 1.0 / dt
    if a.graph:
        run.use_graph(a.graph)
        run.iterate(a.graph)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.iterate(a.iters)
        run.poll()
        dt = (time.perf_counter() - t0) / a.iters
        out["graph_iter_ms"] = dt * 1e3
        out["graph_it_per_s"] = 1.0 / dt
    run.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
