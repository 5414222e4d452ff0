#!/usr/bin/env python3
"""Distributed persistent PCG on ONE GPU (emulated ranks, dist_persist.EmulatedGroup): solve / fixed-iteration
parity against the single-GPU persistent schedule and per-iteration time, for a list of rank counts.

    python tools/dist_persist_check.py [--n 24] [--ranks 1 2 4] [--iters 1 5 50] [--rtol 1e-9] [--gv]

--gv: the pipelined build (FEM_TUNE_PK_GV) for the ranks and the single-GPU reference alike.
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
from fem355 import _capi as C, dist_persist as DP, mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--iters", type=int, nargs="+", default=[1, 5, 50])
    ap.add_argument("--rtol", type=float, default=1e-9)
    ap.add_argument("--time-iters", type=int, default=0)
    ap.add_argument("--prof", action="store_true")
    ap.add_argument("--gv", action="store_true")
    a = ap.parse_args()
    tune = (C.TUNE_DEFAULT | C.TUNE_PK_GV) if a.gv else None
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    f, fixed = mesh.cube_poisson_case(c)
    b = f.reshape(-1).to(torch.float64)
    mask = torch.zeros(c.shape[0], dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    A = system.assemble_tet4_system(c, t, "poisson")
    w = A.jacobi(mask)
    ref = {}
    for k in a.iters:
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=3, tune=tune)
        run.start()
        run.iterate(k)
        ref[k] = (run.poll(), run.x.clone())
        run.close()
    tol = a.rtol * float(torch.sqrt(torch.dot(b, w * b)))
    r3 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=3, tune=tune)
    out = {"n": a.n, "rows": A.n, "gv": a.gv, "single": {"solve_iters": r3.iterations, "status": r3.status}}
    for P in a.ranks:
        res = {}
        for k in a.iters:
            grp = DP.EmulatedGroup(c, t, P, b, fixed_mask=mask, tol=0.0, gv=a.gv)
            grp.start()
            t0 = time.perf_counter()
            grp.iterate(k)
            dt = time.perf_counter() - t0
            polls = [rr.poll() for rr in grp.ranks]
            if any(p[1] == C.PCG_SYNC_TIMEOUT for p in polls):   # diagnostics of a failed hand-off
                G = grp.ranks[0].debug(0, 1)  # noqa
                for r, rr in enumerate(grp.ranks):
                    import ctypes as _ct
                    g = (len(rr.debug(2, 1 << 16)) and None)
                    Gr = int(rr.lib.fem_pcg_get_schedule(rr.h)) and None
                    nG = 256 // P // 8 * 8
                    win = rr.debug(0, 2 * nG + 2)
                    flags = rr.debug(1, P * nG)
                    pub = rr.debug(2, nG * P * 2)
                    print(json.dumps({"rank": r, "G": nG, "win_lo": win[:nG], "win_hi": win[nG:2 * nG],
                                      "colwin": win[2 * nG:], "flags": flags, "pub": pub,
                                      "rflags": rr.debug(3, P), "sync": rr.debug(4, 18)}), flush=True)
            x = grp.x()
            res[f"k{k}"] = {"polls": polls, "ref_poll": ref[k][0],
                            "x_rel": float((x - ref[k][1]).abs().max() / ref[k][1].abs().max().clamp_min(1e-300)),
                            "wall_ms": dt * 1e3}
            grp.close()
        grp = DP.EmulatedGroup(c, t, P, b, fixed_mask=mask, tol=tol, gv=a.gv)
        it, stt = grp.solve(max_iter=20000, chunk=512)
        x = grp.x()
        res["solve"] = {"iters": it, "status": stt,
                        "x_rel": float((x - r3.x).abs().max() / r3.x.abs().max())}
        grp.close()
        if a.time_iters:
            grp = DP.EmulatedGroup(c, t, P, b, fixed_mask=mask, tol=0.0, gv=a.gv)
            grp.start()
            grp.iterate(5)
            t0 = time.perf_counter()
            grp.iterate(a.time_iters)
            res["us_per_it"] = (time.perf_counter() - t0) / a.time_iters * 1e6
            if a.prof:   # phase clocks of the distributed kernel (PROF build), per rank: mean / max over workgroups
                G = 256 // P // 8 * 8
                bufs = []
                for rr in grp.ranks:
                    buf = torch.zeros(G * 24, dtype=torch.int64, device=dev)
                    rr.set_prof(buf)
                    bufs.append(buf)
                grp.iterate(a.time_iters)
                phases = ("u_wait", "spmv", "block_sum", "barrier_ranksum", "step", "update_flag", "prologue",
                          "epilogue")
                prof = []
                for buf in bufs:
                    v = buf.cpu().to(torch.float64) / 2.4e3
                    ph = v[: G * 8].view(G, 8)
                    ph[:, :6] /= a.time_iters
                    prof.append({n: [round(float(ph[:, i].mean()), 2), round(float(ph[:, i].max()), 2)]
                                 for i, n in enumerate(phases)})
                res["prof"] = prof
            grp.close()
        out[f"P{P}"] = res
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
