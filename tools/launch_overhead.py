#!/usr/bin/env python3
"""Fixed cost of a persistent-schedule launch (GPU box): wall and hip-event time of K iterations as one launch,
for several K, on the 10M-tet Poisson bench system -> per-launch overhead (host + kernel prologue/epilogue).

    python tools/launch_overhead.py [--n 119] [--ks 1 2 5 20 100 500] [--reps 5]
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
from fem355 import mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 2, 5, 20, 100, 500])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tune", type=int, default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    f, fixed = mesh.cube_poisson_case(coords)
    mask = torch.zeros(A.n, dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask)
    b = f.reshape(-1).to(torch.float64).contiguous()
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    if a.tune is not None:
        run.set_tuning(a.tune)
    run.start()
    run.iterate(50)
    torch.cuda.synchronize()
    out = {"n": a.n, "rows": A.n, "rows_per_k": {}}
    for k in a.ks:
        walls, evs = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ms, cnt = run.profile(k, every=k)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            evs.append(ms[0] * 1e-3)
        out["rows_per_k"][k] = {"wall_us": min(walls) * 1e6, "event_us": min(evs) * 1e6,
                                "wall_us_per_it": min(walls) / k * 1e6, "event_us_per_it": min(evs) / k * 1e6,
                                "host_us": (min(walls) - min(evs)) * 1e6}
    # plain iterate (no events)
    walls = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.iterate(20)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    out["iterate20_wall_us"] = min(walls) * 1e6
    ks = sorted(out["rows_per_k"])
    k0, k1 = ks[0], ks[-1]
    e0, e1 = out["rows_per_k"][k0]["event_us"], out["rows_per_k"][k1]["event_us"]
    per = (e1 - e0) / (k1 - k0)
    out["fit"] = {"per_iteration_us": per, "per_launch_fixed_us": e0 - per * k0}
    run.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
