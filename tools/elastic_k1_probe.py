"""Elastic 10M K1 (k_pcg_spmv_dot) spread between runs: the same matrix and code measured 310-370 us per SpMV on
different boxes / allocation histories. This probe re-creates the solver context (a fresh hipMalloc of its 1.85 GB
plane-paired matrix copy) several times in one process, with and without spacer allocations in between, and
prints K1 / update / pupdate per trial, to separate placement effects from box effects.

    python tools/elastic_k1_probe.py [--n 119] [--trials 6] [--iters 40]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fem355 import _capi as C, mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C.lib()
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    f, fixed = mesh.cube_elasticity_case(coords)
    A = system.assemble_tet4_system(coords, tets, "elastic", 113.8e9, 0.342)
    mask = torch.zeros((coords.shape[0], 3), dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1).to(torch.float64).contiguous()
    torch.cuda.synchronize()
    res = []
    spacers = []
    for t in range(a.trials):
        # odd trials: leave a spacer allocation behind before the next context (shifts where its copy lands)
        run = system.PcgRunner(A, b, w, tol=0.0)
        run.start()
        run.iterate(5)
        ms, cnt = run.profile(a.iters, every=1)
        k1 = [m / max(c, 1) * 1e3 for m, c in zip(ms, cnt)]
        ms2, cnt2 = run.profile(a.iters, every=1)
        k1b = [m / max(c, 1) * 1e3 for m, c in zip(ms2, cnt2)]
        run.close()
        rec = {"trial": t, "spacer_MB": sum(s.numel() * 8 for s in spacers) >> 20,
               "k1_us": round(k1[0], 1), "update_us": round(k1[1], 1), "pupdate_us": round(k1[2], 1),
               "k1_us_again": round(k1b[0], 1)}
        print(json.dumps(rec), flush=True)
        res.append(rec)
        if t % 2 == 0:
            spacers.append(torch.empty((97 + 31 * t) << 17, dtype=torch.float64, device=dev))
        torch.cuda.synchronize()
    print(json.dumps({"probe": "elastic_k1", "n": a.n, "trials": res}))


if __name__ == "__main__":
    main()
