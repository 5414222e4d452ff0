#!/usr/bin/env python3
"""configs[4] scalar-mass and stiffness tile assemblies alone (GPU box): per family the median of --reps launches of
`SellMatrix(g, 1).add_element_matrices(Me, el)` and of the bs = 3 `add_element_matrices(K, el)` on fresh matrices,
hip events on the library's stream, plus a checksum of the mass values (the A/B builds must give the same bits).

    [FEM355_LIB=...] python tools/mass_tile_probe.py [--reps 7]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import element, mesh, system  # noqa: E402

FAMILIES = [("c3d8", "hex_box", 88), ("c3d6", "wedge_box", 70), ("c3d10", "tet10_cube", 48)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    for et, gen, n in FAMILIES:
        c, el = getattr(mesh, gen)(n, jitter=0.1, device=dev)
        K = element.compute_K_matrix(c, el, et, 113.8e9, 0.342, device=dev, dtype=torch.float64)
        Me = element.compute_M_matrix(c, el, et, 7850.0, device=dev, dtype=torch.float64, scalar=True)
        g = system.build_graph(el, c.shape[0])
        res = {}
        for name, bs, mat in (("mass", 1, Me), ("stiffness", 3, K)):
            ts, last = [], None
            for _ in range(a.reps):
                A = system.SellMatrix(g, bs)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                A.add_element_matrices(mat, el)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
                last = A
            v = last.plain_values()
            res[name] = {"ms_median": sorted(ts)[len(ts) // 2], "ms_min": min(ts),
                         "bits_sum": int(v.view(torch.int64).sum().item())}
        out[et] = res
        del K, Me, g
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
