#!/usr/bin/env python3
"""Assembly of stored element matrices (fem_assemble_from_ke) on the configs[4] families, for rocprofv3 passes:
python tools/ke_assemble_probe.py [--family c3d10] [--n 48] [--reps 3]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import element, mesh, system  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="c3d10")
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[a.family]
    c, el = gen(a.n, jitter=0.1, device=dev)
    K = element.compute_K_matrix(c, el, a.family, 113.8e9, 0.342, device=dev, dtype=torch.float64)
    g = system.build_graph(el, c.shape[0])
    for _ in range(a.reps):
        A = system.SellMatrix(g, 3).add_element_matrices(K, el)
        torch.cuda.synchronize()
        del A
    print("Ke bytes", K.numel() * 8, "sell blocks", g.sell_entries, "nnz blocks", g.nnz, "rows", g.n_nodes)


if __name__ == "__main__":
    main()
