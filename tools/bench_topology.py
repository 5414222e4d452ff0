#!/usr/bin/env python3
"""Mesh topology measurement on the 10M-tet Kuhn cube (n=119): wall time (synchronised) of
identify_tetrahedral_shared_faces, compute_tetrahedral_surface_faces_with_fourth_node, element_to_edge and the
element adjacency CSR through the reference API, faces per second, and the oracle (the reference's torch-CPU op
sequence) on a bounded sample.

    python tools/bench_topology.py [--n 119] [--cpu-n 40]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, element, mesh, topology as T  # noqa: E402


def wall(fn, reps=3):
    ts = []
    out = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--cpu-n", type=int, default=40)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    M = t.shape[0]
    out = {"workload": f"{M:,}-tet Kuhn cube n={a.n} ({4 * M:,} faces, {6 * M:,} edges)"}
    element.identify_tetrahedral_shared_faces(t, device=dev)   # warm (hipCUB kernels, module load)
    s, pairs = wall(lambda: element.identify_tetrahedral_shared_faces(t, device=dev))
    out["shared_faces"] = {"s": s, "pairs": pairs.shape[0], "faces_per_s": 4 * M / s}
    s, (f, _) = wall(lambda: element.compute_tetrahedral_surface_faces_with_fourth_node(t, device=dev))
    out["surface_faces"] = {"s": s, "faces": f.shape[0], "faces_per_s": 4 * M / s}
    s, e = wall(lambda: element.element_to_edge(t, device=dev))
    out["edges"] = {"s": s, "edges": e.shape[1], "edges_per_s": 6 * M / s}
    s, (rp, _) = wall(lambda: element.element_adjacency(t, device=dev))
    out["element_adjacency"] = {"s": s, "nnz": int(rp[-1])}
    print(json.dumps(out), flush=True)

    from oracle import ref_cpu as R
    cc, ct = mesh.kuhn_cube(a.cpu_n)
    t0 = time.perf_counter()
    R.shared_faces(ct, T.TET_SHARED)
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": 4 * ct.shape[0] / dt, "unit": "faces/s (identify_tetrahedral_shared_faces)",
                           "cores": torch.get_num_threads(), "kind": "port",
                           "sample": f"oracle shared_faces, {ct.shape[0]:,}-tet cube n={a.cpu_n}"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
