#!/usr/bin/env python3
"""Node-graph pattern build alone (for rocprofv3 passes): python tools/pattern_only.py [--family c3d10] [--reps 3]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, mesh, system  # noqa: E402

GEN = {"c3d4": (mesh.kuhn_cube, 119), "c3d8": (mesh.hex_box, 88), "c3d6": (mesh.wedge_box, 70),
       "c3d10": (mesh.tet10_cube, 48)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="c3d10", choices=sorted(GEN))
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    gen, n = GEN[a.family]
    c, t = gen(n, device=dev)
    out = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g = system.build_graph(t, c.shape[0])
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
        del g
    print(json.dumps({"family": a.family, "nodes": c.shape[0], "elements": t.shape[0], "graph_ms": out}))


if __name__ == "__main__":
    main()
