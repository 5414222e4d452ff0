#!/usr/bin/env python3
"""VTK reader measurement: write the 10M-tet Kuhn cube (n=119) as a BINARY legacy VTK 4.2
file and an ASCII one of a smaller cube, then time the native reader (host parse) and vtk_loader_to_torch onto
the GPU. pyvista (the reference's reader) is not installed: no reference timing exists here.

    python tools/bench_vtk.py [--n 119] [--ascii-n 40] [--dir /tmp]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import element, mesh  # noqa: E402


def write_binary(path, c, t):
    M = t.shape[0]
    with open(path, "wb") as f:
        f.write(b"# vtk DataFile Version 4.2\nfem355 bench\nBINARY\nDATASET UNSTRUCTURED_GRID\n")
        f.write(f"POINTS {c.shape[0]} double\n".encode())
        f.write(c.numpy().astype(">f8").tobytes())
        f.write(f"\nCELLS {M} {5 * M}\n".encode())
        cells = np.concatenate([np.full((M, 1), 4, dtype=np.int64), t.numpy()], 1).astype(">i4")
        f.write(cells.tobytes())
        f.write(f"\nCELL_TYPES {M}\n".encode())
        f.write(np.full(M, 10, dtype=">i4").tobytes())
        f.write(b"\n")


def write_ascii(path, c, t):
    M = t.shape[0]
    with open(path, "w") as f:
        f.write("# vtk DataFile Version 4.2\nfem355 bench\nASCII\nDATASET UNSTRUCTURED_GRID\n")
        f.write(f"POINTS {c.shape[0]} double\n")
        np.savetxt(f, c.numpy(), fmt="%.17g")
        f.write(f"CELLS {M} {5 * M}\n")
        np.savetxt(f, np.concatenate([np.full((M, 1), 4), t.numpy()], 1), fmt="%d")
        f.write(f"CELL_TYPES {M}\n")
        np.savetxt(f, np.full(M, 10), fmt="%d")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--ascii-n", type=int, default=40)
    ap.add_argument("--dir", default="/tmp")
    a = ap.parse_args()
    out = {}
    for kind, n, writer in (("binary", a.n, write_binary), ("ascii", a.ascii_n, write_ascii)):
        c, t = mesh.kuhn_cube(n)
        path = os.path.join(a.dir, f"fem355_bench_{kind}_{n}.vtk")
        writer(path, c, t)
        size = os.path.getsize(path)
        t0 = time.perf_counter()
        pts, cells, _ = element.read_vtk(path)
        t_parse = time.perf_counter() - t0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p, e = element.vtk_loader_to_torch(path, "c3d4", device="cuda:0", dtype=torch.float64)
        torch.cuda.synchronize()
        t_load = time.perf_counter() - t0
        assert torch.equal(e.cpu(), t) and torch.equal(p.cpu(), c)
        out[kind] = {"tets": t.shape[0], "file_MB": size / 1e6, "parse_s": t_parse, "parse_MBps": size / 1e6 / t_parse,
                     "loader_to_gpu_s": t_load}
        os.remove(path)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
