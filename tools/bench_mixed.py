#!/usr/bin/env python3
"""BASELINE configs[4]: "2M-element P2 tet + hex/wedge mixed mesh, mass+stiffness assembly, 1 x MI355X".

Three separate boxes (P2/linear faces are nonconforming): c3d8 88^3 = 681,472 hexes, c3d6 2*70^3 =
686,000 wedges, c3d10 6*48^3 = 663,552 quadratic tets (jittered). Per family: element stiffness through the
reference API (compute_K_matrix, default rule, single=True) timed with events, then the global assembly (pattern +
row-gather) of those matrices, then the consistent mass (compute_M_matrix: no reference function, parity unpinned)
and its global assembly on the same pattern; plus the c3d4 consistent mass of the 10M cube (compute_c3d4_M_matrix,
the only mass the reference's notebook calls). Output bytes per family give the write bandwidth; the oracle (reference op sequence on
torch-CPU) element stiffness on a bounded sample gives the CPU baseline.

    python tools/bench_mixed.py [--cpu-sample 20000]
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, element, mesh, system  # noqa: E402

E, NU, RHO = 113.8e9, 0.342, 4.47e-3
F64 = torch.float64
FAMILIES = (("c3d8", mesh.hex_box, 88), ("c3d6", mesh.wedge_box, 70), ("c3d10", mesh.tet10_cube, 48))


def ev_ms(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-sample", type=int, default=20000)
    a = ap.parse_args()
    C.lib()
    dev = torch.device("cuda", 0)
    out = {"config": "BASELINE configs[4]: c3d8 88^3 + c3d6 2*70^3 + c3d10 6*48^3 (2,031,024 elements), fp64"}
    total_el = 0
    for et, gen, n in FAMILIES:
        c, el = gen(n, jitter=0.1, device=dev)
        total_el += el.shape[0]
        # one untimed pass of the whole family (module load, allocator pools), then the best of three timed passes
        reps = []
        for _ in range(4):
            ms_k, K = ev_ms(lambda: element.compute_K_matrix(c, el, et, E, NU, device=dev, dtype=F64))
            ms_g, g = ev_ms(lambda: system.build_graph(el, c.shape[0]))
            ms_a, A = ev_ms(lambda: system.SellMatrix(g, 3).add_element_matrices(K, el))
            del K
            ms_m, Me = ev_ms(lambda: element.compute_M_matrix(c, el, et, RHO, device=dev, dtype=F64))
            ms_ma, Am = ev_ms(lambda: system.SellMatrix(g, 3).add_element_matrices(Me, el))
            reps.append((ms_k, ms_g, ms_a, ms_m, ms_ma))
            if len(reps) < 4:
                del Me, A, Am, g
        ms_k, ms_g, ms_a, ms_m, ms_ma = (min(r[i] for r in reps[1:]) for i in range(5))
        del Me, A, Am, g
        # the family's whole job as one timed region (host clock, device idle at both ends): K_e and M_e enqueued
        # on the current stream, the pattern (node graph, SELL layout) built meanwhile on a second stream -- its
        # latency-bound kernels overlap the write-bound element kernels -- then both global assemblies
        # (the pattern build and the element kernels each read a few sizes back to the host, so the pattern runs in a
        # second host thread -- ctypes calls release the GIL -- on its own stream)
        side = torch.cuda.Stream(device=dev)
        pipe = []

        def pattern(box):
            torch.cuda.set_device(dev)
            with torch.cuda.stream(side):
                box.append(system.build_graph(el, c.shape[0]))
        for _ in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            box = []
            th = threading.Thread(target=pattern, args=(box,))
            th.start()
            K = element.compute_K_matrix(c, el, et, E, NU, device=dev, dtype=F64)
            Me = element.compute_M_matrix(c, el, et, RHO, device=dev, dtype=F64)
            th.join()
            g = box[0]
            torch.cuda.current_stream(dev).wait_stream(side)
            A = system.SellMatrix(g, 3).add_element_matrices(K, el)
            Am = system.SellMatrix(g, 3).add_element_matrices(Me, el)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) * 1e3)
            del K, A
            if len(pipe) < 4:
                del Me, Am, g
        out[et] = {"elements": int(el.shape[0]), "nodes": int(c.shape[0]), "Ke_ms": ms_k,
                   "Ke_write_GBps": Me.numel() * 8 / (ms_k * 1e-3) / 1e9, "pattern_ms": ms_g, "assemble_ms": ms_a,
                   "Me_ms": ms_m, "Me_write_GBps": Me.numel() * 8 / (ms_m * 1e-3) / 1e9, "mass_assemble_ms": ms_ma,
                   "total_mass": float(Am.vals.sum()) / 3, "nnz_blocks": g.nnz,
                   "serial_sum_ms": ms_k + ms_g + ms_a + ms_m + ms_ma, "pipelined_ms": min(pipe[1:]),
                   "pipelined_passes_ms": [round(v, 3) for v in pipe]}
        del Me, Am, g
        torch.cuda.empty_cache()
        print(json.dumps(out), flush=True)
    c, t = mesh.kuhn_cube(119, device=dev)
    element.compute_c3d4_M_matrix(c, t[:64], RHO, device=dev, dtype=F64)
    ms_m = []
    for _ in range(3):
        m, Mm = ev_ms(lambda: element.compute_c3d4_M_matrix(c, t, RHO, device=dev, dtype=F64))
        ms_m.append(m)
        del Mm
    ms_m = min(ms_m)
    out["c3d4_mass_10M"] = {"elements": int(t.shape[0]), "ms": ms_m, "write_GBps": t.shape[0] * 144 * 8 / (ms_m * 1e-3) / 1e9}
    out["elements_total"] = total_el
    out["set_serial_ms"] = sum(out[et]["serial_sum_ms"] for et, _, _ in FAMILIES)
    out["set_pipelined_ms"] = sum(out[et]["pipelined_ms"] for et, _, _ in FAMILIES)
    print(json.dumps(out), flush=True)

    if a.cpu_sample <= 0:   # profiling passes: GPU work only
        return
    from oracle import ref_cpu as R
    cpu = {}
    for et, gen, n in FAMILIES:
        cc, ce = gen(n, jitter=0.1)
        ce = ce[: a.cpu_sample]
        t0 = time.perf_counter()
        R.iso_K(cc, ce, et, E, NU)
        cpu[et] = ce.shape[0] / (time.perf_counter() - t0)
    out["cpu_baseline"] = {"value": cpu, "unit": "element stiffness matrices/s", "cores": torch.get_num_threads(),
                           "kind": "port", "sample": f"oracle iso_K on the first {a.cpu_sample} elements per family"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
