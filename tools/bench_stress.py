#!/usr/bin/env python3
"""Stress recovery measurement on the 10M-tet Kuhn cube (n=119) with a smooth displacement.

Kernels timed with hip events on the current stream (median of --reps launches through the C-ABI):
  * k_tet4_stress   : compute_c3d4_element_stress; algorithmic bytes per launch = M (32 conn + 72 tensor + 8 vm)
                      + N (24 coords + 24 u) (each node row once; the 4 gathers per element are L2 / MALL reuse)
  * k_node_average  : compute_node_vm_stress; bytes = 4 (N+1) + 4 * 4M (incidence) + 8 M (vm) + 8 N
  * k_iso_stress<8> : compute_c3d8_element_stress (single) on a hex box of similar node count
Plus the reference-API wall time and the oracle (reference op sequence on torch-CPU) on a bounded sample.

    python tools/bench_stress.py [--n 119] [--reps 20] [--cpu-n 50]
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
from fem355 import _capi as C, element, mesh  # noqa: E402

E, NU = 113.8e9, 0.342
F64 = torch.float64


def med_ms(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu-n", type=int, default=50)
    a = ap.parse_args()
    lib = C.lib()
    dev = torch.device("cuda", 0)
    c, t = mesh.kuhn_cube(a.n, device=dev)
    M, N = t.shape[0], c.shape[0]
    u = torch.stack([torch.sin(3 * c[:, 0]) * c[:, 1], c[:, 2] ** 2, c[:, 0] * c[:, 1] * c[:, 2]], 1) * 1e-4
    u = u.contiguous()
    sig = torch.empty((M, 3, 3), dtype=F64, device=dev)
    vm = torch.empty(M, dtype=F64, device=dev)
    st = C.stream(dev)
    out = {"workload": f"{M:,}-tet c3d4 Kuhn cube n={a.n}, {N:,} nodes, smooth displacement field"}

    def tet():
        C.check(lib.fem_tet4_stress(C.ptr(c), C.ptr(t), M, C.ptr(u), E, NU, C.ptr(sig), C.ptr(vm), None, st), "s")
    tet()
    ms = med_ms(tet, a.reps)
    alg = M * (32 + 72 + 8) + N * 48
    out["k_tet4_stress"] = {"ms": ms, "algorithmic_bytes": alg, "GBps": alg / (ms * 1e-3) / 1e9,
                            "frac_of_8TBps": alg / (ms * 1e-3) / 8e12, "elements_per_s": M / (ms * 1e-3)}
    inc_ptr, inc = element.cached_incidence(t, N)
    nv = torch.empty(N, dtype=F64, device=dev)

    def avg():
        C.check(lib.fem_node_average(C.ptr(vm), 4, C.ptr(inc_ptr), C.ptr(inc), N, C.ptr(nv), st), "avg")
    avg()
    ms = med_ms(avg, a.reps)
    alg = 4 * (N + 1) + 16 * M + 8 * M + 8 * N
    out["k_node_average"] = {"ms": ms, "algorithmic_bytes": alg, "GBps": alg / (ms * 1e-3) / 1e9,
                             "frac_of_8TBps": alg / (ms * 1e-3) / 8e12}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s_api, v_api = element.compute_c3d4_element_stress(c, t, u, E, NU, device=dev, dtype=F64)
    n_api = element.compute_node_vm_stress(c, t, v_api, device=dev, dtype=F64)
    torch.cuda.synchronize()
    out["api_wall_s"] = {"element_stress+node_vm": time.perf_counter() - t0}
    assert torch.equal(s_api, sig) and torch.equal(n_api, nv)
    del sig, s_api

    # c3d8 on a hex box with a similar node count (n^3 hexes)
    hc, he = mesh.hex_box(a.n, device=dev)
    uh = (hc @ torch.tensor([[1.0, 0.2, 0], [0, 1.0, 0.3], [0.1, 0, 1.0]], dtype=F64, device=dev).t() * 1e-4)
    uh = uh.contiguous()
    Mh, Nh = he.shape[0], hc.shape[0]
    p, w = element._points_weights("c3d8", None)
    dN = element._dn_table("c3d8", p, dev)
    w = w.to(dev, F64).contiguous()
    sh = torch.empty((Mh, 3, 3), dtype=F64, device=dev)
    vh = torch.empty(Mh, dtype=F64, device=dev)

    def hexs():
        C.check(lib.fem_iso_stress(C.ptr(hc), C.ptr(he), Mh, 8, C.ptr(uh), E, NU, C.ptr(dN), C.ptr(w), 8, 0,
                                   C.ptr(sh), C.ptr(vh), st), "iso")
    hexs()
    ms = med_ms(hexs, a.reps)
    alg = Mh * (64 + 72 + 8) + Nh * 48
    out["k_iso_stress_c3d8"] = {"elements": Mh, "ms": ms, "algorithmic_bytes": alg, "GBps": alg / (ms * 1e-3) / 1e9,
                                "frac_of_8TBps": alg / (ms * 1e-3) / 8e12, "elements_per_s": Mh / (ms * 1e-3)}
    print(json.dumps(out), flush=True)

    from oracle import ref_cpu as R
    cc, ct = mesh.kuhn_cube(a.cpu_n)
    uc = torch.stack([torch.sin(3 * cc[:, 0]) * cc[:, 1], cc[:, 2] ** 2, cc[:, 0] * cc[:, 1] * cc[:, 2]], 1) * 1e-4
    t0 = time.perf_counter()
    _, vc = R.tet4_stress(cc, ct, uc, E, NU)
    R.node_average(ct, vc, cc.shape[0])
    dt = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": ct.shape[0] / dt, "unit": "elements/s (stress + node average)",
                           "cores": torch.get_num_threads(), "kind": "port",
                           "sample": f"oracle tet4_stress + node_average, {ct.shape[0]:,}-tet cube n={a.cpu_n}"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
