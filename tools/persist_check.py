#!/usr/bin/env python3
"""Persistent PCG (schedule 3) against the deferred schedule (2) on the GPU box: solve-to-tolerance parity (iteration
count, status, x) and fixed-iteration throughput on Kuhn-cube Poisson meshes.

    python tools/persist_check.py [--n 20 119] [--iters 500] [--chunk 500]
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
from fem355 import _capi as C, mesh, system  # noqa: E402


def case(n, dev):
    coords, tets = mesh.kuhn_cube(n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    f, fixed = mesh.cube_poisson_case(coords)
    mask = torch.zeros((coords.shape[0], 1), dtype=torch.uint8, device=dev)
    mask[fixed] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1).to(torch.float64).contiguous()
    return A, b, w


def rate(A, b, w, sched, warm, iters, chunk, tune=None):
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
    if tune is not None:
        run.set_tuning(tune)
    run.start()
    eff = run.effective_schedule()
    uni = run.uniform_slices()[:2]
    run.iterate(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    while done < iters:
        k = min(chunk, iters - done)
        run.iterate(k)
        done += k
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    it, stt, rz = run.poll()
    x = run.x.clone()
    run.close()
    return {"sched": eff, "uniform_slices": list(uni), "it_per_s": iters / dt, "us_per_it": dt / iters * 1e6, "iter": it, "status": stt,
            "rz": rz}, x


PHASES = ("u_wait", "spmv", "block_sum", "barrier_sums", "step", "update_flag", "prologue_per_launch",
          "epilogue_per_launch")


def phase_profile(A, b, w, warm, iters, ghz=2.4, per_wg=False, tune=None, sched=3):
    """Per-iteration phase times (us at `ghz` shader clock) of the instrumented persistent kernel (schedule 3 or the
    a variant): mean and max over workgroups."""
    import ctypes
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
    if tune is not None:
        run.set_tuning(tune)
    run.start()
    assert run.effective_schedule() == sched
    names = PHASES
    run.iterate(warm)
    G = 256
    buf = (ctypes.c_ulonglong * (G * (len(PHASES) + 16)))()
    g = ctypes.c_int()
    C.check(run.lib.fem_pcg_persist_profile(run.h, int(iters), buf, ctypes.byref(g)), "fem_pcg_persist_profile")
    run.close()
    allv = torch.tensor(list(buf), dtype=torch.float64) / (ghz * 1e3)
    t = allv[: G * len(PHASES)].view(G, len(PHASES))[: g.value].clone()
    tw = allv[G * len(PHASES):].view(G, 16)[: g.value] / iters   # per-wave own SpMV, us per iteration
    t[:, :6] /= iters   # per iteration; prologue / epilogue stay per launch
    out = {p: {"mean_us": float(t[:, i].mean()), "max_us": float(t[:, i].max()), "min_us": float(t[:, i].min())}
           for i, p in enumerate(names)} | {"total_mean_us": float(t[:, :6].sum(1).mean())}
    busy = tw > 0
    out["wave_spmv_us"] = {"mean_busy": float(tw[busy].mean()) if busy.any() else 0.0, "max": float(tw.max()),
                           "min_busy": float(tw[busy].min()) if busy.any() else 0.0,
                           "wg_max_mean": float(tw.max(1).values.mean()), "wg_max_max": float(tw.max(1).values.max())}
    if per_wg:   # packed assignment: WG L owns [L S / G, (L+1) S / G), its waves ceil(maxL / 16) slices each in order
        G = g.value
        sp = A.g.slice_ptr.cpu()
        S = sp.numel() - 1
        pack = (-(-S // G) + 15) // 16
        ent, went = [], []
        for L in range(G):
            a0, a1 = L * S // G, (L + 1) * S // G
            ent.append(int(sp[a1] - sp[a0]))
            for wv in range(16):
                lo = min(a0 + wv * pack, a1)
                hi = min(lo + pack, a1)
                went.append(int(sp[hi] - sp[lo]))
        out["per_wg"] = {"spmv_us": [round(float(v), 3) for v in t[:, 1]], "entries": ent,
                         "wave_spmv_us": [round(float(v), 3) for v in tw.reshape(-1)], "wave_entries": went}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[20, 119])
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--warm", type=int, default=50)
    ap.add_argument("--chunk", type=int, default=500)
    ap.add_argument("--prof", action="store_true", help="phase breakdown of the instrumented persistent kernel")
    ap.add_argument("--skip-solve", action="store_true")
    ap.add_argument("--tune", type=int, nargs="*", default=[], help="extra FEM_TUNE_* flag sets for schedule 3")
    ap.add_argument("--per-wg", action="store_true", help="with --prof: SpMV time and matrix entries per workgroup")
    ap.add_argument("--scheds", type=int, nargs="+", default=[2, 3], help="schedules to solve / rate")
    ap.add_argument("--prof-scheds", type=int, nargs="+", default=[3], help="schedules to phase-profile (3, 4)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for n in a.n:
        A, b, w = case(n, dev)
        out = {"n": n, "rows": A.n}
        tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
        if a.prof:
            for ps in a.prof_scheds:
                out["prof" if ps == 3 else f"prof{ps}"] = phase_profile(A, b, w, a.warm, a.iters, per_wg=a.per_wg,
                                                                         sched=ps)
        sol = {}
        for sched in (() if a.skip_solve else a.scheds):
            t0 = time.perf_counter()
            r = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64, schedule=sched)
            torch.cuda.synchronize()
            out[f"solve{sched}"] = {"iters": r.iterations, "status": r.status, "rz": r.rz,
                                    "ms": (time.perf_counter() - t0) * 1e3}
            sol[sched] = r.x
        s0 = a.scheds[0]
        for sched in sol:
            if sched != s0:
                out[f"solve_dx_rel_{sched}"] = float((sol[s0] - sol[sched]).norm() / sol[s0].norm())
        if a.prof:
            print(json.dumps({"n": n, "prof_only": out.get("prof")}), flush=True)
        xs = {}
        for sched in a.scheds:
            try:
                out[f"rate{sched}"], xs[sched] = rate(A, b, w, sched, a.warm, a.iters, a.chunk)
            except RuntimeError as e:   # timing probes with wrong scalars may end in a give-up
                out[f"rate{sched}"] = {"error": str(e)}
        for sched in xs:
            if sched != s0:
                out[f"rate_dx_rel_{sched}"] = float((xs[s0] - xs[sched]).norm() / xs[s0].norm())
        for t in a.tune:   # extra tuning-flag sets of the persistent schedule (FEM_TUNE_*), x compared bitwise
            out[f"rate3_t{t}"], xt = rate(A, b, w, 3, a.warm, a.iters, a.chunk, tune=t)
            out[f"rate3_t{t}"]["x_equal"] = bool(torch.equal(xt, xs[3]))
            out[f"rate3_t{t}"]["dx_rel"] = float((xt - xs[3]).norm() / xs[3].norm())
            if a.prof:
                out[f"prof_t{t}"] = phase_profile(A, b, w, a.warm, a.iters, tune=t)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
