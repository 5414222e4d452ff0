#!/usr/bin/env python3
"""fem355 benchmark: BASELINE.json metric "CG iterations/sec + DOFs/sec (assembly+solve), 10M P1-tet Poisson".

Workload: Kuhn-cube mesh n=119 -> 10,110,954 P1 tets, 1,728,000 nodes/DOFs, scalar Poisson
(kappa=1), z=0 face Dirichlet, unit nodal source; fp64 values, SELL-64 global matrix with 16-bit column deltas
(int32 columns when a delta does not fit).
  * a "step" = one Jacobi-PCG iteration (SpMV + 2 dots + vector updates) on that system, tol=0 (no early exit);
    `value` = steps/s of the whole job (for N>1: the same global system element-partitioned over the ranks,
    strong scaling), measured between barrier+synchronize brackets, max over ranks.
  * DOFs/s = n_DOF / (assembly incl. pattern build + PCG solve to rtol 1e-8 on sqrt(r.z)), reported beside:
    steady state (`dofs_per_s`: the median by total of --dof-passes identical passes after the first, all listed in
    `dofs_passes_ms`; `dofs_per_s_split_medians`: median assembly + median solve) and first use (`dofs_per_s_cold`, which also pays the device allocations of this mesh size).
  * roofline: the dominant kernel of the active schedule, algorithmic bytes (8 + idx) nnz + 4 (n+1) + 16 n
    (§8(d); idx = 2 for 16-bit deltas, 4 for int32) over its device time measured live with hip events on the
    solver stream inside the timed region. bs=1 default (persistent schedule, k_pcg_persist): per ITERATION —
    the whole PCG iteration moves just those bytes (matrix, u gather, u store); other schedules: per SpMV launch
    (k_pcg_d1 deferred, k_pcg_spmv_dot three-kernel).
  * cpu_baseline: the oracle (torch-CPU restatement of the reference's EBE PCG, oracle/ref_cpu.py) timed on the
    host cores on a bounded sample of the same 10M system (element assembly, EBE matvec, 50 fixed PCG iterations:
    BASELINE.md §3), rank 0 at N=1 only. Measured ratio: the CPU's assembly + 50 iterations against the GPU's
    assembly + 50 timed iterations; the whole-solve wall is projected from the CPU iteration rate (labelled so).

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import fem355  # noqa: E402
from fem355 import _capi as C, mesh, system  # noqa: E402

METRIC = "CG iterations/sec + DOFs/sec (assembly+solve), 10M P1-tet Poisson, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--n", "--cube-n", dest="n", type=int, default=119,
                    help="Kuhn cube size (119 -> 10.1M tets); --cube-n under torch.distributed.run (--n is ambiguous there)")
    ap.add_argument("--kind", default="poisson", choices=["poisson", "elastic"])
    ap.add_argument("--sample-every", type=int, default=10, help="event-sample every k-th step")
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--dof-passes", type=int, default=3,
                    help="steady-state assembly + solve passes after the cold one; DOFs/s is the median pass")
    ap.add_argument("--cpu-iters", type=int, default=50,
                    help="CPU-baseline PCG iterations (Poisson; BASELINE.md §3: a fixed 50)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--elastic", type=int, default=1,
                    help="poisson runs: also measure the 10M-tet linear-elasticity system (BASELINE configs[2]/[3]) "
                         "with the same steps, reported under \"elasticity\" in the same JSON line")
    ap.add_argument("--mf-graph", type=int, default=0,
                    help="matrix-free companion: time hipGraph replays (1; measured equal to plain launches: the "
                         "~11 us between the two kernels of an iteration is device-side) or plain launches (0)")
    ap.add_argument("--matfree", type=int, default=1,
                    help="elasticity companion: also the element-chunk (matrix-free) operator, under \"matfree\"")
    ap.add_argument("--elastic-timeout", type=float, default=240.0,
                    help="seconds the elasticity companion may take before the line is printed without it")
    ap.add_argument("--cpu-iters-elastic", type=int, default=50, help="CPU-baseline PCG iterations (elasticity)")
    ap.add_argument("--reference-api", type=int, default=1,
                    help="elasticity companion: also the time to solution through the reference's own hand-off "
                         "(compute_c3d4_K_matrix -> compute_diagonal_preconditioner -> "
                         "preconditioned_conjugate_gradient_solver), under \"reference_api\"")
    ap.add_argument("--mixed", type=int, default=1,
                    help="poisson runs: also BASELINE configs[4] (2M-element c3d8 / c3d6 / c3d10 stiffness + mass "
                         "assembly) under \"mixed\"")
    ap.add_argument("--mixed-ke", default="full", choices=["full", "packed"],
                    help="configs[4] stiffness: the full [M, d, d] K_e of compute_K_matrix, or its packed symmetric "
                         "form (upper blocks; fem_iso_ke_sym + fem_assemble_from_ke_sym)")
    ap.add_argument("--mixed-km", default="split", choices=["fused", "split"],
                    help="configs[4] global assemblies: two separate calls, or stiffness and mass in one pass "
                         "(fem_assemble_from_ke_mass_sl, bit-identical; measured no faster: DESIGN §8i)")
    ap.add_argument("--schedule", type=int, default=None, help="PCG kernel schedule (0 three-kernel, 1 fused, 2 deferred, 3 persistent; "
                    "default: persistent for bs=1, three-kernel for bs=3)")
    ap.add_argument("--graph", type=int, default=0, help="capture k iterations per hipGraph (0 = plain launches)")
    ap.add_argument("--permute", type=int, default=0,
                    help="seed > 0: randomly renumber the cube's nodes first (a mesh in file order, untimed)")
    ap.add_argument("--reorder", default="none", choices=["none", "rcm"],
                    help="rcm: renumber the nodes by device reverse Cuthill-McKee inside every assembly pass "
                         "(timed with it; reported as reorder_ms)")
    ap.add_argument("--config1", type=int, default=1,
                    help="1: also measure BASELINE configs[1] (1M-tet Poisson) on the single-reduction and the "
                         "pipelined persistent kernels, reported under \"config1\"")
    ap.add_argument("--pipelined", type=int, default=0,
                    help="1: the pipelined (Ghysels-Vanroose) persistent iteration for bs = 1 systems of <= 2 slices "
                         "per wave (FEM_TUNE_PK_GV; the 1M cube, a rank share of the 10M one); ignored elsewhere")
    ap.add_argument("--force-dist", action="store_true", help="run the RCCL element-partitioned path even at N=1")
    ap.add_argument("--dist-variant", type=int, default=1,
                    help="N>1: 1 = single-reduction PCG (one all-reduce per iteration), 0 = two reductions")
    ap.add_argument("--dist-exchange", default="p2p", choices=["p2p", "allreduce"],
                    help="N>1 single-reduction exchange: grouped ncclSend/Recv with every other rank + fixed-order sum "
                         "(p2p), or one all-reduce over the global interface vector")
    ap.add_argument("--dist-fused", type=int, default=0,
                    help="N>1 single reduction: 1 = one launch per iteration (k_cg1_fused), 0 = update + SpMV kernels")
    ap.add_argument("--dist-path", default="auto", choices=["auto", "persist", "rccl"],
                    help="N>1: the persistent multi-GPU schedule (rows partitioned, in-kernel hand-offs over xGMI; "
                         "Poisson; auto falls back to RCCL if its self-check fails) or the RCCL element partition")
    ap.add_argument("--dist-graph", type=int, default=50,
                    help="distributed path: capture k iterations (kernels + RCCL) per hipGraph, 0 = plain launches")
    return ap.parse_args()


def sync():
    torch.cuda.synchronize()


def traffic_from_profiles(workload_key, kernel, alg):
    """HBM bytes per launch of `kernel` from the committed PMC summary (tools/pmc_traffic.py), or None when the
    summary was taken on another kernel / matrix format."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path)).get(workload_key, {})
    except Exception:
        return None
    if d.get("kernel") != kernel or d.get("algorithmic_bytes") != alg:
        return None
    return d.get("bytes_per_launch")


def traffic_source(workload_key):
    """Where `traffic` comes from: a PMC run of this bench command (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate
    passes, tools/pmc_traffic.py), committed under profiles/ -- not counted live in this run (no in-process PMC)."""
    try:
        src = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json"))).get(workload_key, {}).get("source")
    except Exception:
        src = None
    return f"profiles/pmc_traffic.json[{workload_key}] <- {src} (committed rocprofv3 PMC passes, not this run)" \
        if src else None


def cpu_model():
    """The host CPU's model name (report it beside the core count)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def s8d_models(n, nnz, spmv_ms, iter_ms, persist):
    """SURVEY §8(d) byte models for n rows / nnz scalar nonzeros: B_spmv over the SpMV launch (persistent schedule:
    the whole iteration, which contains it) and B_iter over the whole iteration, each as a fraction of 8 TB/s."""
    b_spmv = 12 * nnz + 4 * (n + 1) + 16 * n
    b_iter = b_spmv + 88 * n
    return {"B_spmv": b_spmv, "B_iter": b_iter, "iteration_ms": iter_ms,
            "spmv_ms": spmv_ms, "spmv_time_is": "whole iteration" if persist else "SpMV launch",
            "frac_spmv": b_spmv / (spmv_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "frac_iter": b_iter / (iter_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}


def cpu_threads():
    """Host threads for the CPU baseline and what they are based on (torch.set_num_threads with the
    core count stated). The affinity mask sizes it; a thread cap in the environment (OMP_NUM_THREADS: the GPU box
    sets 16, its CPU share, while the mask and os.cpu_count() show the whole machine) bounds it."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(aff, int(cap)) if cap.isdigit() and int(cap) > 0 else aff
    quota = None
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            quota = int(q[0]) / int(q[1])
    except (OSError, ValueError, IndexError):
        pass
    if quota:   # a CPU quota below the mask (a container's share of the host) bounds it as well
        threads = max(1, min(threads, int(quota + 0.999)))
    return threads, {"affinity_cpus": aff, "os_cpu_count": os.cpu_count(), "omp_num_threads": cap or None,
                     "cgroup_cpu_quota": quota}


def cpu_baseline(n, kind, iters, solve_iters=None):
    """Oracle (the reference's op sequence on torch-CPU, oracle/ref_cpu.py) on the same mesh, BASELINE.md §3's
    three numbers: element assembly (`compute_c3d4_K_matrix`, `solver/element.py:883-903`), the EBE matvec
    (`compute_nodal_forces`, `:429-464`) and `iters` Jacobi-PCG iterations (`solver/solver.py:766-812`), timed
    on the host cores with torch.set_num_threads(threads) (cpu_threads). The assembly + fixed-iteration wall is
    measured; the wall of the GPU line's whole solve (solve_iters iterations) is projected from the iteration rate."""
    from oracle import ref_cpu as R
    threads, tinfo = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        coords, tets = mesh.kuhn_cube(n)
        t0 = time.perf_counter()
        K = R.tet4_poisson_K(coords, tets) if kind == "poisson" else R.tet4_K(coords, tets, 113.8e9, 0.342)
        t_asm = time.perf_counter() - t0
        N = coords.shape[0]
        dpn = 1 if kind == "poisson" else 3
        f, fixed = mesh.cube_poisson_case(coords) if kind == "poisson" else mesh.cube_elasticity_case(coords)
        t0 = time.perf_counter()
        Minv = R.diag_preconditioner(K, tets, N, dpn=dpn)
        Minv[fixed] = 0.0
        t_setup = time.perf_counter() - t0
        p = torch.ones(N, dpn, dtype=torch.float64)
        R.nodal_forces(K, tets, p)                     # first touch of the gather / scatter buffers
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            R.nodal_forces(K, tets, p)
        t_mv = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        R.pcg(K, tets, f.view(N, dpn), Minv, tol=0.0, max_iter=iters)
        t_it = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    out = {"value": iters / t_it, "unit": "CG iterations/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "threads_basis": tinfo,
           "sample": f"oracle/ref_cpu.py torch-CPU (the reference's op sequence) on the same {tets.shape[0]:,}-tet "
                     f"{kind} system: element assembly, {reps} EBE matvecs, {iters} Jacobi-PCG iterations; fp64",
           "assembly_s": t_asm, "setup_s": t_setup, "ebe_matvec_ms": t_mv * 1e3, "cg_iters": iters,
           "cg_s": t_it, "assembly_plus_fixed_iters_wall_s": t_asm + t_setup + t_it}
    if solve_iters:
        out["solve_iters"] = solve_iters
        out["projected_assembly_plus_solve_wall_s"] = t_asm + t_setup + solve_iters * t_it / iters
    return out


def attach_cpu_baseline(out, cb):
    """cpu_baseline into the bench dict, with the assembly + CG wall-clock ratios GPU vs CPU (north_star: >= 10x the
    reference CPU's assembly + CG wall-clock at 1 GPU): measured on the same fixed iteration count (the CPU's
    assembly + its `cg_iters` iterations against the GPU's assembly + as many timed iterations), and projected to the
    whole solve to rtol (the CPU iteration rate times the GPU line's iteration count; a projection, so named)."""
    out["cpu_baseline"] = cb
    k = cb.get("cg_iters")
    if k and out.get("ms_per_step"):
        gpu_fixed_s = (out.get("assembly_ms", 0.0) + k * out["ms_per_step"]) * 1e-3
        out["vs_cpu_assembly_plus_fixed_iters"] = {
            "ratio": cb["assembly_plus_fixed_iters_wall_s"] / gpu_fixed_s, "iterations": k,
            "cpu_wall_s": cb["assembly_plus_fixed_iters_wall_s"], "gpu_wall_s": gpu_fixed_s,
            "gpu_basis": "assembly_ms (steady pass) + iterations x ms_per_step (timed region)"}
    proj = cb.get("projected_assembly_plus_solve_wall_s")
    gpu_s = (out.get("assembly_ms", 0.0) + out.get("solve_ms", 0.0)) * 1e-3
    if proj and gpu_s > 0:
        out["projected_vs_cpu_assembly_plus_solve"] = proj / gpu_s


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or a.force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("RANK", str(rank))
        from fem355 import dist
        return dist.bench_main(a, METRIC)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    C.lib()

    # ---- warm the kernels (module load, first-launch costs) on a small mesh
    c0, t0_ = mesh.kuhn_cube(20, device=dev)   # 9k rows: enough slices for the persistent kernel's grid
    A0 = system.assemble_tet4_system(c0, t0_, a.kind, 1.0, 0.3)
    b0 = torch.ones(A0.n, dtype=torch.float64, device=dev)
    A0.matvec(b0)
    A0.pcg(b0, None, w=A0.jacobi(torch.zeros(A0.n, dtype=torch.uint8, device=dev)), mode=C.MODE_PCG, tol=0.0,
           max_iter=4, chunk=4)   # the solver kernels (the persistent one included)
    del A0, b0
    sync()

    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    if a.permute:
        coords, tets = permute_nodes(coords, tets, a.permute)
    out = measure(a, a.kind, coords, tets, dev)
    if not a.no_cpu_baseline and rank == 0:
        attach_cpu_baseline(out, cpu_baseline(a.n, a.kind, a.cpu_iters, out["solve_iters"]))
    # BASELINE configs[2] beside the metric: the same steps on the 10M-tet linear-elasticity system (north_star:
    # CG it/s on elasticity at 1/2/4/8 GPUs), its own CPU-oracle sample; a failure is reported, never fatal
    if a.kind == "poisson" and (a.elastic or a.mixed):
        from fem355 import dist

        def companion():
            d = measure(a, "elastic", coords, tets, dev)
            if a.matfree:
                try:
                    d["matfree"] = measure_matfree(a, coords, tets, dev, d)
                except Exception as e:   # reported, never fatal to the line
                    d["matfree"] = {"error": f"{type(e).__name__}: {e}"}
            if a.reference_api:
                try:
                    d["reference_api"] = measure_reference_api(a, coords, tets, dev, d)
                except Exception as e:   # reported, never fatal to the line
                    d["reference_api"] = {"error": f"{type(e).__name__}: {e}"}
            if not a.no_cpu_baseline:
                attach_cpu_baseline(d, cpu_baseline(a.n, "elastic", a.cpu_iters_elastic, d["solve_iters"]))
            return d
        guard = dist.CompanionGuard(out, "elasticity", rank=0, timeout=a.elastic_timeout)
        if a.elastic:
            guard.run(companion)
        if a.mixed:
            del coords, tets
            torch.cuda.empty_cache()
            try:
                out["mixed"] = measure_mixed(a, dev)
            except Exception as e:   # reported, never fatal to the line
                out["mixed"] = {"error": f"{type(e).__name__}: {e}"}
        if a.config1:
            try:
                out["config1"] = measure_config1(a, dev)
            except Exception as e:   # reported, never fatal to the line
                out["config1"] = {"error": f"{type(e).__name__}: {e}"}
        guard.emit()
        guard.close()
    else:
        print(json.dumps(out), flush=True)


def permute_nodes(coords, tets, seed):
    """The cube under a random node numbering (what a mesh file's order looks like to the pattern)."""
    perm = torch.randperm(coords.shape[0], generator=torch.Generator().manual_seed(seed)).to(coords.device)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel(), device=coords.device)
    return coords[perm].contiguous(), inv[tets].contiguous()


MF_FLOPS_PER_ELEMENT = 197   # csrc/matfree.hpp mf_element (elastic, FMA = 2) + the 12 node-sum adds
FP64_PEAK_TFLOPS = 78.6       # MI355X_MICROARCH.md: fp64 vector


def measure_matfree(a, coords, tets, dev, ref):
    """The 10M elasticity system on the element-chunk operator (system.MatFreeOperator: K p formed from the
    coordinates in every iteration, no matrix): DOFs/s (operator build + Jacobi + solve to rtol, median of the passes
    after a cold one), the fixed-iteration CG it/s with its kernel split, and the solve's agreement with the assembled
    operator's (`ref`, measure()'s elasticity dict: iterations +-2)."""
    M, N = tets.shape[0], coords.shape[0]
    f, fixed = mesh.cube_elasticity_case(coords)
    E, nu = 113.8e9, 0.342

    def build_and_solve():
        t0 = time.perf_counter()
        A = system.MatFreeOperator(coords, tets, "elastic", E, nu)
        mask = torch.zeros((N, 3), dtype=torch.uint8, device=dev)
        mask.index_fill_(0, fixed, 1)   # a fill kernel: no host-to-device copy (and host wait) of the 1
        w = A.jacobi(mask.view(-1))
        sync()
        t_b = time.perf_counter() - t0
        b = f.reshape(-1).to(torch.float64).contiguous()
        tol = a.rtol * float(torch.sqrt(torch.dot(b, w * b)))
        sync()
        t0 = time.perf_counter()
        res = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64)
        sync()
        return A, w, b, res, t_b, time.perf_counter() - t0

    A, w, b, res, tb_cold, ts_cold = build_and_solve()
    passes = []
    for _ in range(max(a.dof_passes, 1)):
        del A, w, b, res
        A, w, b, res, t_b, t_s = build_and_solve()
        passes.append((t_b, t_s))
    t_b, t_s = sorted(passes, key=lambda p: p[0] + p[1])[len(passes) // 2]
    assert abs(res.iterations - ref["solve_iters"]) <= 2, (res.iterations, ref["solve_iters"])
    run = system.PcgRunner(A, b, w, tol=0.0)
    run.start()
    # the timed steps replay hipGraphs of G iterations (two launches per iteration: the host's launch cost leaves
    # gaps between the kernels otherwise); the kernel split comes from a separate event-sampled pass after them
    G = math.gcd(a.steps, a.warmup) if a.mf_graph and a.warmup > 0 else 0
    G = min(G, 50)
    if G:
        run.use_graph(G)
    run.iterate(a.warmup)
    sync()
    t0 = time.perf_counter()
    if G:
        run.iterate(a.steps)
    else:
        ms, cnt = run.profile(a.steps, every=a.sample_every)
    sync()
    dt = time.perf_counter() - t0
    it, _, _ = run.poll()
    assert it == a.warmup + a.steps
    if G:
        ms, cnt = run.profile(min(a.steps, 50), every=1)
    run.close()
    info = A.info()
    k1 = ms[0] / max(cnt[0], 1)
    upd = ms[1] / max(cnt[1], 1)
    flops = MF_FLOPS_PER_ELEMENT * M
    # HBM bytes one K1 must move: the static layout (element local ids, pair lists, chunk tables, the node-major slot
    # positions spos -- carried in the walk's prefetch records since round 5), the coordinates and p once, the slot
    # values written; the merged update reads the slots back with the node -> slot pointers (nptr, not K1's)
    alg = info["static_bytes"] - 4 * (N + 1) + 24 * N + 24 * N + 24 * info["slots"]
    return {
        "value": a.steps / dt, "unit": "CG iterations/s", "ms_per_step": dt / a.steps * 1e3,
        "vs_assembled": (a.steps / dt) / ref["value"],
        "kernel_ms": {"k_pcg_mf_dot": k1, "update_with_slot_sums": upd, "sampled_launches": cnt[0]},
        "timed_launches": (f"hipGraph replays of {G} iterations" if G else "plain launches"),
        "dofs_per_s": 3 * N / (t_b + t_s), "build_ms": t_b * 1e3, "solve_ms": t_s * 1e3,
        "dofs_per_s_cold": 3 * N / (tb_cold + ts_cold), "solve_iters": res.iterations,
        "solve_iters_assembled": ref["solve_iters"], "layout": info,
        "roofline": {"bound": "fp64 VALU issue / latency", "kernel": "k_pcg_mf_dot<3>",
                     "flops_per_launch": flops, "achieved_TFLOPs": flops / (k1 * 1e-3) / 1e12,
                     "peak_TFLOPs": FP64_PEAK_TFLOPS, "frac_flops": flops / (k1 * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                     "algorithmic_bytes": alg, "achieved_GBps": alg / (k1 * 1e-3) / 1e9,
                     "frac_hbm": alg / (k1 * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                     # PMC HBM bytes of one K1 launch (FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_mf.sh), None unless taken
                     # on this layout (same algorithmic bytes)
                     "traffic": traffic_from_profiles(f"kuhn{a.n}_elastic_matfree", "k_pcg_mf_dot<3>", alg),
                     "model": f"{MF_FLOPS_PER_ELEMENT} flops per element; bytes: layout (incl. spos) + coordinates + p "
                              "+ slots"},
        "operator": "element-chunk (matrix-free): Morton-ordered chunks of <= 512 elements / 240 nodes, "
                    "fixed-order slot sums (csrc/matfree.hip)",
    }


MIXED_FAMILIES = (("c3d8", "hex_box", 88), ("c3d6", "wedge_box", 70), ("c3d10", "tet10_cube", 48))
RHO = 4.47e-3   # solver_example.ipynb:38-40


def measure_mixed(a, dev):
    """BASELINE configs[4]: "2M-element P2 tet + hex/wedge mixed mesh, mass+stiffness assembly, 1 x MI355X" -- three
    separate boxes (P2 / linear faces are nonconforming): c3d8 88^3 = 681,472 hexes, c3d6 2 x 70^3 =
    686,000 wedges, c3d10 6 x 48^3 = 663,552 quadratic tets, jittered. Per family one job: element stiffness through
    the reference API (`compute_K_matrix`, `solver/element.py:419-427`, default rule / single=True; --mixed-ke packed:
    its packed symmetric form, upper 3x3 blocks only, `element._solid_ke_sym` + `SellMatrix.add_element_matrices_sym`,
    the same sums, measured slower overall) and the consistent
    mass (`compute_M_matrix(..., scalar=True)`: its factor M_s of M = M_s (x) I3, [M, npe, npe] -- the 3x3 blocks of a
    vector-field mass are multiples of I3, so the stored and assembled mass is the bs = 1 M_s on the same node pattern;
    no reference function: parity unpinned) on the current stream, the pattern (node graph
    + SELL layout) on a second stream from a second host thread meanwhile, then both global assemblies; host clock
    around the whole job, device idle at both ends, best of --dof-passes after a cold pass. Per stage the kernel time
    (hip events, separate passes) and bytes: K_e / M_e written, K_e read + SELL values written by the assembly."""
    import threading
    from fem355 import element
    E, nu = 113.8e9, 0.342
    F64 = torch.float64

    def ev(fn):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        r = fn()
        s1.record()
        sync()
        return s0.elapsed_time(s1), r

    out = {"config": "c3d8 88^3 + c3d6 2 x 70^3 + c3d10 6 x 48^3 hexes / wedges / P2 tets (2,031,024 elements), "
                     "jitter 0.1, stiffness (bs = 3) + consistent mass (its scalar factor M_s, bs = 1: M = M_s (x) I3), "
                     "fp64"}
    total_ms, total_el, total_bytes = 0.0, 0, 0
    fused_km = a.mixed_km == "fused" and a.mixed_ke == "full"
    out["global_assembly"] = ("stiffness + mass in one pass (fem_assemble_from_ke_mass_sl)" if fused_km
                              else "stiffness and mass in separate passes")
    for et, gen, n in MIXED_FAMILIES:
        c, el = getattr(mesh, gen)(n, jitter=0.1, device=dev)
        N = c.shape[0]
        side = torch.cuda.Stream(device=dev)
        if a.mixed_ke == "packed":   # upper 3x3 blocks only (measured slower overall: DESIGN §10)
            def ke_fn():
                return element._solid_ke_sym(c, el, et, E, nu, device=dev)

            def asm_fn(S, K):
                return S.add_element_matrices_sym(K, el)
        else:
            def ke_fn():
                return element.compute_K_matrix(c, el, et, E, nu, device=dev, dtype=F64)

            def asm_fn(S, K):
                return S.add_element_matrices(K, el)

        def job():
            box = []

            def pattern():
                torch.cuda.set_device(dev)
                with torch.cuda.stream(side):
                    box.append(system.build_graph(el, N))
            th = threading.Thread(target=pattern)
            th.start()
            K = ke_fn()
            Me = element.compute_M_matrix(c, el, et, RHO, device=dev, dtype=F64, scalar=True)
            th.join()
            g = box[0]
            torch.cuda.current_stream(dev).wait_stream(side)
            Am = system.SellMatrix(g, 1)
            if fused_km:   # one pass: one column search and one incidence walk for both matrices
                A = system.SellMatrix(g, 3).add_stiffness_and_mass(K, Me, el, Am)
            else:
                A = asm_fn(system.SellMatrix(g, 3), K)
                Am.add_element_matrices(Me, el)
            return K, Me, g, A, Am

        walls = []
        for _ in range(1 + max(a.dof_passes, 1)):
            sync()
            t0 = time.perf_counter()
            K, Me, g, A, Am = job()
            sync()
            walls.append((time.perf_counter() - t0) * 1e3)
            del K, Me, A, Am, g
        # kernel times by stage (events; not overlapped), outside the timed jobs
        ms_k, K = ev(ke_fn)
        ms_g, g = ev(lambda: system.build_graph(el, N))
        ms_a, A = ev(lambda: asm_fn(system.SellMatrix(g, 3), K))
        ms_m, Me = ev(lambda: element.compute_M_matrix(c, el, et, RHO, device=dev, dtype=F64, scalar=True))
        ms_ma, Am = ev(lambda: system.SellMatrix(g, 1).add_element_matrices(Me, el))
        ms_km = None
        if fused_km:
            def km():
                mm = system.SellMatrix(g, 1)
                return system.SellMatrix(g, 3).add_stiffness_and_mass(K, Me, el, mm), mm
            ms_km, (A2, Am2) = ev(km)
            assert torch.equal(Am2.plain_values(), Am.plain_values())   # the fused mass is the separate one's bits
            del A2, Am2
        ke_bytes = K.numel() * 8
        me_bytes = Me.numel() * 8
        sell_bytes = g.sell_entries * 9 * 8
        mass = float(Am.plain_values().sum())
        nnzb = g.nnz
        del K, Me, A, Am, g
        torch.cuda.empty_cache()
        best = min(walls[1:])
        total_ms += best
        total_el += int(el.shape[0])
        total_bytes += 2 * ke_bytes + sell_bytes + 2 * me_bytes + sell_bytes // 9
        out[et] = {"elements": int(el.shape[0]), "nodes": N, "nnz_blocks": nnzb, "job_ms": best,
                   "job_passes_ms": [round(w, 3) for w in walls],
                   "stage_ms": {"Ke": ms_k, "pattern": ms_g, "assemble_K": ms_a, "Me": ms_m, "assemble_M": ms_ma,
                                "assemble_K_and_M_one_pass": ms_km},
                   "Ke_write_GBps": ke_bytes / (ms_k * 1e-3) / 1e9, "Me_write_GBps": me_bytes / (ms_m * 1e-3) / 1e9,
                   "assemble_K_GBps": (ke_bytes + sell_bytes) / (ms_a * 1e-3) / 1e9,
                   "total_mass_over_rho": mass / RHO}
    out["elements_total"] = total_el
    out["set_ms"] = total_ms
    out["value"] = total_el / (total_ms * 1e-3)
    out["unit"] = "elements/s (stiffness + mass, patterns and both global assemblies)"
    out["roofline"] = {"bound": "hbm", "algorithmic_bytes": total_bytes,
                       "achieved_GBps": total_bytes / (total_ms * 1e-3) / 1e9,
                       "frac": total_bytes / (total_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                       "model": "K_e and M_s,e written and each read once by its assembly, the bs = 3 stiffness and "
                                "bs = 1 mass SELL values written once (the set's job time; the pattern excluded)"
                                + ("; K_e in its packed symmetric form (upper blocks)" if a.mixed_ke == "packed" else "")}
    return out


def measure_config1(a, dev):
    """BASELINE configs[1] beside the metric: the 1M-tet P1 Poisson cube (n = 55, 998,250 tets), assembly + Jacobi-PCG,
    on the single-reduction persistent kernel and on the pipelined one (FEM_TUNE_PK_GV, which applies at this size;
    DESIGN §8i) -- 500 timed fixed iterations each, whatever --steps the metric line uses."""
    import copy
    c1, t1 = mesh.kuhn_cube(55, device=dev)
    out = {"config": {"workload": f"{t1.shape[0]:,}-tet P1 poisson Kuhn cube n=55, Jacobi-PCG fixed iterations",
                      "tets": int(t1.shape[0]), "nodes": int(c1.shape[0])}}
    keep = ("value", "unit", "steps", "ms_per_step", "dofs_per_s", "assembly_ms", "solve_ms", "solve_iters",
            "pipelined", "kernel_ms")
    for pl in (0, 1):
        b = copy.copy(a)
        b.n, b.steps, b.warmup, b.pipelined = 55, 500, 50, pl
        d = measure(b, "poisson", c1, t1, dev)
        out["pipelined" if pl else "single_reduction"] = {k: d[k] for k in keep if k in d}
    return out


def measure_reference_api(a, coords, tets, dev, ref):
    """configs[2] through the reference's own hand-off, as the notebooks call it: `compute_c3d4_K_matrix` (K [M,12,12]
    on the device, 11.6 GB at 10M tets; `solver/element.py:883-903`) -> `compute_diagonal_preconditioner` (the exact
    diagonal, fixed DOFs zeroed: the reference's PCG has no other Dirichlet handling, `solver/solver.py:814-833`) ->
    `preconditioned_conjugate_gradient_solver` (`solver/solver.py:766-812`: the stored K_e assembled into SELL, then
    the device PCG) to the bench's tolerance. Time to solution per stage; pass 1 builds the pattern inside the solver
    call, pass 2 finds it cached (a second solve on the same mesh). Iterations must agree with the fused pipeline's
    (`ref`, +-2). The solver's prints go to stderr (the bench's stdout is its JSON line)."""
    import contextlib
    from fem355 import solver as S
    N = coords.shape[0]
    f, fixed = mesh.cube_elasticity_case(coords)
    E, nu = 113.8e9, 0.342
    f = f.to(torch.float64)
    passes = []
    for cold in (True, False):
        if cold:
            S._GRAPH_CACHE.clear()
        sync()
        t0 = time.perf_counter()
        K = S.compute_c3d4_K_matrix(coords, tets, E, nu, device=dev, dtype=torch.float64)
        sync()
        t1 = time.perf_counter()
        Minv = S.compute_diagonal_preconditioner(K, tets, N, device=dev, dtype=torch.float64, exact_diagonal=True)
        Minv[fixed] = 0.0
        sync()
        t2 = time.perf_counter()
        b = f.reshape(-1)
        tol = a.rtol * float(torch.sqrt(torch.dot(b, Minv.reshape(-1) * b)))
        sync()
        t3 = time.perf_counter()
        with contextlib.redirect_stdout(sys.stderr):
            u, res = S.preconditioned_conjugate_gradient_solver(K, tets, f, Minv, tol=tol, max_iter=20000, device=dev,
                                                                dtype=torch.float64, return_info=True)
        sync()
        t4 = time.perf_counter()
        passes.append({"element_K_ms": (t1 - t0) * 1e3, "preconditioner_ms": (t2 - t1) * 1e3,
                       "pcg_call_ms": (t4 - t3) * 1e3, "total_ms": (t1 - t0 + t2 - t1 + t4 - t3) * 1e3,
                       "iterations": res.iterations, "status": res.status})
        del K, Minv, u, res
    torch.cuda.empty_cache()
    assert all(abs(p["iterations"] - ref["solve_iters"]) <= 2 for p in passes), (passes, ref["solve_iters"])
    warm = passes[1]
    return {"route": "compute_c3d4_K_matrix -> compute_diagonal_preconditioner(exact_diagonal=True) -> "
                     "preconditioned_conjugate_gradient_solver (K [M,12,12] fp64 on the device)",
            "cold_pattern": passes[0], "cached_pattern": warm, "time_to_solution_ms": warm["total_ms"],
            "dofs_per_s": 3 * N / (warm["total_ms"] * 1e-3), "solve_iters": warm["iterations"],
            "solve_iters_fused_pipeline": ref["solve_iters"]}


def measure(a, kind, coords, tets, dev):
    """One single-GPU measurement of `kind` on the mesh: DOFs/s (assembly + solve to rtol, two passes) and the
    fixed-iteration CG it/s with its roofline. Returns the bench dict (cpu_baseline None)."""
    M, N = tets.shape[0], coords.shape[0]
    if kind == "poisson":
        f, fixed = mesh.cube_poisson_case(coords)
        E, nu = 1.0, 0.0
    else:
        f, fixed = mesh.cube_elasticity_case(coords)
        E, nu = 113.8e9, 0.342
    sync()

    # ---- assembly (pattern + values + Jacobi) and solve to tolerance: DOFs/s. The first pass pays the first-use
    # device allocations of this mesh size (torch's caching allocator, the solver's buffer cache) and is reported as
    # dofs_per_s_cold; the --dof-passes passes after it, timed the same way, give the steady-state dofs_per_s (their
    # medians; same work every pass: the pattern, the values, the Jacobi weights and the whole solve are recomputed
    # from the mesh)
    reorder_ms = []

    # --pipelined 1: the pipelined persistent iteration where it applies (include/fem355.h FEM_TUNE_PK_GV)
    tune = (C.TUNE_DEFAULT | C.TUNE_PK_GV) if a.pipelined else None

    def assemble_and_solve():
        t0 = time.perf_counter()
        c, t, ff, fx = coords, tets, f, fixed
        if a.reorder == "rcm":   # renumbered mesh, load and constraints (u maps back through inv)
            perm, inv = system.rcm_order(tets, N)
            c, t = system.renumber(coords, tets, perm, inv)
            ff, fx = f[perm], inv[fixed]
            sync()
            reorder_ms.append((time.perf_counter() - t0) * 1e3)
        A = system.assemble_tet4_system(c, t, kind, E, nu)
        mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
        mask.index_fill_(0, fx, 1)   # a fill kernel: no host-to-device copy (and host wait) of the 1
        w = A.jacobi(mask.view(-1))
        sync()
        t_asm = time.perf_counter() - t0
        A.check_singular()
        b = ff.reshape(-1).to(torch.float64).contiguous()
        tol = a.rtol * float(torch.sqrt(torch.dot(b, w * b)))
        sync()
        t0 = time.perf_counter()
        res = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=20000, chunk=64, schedule=a.schedule,
                    tune=tune)
        sync()
        return A, w, b, res, t_asm, time.perf_counter() - t0

    A, w, b, res, t_asm_cold, t_solve_cold = assemble_and_solve()
    res_cold = res
    passes = []
    for _ in range(max(a.dof_passes, 1)):
        del A, w, b, res
        A, w, b, res, t_asm, t_solve = assemble_and_solve()
        assert res.iterations == res_cold.iterations and res.status == res_cold.status
        passes.append((t_asm, t_solve))
    # steady state: the median pass by its assembly + solve total (a measured pass: dofs_per_s, assembly_ms and
    # solve_ms all come from it); the medians of the assembly times and of the solve times taken separately (they
    # may come from different passes) are reported beside it
    t_asm, t_solve = sorted(passes, key=lambda p: p[0] + p[1])[len(passes) // 2]
    t_asm_med = sorted(p[0] for p in passes)[len(passes) // 2]
    t_solve_med = sorted(p[1] for p in passes)[len(passes) // 2]

    # ---- fixed-iteration timing (the metric)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=a.schedule, tune=tune)
    run.start()
    if a.graph:
        run.use_graph(a.graph)
    persist = run.effective_schedule() == system.SCHED_PERSIST
    pipelined = persist and run.pipelined()
    n_uni, n_sl, idx_total = run.uniform_slices()
    # the W warm-up steps go through the same launch path as the timed steps (persistent: one launch, events of the
    # context created here rather than next to the timed launch)
    if persist and a.warmup > 0:
        run.profile(a.warmup, every=a.warmup)
    else:
        run.iterate(a.warmup)
    sync()
    t0 = time.perf_counter()
    # persistent schedule: the K steps are ONE cooperative launch (the kernel stops itself on convergence, so a
    # solve needs no host polling either); hip events around it give the per-iteration time of the whole iteration
    ms, cnt = run.profile(a.steps, every=a.steps if persist else a.sample_every)
    sync()
    dt = time.perf_counter() - t0
    it, stt, _ = run.poll()
    assert it == a.warmup + a.steps, (it, stt)
    kernel = {system.SCHED_THREE: "k_pcg_spmv_dot", system.SCHED_FUSED: "k_pcg_spmv_dot<FUSED>",
              system.SCHED_DEFERRED: "k_pcg_d1",
              system.SCHED_PERSIST: "k_pcg_persist3" if A.bs == 3 else "k_pcg_persist"}[run.effective_schedule()]
    if pipelined:
        kernel = "k_pcg_persist_gv"
    run.close()

    # per launch of the measured kernel: one SpMV (3-kernel / deferred) or one whole iteration (persistent: the
    # matrix, the u gather and the u store are all it moves; r, p, s, x, w stay in registers and LDS)
    spmv_ms = ms[0] / max(cnt[0], 1)
    # column-index bytes of the stored format: slice-uniform slices read one delta list per slice (persistent
    # schedule), the others 2 (int16) or 4 bytes per entry incl. padding
    alg = A.algorithmic_bytes_spmv(index_total=idx_total if (persist and n_uni) else None)
    achieved = alg / (spmv_ms * 1e-3) / 1e9
    # SURVEY §8(d)'s byte models beside the stored-format one: B_spmv = 12 nnz + 4 (n+1) + 16 n (scalar CSR, int32
    # columns) and B_iter = B_spmv + 88 n (11 vector streams of a three-pass Jacobi-PCG iteration), both over the
    # measured iteration time; the SpMV frac uses the SpMV launch alone where the schedule has one
    iter_ms = spmv_ms if persist else spmv_ms + ms[1] / max(cnt[1], 1) + ms[2] / max(cnt[2], 1)
    s8d = s8d_models(A.n, A.g.nnz * A.bs * A.bs, spmv_ms, iter_ms, persist)
    ceiling = system.stream_ceiling(dev)
    # the assembly's value kernel alone, outside every timed region: one launch on a fresh matrix of the same
    # pattern (the store path of the assembly passes) between hip events on the library's stream (torch's current
    # stream), against SURVEY §8(d)'s B_asm = 112 M + 8 nnz (conn + gathered coordinates in, every value written
    # once; nnz counts scalar values, so x bs^2 for the block system). Skipped with --reorder (renumbered mesh).
    asm_roof = None
    if a.reorder != "rcm":
        A2 = system.SellMatrix(A.g, A.bs)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        sync()
        ev[0].record()
        A2.add_tet4(coords, tets, E, nu)
        ev[1].record()
        sync()
        vms = ev[0].elapsed_time(ev[1])
        b_asm = 112 * M + 8 * A.g.nnz * A.bs * A.bs
        asm_roof = {"kernel": f"k_asm_tet4_acc<{A.bs}>", "values_ms": vms, "B_asm": b_asm,
                    "achieved_GBps": b_asm / (vms * 1e-3) / 1e9, "peak": HBM_PEAK_GBPS,
                    "frac": b_asm / (vms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                    "model": "SURVEY 8(d) B_asm = 112 M + 8 nnz (values only; the pattern build excluded)"}
        del A2
    workload_key = f"kuhn{a.n}_{kind}"
    out = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "CG iterations/s",
        "n_gpus": 1,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{M:,}-tet P1 {kind} Kuhn cube n={a.n}, Jacobi-PCG fixed iterations",
                   "tets": M, "nodes": N, "dofs": A.n, "nnz_blocks": A.g.nnz, "format": "SELL-64 fp64 values, " + ("int16 column deltas" if A.use16 else "int32 cols")
                   + (f", slice-uniform deltas in {n_uni} of {n_sl} slices" if (persist and n_uni) else ""),
                   "parallelism": "single GPU"},
        "dofs_per_s": A.n / (t_asm + t_solve),
        "assembly_ms": t_asm * 1e3,
        "solve_ms": t_solve * 1e3,
        "dofs_passes_ms": [[round(x * 1e3, 4), round(y * 1e3, 4)] for x, y in passes],
        "dofs_per_s_split_medians": A.n / (t_asm_med + t_solve_med),
        "assembly_ms_median": t_asm_med * 1e3,
        "solve_ms_median": t_solve_med * 1e3,
        "dofs_per_s_cold": A.n / (t_asm_cold + t_solve_cold),
        "assembly_ms_cold": t_asm_cold * 1e3,
        "solve_ms_cold": t_solve_cold * 1e3,
        "solve_iters": res.iterations,
        "mesh_numbering": ("random (seed %d)" % a.permute if a.permute else "lexicographic")
        + (", device RCM renumbering in every assembly pass" if a.reorder == "rcm" else ""),
        "reorder_ms": (sorted(reorder_ms)[len(reorder_ms) // 2] if reorder_ms else None),
        "solve_status": res.status,
        "pipelined": pipelined,
        "kernel_ms": ({"persist_iteration": spmv_ms, "iterations_per_launch": a.steps} if persist else
                      {"spmv_dot": spmv_ms, "update": ms[1] / max(cnt[1], 1), "pupdate": ms[2] / max(cnt[2], 1),
                       "sampled_launches": cnt[0]}),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic_from_profiles(workload_key, kernel, alg),
                     "traffic_source": traffic_source(workload_key)
                     if traffic_from_profiles(workload_key, kernel, alg) is not None else None,
                     "kernel": kernel, "algorithmic_bytes": alg,
                     "per": "iteration (whole PCG iteration in the persistent kernel)" if persist else "SpMV launch",
                     "stream_ceiling_GBps": ceiling, "frac_of_stream_read": achieved / ceiling["read"],
                     "s8d": s8d},
        "assembly_roofline": asm_roof,
        "cpu_baseline": None,
    }
    return out


if __name__ == "__main__":
    main()
