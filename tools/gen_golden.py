#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE itself (build container only).

The reference (sml2004/CUDA-powered-mesh-handling-and-Iterative-solvers @ 2025-04-18) is pure Python +
PyTorch; it is imported read-only from /root/reference/solver with a stub `pyvista` module (only
`vtk_loader_to_torch` uses it, `solver/element.py:13,53`), every call on device="cpu", dtype=float64
(SURVEY.md §8(c) recipe). Nothing of the reference is copied: only inputs and outputs are stored.

Skips (exit 0) when /root/reference is absent (e.g. on the GPU box). Re-run: python tools/gen_golden.py
"""
from __future__ import annotations

import contextlib
import io
import os
import re
import sys
import types

import numpy as np
import torch

REF = "/root/reference/solver"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

import fem355  # noqa: E402  (synthetic meshes only)
from fem355 import mesh  # noqa: E402

E, NU = 113.8e9, 0.342          # solver_example.ipynb:38-40
CPU, F64 = "cpu", torch.float64


def load_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("pyvista", types.ModuleType("pyvista"))
    sys.path.insert(0, REF)
    import element  # noqa
    import solver   # noqa
    return element, solver


def run_quiet(fn, *a, **k):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = fn(*a, **k)
    return out, buf.getvalue()


def iters_from(text):
    m = re.search(r"Converged after (\d+) iterations", text)
    return int(m.group(1)) if m else -1


def save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()})
    print(f"{name}: {os.path.getsize(path)/1024:.1f} KiB  keys={sorted(arrays)}")


def masked_residual(el, K, elems, F, u, fixed):
    r = F - el.compute_nodal_forces(K, elems, u, device=CPU, dtype=F64)
    r[fixed] = 0.0
    return float(torch.linalg.norm(r))


def gen_tet4_n4(el, so):
    coords, tets = mesh.kuhn_cube(4, jitter=0.15)
    N = coords.shape[0]
    V = el.compute_tetrahedral_volumes(coords, tets, device=CPU, dtype=F64)
    B = el.compute_c3d4_B_matrix(coords, tets, device=CPU, dtype=F64)
    K = el.compute_K_matrix(coords, tets, "c3d4", E, NU, device=CPU, dtype=F64)
    D = el.compute_elasticity_matrix(E, NU, device=CPU, dtype=F64)
    F, fixed = mesh.cube_elasticity_case(coords)
    Minv_bug = so.compute_diagonal_preconditioner(K, tets, N, device=CPU, dtype=F64)
    # true diagonal (the function's documented intent), fixed DOFs zeroed -> PCG on K_ff
    dofs = (tets.unsqueeze(-1) * 3 + torch.arange(3)).reshape(-1)
    diag = torch.zeros(3 * N, dtype=F64).index_add_(0, dofs, torch.diagonal(K, dim1=1, dim2=2).reshape(-1))
    Minv = (1.0 / diag).view(N, 3)
    Minv[fixed] = 0.0
    p = torch.from_numpy(np.random.default_rng(7).standard_normal((N, 3)))
    y = el.compute_nodal_forces(K, tets, p, device=CPU, dtype=F64)

    tol = 1e-6
    u_cg, txt = run_quiet(so.stable_conjugate_gradient_solver, K, tets, F, fixed, tol=tol, max_iter=1000,
                          device=CPU, dtype=F64)
    n_cg = iters_from(txt)
    hist = []
    for k in range(1, min(n_cg, 40) + 1):   # reference returns no history: re-run with max_iter=k
        uk, _ = run_quiet(so.stable_conjugate_gradient_solver, K, tets, F, fixed, tol=0.0, max_iter=k,
                          device=CPU, dtype=F64)
        hist.append(masked_residual(el, K, tets, F, uk, fixed))
    u_pcg, txt2 = run_quiet(so.preconditioned_conjugate_gradient_solver, K, tets, F, Minv, tol=1e-6,
                            max_iter=1000, device=CPU, dtype=F64)
    n_pcg = iters_from(txt2)
    save("tet4_cube_n4_jit", coords=coords, tets=tets, V=V, B=B, K=K, D=D, F=F, fixed=fixed, p=p, y=y,
         Minv_bug=Minv_bug, Minv=Minv, tol=tol, u_cg=u_cg, n_cg=n_cg, cg_hist=np.array(hist),
         u_pcg=u_pcg, n_pcg=n_pcg, cg_stdout=np.array(txt.strip()), pcg_stdout=np.array(txt2.strip()))


def gen_tet4_n6(el, so):
    coords, tets = mesh.kuhn_cube(6)
    N = coords.shape[0]
    K = el.compute_c3d4_K_matrix(coords, tets, E, NU, device=CPU, dtype=F64)
    p = torch.from_numpy(np.random.default_rng(11).standard_normal((N, 3)))
    y = el.compute_nodal_forces(K, tets, p, device=CPU, dtype=F64)
    F, fixed = mesh.cube_elasticity_case(coords)
    u, txt = run_quiet(so.stable_conjugate_gradient_solver, K, tets, F, fixed, tol=1e-6, max_iter=2000,
                       device=CPU, dtype=F64)
    save("tet4_cube_n6", coords=coords, tets=tets, p=p, y=y, F=F, fixed=fixed, u_cg=u, n_cg=iters_from(txt),
         tol=1e-6, K_diag=torch.diagonal(K, dim1=1, dim2=2).contiguous())


def gen_poisson(el, so):
    """Scalar P1 Poisson pinned on the reference: K^P = V G G^T from the reference's own B rows/volumes;
    the solve uses the reference PCG on K^P (x) I3 (three decoupled copies of the scalar system)."""
    coords, tets = mesh.kuhn_cube(4, jitter=0.15)
    N = coords.shape[0]
    B = el.compute_c3d4_B_matrix(coords, tets, device=CPU, dtype=F64)
    V = el.compute_tetrahedral_volumes(coords, tets, device=CPU, dtype=F64)
    G = torch.stack([B[:, 0, 0::3], B[:, 1, 1::3], B[:, 2, 2::3]], dim=2)       # [M,4,3]
    KP = torch.matmul(G, G.transpose(1, 2)) * V.view(-1, 1, 1)
    Kx = torch.kron(KP.contiguous(), torch.eye(3, dtype=F64).unsqueeze(0))     # [M,12,12]
    f, fixed = mesh.cube_poisson_case(coords)
    dofs = tets.reshape(-1)
    diag = torch.zeros(N, dtype=F64).index_add_(0, dofs, torch.diagonal(KP, dim1=1, dim2=2).reshape(-1))
    dinv = 1.0 / diag
    dinv[fixed] = 0.0
    F3 = f.expand(N, 3).contiguous()
    u3, txt = run_quiet(so.preconditioned_conjugate_gradient_solver, Kx, tets, F3, dinv.view(N, 1).expand(N, 3),
                        tol=1e-9, max_iter=2000, device=CPU, dtype=F64)
    p = torch.from_numpy(np.random.default_rng(5).standard_normal((N, 3)))
    y3 = el.compute_nodal_forces(Kx, tets, p, device=CPU, dtype=F64)
    save("poisson_tet4_n4_jit", coords=coords, tets=tets, KP=KP, f=f[:, 0], fixed=fixed, dinv=dinv,
         u=u3[:, 0], n_pcg=iters_from(txt), tol=1e-9, p=p[:, 0], y=y3[:, 0])


def jittered_single_cells(etype, n_cells, seed):
    rng = np.random.default_rng(seed)
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    coords, el = gen(2, jitter=0.2, seed=seed)
    coords = coords + torch.from_numpy(rng.uniform(-0.03, 0.03, coords.shape))   # boundary nodes too
    pick = torch.from_numpy(rng.choice(el.shape[0], size=min(n_cells, el.shape[0]), replace=False))
    el = el[pick]
    # include both orientations: mirror half of the picked cells (reverses the Jacobian sign)
    flip = {"c3d8": [0, 3, 2, 1, 4, 7, 6, 5], "c3d6": [0, 2, 1, 3, 5, 4],
            "c3d10": [0, 2, 1, 3, 6, 5, 4, 7, 9, 8]}[etype]
    el[::2] = el[::2][:, flip]
    return coords, el.contiguous()


def gen_solids(el, so):
    for etype, ncell, seed in (("c3d8", 8, 101), ("c3d6", 8, 102), ("c3d10", 6, 103)):
        coords, cells = jittered_single_cells(etype, ncell, seed)
        pts, w = el.integral_points(etype, device=CPU)
        pts, w = pts.to(F64), w.to(F64)
        if etype == "c3d6":   # dtype quirk Q7: build in the reference's own way at float64
            pts, w = el.c3d6_integration_points(device=CPU, dtype=F64)
        if etype == "c3d10":
            pts, w = el.c3d10_integration_points(device=CPU, dtype=F64)
        if etype == "c3d8":
            pts, w = el.c3d8_integration_points(device=CPU, dtype=F64)
        Js, Gs, Bs = [], [], []
        for q in range(pts.shape[0]):
            Js.append({"c3d8": el.compute_c3d8_Jacobian, "c3d6": el.compute_c3d6_Jacobian,
                       "c3d10": el.compute_c3d10_Jacobian}[etype](coords, cells, pts[q], device=CPU, dtype=F64))
            Gs.append({"c3d8": el.compute_c3d8_shape_gradients, "c3d6": el.compute_c3d6_shape_gradients,
                       "c3d10": el.compute_c3d10_shape_gradients}[etype](coords, cells, pts[q], device=CPU, dtype=F64))
            Bs.append({"c3d8": el.compute_c3d8_B_matrix, "c3d6": el.compute_c3d6_B_matrix,
                       "c3d10": el.compute_c3d10_B_matrix}[etype](coords, cells, pts[q], device=CPU, dtype=F64))
        K1 = el.compute_K_matrix(coords, cells, etype, E, NU, single=True, device=CPU, dtype=F64)
        K0 = el.compute_K_matrix(coords, cells, etype, E, NU, single=False, device=CPU, dtype=F64)
        extra = {}
        if etype == "c3d6":
            extra["vol"] = el.compute_wedge_volumes(coords, cells, device=CPU, dtype=F64)
        if etype == "c3d8":
            extra["vol"] = el.compute_hexahedral_volumes(coords, cells, device=CPU, dtype=F64)
        save(f"{etype}_cells", coords=coords, elements=cells, points=pts, weights=w, J=torch.stack(Js),
             grads=torch.stack(Gs), B=torch.stack(Bs), K_single=K1, K_multi=K0, **extra)


def mixed_box():
    """Conforming-node box [0,1]^3 on an n=3 grid: hex cells with i==0, wedges i==1, Kuhn tets i==2."""
    n = 3
    coords = mesh.grid_coords(n, jitter=0.1, seed=77)
    hexes = mesh._hex_corner_nodes(n)
    i = torch.arange(n).repeat_interleave(n * n)
    h8 = hexes[i == 0]
    w6 = torch.stack([hexes[i == 1][:, list(s)] for s in mesh.WEDGE_SPLIT], 1).reshape(-1, 6)
    t4 = torch.stack([hexes[i == 2][:, list(t)] for t in mesh.KUHN_TETS], 1).reshape(-1, 4)
    return coords, t4.contiguous(), w6.contiguous(), h8.contiguous()


def gen_mixed(el, so):
    coords, t4, w6, h8 = mixed_box()
    N = coords.shape[0]
    F3, fixed = mesh.cube_elasticity_case(coords)
    force = torch.zeros((N, 6), dtype=F64)
    force[:, :3] = F3
    u, txt = run_quiet(so.static_structure_solver, coords, force, fixed, c3d4=t4, c3d6=w6, c3d8=h8,
                       material={"E": E, "nu": NU}, tol=1e-6, max_iter=3000, device=CPU, dtype=F64)
    save("mixed_static", coords=coords, c3d4=t4, c3d6=w6, c3d8=h8, force=force, fixed=fixed, u=u,
         n_iter=iters_from(txt), tol=1e-6)


def gen_partition(el, so):
    coords, tets = mesh.kuhn_cube(4)
    cent = coords[tets].mean(1)
    parts = [torch.nonzero((cent[:, 0] >= a) & (cent[:, 0] < b), as_tuple=True)[0]
             for a, b in ((0, 0.25), (0.25, 0.5), (0.5, 0.75), (0.75, 1.01))]
    out = {"tets": tets}
    for k, ids in enumerate(parts):   # global->local map exactly as subdivision.ipynb:254-259
        elems = tets[ids]
        g = torch.unique(elems)
        g2l = {int(v): j for j, v in enumerate(g.tolist())}
        loc = torch.tensor([[g2l[int(v)] for v in row] for row in elems.tolist()], dtype=torch.long)
        out[f"ids{k}"], out[f"nodes{k}"], out[f"local{k}"] = ids, g, loc
    save("partition_ref", **out)


def constrained_case():
    """Jittered n=4 c3d4 cube with an SPC'd base (one prescribed non-zero value), a rigid RBE2 top plate driven
    from its centre node (case A), and an RBE2 side group + weighted RBE3 top master + nodal loads (case B)."""
    coords, tets = mesh.kuhn_cube(4, jitter=0.15)
    z = coords[:, 2]
    base = torch.nonzero(z < 1e-9).view(-1).tolist()
    top = torch.nonzero(z > 1 - 1e-9).view(-1).tolist()
    master = top[len(top) // 2]
    slaves = [t for t in top if t != master]
    spc = [{"node": b, "dofs": [0, 1, 2], "value": 0.0} for b in base]
    spc[0] = {"node": base[0], "dofs": [0], "value": 1e-5}
    rbe2_a = [{"master": master, "slaves": slaves, "dofs": [0, 1, 2]}]
    side = [s for s in torch.nonzero(coords[:, 0] > 1 - 1e-9).view(-1).tolist() if s not in base and s not in top]
    rbe2_b = [{"master": side[0], "slaves": side[1:4], "dofs": [0, 2]}]
    rbe3_b = [{"master": master, "slaves": slaves[:6], "dofs": [0, 1, 2], "weights": [1.0, 2.0, 1.0, 0.5, 1.5, 1.0]},
              {"master": slaves[7], "slaves": slaves[8:11], "dofs": [2, 1], "weights": [1.0, 1.0, 2.0]}]
    loads_b = [{"node": s, "force": [1e4, 0.0, -1e5]} for s in top]
    return coords, tets, master, spc, rbe2_a, rbe2_b, rbe3_b, loads_b


def gen_constrained(el, so):
    import json
    coords, tets, master, spc, rbe2_a, rbe2_b, rbe3_b, loads_b = constrained_case()
    N = coords.shape[0]
    K = el.compute_K_matrix(coords, tets, "c3d4", E, NU, device=CPU, dtype=F64)
    F = torch.zeros((N, 3), dtype=F64)
    F[master, 2] = -1e6
    tol = 1e-3
    ua, ta = run_quiet(so.constrained_conjugate_gradient_solver, K, tets, F, rbe2_a, spc, tol=tol, max_iter=3000,
                       device=CPU)
    ub, tb = run_quiet(so.new_constrained_conjugate_gradient_solver, K, tets, N, rbe2_b, rbe3_b, spc, loads_b, tol=tol,
                       max_iter=3000, device=CPU)
    it = [int(re.search(r"Converged @ iter (\d+)", t).group(1)) for t in (ta, tb)]
    cons = json.dumps({"spc": spc, "rbe2_a": rbe2_a, "rbe2_b": rbe2_b, "rbe3_b": rbe3_b, "loads_b": loads_b})
    save("constrained_tet4", coords=coords, tets=tets, F=F, u_a=ua, u_b=ub, n_iter_a=it[0], n_iter_b=it[1], tol=tol,
         constraints=np.array(cons))


def gen_stress(el, so):
    """Stress recovery on the golden meshes with seeded displacements."""
    g = np.load(os.path.join(OUT, "tet4_cube_n4_jit.npz"))
    coords, tets = torch.from_numpy(g["coords"]), torch.from_numpy(g["tets"])
    u = torch.from_numpy(g["u_cg"])
    out = {}
    s4, v4 = el.compute_element_stress(coords, tets, u, E, NU, "c3d4", device=CPU, dtype=F64)
    out.update(c3d4_sig=s4, c3d4_vm=v4,
               c3d4_node_vm=el.compute_node_vm_stress(coords, tets, v4, device=CPU, dtype=F64))
    rng = np.random.default_rng(7)
    normals = torch.from_numpy(rng.standard_normal((tets.shape[0], 4, 3)))
    ff = el.compute_c3d4_surface_forces(normals, s4, device=CPU)
    S = 40
    sidx = torch.stack([torch.from_numpy(rng.integers(0, tets.shape[0], (S, 2))),
                        torch.from_numpy(rng.integers(0, 4, (S, 2)))], dim=-1)   # [S, 2, (elem, face)]
    out.update(normals=normals, face_forces=ff, shared_idx=sidx,
               shared_sum=el.compute_c3d4_shared_face_forces_sum(sidx, ff, device=CPU))
    voigt = torch.from_numpy(rng.standard_normal((16, 6)))
    T = el.compute_stress_tensor(voigt)
    out.update(voigt=voigt, voigt_tensor=T, voigt_vm=el.compute_von_mises_stress(T))
    for etype in ("c3d8", "c3d6", "c3d10"):
        c = np.load(os.path.join(OUT, f"{etype}_cells.npz"))
        cc, ce = torch.from_numpy(c["coords"]), torch.from_numpy(c["elements"])
        ue = torch.from_numpy(rng.standard_normal((cc.shape[0], 3))) * 1e-3
        s1, v1 = el.compute_element_stress(cc, ce, ue, E, NU, etype, single=True, device=CPU, dtype=F64)
        s0, v0 = el.compute_element_stress(cc, ce, ue, E, NU, etype, single=False, device=CPU, dtype=F64)
        out.update({f"{etype}_u": ue, f"{etype}_sig1": s1, f"{etype}_vm1": v1, f"{etype}_sig0": s0,
                    f"{etype}_vm0": v0, f"{etype}_node_vm": el.compute_node_vm_stress(cc, ce, v1, device=CPU,
                                                                                        dtype=F64)})
    save("stress", **out)


def gen_topology(el, so):
    """Topology on small jittered meshes with some elements removed (holes -> inner
    surfaces), tets / hexes / wedges / c3d10."""
    out = {}
    rng = np.random.default_rng(11)
    ct, tt = mesh.kuhn_cube(3, jitter=0.15, seed=5)
    tt = tt[torch.from_numpy(np.sort(rng.choice(tt.shape[0], tt.shape[0] - 9, replace=False)))]
    f, x = el.compute_tetrahedral_surface_faces_with_fourth_node(tt, device=CPU)
    out.update(tet_coords=ct, tets=tt, tet_surf=f, tet_surf_x=x,
               tet_surf_n=el.compute_tetrahdral_surface_normals(ct, tt, device=CPU, dtype=F64),
               tet_area_n=el.compute_tetrahedral_normals_and_area(ct, tt, device=CPU, dtype=F64),
               tet_shared=el.identify_tetrahedral_shared_faces(tt, device=CPU),
               tet_edges=el.element_to_edge(tt, device=CPU))
    ch, hh = mesh.hex_box(3, jitter=0.15, seed=6)
    hh = hh[torch.from_numpy(np.sort(rng.choice(hh.shape[0], hh.shape[0] - 3, replace=False)))]
    f, x = el.compute_hexahedral_surface_faces_with_extra_node(hh, device=CPU)
    out.update(hex_coords=ch, hexes=hh, hex_surf=f, hex_surf_x=x,
               hex_surf_n=el.compute_hexahedral_surface_normals(ch, hh, device=CPU, dtype=F64),
               hex_area_n=el.compute_hexahedral_normals_and_area(ch, hh, device=CPU, dtype=F64),
               hex_shared=el.identify_hexahedral_shared_faces(hh, device=CPU),
               hex_tets=el.c3d8_to_c3d4(hh, device=CPU))
    cw, ww = mesh.wedge_box(2, jitter=0.1, seed=7)
    # compute_wedge_normals_and_area raises in the reference itself (torch.cross(..., dim=3) on [M, 3, 3]
    # tensors, `solver/element.py:2409,2415`): not a fixture
    (fq, ft), (xq, xt) = el.compute_wedge_surface_faces_with_extra_node(ww, device=CPU)
    nq, nt = el.compute_wedge_surface_normals(cw, ww, device=CPU, dtype=F64)
    out.update(wedge_coords=cw, wedges=ww, wedge_surf_q=fq, wedge_surf_t=ft, wedge_surf_xq=xq, wedge_surf_xt=xt,
               wedge_surf_nq=nq, wedge_surf_nt=nt,
               wedge_tets=el.c3d6_to_c3d4(ww, device=CPU))
    c10, t10 = mesh.tet10_cube(1)
    out.update(tet10=t10, tet10_tets=el.c3d10_to_c3d4(t10, device=CPU))
    save("topology", **out)


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return 0
    os.makedirs(OUT, exist_ok=True)
    el, so = load_reference()
    torch.manual_seed(0)
    gen_tet4_n4(el, so)
    gen_tet4_n6(el, so)
    gen_poisson(el, so)
    gen_solids(el, so)
    gen_mixed(el, so)
    gen_partition(el, so)
    gen_constrained(el, so)
    gen_stress(el, so)
    gen_topology(el, so)
    return 0


if __name__ == "__main__":
    sys.exit(main())
