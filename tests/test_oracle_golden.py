"""Tier 1 (CPU): the oracle restatement against golden vectors produced by the reference itself
(tools/gen_golden.py). Bit-exact where the op sequence is the reference's."""
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

E, NU = 113.8e9, 0.342


def test_tet4_element_algebra():
    g = load_golden("tet4_cube_n4_jit")
    c, t = g["coords"], g["tets"]
    assert rel(R.tet_volumes(c, t), g["V"]) == 0.0
    assert rel(R.tet4_B(c, t), g["B"]) == 0.0
    assert rel(R.tet4_K(c, t, E, NU), g["K"]) == 0.0
    assert rel(R.elasticity_matrix(E, NU), g["D"]) < 1e-15


def test_ebe_operator_and_preconditioner():
    g = load_golden("tet4_cube_n4_jit")
    K, t = g["K"], g["tets"]
    assert rel(R.nodal_forces(K, t, g["p"]), g["y"]) == 0.0
    assert rel(R.diag_preconditioner(K, t, g["coords"].shape[0], compat_colzero=True), g["Minv_bug"]) == 0.0
    g6 = load_golden("tet4_cube_n6")
    K6 = R.tet4_K(g6["coords"], g6["tets"], E, NU)
    assert rel(R.nodal_forces(K6, g6["tets"], g6["p"]), g6["y"]) < 1e-15


def test_stable_cg_and_pcg_match_reference_iterations():
    g = load_golden("tet4_cube_n4_jit")
    K, t = g["K"], g["tets"]
    hist = []
    u, n, s = R.stable_cg(K, t, g["F"], g["fixed"], tol=float(g["tol"]), history=hist)
    assert s == "converged" and n == int(g["n_cg"])
    assert rel(u, g["u_cg"]) == 0.0
    u, n, s = R.pcg(K, t, g["F"], g["Minv"], tol=1e-6)
    assert n == int(g["n_pcg"]) and rel(u, g["u_pcg"]) == 0.0
    assert str(g["cg_stdout"]).startswith(f"Converged after {int(g['n_cg'])} iterations.")


def test_cg_residual_history_first_iterations():
    """Contract: the true masked residual after k iterations matches the reference's."""
    g = load_golden("tet4_cube_n4_jit")
    K, t, F, fixed = g["K"], g["tets"], g["F"], g["fixed"]
    ref = g["cg_hist"]
    for k in (1, 5, 10, 20):
        u, _, _ = R.stable_cg(K, t, F, fixed, tol=0.0, max_iter=k)
        r = F - R.nodal_forces(K, t, u)
        r[fixed] = 0.0
        assert abs(float(torch.linalg.norm(r)) - float(ref[k - 1])) <= 1e-10 * float(ref[k - 1])


def test_isoparametric_solids():
    for et in ("c3d8", "c3d6", "c3d10"):
        g = load_golden(f"{et}_cells")
        c, e = g["coords"], g["elements"]
        p, w = R.POINTS[et]()
        assert rel(p, g["points"]) == 0.0 and rel(w, g["weights"]) == 0.0
        assert rel(R.iso_K(c, e, et, E, NU), g["K_single"]) == 0.0, et
        assert rel(R.iso_K(c, e, et, E, NU, single=False), g["K_multi"]) == 0.0, et
        for q in range(p.shape[0]):
            dN = R.DN[et](*[float(v) for v in p[q]])
            assert rel(R.iso_jacobian(c, e, dN), g["J"][q]) < 1e-15
            assert rel(R.iso_gradients(c, e, dN), g["grads"][q]) < 1e-14
        if et == "c3d8":   # compute_hexahedral_volumes (`solver/element.py:1248-1291`)
            assert rel(R.hex_volumes(c, e), g["vol"]) == 0.0
        if et == "c3d6":
            assert rel(R.wedge_volumes(c, e), g["vol"]) < 1e-15


def test_poisson_derivation_and_solve():
    g = load_golden("poisson_tet4_n4_jit")
    c, t = g["coords"], g["tets"]
    assert rel(R.tet4_poisson_K(c, t), g["KP"]) == 0.0
    u, n, _ = R.pcg(g["KP"], t, g["f"].view(-1, 1), g["dinv"].view(-1, 1), tol=float(g["tol"]))
    assert n == int(g["n_pcg"]) and rel(u[:, 0], g["u"]) < 1e-14
    assert rel(R.nodal_forces(g["KP"], t, g["p"].view(-1, 1))[:, 0], g["y"]) < 1e-14


def test_static_structure_mixed():
    g = load_golden("mixed_static")
    u, n, s = R.static_structure(g["coords"], g["force"], g["fixed"],
                                 {"c3d4": g["c3d4"], "c3d6": g["c3d6"], "c3d8": g["c3d8"]}, E, NU, tol=1e-6,
                                 max_iter=3000)
    assert s == "converged" and n == int(g["n_iter"]) and rel(u, g["u"]) == 0.0


def test_coo_coalesce_equals_ebe_and_partition_maps():
    g = load_golden("tet4_cube_n4_jit")
    K, t, p = g["K"], g["tets"], g["p"]
    rp, ci, v = R.coo_to_csr(K, t, 3)
    y = R.csr_matvec(rp, ci, v, p.reshape(-1)).view(-1, 3)
    assert rel(y, g["y"]) < 1e-14
    rpn, cin = R.node_pattern(t, g["coords"].shape[0])
    # the dof pattern is the node pattern expanded by 3x3 blocks
    assert int(rp[-1]) == 9 * int(rpn[-1])
    pr = load_golden("partition_ref")
    for k in range(4):
        nodes, loc = R.partition_local_maps(pr["tets"], pr[f"ids{k}"])
        assert torch.equal(nodes, pr[f"nodes{k}"]) and torch.equal(loc, pr[f"local{k}"])


def constrained_fixture():
    import json
    g = load_golden("constrained_tet4")
    return g, json.loads(str(g["constraints"]))


def test_constrained_cg_oracle_matches_reference():
    """`constrained_conjugate_gradient_solver` (RBE2 plate + SPC with a prescribed value) and
    `new_constrained_conjugate_gradient_solver` (SPC, RBE2, weighted RBE3 sets, nodal loads)."""
    g, c = constrained_fixture()
    K = R.tet4_K(g["coords"], g["tets"], E, NU)
    tol = float(g["tol"])
    u, n, s = R.constrained_cg(K, g["tets"], g["F"], c["rbe2_a"], c["spc"], tol=tol, max_iter=3000)
    assert s == "converged" and n == int(g["n_iter_a"]) and rel(u, g["u_a"]) == 0.0
    Fb = R.loads_to_F(g["coords"].shape[0], c["loads_b"])
    u, n, s = R.constrained_cg(K, g["tets"], Fb, c["rbe2_b"], c["spc"], c["rbe3_b"], tol=tol, max_iter=3000)
    assert s == "converged" and n == int(g["n_iter_b"]) and rel(u, g["u_b"]) == 0.0


def test_stress_recovery_oracle_matches_reference():
    """compute_*_element_stress / compute_node_vm_stress / surface + shared-face forces (§8(f) row 2)."""
    s = load_golden("stress")
    g = load_golden("tet4_cube_n4_jit")
    c, t = g["coords"], g["tets"]
    sig, vm = R.tet4_stress(c, t, g["u_cg"], E, NU)
    assert rel(sig, s["c3d4_sig"]) == 0.0 and rel(vm, s["c3d4_vm"]) == 0.0
    assert rel(R.node_average(t, vm, c.shape[0]), s["c3d4_node_vm"]) == 0.0
    assert rel(R.face_forces(s["normals"], sig), s["face_forces"]) == 0.0
    assert rel(R.shared_face_sum(s["shared_idx"], s["face_forces"]), s["shared_sum"]) == 0.0
    T = R.stress_tensor(s["voigt"])
    assert rel(T, s["voigt_tensor"]) == 0.0 and rel(R.von_mises(T), s["voigt_vm"]) == 0.0
    for et in ("c3d8", "c3d6", "c3d10"):
        cg = load_golden(f"{et}_cells")
        cc, ce, u = cg["coords"], cg["elements"], s[f"{et}_u"]
        s1, v1 = R.iso_stress(cc, ce, u, et, E, NU, single=True)
        s0, v0 = R.iso_stress(cc, ce, u, et, E, NU, single=False)
        assert rel(s1, s[f"{et}_sig1"]) < 1e-15 and rel(v1, s[f"{et}_vm1"]) < 1e-15, et
        assert rel(s0, s[f"{et}_sig0"]) < 1e-15 and rel(v0, s[f"{et}_vm0"]) < 1e-15, et
        assert rel(R.node_average(ce, s[f"{et}_vm1"], cc.shape[0]), s[f"{et}_node_vm"]) == 0.0, et


def test_topology_oracle_matches_reference():
    """Surface faces / normals, shared faces, edges and element splits (§8(f) row 3)."""
    from fem355 import topology as T
    g = load_golden("topology")
    c, t = g["tet_coords"], g["tets"]
    f, x = R.boundary_faces(t, T.TET_SURFACE, T.TET_SURFACE_X)
    assert torch.equal(f, g["tet_surf"]) and torch.equal(x, g["tet_surf_x"])
    assert rel(R.surface_normals(c, f, x, 2), g["tet_surf_n"]) == 0.0
    assert rel(R.element_face_normals(c, t, T.TET_SHARED, T.TET_SHARED, T.TET_SHARED_X, scale=0.5),
               g["tet_area_n"]) == 0.0
    assert torch.equal(R.shared_faces(t, T.TET_SHARED), g["tet_shared"])
    assert torch.equal(R.unique_edges(t, T.EDGES), g["tet_edges"])
    ch, h = g["hex_coords"], g["hexes"]
    f, x = R.boundary_faces(h, T.HEX, T.HEX_SURFACE_X)
    assert torch.equal(f, g["hex_surf"]) and torch.equal(x, g["hex_surf_x"])
    assert rel(R.surface_normals(ch, f, x, 2), g["hex_surf_n"]) == 0.0
    rows = [[r[0], r[1], r[3]] for r in T.HEX]
    assert rel(R.element_face_normals(ch, h, T.HEX, rows, T.HEX_AREA_X), g["hex_area_n"]) == 0.0
    assert torch.equal(R.shared_faces(h, T.HEX), g["hex_shared"])
    cw, w = g["wedge_coords"], g["wedges"]
    fq, xq = R.boundary_faces(w, T.WEDGE_QUAD, T.WEDGE_QUAD_X)
    ft, xt = R.boundary_faces(w, T.WEDGE_TRI, T.WEDGE_TRI_X)
    assert torch.equal(fq, g["wedge_surf_q"]) and torch.equal(ft, g["wedge_surf_t"])
    assert torch.equal(xq, g["wedge_surf_xq"]) and torch.equal(xt, g["wedge_surf_xt"])
    assert rel(R.surface_normals(cw, fq, xq, 3), g["wedge_surf_nq"]) == 0.0
    assert rel(R.surface_normals(cw, ft, xt, 2), g["wedge_surf_nt"]) == 0.0
    assert torch.equal(R.split_elements(h, T.SPLIT[8]), g["hex_tets"])
    assert torch.equal(R.split_elements(w, T.SPLIT[6]), g["wedge_tets"])
    assert torch.equal(R.split_elements(g["tet10"], T.SPLIT[10]), g["tet10_tets"])
