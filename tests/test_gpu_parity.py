"""Tier 2/3 (GPU): the HIP path through the C-ABI against the oracle and the reference's golden vectors.

Tolerances (fp64): element quantities 1e-12 relative (closed-form vs LU rounding), operators 1e-12, solutions
1e-10 relative with iteration counts within ±2 of the reference (SURVEY §8(c) contract); integer patterns
bit-exact."""
import pytest
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64 = torch.float64


def CAPI():
    from fem355 import _capi
    return _capi


C_MODE = {"cg": 0, "pcg": 1}


def _mods():
    import fem355  # noqa: F401
    from fem355 import element, mesh, solver, system
    return element, mesh, solver, system


# ------------------------------------------------------------------ L1 element kernels
def test_tet4_element_matrices_vs_golden(gpu):
    el, *_ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    c, t = g["coords"], g["tets"]
    assert rel(el.compute_tetrahedral_volumes(c, t, device=gpu, dtype=F64), g["V"]) < 1e-13
    assert rel(el.compute_c3d4_B_matrix(c, t, device=gpu, dtype=F64), g["B"]) < 1e-12
    assert rel(el.compute_c3d4_K_matrix(c, t, E, NU, device=gpu, dtype=F64), g["K"]) < 1e-12
    assert rel(el.compute_K_matrix(c, t, "C3D4", E, NU, device=gpu, dtype=F64), g["K"]) < 1e-12
    # reference default dtype (float32 output) still computed in fp64
    K32 = el.compute_c3d4_K_matrix(c, t, E, NU, device=gpu)
    assert K32.dtype == torch.float32 and rel(K32, g["K"]) < 1e-6


def test_poisson_and_mass_element_matrices(gpu):
    el, mesh, *_ = _mods()
    g = load_golden("poisson_tet4_n4_jit")
    assert rel(el.compute_c3d4_poisson_K_matrix(g["coords"], g["tets"], device=gpu, dtype=F64), g["KP"]) < 1e-12
    c, t = mesh.kuhn_cube(3, jitter=0.1)
    Mm = el.compute_c3d4_M_matrix(c, t, 4.47e-3, device=gpu, dtype=F64).cpu()
    # parity unpinned (no reference source): check total mass and symmetry
    assert abs(float(Mm.sum()) / 3 - 4.47e-3) < 1e-15 and rel(Mm, Mm.transpose(1, 2)) == 0.0


@pytest.mark.parametrize("etype", ["c3d8", "c3d6", "c3d10"])
def test_isoparametric_mass_matrices(gpu, etype):
    """Consistent mass of c3d8 / c3d6 / c3d10 (BASELINE configs[4] "mass+stiffness"; no reference function: parity
    unpinned): the GPU kernel equals the oracle's restatement of the same rule to 1e-13 on jittered meshes, totals
    rho x volume, and assembled into the bs = 3 global matrix it equals the element-by-element product."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    rho = 4.47e-3
    c, t = gen(3, jitter=0.1)
    Me = el.compute_M_matrix(c, t, etype.upper(), rho, device=gpu, dtype=F64)
    pts, wts = el.mass_integration_points(etype)
    ref = R.iso_mass(c, t, el._N[etype], el._ISO[etype][1], pts, wts, rho)
    assert rel(Me, ref) < 1e-13
    assert el.compute_M_matrix(c, t, etype, rho, device=gpu).dtype == torch.float32
    cu, tu = gen(3)
    assert abs(float(el.compute_M_matrix(cu, tu, etype, rho, device=gpu, dtype=F64).sum()) / 3 - rho) < 1e-15
    N = c.shape[0]
    g = system.build_graph(t.to(gpu), N)
    A = system.SellMatrix(g, 3).add_element_matrices(Me, t.to(gpu))
    x = torch.randn(N * 3, dtype=F64, generator=torch.Generator().manual_seed(7))
    assert rel(A.matvec(x.to(gpu)), R.nodal_forces(ref, t, x.view(N, 3)).reshape(-1)) < 1e-13
    with pytest.raises(ValueError):
        el.compute_M_matrix(c, t, "c3d20", rho, device=gpu)


def test_singular_element_raises(gpu):
    el, *_ = _mods()
    c = torch.tensor([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]], dtype=F64)
    t = torch.tensor([[0, 1, 2, 3]])
    with pytest.raises(ValueError, match="Singular matrix"):
        el.compute_c3d4_K_matrix(c, t, E, NU, device=gpu)
    with pytest.raises(ValueError, match="Unsupported element type"):
        el.compute_K_matrix(c, t, "c3d15", E, NU, device=gpu)


@pytest.mark.parametrize("etype", ["c3d8", "c3d6", "c3d10"])
def test_isoparametric_vs_golden(gpu, etype):
    el, *_ = _mods()
    g = load_golden(f"{etype}_cells")
    c, e = g["coords"], g["elements"]
    K1 = el.compute_K_matrix(c, e, etype, E, NU, single=True, device=gpu, dtype=F64)
    K0 = el.compute_K_matrix(c, e, etype, E, NU, single=False, device=gpu, dtype=F64)
    assert rel(K1, g["K_single"]) < 1e-12
    assert rel(K0, g["K_multi"]) < 1e-12
    fn = {"c3d8": (el.compute_c3d8_Jacobian, el.compute_c3d8_shape_gradients, el.compute_c3d8_B_matrix),
          "c3d6": (el.compute_c3d6_Jacobian, el.compute_c3d6_shape_gradients, el.compute_c3d6_B_matrix),
          "c3d10": (el.compute_c3d10_Jacobian, el.compute_c3d10_shape_gradients, el.compute_c3d10_B_matrix)}[etype]
    for q in range(g["points"].shape[0]):
        ip = g["points"][q]
        assert rel(fn[0](c, e, ip, device=gpu, dtype=F64), g["J"][q]) < 1e-13
        assert rel(fn[1](c, e, ip, device=gpu, dtype=F64), g["grads"][q]) < 1e-12
        assert rel(fn[2](c, e, ip, device=gpu, dtype=F64), g["B"][q]) < 1e-12
    if etype == "c3d6":
        assert rel(el.compute_wedge_volumes(c, e, device=gpu, dtype=F64), g["vol"]) < 1e-13
    if etype == "c3d8":   # compute_hexahedral_volumes (`solver/element.py:1248-1291`), both orientations
        v = el.compute_hexahedral_volumes(c, e, device=gpu, dtype=F64)
        assert v.shape == (e.shape[0],) and rel(v, g["vol"]) < 1e-13
        assert el.compute_hexahedral_volumes(c, e, device=gpu).dtype == torch.float32   # the reference's default


@pytest.mark.parametrize("etype,n", [("c3d8", 7), ("c3d6", 6), ("c3d10", 4)])
def test_packed_symmetric_ke_assembly(gpu, etype, n, monkeypatch):
    """configs[4]'s internal path: K_e stored as its upper 3x3 blocks only
    (`element._solid_ke_sym`, include/fem355.h fem_iso_ke_sym) equals compute_K_matrix's upper blocks bit for bit, and
    the global matrix assembled from it (lower blocks read as transposes) equals the one assembled from the full K_e:
    bit for bit for c3d10 (whose full K_e mirrors its upper blocks), to 1e-14 for c3d8 / c3d6 (their lower blocks are
    formed directly, rounding in another order) -- stored first, then added on top, in the solver layout and in the
    plain planes."""
    el, mesh, _, system = _mods()
    from fem355 import _capi as C
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, e = gen(n, jitter=0.1)
    c, e = c.to(gpu), e.to(gpu)
    npe = e.shape[1]
    K = el.compute_K_matrix(c, e, etype, E, NU, device=gpu, dtype=F64)
    Kp = el._solid_ke_sym(c, e, etype, E, NU, device=gpu)
    stride = int(C.lib().fem_ke_sym_stride(npe))
    assert Kp.shape == (e.shape[0], stride) and stride == (9 * npe * (npe + 1) // 2 + 1) // 2 * 2
    blocks = [(a, b) for a in range(npe) for b in range(a, npe)]
    up = torch.stack([K[:, 3 * a:3 * a + 3, 3 * b:3 * b + 3].reshape(-1, 9) for a, b in blocks], 1).reshape(-1, 9 * len(blocks))
    assert torch.equal(Kp[:, :up.shape[1]], up)
    assert not Kp[:, up.shape[1]:].any()
    g = system.build_graph(e, c.shape[0])
    for sl in ("1", "0"):
        monkeypatch.setenv("FEM355_SL", sl)
        Af = system.SellMatrix(g, 3).add_element_matrices(K, e)
        As = system.SellMatrix(g, 3).add_element_matrices_sym(Kp, e)
        assert Af.solver_layout == As.solver_layout == (sl == "1")
        for step in range(2):
            vf, vs = Af.plain_values(), As.plain_values()
            if etype == "c3d10":
                assert torch.equal(vf, vs), (sl, step)
            else:
                assert rel(vs, vf) < 1e-14, (sl, step)
            Af.add_element_matrices(K, e)
            As.add_element_matrices_sym(Kp, e)


@pytest.mark.parametrize("etype,n", [("c3d8", 7), ("c3d6", 6), ("c3d10", 4), ("c3d10", 9)])
def test_fused_stiffness_mass_assembly(gpu, etype, n, monkeypatch):
    """configs[4]'s one-pass stiffness + mass assembly (include/fem355.h fem_assemble_from_ke_mass_sl,
    `SellMatrix.add_stiffness_and_mass`): the bs = 3 stiffness (solver layout) and the bs = 1 mass factor (plain
    planes) of one pass equal the two separate tile assemblies bit for bit -- stored fresh, then added on top; an
    element listing a node twice takes the ordered branch in both; FEM355_KM_SPLIT=1 runs the two calls and gives
    the same bits."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, e = gen(n, jitter=0.1)
    if n == 4:   # one element repeats a node (a degenerate element: its values are summed in (b) order)
        e = e.clone()
        e[3, 1] = e[3, 0]
    c, e = c.to(gpu), e.to(gpu)
    K = el.compute_K_matrix(c, e, etype, E, NU, device=gpu, dtype=F64)
    Me = el.compute_M_matrix(c, e, etype, 7850.0, device=gpu, dtype=F64, scalar=True)
    g = system.build_graph(e, c.shape[0])

    def bits(A):   # NaN-safe bit comparison (a degenerate element's K_e is not finite)
        return A.plain_values().view(torch.int64)

    for steps in (1, 2):   # stored fresh; stored, then added (no read in between: both calls fused)
        Ks, Ms = system.SellMatrix(g, 3), system.SellMatrix(g, 1)
        Kf, Mf = system.SellMatrix(g, 3), system.SellMatrix(g, 1)
        Kx, Mx = system.SellMatrix(g, 3), system.SellMatrix(g, 1)
        for _ in range(steps):
            Ks.add_element_matrices(K, e)
            Ms.add_element_matrices(Me, e)
            Kf.add_stiffness_and_mass(K, Me, e, Mf)
            assert Kf.solver_layout and Mf._plain_ok and not Mf.solver_layout   # the fused call ran
            with monkeypatch.context() as mp:
                mp.setenv("FEM355_KM_SPLIT", "1")
                Kx.add_stiffness_and_mass(K, Me, e, Mx)
        assert Kf.solver_layout == Ks.solver_layout
        assert torch.equal(bits(Kf), bits(Ks)), steps
        assert torch.equal(bits(Mf), bits(Ms)), steps
        assert torch.equal(bits(Kx), bits(Ks)) and torch.equal(bits(Mx), bits(Ms))
        assert float(Mf.plain_values().sum()) > 0.0
        if steps == 1:   # against the independent forms: column-owner K (FEM355_KE_COLS), wave-per-row mass
            with monkeypatch.context() as mp:
                mp.setenv("FEM355_KE_COLS", "1")
                assert torch.equal(bits(system.SellMatrix(g, 3).add_element_matrices(K, e)), bits(Ks))
            with monkeypatch.context() as mp:
                mp.setenv("FEM355_KE_ROWS", "1")
                assert torch.equal(bits(system.SellMatrix(g, 1).add_element_matrices(Me, e)), bits(Ms))


# ------------------------------------------------------------------ L2 operators
def test_ebe_operator_vs_golden(gpu):
    el, *_ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    y = el.compute_nodal_forces(g["K"], g["tets"], g["p"], device=gpu, dtype=F64)
    assert y.device.type == "cuda" and rel(y, g["y"]) < 1e-13
    g6 = load_golden("tet4_cube_n6")
    K6 = el.compute_c3d4_K_matrix(g6["coords"], g6["tets"], E, NU, device=gpu, dtype=F64)
    assert rel(el.compute_nodal_forces(K6, g6["tets"], g6["p"], device=gpu, dtype=F64), g6["y"]) < 1e-12
    # device="cpu" is served by the GPU and handed back on the host
    ycpu = el.compute_nodal_forces(g["K"], g["tets"], g["p"], device="cpu", dtype=F64)
    assert ycpu.device.type == "cpu" and rel(ycpu, g["y"]) < 1e-13


def test_pattern_bit_exact_vs_oracle(gpu):
    _, mesh, _, system = _mods()
    for (c, t) in (mesh.kuhn_cube(5, jitter=0.1), mesh.hex_box(4), mesh.wedge_box(3), mesh.tet10_cube(2)):
        N = c.shape[0]
        gph = system.build_graph(t.to(gpu), N)
        rp, ci = R.node_pattern(t, N)
        assert torch.equal(gph.rowptr.cpu().long(), rp)
        assert torch.equal(gph.colidx.cpu().long(), ci)
        # diagonal positions point at the diagonal
        rows = torch.arange(N)
        assert torch.equal(gph.colidx.cpu().long()[gph.diagpos.cpu().long()], rows)
        # incidence is sorted and complete
        ip, inc = gph.inc_ptr.cpu().long(), gph.inc.cpu().long()
        assert int(ip[-1]) == t.numel()
        assert torch.equal(torch.sort(inc)[0], torch.arange(t.numel()))          # every (e, local) once
        seg = torch.repeat_interleave(torch.arange(N), ip[1:] - ip[:-1])
        same = seg[1:] == seg[:-1]
        assert bool((inc[1:][same] > inc[:-1][same]).all())                      # ascending per node
        assert torch.equal(t.reshape(-1)[inc], seg)                               # entry belongs to its node


def test_incidence_bucket_sort_equals_radix_sort(gpu, monkeypatch):
    """The incidence by the two-level bucket sort (default) is the radix sort's (FEM355_INC_RADIX) entry for entry:
    a randomly numbered cube, c3d10 elements repeated 9 times (buckets past the LDS capacity: the global path), a
    700-tet fan (one node in every element) and a mesh with unused nodes."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(9)
    perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(2))
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    _, t10 = mesh.tet10_cube(3)
    a = torch.arange(1, 701)
    fan = torch.stack([torch.zeros_like(a), a, a + 1, a + 2], 1)
    cases = [(inv[t], c.shape[0]), (t10.repeat(9, 1), int(t10.max()) + 1), (fan, 703), (t + 5, c.shape[0] + 9)]
    for el, N in cases:
        eg = el.to(gpu).contiguous()
        monkeypatch.delenv("FEM355_INC_RADIX", raising=False)
        ip1, in1 = system.incidence(eg, N)
        monkeypatch.setenv("FEM355_INC_RADIX", "1")
        ip2, in2 = system.incidence(eg, N)
        monkeypatch.delenv("FEM355_INC_RADIX", raising=False)
        assert torch.equal(ip1, ip2) and torch.equal(in1, in2), (el.shape, N)
    bad = torch.tensor([[0, 1, 2, 3], [1, 2, 3, 9]])
    with pytest.raises(IndexError):
        system.build_graph(bad.to(gpu), 5)


def test_pattern_wide_rows_vs_oracle(gpu):
    """Rows past every LDS tier: > 2048 candidates (c3d10 x9 repeats, hash tier) and > 512 unique neighbours
    (a fan of 700 tets around node 0, selection tier); bit-exact against the oracle, also through the CSR C-ABI."""
    _, mesh, _, system = _mods()
    c10, t10 = mesh.tet10_cube(3)
    a = torch.arange(1, 701)
    fan = torch.stack([torch.zeros_like(a), a, a + 1, a + 2], 1)
    fan = torch.cat([fan, torch.tensor([[5, 9, 400, 702]])])             # a short row next to the fan
    for t, N in ((t10.repeat(9, 1), c10.shape[0]), (fan, 703)):
        gph = system.build_graph(t.to(gpu), N)
        rp, ci = R.node_pattern(t, N)
        assert torch.equal(gph.rowptr.cpu().long(), rp) and torch.equal(gph.colidx.cpu().long(), ci)
        assert torch.equal(gph.colidx.cpu().long()[gph.diagpos.cpu().long()], torch.arange(N))
    assert int(rp[1] - rp[0]) == 703


def test_assembled_operator_equals_ebe_and_coo(gpu):
    el, mesh, solver, system = _mods()
    g = load_golden("tet4_cube_n4_jit")
    K, t, p = g["K"], g["tets"], g["p"]
    A = solver.assemble(K, t, g["coords"].shape[0], gpu)
    y = A.matvec(p.to(gpu).reshape(-1)).view(-1, 3)
    assert rel(y, g["y"]) < 1e-13
    # block CSR export == oracle's coalesced COO
    rp, ci, v = A.csr()
    orp, oci, ov = R.coo_to_csr(K, t, 3)
    dense = torch.zeros(3 * g["coords"].shape[0], 3 * g["coords"].shape[0], dtype=F64)
    rows = torch.repeat_interleave(torch.arange(orp.numel() - 1), orp[1:] - orp[:-1])
    dense[rows, oci] = ov
    mine = torch.zeros_like(dense)
    rpc, cic, vc = rp.cpu().long(), ci.cpu().long(), v.cpu()
    nrow = torch.repeat_interleave(torch.arange(rpc.numel() - 1), rpc[1:] - rpc[:-1])
    for a in range(3):
        for b in range(3):
            mine[3 * nrow + a, 3 * cic + b] = vc[:, a, b]
    assert rel(mine, dense) < 1e-13


def test_fused_tet4_assembly_matches_element_path(gpu):
    el, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(6, jitter=0.12)
    N = c.shape[0]
    x = torch.randn(N * 3, dtype=F64)
    for kind, bs in (("elastic", 3), ("poisson", 1)):
        A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, E if bs == 3 else 2.5, NU)
        Ke = R.tet4_K(c, t, E, NU) if bs == 3 else 2.5 * R.tet4_poisson_K(c, t)
        xx = x[: N * bs]
        y_ref = R.nodal_forces(Ke, t, xx.view(N, bs)).reshape(-1)
        assert rel(A.matvec(xx.to(gpu)), y_ref) < 1e-12, kind


def test_cols16_matches_int32_and_falls_back(gpu):
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    for kind, bs in (("poisson", 1), ("elastic", 3)):
        A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, 1.0 if bs == 1 else E, NU)
        assert A.use16
        x = torch.randn(A.n, dtype=F64, device=gpu)
        y16 = A.matvec(x)
        A.use16 = False
        y32 = A.matvec(x)
        assert torch.equal(y16, y32)     # same arithmetic, only the index encoding differs
        A.use16 = True
        assert A.algorithmic_bytes_spmv() < A.algorithmic_bytes_spmv(index_bytes=4)
    # a random node numbering on a 35,937-node mesh has |col - row| > 32767 somewhere -> int32 columns
    c, t = mesh.kuhn_cube(32)
    perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(3))
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    cp, tp = c[perm], inv[t]
    A = system.assemble_tet4_system(cp.to(gpu), tp.to(gpu), "poisson")
    assert not A.use16
    Ko = R.tet4_poisson_K(cp, tp)
    x = torch.randn(A.n, dtype=F64)
    assert rel(A.matvec(x.to(gpu)), R.nodal_forces(Ko, tp, x.view(-1, 1)).view(-1)) < 1e-12


def test_spmv_large_cube_properties(gpu):
    """Full-size check without the oracle: the assembled Laplacian annihilates constants and is symmetric
    in the bilinear sense x.Ay == y.Ax (10M-tet scale runs in bench.py; here n=60)."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(60, device=gpu)
    A = system.assemble_tet4_system(c, t, "poisson")
    one = torch.ones(A.n, dtype=F64, device=gpu)
    assert float(A.matvec(one).abs().max()) < 1e-12
    x, y = torch.randn(A.n, dtype=F64, device=gpu), torch.randn(A.n, dtype=F64, device=gpu)
    a, b = float(torch.dot(x, A.matvec(y))), float(torch.dot(y, A.matvec(x)))
    assert abs(a - b) <= 1e-12 * abs(a)
    E3 = system.assemble_tet4_system(c, t, "elastic", E, NU)
    rigid = torch.zeros(A.n_rows, 3, dtype=F64, device=gpu)
    rigid[:, 0] = 1.0
    assert float(E3.matvec(rigid.view(-1)).abs().max()) < 1e-6 * E * (1.0 / 60)


# ------------------------------------------------------------------ L3 solvers
def test_stable_cg_vs_reference(gpu, capsys):
    _, _, solver, _ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    u, res = solver.stable_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=float(g["tol"]),
                                                     device=gpu, return_info=True)
    out = capsys.readouterr().out
    assert abs(res.iterations - int(g["n_cg"])) <= 2, (res.iterations, int(g["n_cg"]))
    assert rel(u, g["u_cg"]) < 1e-10
    assert out.startswith(f"Converged after {res.iterations} iterations. Residual norm:")
    # residual contract: first iterations track the reference's history
    _, r5 = solver.stable_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=0.0, max_iter=20,
                                                    device=gpu, return_info=True)
    assert "did not converge" in capsys.readouterr().out
    assert r5.iterations == 20


def test_final_solver_is_stable_cg_without_maxiter_message(gpu, capsys):
    """`final_solver` (`solver/solver.py:231-295`): the stable CG iteration out of place; the same stop prints, none
    at max_iter (no for-else in the reference)."""
    _, _, solver, _ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    u, res = solver.final_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=float(g["tol"]), device=gpu,
                                 return_info=True)
    out = capsys.readouterr().out
    us, rs = solver.stable_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=float(g["tol"]),
                                                     device=gpu, return_info=True)
    capsys.readouterr()
    assert res.iterations == rs.iterations and torch.equal(u, us)
    assert abs(res.iterations - int(g["n_cg"])) <= 2 and rel(u, g["u_cg"]) < 1e-10
    assert out.startswith(f"Converged after {res.iterations} iterations. Residual norm:")
    _, r5 = solver.final_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=0.0, max_iter=20, device=gpu,
                                return_info=True)
    assert capsys.readouterr().out == "" and r5.iterations == 20


def test_pcg_vs_reference(gpu, capsys):
    _, _, solver, _ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    u, res = solver.preconditioned_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["Minv"], tol=1e-6,
                                                             device=gpu, dtype=F64, return_info=True)
    assert abs(res.iterations - int(g["n_pcg"])) <= 2 and rel(u, g["u_pcg"]) < 1e-10
    assert capsys.readouterr().out.strip() == f"Converged after {res.iterations} iterations."


def test_diagonal_preconditioner_quirk_and_exact(gpu):
    _, _, solver, _ = _mods()
    g = load_golden("tet4_cube_n4_jit")
    N = g["coords"].shape[0]
    Mb = solver.compute_diagonal_preconditioner(g["K"], g["tets"], N, device=gpu, dtype=F64)
    assert rel(Mb, g["Minv_bug"]) < 1e-15
    Me = solver.compute_diagonal_preconditioner(g["K"], g["tets"], N, device=gpu, dtype=F64, exact_diagonal=True)
    Mref = g["Minv"].clone()
    free = Mref != 0
    assert rel(Me[free], Mref[free]) < 1e-15


def test_unused_node_gets_zero_jacobi_weight(gpu):
    """A point no element touches (common in VTK files): its row is empty, its diagonal 0, so w = 1/0 -> inf -> 0
    as in the reference (`solver/solver.py:828-831`); the solve equals the oracle's on the same system."""
    _, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(5, jitter=0.1)
    c2 = torch.cat([c[:17], torch.tensor([[4.0, 4.0, 4.0]], dtype=c.dtype), c[17:]])   # point 17: unused
    t2 = t + (t >= 17).to(t.dtype)
    N = c2.shape[0]
    A = system.assemble_tet4_system(c2.to(gpu), t2.to(gpu), "poisson")
    assert int(A.g.diagpos[17]) == -1
    w = A.jacobi(None)
    assert float(w[17]) == 0.0 and bool(torch.isfinite(w).all())
    KP = R.tet4_poisson_K(c2, t2)
    assert rel(w, R.diag_preconditioner(KP, t2, N, dpn=1).view(-1)) < 1e-14   # sums in another order
    f, fixed = mesh.cube_poisson_case(c2)
    u, res, _ = solver.solve_tet4(c2, t2, f, fixed, kind="poisson", tol=1e-10, device=gpu)
    dinv = R.diag_preconditioner(KP, t2, N, dpn=1)
    dinv[fixed] = 0.0
    u_ref, it_ref, _ = R.pcg(KP, t2, f, dinv, tol=1e-10)
    assert abs(res.iterations - it_ref) <= 2 and rel(u, u_ref) < 1e-10
    assert float(u[17].abs().max()) == 0.0


def test_poisson_pcg_vs_reference(gpu):
    _, _, solver, _ = _mods()
    g = load_golden("poisson_tet4_n4_jit")
    u, res, A = solver.solve_tet4(g["coords"], g["tets"], g["f"].view(-1, 1), g["fixed"], kind="poisson",
                                  tol=float(g["tol"]), device=gpu)
    assert abs(res.iterations - int(g["n_pcg"])) <= 2
    assert rel(u[:, 0], g["u"]) < 1e-10


def test_static_structure_mixed_vs_reference(gpu):
    _, _, solver, _ = _mods()
    g = load_golden("mixed_static")
    u, res = solver.static_structure_solver(g["coords"], g["force"], g["fixed"], c3d4=g["c3d4"], c3d6=g["c3d6"],
                                            c3d8=g["c3d8"], material={"E": E, "nu": NU}, tol=1e-6, max_iter=3000,
                                            device=gpu, return_info=True)
    assert abs(res.iterations - int(g["n_iter"])) <= 2 and rel(u, g["u"]) < 1e-10


@pytest.mark.parametrize("sched", ["three_kernel", "default"])
def test_golden_solvers_per_schedule(gpu, sched, monkeypatch, capsys):
    """The reference-API solvers on the golden fixtures under each schedule the library can pick: the three-kernel
    schedule (0) and the default -- the persistent kernels (k_pcg_persist for bs = 1, k_pcg_persist3 for these
    bs = 3 systems, which fit on chip). Both against the reference's own outputs (`solver/solver.py:11-229`,
    `:766-812`)."""
    _, _, solver, system = _mods()
    if sched == "three_kernel":
        monkeypatch.setattr(system, "DEFAULT_SCHEDULE", {1: system.SCHED_THREE, 3: system.SCHED_THREE})
    want = system.SCHED_THREE if sched == "three_kernel" else system.SCHED_PERSIST
    g = load_golden("tet4_cube_n4_jit")
    u, res = solver.stable_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["fixed"], tol=float(g["tol"]),
                                                     device=gpu, return_info=True)
    assert res.schedule == want, res.schedule
    assert abs(res.iterations - int(g["n_cg"])) <= 2 and rel(u, g["u_cg"]) < 1e-10
    u, res = solver.preconditioned_conjugate_gradient_solver(g["K"], g["tets"], g["F"], g["Minv"], tol=1e-6,
                                                             device=gpu, dtype=F64, return_info=True)
    assert res.schedule == want, res.schedule
    assert abs(res.iterations - int(g["n_pcg"])) <= 2 and rel(u, g["u_pcg"]) < 1e-10
    m = load_golden("mixed_static")
    u, res = solver.static_structure_solver(m["coords"], m["force"], m["fixed"], c3d4=m["c3d4"], c3d6=m["c3d6"],
                                            c3d8=m["c3d8"], material={"E": E, "nu": NU}, tol=1e-6, max_iter=3000,
                                            device=gpu, return_info=True)
    assert res.schedule == want, res.schedule
    assert abs(res.iterations - int(m["n_iter"])) <= 2 and rel(u, m["u"]) < 1e-10
    p = load_golden("poisson_tet4_n4_jit")
    u, res, _ = solver.solve_tet4(p["coords"], p["tets"], p["f"].view(-1, 1), p["fixed"], kind="poisson",
                                  tol=float(p["tol"]), device=gpu)
    assert res.schedule == want, res.schedule
    assert abs(res.iterations - int(p["n_pcg"])) <= 2 and rel(u[:, 0], p["u"]) < 1e-10
    capsys.readouterr()


def test_cg_guard_breakdown(gpu, capsys):
    """pAp <= 0 on an indefinite operator (the reference's negative-definite c3d10 rule, Q2) stops at iteration 1."""
    el, mesh, solver, _ = _mods()
    c, t10 = mesh.tet10_cube(1)
    K = el.compute_c3d10_K_matrix(c, t10, E, NU, device=gpu, dtype=F64)
    F = torch.zeros(c.shape[0], 3, dtype=F64)
    F[:, 2] = -1.0
    fixed = mesh.face_nodes(c, 2, 0.0)
    u, res = solver.stable_conjugate_gradient_solver(K, t10, F, fixed, device=gpu, return_info=True)
    out = capsys.readouterr().out
    assert res.iterations == 1 and "Terminating early at iteration 1" in out
    assert float(u.abs().max()) == 0.0


@pytest.mark.parametrize("kind", ["poisson", "elastic"])
def test_fused_and_three_kernel_schedules_agree(gpu, kind):
    _, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(7, jitter=0.1)
    if kind == "poisson":
        f, fixed = mesh.cube_poisson_case(c)
    else:
        f, fixed = mesh.cube_elasticity_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, 1.0 if kind == "poisson" else E, NU)
    mask = torch.zeros((c.shape[0], A.bs), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    b = f.to(gpu).reshape(-1)
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, w=w, tol=tol, max_iter=2000, schedule=0)
    wm = (mask.view(-1) == 0).to(F64)
    c0 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=0)
    for sched in (1, 2):
        r1 = A.pcg(b, w=w, tol=tol, max_iter=2000, schedule=sched, history=True)
        assert r1.status == r0.status == 1 and abs(r1.iterations - r0.iterations) <= 1, sched
        assert rel(r1.x, r0.x) < 1e-10
        # CG mode, fixed max_iter (the fused schedule's deferred x update is applied at the end)
        c1 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=sched)
        assert c1.iterations == c0.iterations == 25 and c1.status == c0.status == 2 and rel(c1.x, c0.x) < 1e-12


def test_deferred_schedule_guard_and_graph(gpu):
    """Deferred schedule: breakdown stop on the indefinite c3d10 rule (Q2) at iteration 1, and graph replay from
    even bank parity equals plain launches."""
    el, mesh, solver, system = _mods()
    c, t10 = mesh.tet10_cube(1)
    K = el.compute_c3d10_K_matrix(c, t10, E, NU, device=gpu, dtype=F64)
    A = solver.assemble(K, t10, c.shape[0], gpu)
    F = torch.zeros(c.shape[0] * 3, dtype=F64, device=gpu)
    F[2::3] = -1.0
    fixed = mesh.face_nodes(c, 2, 0.0).to(gpu)
    w = torch.ones(c.shape[0], 3, dtype=F64, device=gpu)
    w[fixed] = 0.0
    res = A.pcg(F, w=w.view(-1), mode=0, tol=1e-10, max_iter=50, schedule=2)
    assert res.status == 3 and res.iterations == 1 and float(res.x.abs().max()) == 0.0
    c4, t4 = mesh.kuhn_cube(6)
    P = system.assemble_tet4_system(c4.to(gpu), t4.to(gpu), "poisson")
    b = torch.ones(P.n, dtype=F64, device=gpu)
    wj = P.jacobi(None)
    runs = []
    for g in (0, 4):
        run = system.PcgRunner(P, b, wj, tol=0.0, schedule=2)
        run.start()
        if g:
            run.use_graph(g)
        run.iterate(12)
        it, st, rz = run.poll()
        runs.append((it, rz, run.x.clone()))
        run.close()
    assert runs[0][0] == runs[1][0] == 12 and runs[0][1] == runs[1][1] and torch.equal(runs[0][2], runs[1][2])


def test_pcg_history_and_fixed_iterations(gpu):
    _, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(8)
    f, fixed = mesh.cube_poisson_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(A.n, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask)
    res = A.pcg(f.to(gpu), w=w, tol=0.0, max_iter=30, history=True)
    assert res.iterations == 30 and res.status == 2 and res.history.numel() == 30
    # oracle PCG with the same M_inv: the first 20 residuals agree to 1e-10
    KP = R.tet4_poisson_K(c, t)
    hist = []
    R.pcg(KP, t, f, w.cpu().view(-1, 1), tol=0.0, max_iter=30, history=hist)
    h = res.history.cpu()
    for k in range(20):
        assert abs(float(h[k]) - hist[k]) <= 1e-10 * hist[k], k


@pytest.mark.parametrize("etype,n", [("c3d8", 5), ("c3d6", 4), ("c3d10", 3)])
def test_assembly_from_element_matrices_wide_rows(gpu, etype, n):
    """Assembly from stored K_e (wave-per-row kernel) across column groups and >64 incident elements per row:
    assembled matvec == element-by-element product of the same K_e (bs=3 and the scalar bs=1 sub-block)."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, t = gen(n, jitter=0.1)
    t = t.repeat(9, 1)                      # each element nine times: rows see > 64 incident elements
    N = c.shape[0]
    K = el.compute_K_matrix(c.to(gpu), t.to(gpu), etype, E, NU, device=gpu, dtype=F64)
    g = system.build_graph(t.to(gpu), N)
    inc_ptr = g.inc_ptr.cpu()
    assert int((inc_ptr[1:] - inc_ptr[:-1]).max()) > 64
    for bs in (3, 1):
        Kb = K if bs == 3 else K[:, 0::3, 0::3].contiguous()
        A = system.SellMatrix(g, bs).add_element_matrices(Kb, t.to(gpu))
        x = torch.randn(N * bs, dtype=F64, generator=torch.Generator().manual_seed(3))
        y_ref = R.nodal_forces(Kb.cpu(), t, x.view(N, bs)).reshape(-1)
        assert rel(A.matvec(x.to(gpu)), y_ref) < 1e-12, (etype, bs)


@pytest.mark.parametrize("etype,n", [("c3d8", 4), ("c3d6", 4), ("c3d10", 3)])
def test_fresh_matrix_store_equals_zero_and_add(gpu, etype, n):
    """A fresh SellMatrix's first add_element_matrices stores every value (no memset, no read of the matrix): the
    whole value buffer -- padding entries included -- equals zeroing + adding bit for bit, for bs = 3 (block-CSR
    store path) and bs = 1 (in-place path behind a memset); a second family adds on top exactly as before."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, t = gen(n, jitter=0.1)
    tg = t.to(gpu)
    K = el.compute_K_matrix(c.to(gpu), tg, etype, E, NU, device=gpu, dtype=F64)
    Me = el.compute_M_matrix(c.to(gpu), tg, etype, 4.47e-3, device=gpu, dtype=F64)
    g = system.build_graph(tg, c.shape[0])
    for bs in (3, 1):
        Kb = K if bs == 3 else K[:, 0::3, 0::3].contiguous()
        Mb = Me if bs == 3 else Me[:, 0::3, 0::3].contiguous()
        fresh = system.SellMatrix(g, bs)
        fresh._plain_buf().fill_(float("nan"))          # garbage: every value must be written by the store pass
        fresh.add_element_matrices(Kb, tg)
        zeroed = system.SellMatrix(g, bs)
        zeroed.vals                               # zero first, then the add path
        zeroed.add_element_matrices(Kb, tg)
        assert torch.equal(fresh.vals, zeroed.vals), (etype, bs)
        fresh.add_element_matrices(Mb, tg)
        zeroed.add_element_matrices(Mb, tg)
        assert torch.equal(fresh.vals, zeroed.vals), (etype, bs, "second family")


@pytest.mark.parametrize("kind", ["poisson", "elastic"])
def test_paired_matrix_copy_is_bit_identical(gpu, kind):
    """FEM_TUNE_PAIR (16-byte-value copy: bs = 1 lane-paired, bs = 3 plane-paired layout A) keeps every row's
    summation order, so fixed-iteration PCG iterates equal the plain layout's bit for bit, in every schedule."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(9, jitter=0.1)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, 1.0 if kind == "poisson" else E, NU)
    assert A.use16
    b = torch.randn(A.n, dtype=F64, device=gpu)
    w = A.jacobi(None)
    for sched in (0, 2):
        xs = []
        for flags in (1, 3):   # FEM_TUNE_REVERSE, FEM_TUNE_REVERSE | FEM_TUNE_PAIR
            run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
            run.set_tuning(flags)
            run.start()
            run.iterate(30)
            it, _, _ = run.poll()
            assert it == 30
            xs.append(run.x.clone())
            run.close()
        assert torch.equal(xs[0], xs[1]), (kind, sched)


# ------------------------------------------------------------------ persistent schedule (csrc/pcg_persist.hpp)
def _poisson_case(system, mesh, n, gpu, jitter=0.0):
    c, t = mesh.kuhn_cube(n, jitter=jitter, device=gpu) if jitter == 0.0 else mesh.kuhn_cube(n, jitter=jitter)
    f, fixed = mesh.cube_poisson_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros(A.n, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    return A, f.to(gpu).reshape(-1).to(F64), mask


@pytest.mark.parametrize("n,jitter", [(7, 0.1), (40, 0.0)])
def test_persistent_schedule_matches_three_kernel(gpu, n, jitter):
    """Schedule 3 (single-reduction iteration in one cooperative launch) against the 3-kernel schedule: PCG to
    tolerance (iterations +-1, x 1e-10), CG mode with masked rows at fixed iterations (x 1e-12), history."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, n, gpu, jitter)
    w = A.jacobi(mask)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    assert run.effective_schedule() == 3
    run.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=0, history=True)
    r3 = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=3, history=True)
    assert r0.status == r3.status == 1 and abs(r0.iterations - r3.iterations) <= 1
    assert rel(r3.x, r0.x) < 1e-10
    k = min(r0.iterations, r3.iterations) - 1
    assert rel(r3.history[:k], r0.history[:k]) < 1e-8
    wm = (mask == 0).to(F64)
    c0 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=0)
    c3 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=3)
    assert c0.iterations == c3.iterations == 25 and c0.status == c3.status == 2 and rel(c3.x, c0.x) < 1e-12


def test_persistent_initial_guess(gpu):
    """Non-zero x0 (r0 = b - A x0 before the first launch; x carried in LDS): schedule 3 equals the 3-kernel
    schedule in PCG and CG (masked) modes."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 16, gpu, jitter=0.1)
    w = A.jacobi(mask)
    x0 = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(5)).to(gpu)
    x0[mask.bool()] = 0.0
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, x0, w=w, tol=tol, max_iter=3000, schedule=0)
    r3 = A.pcg(b, x0, w=w, tol=tol, max_iter=3000, schedule=3)
    assert r0.status == r3.status == 1 and abs(r0.iterations - r3.iterations) <= 1 and rel(r3.x, r0.x) < 1e-10
    wm = (mask == 0).to(F64)
    c0 = A.pcg(b, x0, w=wm, mode=0, tol=0.0, max_iter=30, schedule=0)
    c3 = A.pcg(b, x0, w=wm, mode=0, tol=0.0, max_iter=30, schedule=3)
    assert c0.iterations == c3.iterations == 30 and rel(c3.x, c0.x) < 1e-12


def test_persistent_chunks_are_bit_identical(gpu):
    """Chunk boundaries add no arithmetic: 4 launches of 9 iterations == one launch of 36, bit for bit, and the
    poll reports the same state; both u hand-off forms (sc1 gathers, acquire + plain gathers) agree bit for bit."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 24, gpu)
    w = A.jacobi(mask)
    outs = []
    for chunks, flags in (((36,), 15), ((9, 9, 9, 9), 15), ((36,), 11)):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
        run.set_tuning(flags)   # 15: sc1 gathers (default), 11: agent acquire + plain gathers
        run.start()
        for k in chunks:
            run.iterate(k)
        outs.append((run.poll(), run.x.clone()))
        run.close()
    assert outs[0][0] == outs[1][0] == outs[2][0] and outs[0][0][0] == 36
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][1], outs[2][1])


@pytest.mark.parametrize("kind", ["poisson", "elastic"])
def test_persistent_bad_window_is_an_error(gpu, kind):
    """A gather window outside the u-flag array (injected through the debug knob after start) is reported, not
    clamped into silently wrong iterates: the launch ends, fem_pcg_poll returns FEM_ESTATE -> FemError, and the next
    context on the same device runs normally (no fault, no hang)."""
    _, mesh, _, system = _mods()
    from fem355 import _capi as C
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    f, fixed = mesh.cube_poisson_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), kind, E=1.0, nu=0.3)
    mask = torch.zeros(A.n // A.bs, dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    if A.bs == 3:
        mask = mask.repeat_interleave(3)
    w = A.jacobi(mask)
    b = torch.ones(A.n, dtype=F64, device=gpu) * (1 - mask.to(F64))
    for lo, hi in ((0, 1 << 20), (-7, 2)):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
        run.start()
        assert run.effective_schedule() == 3
        run.debug_window(1, lo, hi)
        run.iterate(5)
        with pytest.raises(C.FemError, match="gather window"):
            run.poll()
        run.close()
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    run.iterate(5)
    assert run.poll()[:2] == (5, 0)
    run.close()


def _fixed_iterates(system, A, b, w, sched, flags, k):
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
    if flags is not None:
        run.set_tuning(flags)
    run.start()
    uni = run.uniform_slices()
    run.iterate(k)
    it, st, rz = run.poll()
    assert it == k and st == 0
    x = run.x.clone()
    run.close()
    return uni, rz, x


@pytest.mark.parametrize("case", ["kuhn", "kuhn_unused_node", "permuted"])
def test_slice_uniform_deltas_are_bit_identical(gpu, case):
    """FEM_TUNE_PK_UNI (default): slices whose rows share one sorted delta list store it once and hold zeros where
    a row lacks an offset. Every row adds the same products in the same order, so the persistent and the deferred
    schedules give the same iterates bit for bit with and without it. Kuhn cubes: every full slice qualifies (the
    partial last slice never does); an unused node (empty row) and a random node numbering (no common lists) fall
    back per slice."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(13, jitter=0.1)
    N = c.shape[0]
    if case == "kuhn_unused_node":
        c = torch.cat([c[:700], torch.tensor([[4.0, 4.0, 4.0]], dtype=c.dtype), c[700:]])
        t = t + (t >= 700).to(t.dtype)
        N += 1
    elif case == "permuted":
        perm = torch.randperm(N, generator=torch.Generator().manual_seed(11))
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(N)
        c, t = c[perm], inv[t]
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    b = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(2)).to(gpu)
    w = A.jacobi(None)
    for sched in (3, 2):
        uni, rz1, x1 = _fixed_iterates(system, A, b, w, sched, None, 40)        # defaults (PK_UNI on)
        off, rz0, x0 = _fixed_iterates(system, A, b, w, sched, 1 | 2 | 4 | 8, 40)
        nsl = (N + 63) // 64
        assert uni[1] == off[1] == nsl and off[0] == 0
        if case == "permuted":
            assert uni[0] <= nsl // 10
        elif case == "kuhn":
            # all but the slices near either end (a padded column row + delta would leave [0, N)) and the partial one
            assert nsl - 9 <= uni[0] < nsl
        else:
            assert 0 < uni[0] < nsl   # slices whose rows' offsets change at the inserted node fall back
        assert uni[2] < off[2] or uni[0] == 0
        assert torch.equal(x1, x0) and rz1 == rz0, (case, sched)


@pytest.mark.parametrize("case", ["kuhn", "kuhn_unused_node", "permuted", "wide"])
def test_solver_layout_is_bit_identical_to_plain(gpu, case, monkeypatch):
    """P1 assembly straight into the solver layout (lane-paired entries, slice-uniform delta lists
    from the pattern, the persistent schedule's gather windows formed with the pattern) against the plain SELL matrix
    whose contexts build their own paired copy at every start (FEM355_SL=0): the plain values formed back from the
    solver layout, Jacobi weights, the operator, fixed iterations of the persistent / deferred / 3-kernel schedules
    and a solve to tolerance -- all bit for bit; a second assembly added onto the first as well. Cases: Kuhn cube,
    an unused node (empty row, partial uniformity), a random numbering (no uniform slice), a fan (a 43-column row:
    the 32-column accumulator window, two sweeps)."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(13, jitter=0.1)
    N = c.shape[0]
    if case == "kuhn_unused_node":
        c = torch.cat([c[:700], torch.tensor([[4.0, 4.0, 4.0]], dtype=c.dtype), c[700:]])
        t = t + (t >= 700).to(t.dtype)
        N += 1
    elif case == "permuted":
        perm = torch.randperm(N, generator=torch.Generator().manual_seed(11))
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(N)
        c, t = c[perm], inv[t]
    elif case == "wide":   # a hub row of 43 columns: the 32-column window, two sweeps
        c, t = _helix_fan(40)
        N = c.shape[0]
    cg, tg = c.to(gpu), t.to(gpu)
    monkeypatch.setenv("FEM355_SL", "0")
    P = system.assemble_tet4_system(cg, tg, "poisson", 1.7)
    monkeypatch.delenv("FEM355_SL", raising=False)
    S = system.assemble_tet4_system(cg, tg, "poisson", 1.7)
    assert S.solver_layout and not P.solver_layout
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask[::7] = 1
    wS, wP = S.jacobi(mask), P.jacobi(mask)
    assert torch.equal(wS, wP)
    x = torch.randn(N, dtype=F64, generator=torch.Generator().manual_seed(3)).to(gpu)
    assert torch.equal(S.matvec(x), P.matvec(x))
    b = torch.randn(N, dtype=F64, generator=torch.Generator().manual_seed(2)).to(gpu)
    for sched in (3, 2, 0):
        _, rzS, xS = _fixed_iterates(system, S, b, wS, sched, None, 30)
        _, rzP, xP = _fixed_iterates(system, P, b, wP, sched, None, 30)
        assert torch.equal(xS, xP) and rzS == rzP, (case, sched)
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, wP * b)))
    rS, rP = S.pcg(b, w=wS, tol=tol, max_iter=3000), P.pcg(b, w=wP, tol=tol, max_iter=3000)
    assert rS.iterations == rP.iterations and torch.equal(rS.x, rP.x)
    assert S.solver_layout   # nothing above needed the plain copy
    assert torch.equal(S.vals, P.vals)   # the plain values formed back from the solver layout
    # adding a second assembly onto the solver layout
    S2 = system.assemble_tet4_system(cg, tg, "poisson", 1.7)
    S2.add_tet4(cg, tg, 0.3)
    monkeypatch.setenv("FEM355_SL", "0")
    P2 = system.assemble_tet4_system(cg, tg, "poisson", 1.7)
    P2.add_tet4(cg, tg, 0.3)
    assert S2.solver_layout and torch.equal(S2.vals, P2.vals)


@pytest.mark.parametrize("case", ["tet4", "tet4_permuted", "c3d8", "tet4_plus_ke"])
def test_solver_layout_elastic_is_bit_identical_to_plain(gpu, case, monkeypatch):
    """bs = 3 solver layout: the c3d4 accumulator kernel and the stored-K_e tile kernel write the
    plane-paired layout A the paired schedules read, so no start converts the matrix and one copy is resident.
    Against the plain matrix (FEM355_SL=0, whose contexts build their layout-A copy at start): Jacobi weights, the
    operator, fixed iterations of the persistent / deferred / 3-kernel schedules, a solve to tolerance and the plain
    values formed back -- bit for bit. Cases: a jittered Kuhn cube, the same renumbered at random (wide slices), a
    hexahedral box from stored K_e (stored then added; the reference's c3d10 rule is not positive definite, Q2), and c3d4 values plus the same operator's K_e added on top."""
    el, mesh, _, system = _mods()
    if case == "c3d8":
        c, t = mesh.hex_box(7, jitter=0.1)
    else:
        c, t = mesh.kuhn_cube(9, jitter=0.1)
    if case == "tet4_permuted":
        perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(11))
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel())
        c, t = c[perm], inv[t]
    N = c.shape[0]
    cg, tg = c.to(gpu), t.to(gpu)
    g = system.build_graph(tg, N)
    K = None if case.startswith("tet4") and case != "tet4_plus_ke" else \
        el.compute_K_matrix(cg, tg, "c3d8" if case == "c3d8" else "c3d4", E, NU, device=gpu, dtype=F64)

    def build():
        A = system.SellMatrix(g, 3)
        if case == "c3d8":
            A.add_element_matrices(K, tg)
            A.add_element_matrices(K, tg)
        else:
            A.add_tet4(cg, tg, E, NU)
            if K is not None:
                A.add_element_matrices(K, tg)
        return A
    monkeypatch.setenv("FEM355_SL", "0")
    P = build()
    monkeypatch.delenv("FEM355_SL", raising=False)
    S = build()
    assert S.solver_layout and not P.solver_layout
    mask = torch.zeros(3 * N, dtype=torch.uint8, device=gpu)
    mask[::11] = 1
    wS, wP = S.jacobi(mask), P.jacobi(mask)
    assert torch.equal(wS, wP)
    x = torch.randn(3 * N, dtype=F64, generator=torch.Generator().manual_seed(3)).to(gpu)
    assert torch.equal(S.matvec(x), P.matvec(x))
    b = torch.randn(3 * N, dtype=F64, generator=torch.Generator().manual_seed(2)).to(gpu)
    for sched in (3, 2, 0):
        _, rzS, xS = _fixed_iterates(system, S, b, wS, sched, None, 25)
        _, rzP, xP = _fixed_iterates(system, P, b, wP, sched, None, 25)
        assert torch.equal(xS, xP) and rzS == rzP, (case, sched)
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, wP * b)))
    rS, rP = S.pcg(b, w=wS, tol=tol, max_iter=4000), P.pcg(b, w=wP, tol=tol, max_iter=4000)
    assert rS.iterations == rP.iterations and torch.equal(rS.x, rP.x)
    assert S.solver_layout
    assert torch.equal(S.vals, P.vals)


@pytest.mark.parametrize("n,jitter", [(20, 0.1), (66, 0.0), (80, 0.05)])
def test_persistent_slot_builds_are_bit_identical(gpu, n, jitter):
    """When every wave owns at most 1 / 2 / 4 slices the persistent schedule runs a one- / two- / four-slot build with
    8 / 4 / 4 lane pairs in flight instead of the 7-slot build's 2 (n = 20: 145 slices, 1 per wave; n = 66: 4,714
    slices, 2; n = 80: 8,303 slices, 3). Only the loads in flight differ: 60 fixed iterations equal the 7-slot build's
    (FEM_TUNE_PK_WIDE) bit for bit."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(n, jitter=jitter)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    b = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(5)).to(gpu)
    w = A.jacobi(None)
    dflt = 1 | 2 | 4 | 8 | 128
    _, rz1, x1 = _fixed_iterates(system, A, b, w, 3, dflt, 60)
    _, rz0, x0 = _fixed_iterates(system, A, b, w, 3, dflt | 256, 60)   # FEM_TUNE_PK_WIDE
    assert torch.equal(x1, x0) and rz1 == rz0, n


def test_persistent_full_geometry_10m(gpu):
    """The 10M-tet bench system (27,000 slices: 6-7 slots per wave, every register slot and the LDS v slots in use):
    50 fixed iterations equal the deferred schedule's to 1e-12; a solve to tolerance stops mid-launch at the
    same iteration count."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 119, gpu)
    w = A.jacobi(mask)
    xs = []
    for sched in (2, 3):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
        run.start()
        assert run.effective_schedule() == sched
        run.iterate(50)
        it, st, rz = run.poll()
        assert it == 50 and st == 0
        xs.append((rz, run.x.clone()))
        run.close()
    assert rel(xs[1][1], xs[0][1]) < 1e-12 and abs(xs[1][0] - xs[0][0]) <= 1e-10 * abs(xs[0][0])
    # the u hand-off through an agent acquire + plain gathers (FEM_TUNE_PK_SC1 off) gives the same bits
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.set_tuning(1 | 2 | 8)   # REVERSE | PAIR | PK_PACK, without PK_SC1
    run.start()
    run.iterate(50)
    assert run.poll()[0] == 50 and torch.equal(run.x, xs[1][1])
    run.close()
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    r2 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=2)
    r3 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=3)
    assert r2.status == r3.status == 1 and abs(r2.iterations - r3.iterations) <= 1 and rel(r3.x, r2.x) < 1e-10


def test_persistent_overflow_past_register_capacity(gpu):
    """A 13.2M-tet mesh (2.25M rows: more than 7 slices per wave): the overflow build keeps the rows past the register
    slots in HBM inside the same launch; fixed iterations equal the deferred schedule's to 1e-12, a solve to
    tolerance stops at the same iteration."""
    _, mesh, _, system = _mods()
    A, b, mask = _poisson_case(system, mesh, 130, gpu)
    w = A.jacobi(mask)
    xs = []
    for sched in (2, 3):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=sched)
        run.start()
        assert run.effective_schedule() == sched
        run.iterate(30)
        assert run.poll()[0] == 30
        xs.append(run.x.clone())
        run.close()
    assert rel(xs[1], xs[0]) < 1e-12
    tol = 1e-8 * float(torch.sqrt(torch.dot(b, w * b)))
    r2 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=2)
    r3 = A.pcg(b, w=w, tol=tol, max_iter=3000, schedule=3)
    assert r2.status == r3.status == 1 and abs(r2.iterations - r3.iterations) <= 1 and rel(r3.x, r2.x) < 1e-10


def test_persistent_falls_back_and_guards(gpu):
    """bs = 3 runs the persistent schedule when asked (3) and by default while its state fits on chip (auto, 4); a
    guard stop (CG breakdown on the scalar block of the indefinite c3d10 rule) reports the same status and
    iteration as the 3-kernel schedule."""
    el, mesh, solver, system = _mods()
    c, t = mesh.kuhn_cube(6)
    Ael = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", E, NU)
    for sched in (3, None):
        run = system.PcgRunner(Ael, torch.ones(Ael.n, dtype=F64, device=gpu), Ael.jacobi(None), tol=0.0,
                               schedule=sched)
        run.start()
        assert run.effective_schedule() == 3, sched
        run.close()
    c10, t10 = mesh.tet10_cube(1)
    K = el.compute_c3d10_K_matrix(c10, t10, E, NU, device=gpu, dtype=F64)[:, 0::3, 0::3].contiguous()
    g = system.build_graph(t10.to(gpu), c10.shape[0])
    A = system.SellMatrix(g, 1).add_element_matrices(K, t10.to(gpu))
    F = -torch.ones(A.n, dtype=F64, device=gpu)
    fixed = mesh.face_nodes(c10, 2, 0.0).to(gpu)
    wv = torch.ones(A.n, dtype=F64, device=gpu)
    wv[fixed] = 0.0
    res = [A.pcg(F, w=wv, mode=0, tol=1e-10, max_iter=50, schedule=s) for s in (0, 3)]
    assert res[0].status == res[1].status and res[0].iterations == res[1].iterations
    assert rel(res[1].x, res[0].x) < 1e-10 or float(res[0].x.abs().max()) == float(res[1].x.abs().max()) == 0.0


@pytest.mark.parametrize("etype,n,rep", [("c3d8", 5, 1), ("c3d6", 4, 1), ("c3d10", 4, 1), ("c3d10", 3, 9)])
def test_element_row_assembly_bit_identical_to_column_form(gpu, etype, n, rep, monkeypatch):
    """bs = 3 assembly from stored K_e: the tile kernel (k_assemble_ke_tile3, default), the element-row kernel
    (k_assemble_ke_rows3 + block-CSR buffer, FEM355_KE_ROWS; its direct-SELL variant FEM355_KE_SELLW) and the
    column-owner kernel (k_assemble_ke_w, FEM355_KE_COLS) give the same SELL values bit for bit, stored and added -- also with every element
    repeated (rows past 64 incident elements and past the 64-column window) and with a node listed twice in one
    element (the ordered duplicate path)."""
    el, mesh, _, system = _mods()
    gen = {"c3d8": mesh.hex_box, "c3d6": mesh.wedge_box, "c3d10": mesh.tet10_cube}[etype]
    c, t = gen(n, jitter=0.1)
    t = t.repeat(rep, 1)
    K = el.compute_K_matrix(c.to(gpu), t.to(gpu), etype, E, NU, device=gpu, dtype=F64)
    if rep == 1:   # assembled over a connectivity where element 3 lists its first node twice
        t = t.clone()
        t[3, -1] = t[3, 0]
    tg = t.to(gpu)
    g = system.build_graph(tg, c.shape[0])
    if rep > 1:
        rp = g.rowptr.cpu()
        assert int((rp[1:] - rp[:-1]).max()) > 64 or int((g.inc_ptr[1:] - g.inc_ptr[:-1]).max()) > 64
    def fresh(twice=False):
        A = system.SellMatrix(g, 3)
        A._plain_buf().fill_(float("nan"))   # a fresh matrix is stored whole: no entry may be left unwritten
        A.add_element_matrices(K, tg)
        if twice:                     # and adding onto stored values
            A.add_element_matrices(K, tg)
        return A.vals.clone()
    for v in ("FEM355_KE_COLS", "FEM355_KE_ROWS", "FEM355_KE_SELLW"):
        monkeypatch.delenv(v, raising=False)
    a, a2 = fresh(), fresh(True)          # tile form (default: rows of a slice together, straight into SELL)
    monkeypatch.setenv("FEM355_KE_ROWS", "1")       # element-row form + block-CSR buffer + slice pass
    r, r2 = fresh(), fresh(True)
    monkeypatch.setenv("FEM355_KE_SELLW", "1")      # element-row form, row sums straight into the SELL planes
    d = fresh()
    monkeypatch.delenv("FEM355_KE_SELLW", raising=False)
    monkeypatch.delenv("FEM355_KE_ROWS", raising=False)
    monkeypatch.setenv("FEM355_KE_COLS", "1")       # column-owner form
    b = fresh()
    monkeypatch.delenv("FEM355_KE_COLS", raising=False)
    monkeypatch.setenv("FEM355_SL", "0")            # tile form into the plain planes instead of the solver layout
    p, p2 = fresh(), fresh(True)
    assert torch.equal(a, b) and torch.equal(a, r) and torch.equal(a, d) and torch.equal(a2, r2), etype
    assert torch.equal(a, p) and torch.equal(a2, p2), etype


@pytest.mark.parametrize("kind,mode,small", [("elastic", "cg", False), ("elastic", "pcg", False),
                                             ("poisson", "pcg", False), ("elastic", "pcg", True),
                                             ("elastic", "cg", True)])
def test_merged_update_matches_two_kernel_update(gpu, kind, mode, small):
    """3-kernel schedule: the merged r/z + x/p update (k_pcg_update2, FEM_TUNE_UPD1, default) against the two
    vector kernels it replaces, on an odd number of dofs (the scalar tail), stable CG with its history and PCG: same
    stop, iterations +-1, x 1e-12, the first 20 residual norms 1e-12 (p = z + beta p rounds z first, so the bits may
    differ). small: the merged update's grid capped at 8 workgroups (FEM_TUNE_U2_SMALL) on a 50,625-dof system, so
    its loops past the register-cached z (n/2 > 8 x 256 x 8) run as well."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(24 if small else 10, jitter=0.1)   # 15,625 / 1,331 nodes: n odd for both kinds
    N = c.shape[0]
    if kind == "elastic":
        f, fixed = mesh.cube_elasticity_case(c)
        A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", E, NU)
    else:
        f, fixed = mesh.cube_poisson_case(c)
        A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "poisson")
    mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    if mode == "cg":
        w = (w != 0).to(F64)   # CG_STABLE: w is the 0/1 free mask
    md = C_MODE[mode]
    b = f.reshape(-1).to(gpu, F64)
    tol = 1e-9 * float(torch.linalg.norm(b))
    tn0 = CAPI().TUNE_DEFAULT | (CAPI().TUNE_U2_SMALL if small else 0)
    runs = [A.pcg(b, w=w, mode=md, tol=tol, max_iter=5000, history=True, schedule=0, tune=tn)
            for tn in (tn0, CAPI().TUNE_DEFAULT & ~CAPI().TUNE_UPD1)]
    a, o = runs
    assert A.n % 2 == 1 and a.schedule == 0 and o.schedule == 0
    assert not small or A.n // 2 > 8 * 256 * 8
    assert a.status == o.status == CAPI().PCG_CONVERGED and abs(a.iterations - o.iterations) <= 1
    assert rel(a.x, o.x) < 1e-12
    assert rel(a.history[:20], o.history[:20]) < 1e-12


def test_merged_update_give_up_is_all_or_nothing(gpu):
    """a merged-update launch whose wait gives up must end with FEM_PCG_SYNC_TIMEOUT, the give-up
    site 4 (+ 16 x launch) and NO workgroup's x update -- also when the late workgroup arrives afterwards and finishes
    r.z (FEM_TUNE_U2_HOLD holds workgroup 0 back past every other workgroup's 2 s wait). fem_pcg_solve then re-solves
    from x0 with the two-kernel update: the same result as a solve without the merged update."""
    import ctypes
    _, mesh, _, system = _mods()
    cap = CAPI()
    c, t = mesh.kuhn_cube(12, jitter=0.1)
    N = c.shape[0]
    f, fixed = mesh.cube_elasticity_case(c)
    A = system.assemble_tet4_system(c.to(gpu), t.to(gpu), "elastic", E, NU)
    mask = torch.zeros((N, 3), dtype=torch.uint8, device=gpu)
    mask[fixed.to(gpu)] = 1
    w = A.jacobi(mask.view(-1))
    b = f.reshape(-1).to(gpu, F64)
    x0 = torch.randn(A.n, dtype=F64, generator=torch.Generator().manual_seed(5)).to(gpu)
    run = system.PcgRunner(A, b, w, x0=x0, tol=0.0, schedule=0)
    try:
        run.set_tuning(cap.TUNE_DEFAULT | cap.TUNE_U2_HOLD)
        run.start()
        run.iterate(3)
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        cap.check(run.lib.fem_pcg_poll(run.h, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)), "poll")
        site = ctypes.c_int()
        cap.check(run.lib.fem_pcg_sync_site(run.h, ctypes.byref(site)), "site")
        assert stt.value == cap.PCG_SYNC_TIMEOUT and it.value == 0, (it.value, stt.value)
        assert site.value == 4 + 16 * 1, site.value
        assert torch.equal(run.x, x0)            # nobody applied x += alpha p
    finally:
        run.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    held = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=0, tune=cap.TUNE_DEFAULT | cap.TUNE_U2_HOLD)
    plain = A.pcg(b, w=w, tol=tol, max_iter=5000, schedule=0, tune=cap.TUNE_DEFAULT & ~cap.TUNE_UPD1)
    assert held.status == plain.status == cap.PCG_CONVERGED and held.iterations == plain.iterations
    assert torch.equal(held.x, plain.x)


def _helix_fan(m):
    """m non-degenerate tets [0, a, a+1, a+2] around node 0 (a row of m + 3 columns) on a helix of nodes."""
    th = torch.arange(1, m + 3, dtype=F64) * 0.3
    pts = torch.stack([torch.cos(th), torch.sin(th), 0.05 * th], 1)
    c = torch.cat([torch.zeros(1, 3, dtype=F64), pts])
    a = torch.arange(1, m + 1)
    return c, torch.stack([torch.zeros_like(a), a, a + 1, a + 2], 1)


@pytest.mark.parametrize("m,gap", [(60, 0), (60, 40000), (300, 0), (300, 40000), (32700, 0), (33000, 0)])
def test_cols16_flag_from_graph_count_matches_bandwidth(gpu, m, gap):
    """The 16-bit delta decision is taken in the node-graph count kernels (read back in the build's single sync):
    16-bit columns iff every |col - row| <= 32767, for rows in each count kernel -- hashed in registers (60-tet fan,
    63 columns), hashed in LDS (300 tets, 303 columns) and selected in memory (32,700 / 33,000 tets: bandwidth just
    under / over the limit). gap: the hub node is moved 40,000 ids away from its fan."""
    _, _, _, system = _mods()
    c, t = _helix_fan(m)
    if gap:
        c = torch.cat([c, torch.zeros(gap, 3, dtype=F64)])
        t = torch.where(t == 0, torch.full_like(t, c.shape[0] - 1), t)
        c[-1] = 0.0
    g = system.build_graph(t.to(gpu), c.shape[0], compress=True)
    rp = g.rowptr.long().cpu()
    rows = torch.repeat_interleave(torch.arange(c.shape[0]), rp[1:] - rp[:-1])
    bw = int((g.colidx.long().cpu() - rows).abs().max())
    assert (g.dcols is not None) == (bw <= 32767), (m, gap, bw)


@pytest.mark.parametrize("m,spread", [(200_000, 1), (200_000, 7)])
def test_hub_row_pattern_is_bounded_and_exact(gpu, m, spread):
    """A node shared by m = 200,000 tets (a row of 200,003 columns): the node-graph pattern's
    big-row tier (k_graph_big: an LDS bitmap of node ids per 2^20-id window, O(candidates) per window) builds it
    within a stated bound -- 10 s for the whole pattern, warm -- and the pattern equals the oracle's coalesced COO
    (`R.node_pattern`, `subdivision.ipynb:118-139`) bit for bit, diagonal positions included. spread: the fan's node
    ids multiplied by 7 (1.4M ids: two bitmap windows, int32 columns, unused nodes with empty rows)."""
    import time
    _, _, _, system = _mods()
    c, t = _helix_fan(m)
    N = c.shape[0]
    if spread > 1:
        t = t * spread
        N = (N - 1) * spread + 1
    tg = t.to(gpu)
    system.build_graph(tg[:1000], N)                  # module loads / first-use costs outside the bound
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = system.build_graph(tg, N)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert dt < 10.0, dt
    rp, ci = R.node_pattern(t, N)
    assert torch.equal(g.rowptr.long().cpu(), rp) and torch.equal(g.colidx.long().cpu(), ci)
    assert int(rp[1] - rp[0]) == m + 3
    rows = torch.repeat_interleave(torch.arange(N), rp[1:] - rp[:-1])
    dpos = torch.full((N,), -1, dtype=torch.long)
    on = ci == rows
    dpos[rows[on]] = torch.nonzero(on, as_tuple=True)[0]
    assert torch.equal(g.diagpos.long().cpu(), dpos)
    assert (g.dcols is not None) == (spread == 1 and m + 2 <= 32767)


@pytest.mark.parametrize("case", ["kuhn", "permuted", "fan", "repeated", "twice"])
def test_tile_assembly_bit_identical_to_row_kernels(gpu, case, monkeypatch):
    """c3d4 / P1 assembly straight into SELL: the accumulator kernel (k_asm_tet4_acc, default; fresh matrices stored
    whole without a memset) gives the SELL values -- padding included -- of the wave-per-row kernels
    (k_assemble_p1w / k_assemble_el3w onto a zeroed matrix, FEM355_ASM_ROWS) bit for bit, and adding a second time
    onto stored values too. Cases: a jittered cube, a randomly renumbered cube (wide slices), and a 1,500-tet fan (a
    row of 1,503 columns: the CSR segment searched in memory, many output passes), a cube whose element 3 lists a
    node twice (the ordered path for an element hitting one column twice; its entries are NaN -- the element is
    singular -- so the NaN positions and the other entries are compared and the operator check skipped) and a cube with every element listed twice (rows of ~48 incidences: several item batches)."""
    _, mesh, _, system = _mods()
    if case == "fan":
        c, t = _helix_fan(1500)
    else:
        c, t = mesh.kuhn_cube(7, jitter=0.12)
        if case == "repeated":
            t = t.clone()
            t[3, 3] = t[3, 0]
        if case == "twice":
            t = t.repeat(2, 1)
        if case == "permuted":
            perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(11))
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(perm.numel())
            c, t = c[perm], inv[t]
    cg, tg = c.to(gpu), t.to(gpu)
    g = system.build_graph(tg, c.shape[0])
    for kind, bs, Ek in (("poisson", 1, 2.5), ("elastic", 3, E)):
        out = []
        for rows in (False, True):
            if rows:
                monkeypatch.setenv("FEM355_ASM_ROWS", "1")
            else:
                monkeypatch.delenv("FEM355_ASM_ROWS", raising=False)
            A = system.SellMatrix(g, bs)
            A._plain_buf().fill_(float("nan"))    # a fresh matrix's buffer is never read by the store path
            A.add_tet4(cg, tg, Ek, NU)
            first = A.vals.clone()
            A.add_tet4(cg, tg, Ek, NU)
            out.append((first, A.vals.clone()))
        monkeypatch.delenv("FEM355_ASM_ROWS", raising=False)
        if bs == 1 and case in ("kuhn", "twice"):   # the 16-column window (max_width <= 16) vs the 32-column one
            assert 0 < g.max_width <= 16
            mw, g.max_width = g.max_width, 0
            A32 = system.SellMatrix(g, bs)
            A32.add_tet4(cg, tg, Ek, NU)
            g.max_width = mw
            assert torch.equal(A32.vals, out[0][0]), case
            del A32
        if case == "repeated":   # the singular element's entries are NaN in both (payloads may differ)
            for i in (0, 1):
                na, nb = torch.isnan(out[0][i]), torch.isnan(out[1][i])
                assert torch.equal(na, nb) and 0 < int(na.sum()) < na.numel() // 4, (kind, i)
                assert torch.equal(out[0][i][~na], out[1][i][~nb]), (kind, i)
            continue
        assert not bool(torch.isnan(out[0][0]).any())
        assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1]), (case, kind)
        Ko = R.tet4_K(c, t, E, NU) if bs == 3 else 2.5 * R.tet4_poisson_K(c, t)
        x = torch.randn(c.shape[0] * bs, dtype=F64, generator=torch.Generator().manual_seed(5))
        A.check_singular()
        y = system.SellMatrix.matvec(A, x.to(gpu))
        assert rel(y, 2 * R.nodal_forces(Ko, t, x.view(-1, bs)).reshape(-1)) < 1e-12, (case, kind)


def _elastic_case(system, mesh, n, gpu, jitter=0.1):
    c, t = mesh.kuhn_cube(n, jitter=jitter, device=gpu)
    f, fixed = mesh.cube_elasticity_case(c)
    A = system.assemble_tet4_system(c, t, "elastic", E, NU)
    mask = torch.zeros((c.shape[0], 3), dtype=torch.uint8, device=gpu)
    mask[fixed] = 1
    return A, f.reshape(-1).to(F64).contiguous(), mask.view(-1)


@pytest.mark.parametrize("n", [7, 24])
def test_persistent_elastic_matches_three_kernel(gpu, n):
    """bs = 3 persistent schedule (k_pcg_persist3: 3x3 blocks, state on chip) against the 3-kernel schedule on the
    elasticity system: PCG to tolerance (iterations +-1, x 1e-10, residual history 1e-8), CG mode with masked rows at
    fixed iterations (x 1e-12), and chunked launches continue the same iteration."""
    _, mesh, _, system = _mods()
    A, b, mask = _elastic_case(system, mesh, n, gpu)
    w = A.jacobi(mask)
    run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
    run.start()
    assert run.effective_schedule() == 3
    run.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=0, history=True)
    r3 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=3, history=True)
    assert r0.status == r3.status == 1 and abs(r0.iterations - r3.iterations) <= 1, (r0.iterations, r3.iterations)
    assert rel(r3.x, r0.x) < 1e-10
    k = min(r0.iterations, r3.iterations) - 1
    assert rel(r3.history[:k], r0.history[:k]) < 1e-8
    wm = (mask == 0).to(F64)
    c0 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=0)
    c3 = A.pcg(b, w=wm, mode=0, tol=0.0, max_iter=25, schedule=3)
    assert c0.iterations == c3.iterations == 25 and c0.status == c3.status == 2 and rel(c3.x, c0.x) < 1e-12
    # 3 launches of 10 == 1 launch of 30, bit for bit
    xs = []
    for chunks in ((30,), (10, 10, 10)):
        run = system.PcgRunner(A, b, w, tol=0.0, schedule=3)
        run.start()
        for kk in chunks:
            run.iterate(kk)
        assert run.poll()[0] == 30
        torch.cuda.synchronize()
        xs.append(run.x.clone())
        run.close()
    assert torch.equal(xs[0], xs[1])


def test_persistent_elastic_overflow(gpu):
    """Past 2 on-chip slices per wave (n = 80: 8,438 slices > 256 x 16 x 2) the overflow build streams the rest of
    each wave's slices from HBM inside the same launch: equal to the 3-kernel schedule (iterations +-1, x 1e-10)."""
    _, mesh, _, system = _mods()
    A, b, mask = _elastic_case(system, mesh, 80, gpu, jitter=0.0)
    assert (A.g.n_nodes + 63) // 64 > 256 * 16 * 2
    w = A.jacobi(mask)
    run = system.PcgRunner(A, b, w, tol=0.0)   # default (auto): past the on-chip capacity -> three-kernel
    run.start()
    assert run.effective_schedule() == 0
    run.close()
    tol = 1e-9 * float(torch.sqrt(torch.dot(b, w * b)))
    r0 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=0)
    r3 = A.pcg(b, w=w, tol=tol, max_iter=20000, schedule=3)
    assert r0.status == r3.status == 1 and abs(r0.iterations - r3.iterations) <= 1, (r0.iterations, r3.iterations)
    assert rel(r3.x, r0.x) < 1e-10


def test_empty_mesh(gpu, capsys):
    """No elements (M = 0): element matrices [0, 12, 12], a zero operator, and the stable CG stops at iteration 1 on
    p.Kp = 0 with the reference's breakdown message. (The reference itself raises RuntimeError in
    compute_nodal_forces there -- `dofs.view(M, -1)` of an empty tensor, `solver/element.py:452` -- a deliberate
    difference: nothing faults or reads out of bounds.)"""
    element, _, solver, system = _mods()
    coords = torch.rand(10, 3, dtype=F64, generator=torch.Generator().manual_seed(3))
    el = torch.zeros((0, 4), dtype=torch.long)
    K = element.compute_c3d4_K_matrix(coords, el, 1e9, 0.3, device=gpu, dtype=F64)
    assert K.shape == (0, 12, 12)
    y = element.compute_nodal_forces(K, el, torch.rand(10, 3, dtype=F64), device=gpu, dtype=F64)
    assert y.shape == (10, 3) and float(y.abs().max()) == 0.0
    capsys.readouterr()
    F = torch.rand(10, 3, dtype=F64)
    u, res = solver.stable_conjugate_gradient_solver(K, el, F, torch.tensor([0]), device=gpu, max_iter=5,
                                                     return_info=True)
    assert res.iterations == 1 and float(u.abs().max()) == 0.0
    assert capsys.readouterr().out.startswith("Terminating early at iteration 1: p^T K p = 0.000e+00")
    A = system.assemble_tet4_system(coords.to(gpu), el.to(gpu), "poisson")
    assert float(A.matvec(torch.ones(10, dtype=F64, device=gpu)).abs().max()) == 0.0


def test_vals_edits_are_seen_by_solves(gpu):
    """a solver-layout matrix used to keep solving with its layout copy after the caller edited `vals`
    in place. Once handed out, the plain values are the matrix: matvec, Jacobi and the solve see the edit (x2 values:
    twice the product, half the weights, half the solution -- exact in binary floating point)."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(8, jitter=0.1)
    cg, tg = c.to(gpu), t.to(gpu)
    A = system.assemble_tet4_system(cg, tg, "poisson")
    assert A.solver_layout
    N = c.shape[0]
    mask = torch.zeros(N, dtype=torch.uint8, device=gpu)
    mask[:50] = 1
    p = torch.randn(N, dtype=F64, generator=torch.Generator().manual_seed(4)).to(gpu)
    y, w = A.matvec(p), A.jacobi(mask)
    b = torch.ones(N, dtype=F64, device=gpu)
    r1 = A.pcg(b, w=w, tol=0.0, max_iter=30)
    A.vals.mul_(2.0)
    assert not A.solver_layout
    assert torch.equal(A.matvec(p), 2.0 * y)
    w2 = A.jacobi(mask)
    assert torch.equal(w2, 0.5 * w)
    r2 = A.pcg(b, w=w2, tol=0.0, max_iter=30)
    assert torch.equal(r2.x, 0.5 * r1.x)


@pytest.mark.parametrize("etype,gen,n", [("c3d8", "hex_box", 5), ("c3d6", "wedge_box", 5), ("c3d10", "tet10_cube", 4)])
def test_scalar_mass_and_bs1_tile_assembly(gpu, etype, gen, n, monkeypatch):
    """BASELINE configs[4]'s mass as its scalar factor (compute_M_matrix(..., scalar=True), fem_iso_mass_scalar):
    M_e = Ms (x) I3 bit for bit, and the bs = 1 global Ms (k_assemble_ke_tile1) = the diagonal entries of every 3x3
    block of the bs = 3 global mass, off-diagonal entries zero; the tile form equals the wave-per-row kernel
    (FEM355_KE_ROWS) bit for bit when storing and when adding onto stored values. Parity unpinned (no reference mass)."""
    el_mod, mesh, _, system = _mods()
    c, t = getattr(mesh, gen)(n, jitter=0.1)
    cg, tg = c.to(gpu), t.to(gpu)
    N = c.shape[0]
    rho = 4.47e-3
    Ms = el_mod.compute_M_matrix(cg, tg, etype, rho, device=gpu, dtype=F64, scalar=True)
    Me = el_mod.compute_M_matrix(cg, tg, etype, rho, device=gpu, dtype=F64)
    npe = t.shape[1]
    assert Ms.shape == (t.shape[0], npe, npe)
    kron = torch.einsum("mab,ij->maibj", Ms, torch.eye(3, dtype=F64, device=gpu)).reshape(Me.shape)
    assert torch.equal(kron, Me)
    g = system.build_graph(tg, N)
    A1 = system.SellMatrix(g, 1).add_element_matrices(Ms, tg)
    A3 = system.SellMatrix(g, 3).add_element_matrices(Me, tg)
    _, _, v1 = A1.csr()
    _, _, v3 = A3.csr()
    for i in range(3):
        assert torch.equal(v3[:, i, i], v1[:, 0, 0])
    off = v3.clone()
    for i in range(3):
        off[:, i, i] = 0.0
    assert float(off.abs().max()) == 0.0
    assert abs(float(v1.sum()) / rho - 1.0) < 1e-12   # total mass = rho x unit volume
    # tile form vs the wave-per-row kernel: stored, then a second family added on top
    A1.add_element_matrices(Ms, tg)
    monkeypatch.setenv("FEM355_KE_ROWS", "1")
    B1 = system.SellMatrix(g, 1).add_element_matrices(Ms, tg)
    fresh = B1.plain_values().clone()
    B1.add_element_matrices(Ms, tg)
    monkeypatch.delenv("FEM355_KE_ROWS")
    A1b = system.SellMatrix(g, 1).add_element_matrices(Ms, tg)
    assert torch.equal(A1b.plain_values(), fresh)
    assert torch.equal(A1.plain_values(), B1.plain_values())


@pytest.mark.parametrize("case", ["kuhn", "permuted"])
def test_solver_layout_from_the_fill_pass(gpu, case, monkeypatch):
    """build_graph(..., solver_layout=True) forms the bs = 1 solver layout (paired deltas, slice-uniform lists, gather
    windows) inside the SELL fill pass (fem_graph_sell_fill_sl): the same arrays as the separate k_sell_sl_pattern
    pass (FEM355_SL_SEPARATE), bit for bit, and the same solve."""
    _, mesh, _, system = _mods()
    c, t = mesh.kuhn_cube(13, jitter=0.1)
    if case == "permuted":
        perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(5))
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel())
        c, t = c[perm], inv[t]
    cg, tg = c.to(gpu), t.to(gpu)
    N = c.shape[0]
    gf = system.build_graph(tg, N, solver_layout=True)
    monkeypatch.setenv("FEM355_SL_SEPARATE", "1")
    gs = system.build_graph(tg, N, solver_layout=True)
    monkeypatch.delenv("FEM355_SL_SEPARATE")
    assert getattr(gs, "_sl", None) is None and gf._sl is not None
    a, b = gf.solver_layout(), gs.solver_layout()
    ns = (N + 63) // 64
    assert torch.equal(a.pcols, b.pcols) and torch.equal(a.uoff[:ns], b.uoff[:ns]) and torch.equal(a.win, b.win)
    sp = gf.slice_ptr.cpu()
    uo = b.uoff[:ns].cpu()
    for q in torch.nonzero(uo >= 0).view(-1).tolist():   # the written part of the lists: w deltas per uniform slice
        w = int((sp[q + 1] - sp[q]) // 64)
        o = int(uo[q])
        assert torch.equal(a.ucol[o:o + w], b.ucol[o:o + w])
    A1 = system.SellMatrix(gf, 1).add_tet4(cg, tg, 1.0)
    A2 = system.SellMatrix(gs, 1).add_tet4(cg, tg, 1.0)
    assert torch.equal(A1._svals, A2._svals)


def _windows_restated(g, G, pk_waves=16):
    """The persistent schedule's gather windows restated on the host from the pattern's 16-bit deltas (k_pk_window /
    pk_slice_span, csrc/pcg_persist.hpp, sell_pair.hpp): per slice the union of its rows' deltas applied to the whole
    slice, mapped to owner workgroups; per owner the min / max over its slices, (G, -1) for an owner without any."""
    N = g.n_nodes
    ns = (N + 63) // 64
    sp = g.slice_ptr.cpu().tolist()
    d = g.dcols.cpu().to(torch.int64)
    W = G * pk_waves
    owner = lambda r: (((r >> 6) + 1) * W - 1) // ns // pk_waves
    lo = [G] * G
    hi = [-1] * G
    for s in range(ns):
        w = (sp[s + 1] - sp[s]) // 64
        blk = d[sp[s]:sp[s + 1]].view(w, 64)
        rows = min(64, N - s * 64)
        dmin = min(0, int(blk[:, :rows].min())) if w else 0
        dmax = max(0, int(blk[:, :rows].max())) if w else 0
        cl, ch = s * 64 + dmin, min(s * 64 + 63 + dmax, N - 1)
        cl = max(cl, 0)
        cl = min(cl, ch)
        me = owner(s * 64)
        lo[me] = min(lo[me], owner(cl))
        hi[me] = max(hi[me], owner(ch))
    return torch.tensor(lo + hi, dtype=torch.int32)


@pytest.mark.parametrize("case", ["kuhn", "permuted", "ragged"])
def test_gather_windows_from_slice_spans(gpu, case, monkeypatch):
    """Round 5: the gather windows are reduced from per-slice owner spans (k_win_from_spans) instead of two atomics
    per slice. Both producers -- the fill pass (fem_graph_sell_fill_sl) and the separate pass (fem_sell_sl_pattern)
    -- against the host restatement of k_pk_window, exactly: a Kuhn cube, a random numbering (every window spans the
    grid), and a mesh whose last slice is partial."""
    _, mesh, _, system = _mods()
    n = 12 if case == "ragged" else 13
    c, t = mesh.kuhn_cube(n, jitter=0.1)
    if case == "permuted":
        perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(9))
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel())
        c, t = c[perm], inv[t]
    N = c.shape[0]
    assert case != "ragged" or N % 64 != 0
    tg = t.to(gpu)
    gf = system.build_graph(tg, N, solver_layout=True)
    monkeypatch.setenv("FEM355_SL_SEPARATE", "1")
    gs = system.build_graph(tg, N, solver_layout=True)
    monkeypatch.delenv("FEM355_SL_SEPARATE")
    a, b = gf.solver_layout(), gs.solver_layout()
    torch.cuda.synchronize()
    want = _windows_restated(gf, a.G)
    assert torch.equal(a.win.cpu()[: 2 * a.G], want)
    assert torch.equal(b.win.cpu()[: 2 * b.G], want)


def test_span_scratch_across_streams(gpu):
    """The slice spans live in a per-stream scratch kept between calls (runtime.hip stream_scratch, at most 8 kept):
    the solver layout built on twelve streams in turn -- the first streams' buffers evicted, a larger mesh growing a
    stream's buffer -- gives the windows and paired deltas of the first build, exactly."""
    _, mesh, _, system = _mods()
    ref = {}
    for n in (9, 13):
        c, t = mesh.kuhn_cube(n, jitter=0.1)
        tg, N = t.to(gpu), c.shape[0]
        g = system.build_graph(tg, N, solver_layout=True)
        sl = g.solver_layout()
        torch.cuda.synchronize()
        ref[n] = (tg, N, sl.win.cpu(), sl.pcols.cpu(), sl.uoff.cpu())
    streams = [torch.cuda.Stream(device=gpu) for _ in range(12)]
    for k, s in enumerate(streams):
        n = 9 if k % 3 else 13
        tg, N, win, pcols, uoff = ref[n]
        with torch.cuda.stream(s):
            g = system.build_graph(tg, N, solver_layout=True)
            sl = g.solver_layout()
        s.synchronize()
        assert torch.equal(sl.win.cpu(), win) and torch.equal(sl.pcols.cpu(), pcols), (k, n)
        assert torch.equal(sl.uoff.cpu(), uoff), (k, n)


@pytest.mark.gpu
def test_value_kernel_refuses_rows_past_16bit_positions(gpu):
    """The accumulator value kernel keeps column positions in 16-bit fields: a pattern whose widest row has 65,535
    columns or more (here a hub node shared by 21,846 tets, 65,539 columns) is refused with FEM_EARG -> FemError by
    fem_assemble_tet4*, never assembled with aliased positions. A normal pattern on the same device assembles after."""
    _, mesh, _, system = _mods()
    from fem355 import _capi as C
    ne = 21846
    g = torch.Generator().manual_seed(5)
    c = torch.cat([torch.zeros(1, 3, dtype=F64), torch.rand(3 * ne, 3, generator=g, dtype=F64) + 0.5]).to(gpu)
    t = torch.cat([torch.zeros(ne, 1, dtype=torch.int64),
                   torch.arange(1, 3 * ne + 1, dtype=torch.int64).view(ne, 3)], dim=1).to(gpu)
    with pytest.raises(C.FemError, match="columns exceeds"):
        system.assemble_tet4_system(c, t, "poisson", E=1.0, nu=0.3)
    c2, t2 = mesh.kuhn_cube(4, jitter=0.1)
    A = system.assemble_tet4_system(c2.to(gpu), t2.to(gpu), "poisson", E=1.0, nu=0.3)
    assert A.n == c2.shape[0]
