"""GPU: stress recovery (reference `solver/element.py:308-353,409-504,905-937,1127-1189,
1696-1752,2570-2629,3343-3382`) through the C-ABI.

Oracle: `oracle.ref_cpu.{tet4_stress, iso_stress, node_average, face_forces, shared_face_sum}`, pinned to the
reference by `tests/test_oracle_golden.py::test_stress_recovery_oracle_matches_reference` (fixture `stress`).
Tolerances (fp64): stresses / von Mises 1e-12 relative (closed-form / cofactor gradients vs the reference's LU
inverse); node averages and face sums 1e-15; the 10M-tet property test (linear field -> exact constant stress)
1e-9 relative.
"""
import pytest
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64 = torch.float64


def _el():
    import fem355  # noqa: F401
    from fem355 import element, mesh
    return element, mesh


def test_c3d4_stress_and_node_average_vs_reference(gpu):
    el, _ = _el()
    s = load_golden("stress")
    g = load_golden("tet4_cube_n4_jit")
    c, t, u = g["coords"], g["tets"], g["u_cg"]
    sig, vm = el.compute_c3d4_element_stress(c, t, u, E, NU, device=gpu, dtype=F64)
    assert sig.shape == (t.shape[0], 3, 3) and rel(sig, s["c3d4_sig"]) < 1e-12 and rel(vm, s["c3d4_vm"]) < 1e-12
    sig2, vm2 = el.compute_element_stress(c, t, u, E, NU, "C3D4", device=gpu, dtype=F64)
    assert torch.equal(sig2, sig) and torch.equal(vm2, vm)
    nv = el.compute_node_vm_stress(c, t, s["c3d4_vm"], device=gpu, dtype=F64)
    assert rel(nv, s["c3d4_node_vm"]) < 1e-15
    # reference default dtype: float32 output of the fp64 computation
    s32, _ = el.compute_c3d4_element_stress(c, t, u, E, NU, device=gpu)
    assert s32.dtype == torch.float32 and rel(s32, s["c3d4_sig"]) < 1e-6


@pytest.mark.parametrize("etype", ["c3d8", "c3d6", "c3d10"])
def test_iso_stress_vs_reference(gpu, etype):
    el, _ = _el()
    s = load_golden("stress")
    cg = load_golden(f"{etype}_cells")
    cc, ce, u = cg["coords"], cg["elements"], s[f"{etype}_u"]
    s1, v1 = el.compute_element_stress(cc, ce, u, E, NU, etype, single=True, device=gpu, dtype=F64)
    assert rel(s1, s[f"{etype}_sig1"]) < 1e-12 and rel(v1, s[f"{etype}_vm1"]) < 1e-12
    s0, v0 = el.compute_element_stress(cc, ce, u, E, NU, etype, single=False, device=gpu, dtype=F64)
    assert s0.shape == s[f"{etype}_sig0"].shape and v0.shape == s[f"{etype}_vm0"].shape
    assert rel(s0, s[f"{etype}_sig0"]) < 1e-12 and rel(v0, s[f"{etype}_vm0"]) < 1e-12
    nv = el.compute_node_vm_stress(cc, ce, s[f"{etype}_vm1"], device=gpu, dtype=F64)
    assert rel(nv, s[f"{etype}_node_vm"]) < 1e-15
    # custom integration table [n,4] (xi, eta, zeta, w): a single point with weight 2
    pts, w = R.POINTS[etype]()
    ip = torch.cat([pts[:1], torch.full((1, 1), 2.0, dtype=F64)], 1)
    sc, vc = el.compute_element_stress(cc, ce, u, E, NU, etype, integral_point=ip, single=True, device=gpu, dtype=F64)
    ro, rv = R.iso_stress(cc, ce, u, etype, E, NU, points=pts[:1], weights=torch.tensor([2.0], dtype=F64))
    assert rel(sc, ro) < 1e-12 and rel(vc, rv) < 1e-12


def test_tensor_vm_and_face_forces_vs_reference(gpu):
    el, _ = _el()
    s = load_golden("stress")
    T = el.compute_stress_tensor(s["voigt"].to(gpu))
    assert T.device.type == "cuda" and torch.equal(T.cpu(), s["voigt_tensor"])
    assert rel(el.compute_von_mises_stress(T), s["voigt_vm"]) < 1e-15
    ff = el.compute_c3d4_surface_forces(s["normals"], s["c3d4_sig"], device=gpu)
    assert rel(ff, s["face_forces"]) < 1e-15
    sf = el.compute_c3d4_shared_face_forces_sum(s["shared_idx"], s["face_forces"], device=gpu)
    assert torch.equal(sf.cpu(), s["shared_sum"])
    bad = s["shared_idx"].clone()
    bad[0, 0, 1] = 4
    with pytest.raises(IndexError):
        el.compute_c3d4_shared_face_forces_sum(bad, s["face_forces"], device=gpu)


def test_stress_errors(gpu):
    el, mesh = _el()
    c, t = mesh.kuhn_cube(2)
    u = torch.zeros(c.shape[0], 3, dtype=F64)
    t_bad = t.clone()
    t_bad[3, 1] = t_bad[3, 0]          # degenerate tet -> the reference's B-matrix ValueError
    with pytest.raises(ValueError, match="Singular"):
        el.compute_c3d4_element_stress(c, t_bad, u, E, NU, device=gpu)
    t_oob = t.clone()
    t_oob[0, 0] = c.shape[0]
    with pytest.raises(IndexError):
        el.compute_c3d4_element_stress(c, t_oob, u, E, NU, device=gpu)
    with pytest.raises(ValueError):
        el.compute_element_stress(c, t, u, E, NU, "c3d20", device=gpu)
    with pytest.raises(ValueError):
        el.compute_c3d4_element_stress(c, t, torch.zeros(c.shape[0], 6, dtype=F64), E, NU, device=gpu)


def test_linear_field_exact_at_full_size(gpu):
    """10M-tet cube (BASELINE configs[1] mesh): a linear displacement u = G x gives the same strain in every P1
    element, so every element stress equals D eps(G) and every node average equals its von Mises."""
    el, mesh = _el()
    c, t = mesh.kuhn_cube(119, jitter=0.2, device=gpu)
    G = torch.tensor([[1.0, 2.0, -0.5], [0.3, -1.0, 0.7], [0.2, 0.4, 1.5]], dtype=F64, device=gpu) * 1e-4
    u = c @ G.t()
    sig, vm = el.compute_c3d4_element_stress(c, t, u, E, NU, device=gpu, dtype=F64)
    eps = torch.tensor([G[0, 0], G[1, 1], G[2, 2], G[0, 1] + G[1, 0], G[1, 2] + G[2, 1], G[0, 2] + G[2, 0]],
                       dtype=F64)
    D = R.elasticity_matrix(E, NU)
    s_ref = R.stress_tensor((D @ eps).view(1, 6))[0].to(gpu)
    assert float((sig - s_ref).abs().max()) < 1e-9 * float(s_ref.abs().max())
    vm_ref = R.von_mises(s_ref.cpu().view(1, 3, 3))[0]
    assert float((vm - float(vm_ref)).abs().max()) < 1e-9 * float(vm_ref)
    nv = el.compute_node_vm_stress(c, t, vm, device=gpu, dtype=F64)
    assert float((nv - float(vm_ref)).abs().max()) < 1e-9 * float(vm_ref)
