"""GPU: the dof-level CSR C-ABI named in SURVEY §8(b) (fem_solid_ke, fem_csr_pattern, fem_csr_fill,
fem_spmv_csr, fem_pcg_csr), called through ctypes exactly as a foreign caller would.

Oracle: `oracle.ref_cpu.coo_to_csr` (the reference's COO assembly of `subdivision.ipynb:118-139`, coalesced) and the
golden fixtures of the reference itself. Pattern (rowptr, colidx, diagpos) bit-exact; values 1e-13 relative
(summation order); SpMV 1e-13; solutions 1e-10 relative with iteration counts within ±2; solid K 1e-12.
"""
import ctypes

import pytest
import torch

from conftest import load_golden, rel
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
E, NU = 113.8e9, 0.342
F64, I32 = torch.float64, torch.int32


def _lib():
    import fem355  # noqa: F401
    from fem355 import _capi as C
    return C, C.lib()


def _csr(C, lib, tets, N, dpn, dev):
    st = C.stream(dev)
    el = tets.to(dev).long().contiguous()
    rowptr = torch.empty(N * dpn + 1, dtype=I32, device=dev)
    nnz = ctypes.c_int64()
    C.check(lib.fem_csr_pattern(C.ptr(el), el.shape[0], el.shape[1], dpn, N, C.ptr(rowptr), None, None,
                                ctypes.byref(nnz), st), "fem_csr_pattern")
    colidx = torch.empty(nnz.value, dtype=I32, device=dev)
    diag = torch.empty(N * dpn, dtype=I32, device=dev)
    C.check(lib.fem_csr_pattern(C.ptr(el), el.shape[0], el.shape[1], dpn, N, C.ptr(rowptr), C.ptr(colidx),
                                C.ptr(diag), ctypes.byref(nnz), st), "fem_csr_pattern")
    return el, rowptr, colidx, diag


def test_csr_pattern_fill_spmv_vs_reference_coo(gpu):
    C, lib = _lib()
    g = load_golden("tet4_cube_n4_jit")
    N = g["coords"].shape[0]
    el, rowptr, colidx, diag = _csr(C, lib, g["tets"], N, 3, gpu)
    rp_ref, col_ref, val_ref = R.coo_to_csr(g["K"], g["tets"], 3)
    assert torch.equal(rowptr.cpu().long(), rp_ref) and torch.equal(colidx.cpu().long(), col_ref)
    for r in (0, 7, 3 * N - 1):
        assert int(colidx[diag[r]]) == r
    vals = torch.zeros(colidx.numel(), dtype=F64, device=gpu)
    K = g["K"].to(gpu).contiguous()
    C.check(lib.fem_csr_fill(C.ptr(K), C.ptr(el), el.shape[0], 4, 3, N, C.ptr(rowptr), C.ptr(colidx), C.ptr(vals),
                             C.stream(gpu)), "fem_csr_fill")
    assert rel(vals, val_ref) < 1e-13
    p = g["p"].to(gpu).reshape(-1).contiguous()
    y = torch.empty_like(p)
    C.check(lib.fem_spmv_csr(C.ptr(rowptr), C.ptr(colidx), C.ptr(vals), C.ptr(p), C.ptr(y), 3 * N, C.stream(gpu)),
            "fem_spmv_csr")
    assert rel(y.view(N, 3), g["y"]) < 1e-13


def test_csr_poisson_pattern_dpn1(gpu):
    C, lib = _lib()
    g = load_golden("poisson_tet4_n4_jit")
    N = g["coords"].shape[0]
    _, rowptr, colidx, _ = _csr(C, lib, g["tets"], N, 1, gpu)
    rp_ref, col_ref = R.node_pattern(g["tets"], N)
    assert torch.equal(rowptr.cpu().long(), rp_ref) and torch.equal(colidx.cpu().long(), col_ref)


@pytest.mark.parametrize("mode", ["cg", "pcg"])
def test_pcg_csr_vs_reference(gpu, mode):
    C, lib = _lib()
    g = load_golden("tet4_cube_n4_jit")
    N = g["coords"].shape[0]
    el, rowptr, colidx, _ = _csr(C, lib, g["tets"], N, 3, gpu)
    vals = torch.zeros(colidx.numel(), dtype=F64, device=gpu)
    K = g["K"].to(gpu).contiguous()
    C.check(lib.fem_csr_fill(C.ptr(K), C.ptr(el), el.shape[0], 4, 3, N, C.ptr(rowptr), C.ptr(colidx), C.ptr(vals),
                             C.stream(gpu)), "fem_csr_fill")
    b = g["F"].to(gpu).reshape(-1).contiguous()
    x = torch.zeros_like(b)
    fixed = torch.zeros((N, 3), dtype=torch.uint8)
    fixed[g["fixed"]] = 1
    fixed = fixed.view(-1).to(gpu)
    it, st = ctypes.c_int(), ctypes.c_int()
    hist = torch.zeros(3000, dtype=F64, device=gpu)
    if mode == "cg":
        C.check(lib.fem_pcg_csr(C.ptr(rowptr), C.ptr(colidx), C.ptr(vals), 3 * N, C.ptr(b), C.ptr(x), None,
                                C.ptr(fixed), float(g["tol"]), 3000, 1e-30, C.MODE_CG_STABLE, ctypes.byref(it),
                                ctypes.byref(st), C.ptr(hist), C.stream(gpu)), "fem_pcg_csr")
        assert st.value == C.PCG_CONVERGED and abs(it.value - int(g["n_cg"])) <= 2
        assert rel(x.view(N, 3), g["u_cg"]) < 1e-10
    else:
        dinv = g["Minv"].to(gpu).reshape(-1).contiguous()
        C.check(lib.fem_pcg_csr(C.ptr(rowptr), C.ptr(colidx), C.ptr(vals), 3 * N, C.ptr(b), C.ptr(x), C.ptr(dinv),
                                None, 1e-6, 3000, 0.0, C.MODE_PCG, ctypes.byref(it), ctypes.byref(st), None,
                                C.stream(gpu)), "fem_pcg_csr")
        assert st.value == C.PCG_CONVERGED and abs(it.value - int(g["n_pcg"])) <= 2
        assert rel(x.view(N, 3), g["u_pcg"]) < 1e-10


@pytest.mark.parametrize("etype,npe", [("c3d8", 8), ("c3d6", 6), ("c3d10", 10)])
def test_solid_ke_vs_reference(gpu, etype, npe):
    C, lib = _lib()
    g = load_golden(f"{etype}_cells")
    X = g["coords"].to(gpu).contiguous()
    el = g["elements"].to(gpu).long().contiguous()
    M = el.shape[0]
    ip = g["points"].to(gpu).contiguous()
    w = g["weights"].to(gpu).contiguous()
    d = 3 * npe
    K1 = torch.empty((M, d, d), dtype=F64, device=gpu)
    C.check(lib.fem_solid_ke(npe, C.ptr(X), C.ptr(el), M, E, NU, C.ptr(ip), C.ptr(w), ip.shape[0], 1, C.ptr(K1),
                             C.stream(gpu)), "fem_solid_ke")
    assert rel(K1, g["K_single"]) < 1e-12
    K0 = torch.empty(g["K_multi"].shape, dtype=F64, device=gpu)
    C.check(lib.fem_solid_ke(npe, C.ptr(X), C.ptr(el), M, E, NU, C.ptr(ip), C.ptr(w), ip.shape[0], 0, C.ptr(K0),
                             C.stream(gpu)), "fem_solid_ke")
    assert rel(K0, g["K_multi"]) < 1e-12
    with pytest.raises(ValueError):
        C.check(lib.fem_solid_ke(20, C.ptr(X), C.ptr(el), M, E, NU, C.ptr(ip), C.ptr(w), ip.shape[0], 1, C.ptr(K1),
                                 C.stream(gpu)), "fem_solid_ke")


def test_scratch_memory_returns_to_baseline(gpu):
    """the library's stream-ordered scratch (graph build temporaries of fem_csr_pattern, the 9 nnz
    staging of fem_csr_fill) comes from a private pool that keeps at most 256 MB across synchronisations, so the
    device's free memory returns to within that of its baseline after a large pattern + fill (a 1.2M-tet elastic
    cube: ~1 GB of temporaries), and fem_release_scratch trims the rest."""
    C, lib = _lib()
    from fem355 import mesh
    c, t = mesh.kuhn_cube(59)
    N = c.shape[0]
    K = torch.randn(t.shape[0], 12, 12, dtype=F64, generator=torch.Generator().manual_seed(1)).to(gpu)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    el, rowptr, colidx, diag = _csr(C, lib, t, N, 3, gpu)
    vals = torch.zeros(colidx.numel(), dtype=F64, device=gpu)
    C.check(lib.fem_csr_fill(C.ptr(K), C.ptr(el), el.shape[0], 4, 3, N, C.ptr(rowptr), C.ptr(colidx), C.ptr(vals),
                             C.stream(gpu)), "fem_csr_fill")
    torch.cuda.synchronize()
    held = sum(x.numel() * x.element_size() for x in (el, rowptr, colidx, diag, vals))
    del el, rowptr, colidx, diag, vals
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 <= (256 << 20) + (16 << 20), (free0 - free1, held)
    C.check(lib.fem_release_scratch(), "fem_release_scratch")
    torch.cuda.empty_cache()
    free2 = torch.cuda.mem_get_info()[0]
    assert free0 - free2 <= (16 << 20), free0 - free2
