"""CPU tier: the C-ABI library loads, exports every symbol include/fem355.h declares, and the ctypes table
matches the header (no compute calls: no GPU here)."""
import os
import re

import fem355  # noqa: F401
from fem355 import _capi
from conftest import ROOT


def header_functions():
    txt = open(os.path.join(ROOT, "include", "fem355.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fem_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header():
    lib = _capi.load_library()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n


def test_ctypes_table_covers_header():
    names = set(header_functions())
    assert names == set(_capi.SIGNATURES), (names ^ set(_capi.SIGNATURES))


def test_arg_counts_match_header():
    txt = open(os.path.join(ROOT, "include", "fem355.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    for name, (_, args) in _capi.SIGNATURES.items():
        m = re.search(name + r"\s*\(([^)]*)\)", txt, flags=re.S)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, len(params), len(args))


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        return
    from fem355 import element, mesh
    c, t = mesh.kuhn_cube(1)
    try:
        element.compute_c3d4_K_matrix(c, t, 1.0, 0.3, device="cpu")
    except _capi.FemError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("compute ran without a HIP device")


def test_ptr_refuses_host_tensors():
    """A host tensor's address must never reach a kernel (memory fault with XNACK off): C.ptr raises instead."""
    import pytest
    import torch
    assert _capi.ptr(None) is None
    with pytest.raises(_capi.FemError):
        _capi.ptr(torch.zeros(4, dtype=torch.float64))


def test_public_functions_enter_the_named_device(monkeypatch):
    """`device="cuda:1"` with current device 0: the call runs inside a device scope for cuda:1 (the library
    allocates and launches on the CURRENT device), and inside none when the device is already current."""
    import torch
    from fem355 import element, solver
    seen = []

    class Scope:
        def __init__(self, d):
            self.d = d

        def __enter__(self):
            seen.append(("enter", self.d.index))

        def __exit__(self, *a):
            seen.append(("exit", self.d.index))

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(_capi, "device_scope", lambda d: Scope(torch.device(d)) if torch.device(d).index != 0
                        else _capi._NULL_SCOPE)

    @_capi.on_device
    def probe(x, device="cuda:0"):
        seen.append(("call", device))
        return x + 1

    assert probe(1, device="cuda:1") == 2
    assert seen == [("enter", 1), ("call", "cuda:1"), ("exit", 1)]
    seen.clear()
    assert probe(1, "cuda:0") == 2 and seen == [("call", "cuda:0")]
    # the reference-named API is wrapped (functools.wraps keeps the name / signature for the notebooks)
    for fn in (element.compute_c3d4_K_matrix, element.compute_nodal_forces, solver.preconditioned_conjugate_gradient_solver,
               solver.stable_conjugate_gradient_solver, solver.static_structure_solver, solver.final_solver):
        assert hasattr(fn, "__wrapped__"), fn.__name__
