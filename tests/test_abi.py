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
