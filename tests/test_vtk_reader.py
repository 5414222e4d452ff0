"""CPU: the native legacy-VTK reader behind `vtk_loader_to_torch` (reference
`solver/element.py:39-90`, which reads through pyvista).

pyvista is not in this image and the reference ships no VTK file, so parity with pv.read is unpinned: the files
here are written by the small writer below from the VTK legacy format specification (ASCII and big-endian
BINARY, the <= 4.2 count-prefixed CELLS block and the 5.1 OFFSETS / CONNECTIVITY block), and the loader must
return exactly the mesh that was written, reshaped the way the reference reshapes pyvista's `mesh.cells`.
"""
import struct

import numpy as np
import pytest
import torch

import fem355  # noqa: F401
from fem355 import _capi, element, mesh

VTK_TYPE = {4: 10, 8: 12, 6: 13, 10: 24}


def write_vtk(path, pts, cells, version="4.2", binary=False, ptype="double", itype="vtktypeint64", extra=""):
    """Minimal legacy VTK writer (test infrastructure)."""
    pts = np.asarray(pts, dtype=np.float64)
    cells = [list(map(int, c)) for c in cells]
    out = bytearray()

    def text(s):
        out.extend(s.encode())

    def block(values, fmt):
        if binary:
            out.extend(struct.pack(">" + fmt * len(values), *values))
            text("\n")
        else:
            text(" ".join(repr(v) if isinstance(v, float) else str(v) for v in values) + "\n")

    text(f"# vtk DataFile Version {version}\nfem355 test\n{'BINARY' if binary else 'ASCII'}\n")
    text("DATASET UNSTRUCTURED_GRID\n")
    if version.startswith("5"):
        text("METADATA\nINFORMATION 0\n\n")
    text(f"POINTS {pts.shape[0]} {ptype}\n")
    vals = [float(v) for v in pts.reshape(-1)]
    block(vals, "d" if ptype == "double" else "f")
    if version.startswith("5"):
        offs = np.cumsum([0] + [len(c) for c in cells]).tolist()
        conn = [v for c in cells for v in c]
        text(f"CELLS {len(offs)} {len(conn)}\nOFFSETS {itype}\n")
        block(offs, "q" if itype == "vtktypeint64" else "i")
        text(f"CONNECTIVITY {itype}\n")
        block(conn, "q" if itype == "vtktypeint64" else "i")
    else:
        flat = [v for c in cells for v in [len(c)] + c]
        text(f"CELLS {len(cells)} {len(flat)}\n")
        block(flat, "i")
    text(f"CELL_TYPES {len(cells)}\n")
    block([VTK_TYPE.get(len(c), 0) for c in cells], "i")
    text(extra)
    with open(path, "wb") as f:
        f.write(bytes(out))


@pytest.mark.parametrize("version,binary,ptype", [("4.2", False, "double"), ("4.2", True, "double"),
                                                  ("4.2", True, "float"), ("5.1", False, "double"),
                                                  ("5.1", True, "double"), ("3.0", False, "float")])
def test_roundtrip_tets(tmp_path, version, binary, ptype):
    c, t = mesh.kuhn_cube(3, jitter=0.1)
    p = tmp_path / "m.vtk"
    write_vtk(p, c, t, version, binary, ptype, extra="POINT_DATA 64\nSCALARS s float 1\nLOOKUP_TABLE default\n")
    pts, el = element.vtk_loader_to_torch(str(p), "c3d4", device="cpu", dtype=torch.float64)
    want = c.float().double() if ptype == "float" else c
    assert torch.equal(el, t) and el.dtype == torch.long
    assert torch.equal(pts, want)
    pts32, _ = element.vtk_loader_to_torch(p, "c3d4", device="cpu")     # reference default dtype float32
    assert pts32.dtype == torch.float32


@pytest.mark.parametrize("etype,gen", [("c3d8", mesh.hex_box), ("c3d6", mesh.wedge_box), ("c3d10", mesh.tet10_cube)])
def test_other_solids(tmp_path, etype, gen):
    c, e = gen(2)
    p = tmp_path / f"{etype}.vtk"
    write_vtk(p, c, e, "5.1", True, itype="vtktypeint32")
    pts, el = element.vtk_loader_to_torch(p, etype, device="cpu", dtype=torch.float64)
    assert torch.equal(el, e) and torch.equal(pts, c)
    _, cells, types = element.read_vtk(p)
    assert cells.shape[0] == e.shape[0] * (e.shape[1] + 1) and set(types.tolist()) == {VTK_TYPE[e.shape[1]]}


@pytest.mark.parametrize("etype,gen", [("c3d4", mesh.kuhn_cube), ("c3d8", mesh.hex_box), ("c3d6", mesh.wedge_box),
                                       ("c3d10", mesh.tet10_cube)])
def test_one_argument_call_infers_type(tmp_path, etype, gen):
    """`coords, elements = solver.vtk_loader_to_torch(path)` (`solver_example.ipynb:82`): the element type comes
    from the file's cell types; the result equals the explicit-type call."""
    c, e = gen(2)
    p = tmp_path / f"{etype}.vtk"
    write_vtk(p, c, e, "4.2", True)
    if torch.cuda.is_available():
        pts, el = element.vtk_loader_to_torch(str(p))          # literally the notebook's call
    else:
        pts, el = element.vtk_loader_to_torch(str(p), device="cpu")
    pts2, el2 = element.vtk_loader_to_torch(p, etype, device=pts.device)
    assert torch.equal(el, el2) and torch.equal(pts, pts2) and pts.dtype == torch.float32
    assert torch.equal(el.cpu(), e)


def test_one_argument_call_rejects_mixed_cells(tmp_path):
    c, t = mesh.kuhn_cube(1)
    p = tmp_path / "mixed.vtk"
    write_vtk(p, c, [list(t[0]), [0, 1, 2, 3, 4, 5, 6, 7]])
    with pytest.raises(ValueError, match="mixed VTK cell types"):
        element.vtk_loader_to_torch(p, device="cpu")
    assert element.infer_vtk_element_type(np.array([10, 10])) == "c3d4"
    with pytest.raises(ValueError, match="no cells"):
        element.infer_vtk_element_type(np.array([], dtype=np.int64))
    with pytest.raises(ValueError, match="unsupported VTK cell type 42"):
        element.infer_vtk_element_type(np.array([42]))


def test_reference_error_behaviour(tmp_path):
    c, t = mesh.kuhn_cube(1)
    p = tmp_path / "m.vtk"
    write_vtk(p, c, t)
    with pytest.raises(ValueError, match="Invalid element type."):
        element.vtk_loader_to_torch(p, "C3D4", device="cpu")      # no lower-casing, like the reference
    with pytest.raises(FileNotFoundError):
        element.vtk_loader_to_torch(tmp_path / "missing.vtk", "c3d4", device="cpu")
    # mixed cell sizes: the reference's reshape(-1, npe + 1) fails
    write_vtk(p, c, [list(t[0]), list(t[1][:3])])
    with pytest.raises(ValueError):
        element.vtk_loader_to_torch(p, "c3d4", device="cpu")


@pytest.mark.parametrize("bad", ["header", "truncated", "index", "dataset", "count"])
def test_malformed_files_raise(tmp_path, bad):
    c, t = mesh.kuhn_cube(1)
    p = tmp_path / "bad.vtk"
    write_vtk(p, c, t, binary=(bad == "truncated"))
    data = p.read_bytes()
    if bad == "header":
        data = b"# not vtk\n" + data
    elif bad == "truncated":
        data = data[: len(data) // 2]
    elif bad == "index":
        write_vtk(p, c, [[0, 1, 2, 99]])
        data = p.read_bytes()
    elif bad == "dataset":
        data = data.replace(b"UNSTRUCTURED_GRID", b"POLYDATA")
    elif bad == "count":
        data = data.replace(b"POINTS 8", b"POINTS 80000000000")
    p.write_bytes(data)
    with pytest.raises(_capi.FemError):
        element.read_vtk(p)
