#!/usr/bin/env python3
"""why the slot position carried through the chunk walk's prefetch records (before commit
c83e619) came out wrong. Runs the element-chunk operator of the FEM_MF_SPCHECK debug build
(tools/build_variants.sh spcheck "-DFEM_MF_SPCHECK=1"; FEM355_LIB points at it), which carries the position as the
old walk did AND reads it under the chunk's work, and reports per cube size how many slot stores had the two disagree
(fem_mf_spcheck) plus the operator against the assembled one.

    FEM355_LIB=.../build/var_spcheck/libfem355.so python tools/mf_spcheck.py [n ...]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402,F401
from fem355 import _capi as C, mesh, system  # noqa: E402

E, NU = 113.8e9, 0.342


def main():
    lib = C.lib()
    dev = torch.device("cuda", 0)
    buf = (ctypes.c_uint64 * 8)()
    C.check(lib.fem_mf_spcheck(ctypes.byref(buf)), "fem_mf_spcheck")   # reset
    for n in [int(v) for v in sys.argv[1:]] or [20, 40, 60, 80, 119]:
        c, t = mesh.kuhn_cube(n, device=dev)
        A = system.MatFreeOperator(c, t, "elastic", E, NU)
        As = system.assemble_tet4_system(c, t, "elastic", E, NU)
        x = torch.randn(A.n, dtype=torch.float64, device=dev)
        for what, fn in (("apply", lambda: (A.matvec(x), As.matvec(x))), ("diag", lambda: (A.diag(), None))):
            y, ys = fn()
            torch.cuda.synchronize()
            C.check(lib.fem_mf_spcheck(ctypes.byref(buf)), "fem_mf_spcheck")
            rec = {"n": n, "what": what, "chunks": A.info()["chunks"], "stores": buf[0], "mismatches": buf[1],
                   "nonfinite": int((~torch.isfinite(y)).sum())}
            if ys is not None:
                rec["rel_vs_assembled"] = float((y - ys).abs().max() / ys.abs().max())
            if buf[1]:
                rec["first"] = {"chunk": buf[2] >> 16, "thread": buf[2] & 0xffff, "carried": buf[3],
                                "expected": buf[4], "walk_step": buf[5]}
            print(json.dumps(rec), flush=True)
        del A, As


if __name__ == "__main__":
    main()
