#!/usr/bin/env python3
"""Element-chunk operator vs the assembled operator across cube sizes: relative difference, non-finite entries and
the first bad node (diagnostics).  python tools/mf_nan_probe.py [n ...]"""
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
    C.lib()
    dev = torch.device("cuda", 0)
    for n in [int(v) for v in sys.argv[1:]] or [20, 40, 60, 80, 100, 119]:
        c, t = mesh.kuhn_cube(n, device=dev)
        A = system.MatFreeOperator(c, t, "elastic", E, NU)
        As = system.assemble_tet4_system(c, t, "elastic", E, NU)
        x = torch.randn(A.n, dtype=torch.float64, device=dev)
        y, ys = A.matvec(x), As.matvec(x)
        bad = ~torch.isfinite(y)
        d = (y - ys).abs()
        d[bad] = 0
        rec = {"n": n, "info": A.info(), "nonfinite": int(bad.sum()),
               "rel_finite": float(d.max() / ys.abs().max())}
        if rec["nonfinite"]:
            idx = torch.nonzero(bad).view(-1)
            rec["first_bad_dofs"] = idx[:8].tolist()
        dg = A.diag()
        rec["diag_nonfinite"] = int((~torch.isfinite(dg)).sum())
        print(json.dumps(rec), flush=True)
        del A, As


if __name__ == "__main__":
    main()
