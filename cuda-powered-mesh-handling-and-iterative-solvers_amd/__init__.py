"""fem355 — MI355X-native (gfx950) FEM assembly + Jacobi-PCG.

Drop-in for the hot path of sml2004/CUDA-powered-mesh-handling-and-Iterative-solvers: the `element.py`
element stiffness quadrature and the `solver.py` CG / PCG loops, re-implemented as hand-written HIP
kernels behind a C-ABI (`include/fem355.h`, loaded by `_capi.py`). See DESIGN.md.
"""
import os as _os

PKG_DIR = _os.path.dirname(_os.path.abspath(__file__))

from . import mesh  # noqa: E402,F401  (pure torch, no GPU needed)

__all__ = ["mesh", "PKG_DIR"]
