"""Import shim: exposes the package directory `cuda-powered-mesh-handling-and-iterative-solvers_amd/`
(whose name is not a Python identifier) as the importable package ``fem355``.

    import fem355
    from fem355 import element, solver

The reference's own loading style also works unchanged: put that directory on ``sys.path`` and
``import solver`` (what `solver_example.ipynb:20-29` does with the reference's `solver/` directory).
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                         "cuda-powered-mesh-handling-and-iterative-solvers_amd")
_spec = _ilu.spec_from_file_location("fem355", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["fem355"] = _mod
_spec.loader.exec_module(_mod)
