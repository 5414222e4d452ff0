"""`solver/shell.py` (Kirchhoff s3/s4 shells) is OUT OF SCOPE of fem355 (shells are not on
the north_star path). The module exists so that `from shell import *` in the solver mirror resolves as in the
reference (`solver/solver.py:2`); every shell entry point raises."""

__all__ = ["compute_s3_K_matrix", "compute_s4_K_matrix", "compute_shell_nodal_forces"]


def _oos(name):
    def f(*a, **k):
        raise NotImplementedError(f"{name}: shell elements are out of scope of fem355 (SURVEY.md §2 row 13)")
    f.__name__ = name
    return f


compute_s3_K_matrix = _oos("compute_s3_K_matrix")
compute_s4_K_matrix = _oos("compute_s4_K_matrix")
compute_shell_nodal_forces = _oos("compute_shell_nodal_forces")
