import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the fem355 kernels")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: (torch.from_numpy(d[k]) if d[k].dtype.kind in "fiub" else d[k]) for k in d.files}


def rel(a, b):
    a = a.detach().cpu().to(torch.float64)
    b = b.detach().cpu().to(torch.float64)
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-300))


class Cube119:
    """The 10,110,954-tet Kuhn cube of bench.py (BASELINE configs[2]/[3] and the metric) on the host, with the
    oracle's element matrices and reference products formed once per session and shared by every test that checks a
    10M configuration against the oracle (elastic K_e: ~11.6 GB of host memory, ~10 s on the box's cores)."""
    E, NU = 113.8e9, 0.342

    def __init__(self):
        from fem355 import mesh
        self.c, self.t = mesh.kuhn_cube(119)
        self.N = self.c.shape[0]
        self._memo = {}

    def memo(self, key, fn):
        if key not in self._memo:
            self._memo[key] = fn()
        return self._memo[key]

    def K(self, kind):
        from oracle import ref_cpu as R
        if kind == "poisson":
            return self.memo("Kp", lambda: R.tet4_poisson_K(self.c, self.t))
        return self.memo("Ke", lambda: R.tet4_K(self.c, self.t, self.E, self.NU))

    def case(self, kind):
        """(load [N, dpn] fp64, fixed node ids, dinv [N, dpn] exact Jacobi with fixed rows zeroed) of the bench's case."""
        from fem355 import mesh
        from oracle import ref_cpu as R

        def make():
            dpn = 1 if kind == "poisson" else 3
            f, fixed = mesh.cube_poisson_case(self.c) if kind == "poisson" else mesh.cube_elasticity_case(self.c)
            dinv = R.diag_preconditioner(self.K(kind), self.t, self.N, dpn=dpn)
            dinv[fixed] = 0.0
            return f.reshape(self.N, dpn).to(torch.float64), fixed, dinv.reshape(self.N, dpn)
        return self.memo(("case", kind), make)

    def matvec_ref(self, kind, seed):
        """(p [N, dpn] seeded, the oracle's EBE product K p) -- `solver/element.py:429-464`."""
        from oracle import ref_cpu as R

        def make():
            dpn = 1 if kind == "poisson" else 3
            p = torch.randn(self.N, dpn, dtype=torch.float64, generator=torch.Generator().manual_seed(seed))
            return p, R.nodal_forces(self.K(kind), self.t, p).reshape(self.N, dpn)
        return self.memo(("mv", kind, seed), make)

    def pcg_ref(self, kind, iters):
        """The oracle PCG's iterate after `iters` fixed iterations (tol 0) -- `solver/solver.py:766-812`."""
        from oracle import ref_cpu as R

        def make():
            f, _, dinv = self.case(kind)
            u, it, _ = R.pcg(self.K(kind), self.t, f, dinv, tol=0.0, max_iter=iters)
            assert it == iters
            return u.reshape(self.N, -1)
        return self.memo(("pcg", kind, iters), make)


@pytest.fixture(scope="session")
def cube119():
    import fem355  # noqa: F401
    return Cube119()


@pytest.fixture(scope="session")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fem355  # noqa: F401
    from fem355 import _capi
    _capi.lib()
    return "cuda:0"
