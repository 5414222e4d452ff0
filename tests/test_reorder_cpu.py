"""Node renumbering (opt-in RCM, csrc/reorder.hip) -- CPU tier: the oracle's rule (oracle/rcm_ref.py) gives a
permutation, undoes a random numbering of the Kuhn cube down to the bandwidth of scipy's reverse Cuthill-McKee, and
handles several components and nodes no element touches. The device implementation equals this oracle exactly
(tests/test_gpu_reorder.py)."""
import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee
import torch

import fem355  # noqa: F401
from fem355 import mesh
from oracle import ref_cpu as R
from oracle import rcm_ref


def _permuted_cube(n, seed):
    c, t = mesh.kuhn_cube(n)
    perm = torch.randperm(c.shape[0], generator=torch.Generator().manual_seed(seed))
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    return c[perm], inv[t]


def _renumbered_pattern(t, N, inv):
    return R.node_pattern(torch.as_tensor(inv)[t], N)


def test_rcm_oracle_restores_a_narrow_band():
    c, t = _permuted_cube(9, 3)
    N = c.shape[0]
    rp, ci = R.node_pattern(t, N)
    bw0 = rcm_ref.bandwidth(rp, ci)
    perm, inv = rcm_ref.rcm(rp.numpy(), ci.numpy(), N)
    assert np.array_equal(np.sort(perm), np.arange(N)) and np.array_equal(inv[perm], np.arange(N))
    rp2, ci2 = _renumbered_pattern(t, N, inv)
    bw = rcm_ref.bandwidth(rp2, ci2)
    A = sp.csr_matrix((np.ones(ci.numel()), ci.numpy(), rp.numpy()), shape=(N, N))
    q = reverse_cuthill_mckee(A, symmetric_mode=True)
    qi = np.empty(N, dtype=np.int64)
    qi[q] = np.arange(N)
    rp3, ci3 = _renumbered_pattern(t, N, qi)
    bw_scipy = rcm_ref.bandwidth(rp3, ci3)
    assert bw0 > 5 * bw and bw <= 1.5 * bw_scipy, (bw0, bw, bw_scipy)
    # the lexicographic cube's bandwidth is (n+1)^2 + (n+1) + 1; RCM stays within a small factor of it
    assert bw <= 3 * (10 * 10 + 10 + 1)


def test_rcm_oracle_components_and_unused_nodes():
    c, t = mesh.kuhn_cube(3)
    N1 = c.shape[0]
    t2 = torch.cat([t, t + N1 + 5])       # two cubes, 5 unused nodes between them, 3 after
    N = 2 * N1 + 8
    rp, ci = R.node_pattern(t2, N)
    perm, inv = rcm_ref.rcm(rp.numpy(), ci.numpy(), N)
    assert np.array_equal(np.sort(perm), np.arange(N))
    unused = list(range(N1, N1 + 5)) + list(range(2 * N1 + 5, N))
    assert list(perm[N - 8:]) == unused                  # nodes without elements last, ascending
    # each component is contiguous in the new numbering
    new_first = inv[:N1]
    assert new_first.max() - new_first.min() == N1 - 1
