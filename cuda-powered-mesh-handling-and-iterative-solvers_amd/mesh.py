"""Synthetic structured meshes used by the tests, the golden-fixture generator and bench.py.

The reference ships no meshes (its notebooks read the private SimJEB set, `solver_example.ipynb:72-82`),
so every parity case and benchmark runs on these generated boxes:

* ``kuhn_cube(n)``   : unit cube, n^3 hexes, each split into 6 Kuhn tets sharing the 0-6 diagonal
                       (all VTK-positive); nodes numbered ``(i*(n+1)+j)*(n+1)+k`` with i<->x, j<->y, k<->z.
* ``hex_box(n)``     : the same grid as n^3 c3d8 hexes in VTK/Abaqus order (`solver/element.py:1583-1632`).
* ``wedge_box(n)``   : every hex split into 2 c3d6 prisms (bottom triangle 0,1,2 / top 3,4,5, the order
                       `compute_c3d6_Jacobian` assumes, `solver/element.py:2482-2509`).
* ``tet10_cube(n)``  : the Kuhn tets with one mid-edge node per unique edge, in the reference's c3d10 order
                       (mid-edge 4..9 on edges (0,1),(1,2),(2,0),(0,3),(1,3),(2,3); `solver/element.py:1026-1060`).

All generators are vectorised torch code so the 10M-element cases build in about a second on the host or
on the GPU (``device=``). Connectivity is int64 (torch.long), as the reference expects.
"""
from __future__ import annotations

import numpy as np
import torch

# Kuhn split of the unit hex: 6 tets around the 0-6 diagonal, each with positive orientation.
KUHN_TETS = ((0, 1, 2, 6), (0, 2, 3, 6), (0, 3, 7, 6), (0, 7, 4, 6), (0, 4, 5, 6), (0, 5, 1, 6))
# Hex local corner offsets (di, dj, dk) in VTK order.
HEX_CORNERS = ((0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1))
WEDGE_SPLIT = ((0, 1, 3, 4, 5, 7), (1, 2, 3, 5, 6, 7))
TET10_EDGES = ((0, 1), (1, 2), (2, 0), (0, 3), (1, 3), (2, 3))

DEFAULT_SEED = 20250418


def grid_coords(n: int, jitter: float = 0.0, seed: int = DEFAULT_SEED, device="cpu", dtype=torch.float64):
    """Nodes of the (n+1)^3 lattice on [0,1]^3, lexicographic ``(i*(n+1)+j)*(n+1)+k``.

    ``jitter`` moves interior nodes uniformly by up to ±jitter*h per axis (numpy default_rng(seed)),
    so the fixtures are not all congruent elements.
    """
    m = n + 1
    h = 1.0 / n
    ax = torch.arange(m, dtype=dtype) * h
    X, Y, Z = torch.meshgrid(ax, ax, ax, indexing="ij")
    coords = torch.stack([X.reshape(-1), Y.reshape(-1), Z.reshape(-1)], dim=1)
    if jitter:
        rng = np.random.default_rng(seed)
        d = torch.from_numpy(rng.uniform(-jitter * h, jitter * h, size=(m ** 3, 3))).to(dtype)
        idx = torch.arange(m)
        I, J, K = torch.meshgrid(idx, idx, idx, indexing="ij")
        interior = ((I > 0) & (I < n) & (J > 0) & (J < n) & (K > 0) & (K < n)).reshape(-1)
        coords[interior] += d[interior]
    return coords.to(device)


def _hex_corner_nodes(n: int, device="cpu"):
    """[n^3, 8] global node ids of every hex cell, VTK corner order; cells ordered (i, j, k) lexicographic."""
    m = n + 1
    c = torch.arange(n, device=device)
    I, J, K = torch.meshgrid(c, c, c, indexing="ij")
    I, J, K = I.reshape(-1), J.reshape(-1), K.reshape(-1)
    cols = [((I + di) * m + (J + dj)) * m + (K + dk) for (di, dj, dk) in HEX_CORNERS]
    return torch.stack(cols, dim=1).to(torch.long)


def kuhn_cube(n: int, jitter: float = 0.0, seed: int = DEFAULT_SEED, device="cpu", dtype=torch.float64):
    """Unit cube of 6*n^3 linear tets (c3d4). Returns (coords [N,3], elements [M,4] int64)."""
    hexes = _hex_corner_nodes(n, device)
    tets = torch.stack([hexes[:, list(t)] for t in KUHN_TETS], dim=1).reshape(-1, 4).contiguous()
    return grid_coords(n, jitter, seed, device, dtype), tets


def hex_box(n: int, jitter: float = 0.0, seed: int = DEFAULT_SEED, device="cpu", dtype=torch.float64):
    """Unit cube of n^3 trilinear hexes (c3d8)."""
    return grid_coords(n, jitter, seed, device, dtype), _hex_corner_nodes(n, device).contiguous()


def wedge_box(n: int, jitter: float = 0.0, seed: int = DEFAULT_SEED, device="cpu", dtype=torch.float64):
    """Unit cube of 2*n^3 linear prisms (c3d6)."""
    hexes = _hex_corner_nodes(n, device)
    w = torch.stack([hexes[:, list(s)] for s in WEDGE_SPLIT], dim=1).reshape(-1, 6).contiguous()
    return grid_coords(n, jitter, seed, device, dtype), w


def tet10_cube(n: int, jitter: float = 0.0, seed: int = DEFAULT_SEED, device="cpu", dtype=torch.float64):
    """Unit cube of 6*n^3 quadratic tets (c3d10); mid-edge nodes appended after the corner nodes,
    numbered by the sorted unique edge list, placed at the exact edge midpoint."""
    coords, tets = kuhn_cube(n, jitter, seed, device, dtype)
    M = tets.shape[0]
    e = torch.stack([torch.stack([tets[:, a], tets[:, b]], dim=1) for (a, b) in TET10_EDGES], dim=1)  # [M,6,2]
    lo = torch.minimum(e[..., 0], e[..., 1])
    hi = torch.maximum(e[..., 0], e[..., 1])
    key = (lo * coords.shape[0] + hi).reshape(-1)
    uniq, inv = torch.unique(key, return_inverse=True)
    a = uniq // coords.shape[0]
    b = uniq % coords.shape[0]
    mid = 0.5 * (coords[a] + coords[b])
    mids = inv.reshape(M, 6) + coords.shape[0]
    return torch.cat([coords, mid], dim=0), torch.cat([tets, mids], dim=1).contiguous()


def face_nodes(coords: torch.Tensor, axis: int, value: float, atol: float = 1e-12):
    """Indices of nodes lying on the plane coords[:, axis] == value (the fixed / loaded faces)."""
    return torch.nonzero((coords[:, axis] - value).abs() <= atol, as_tuple=True)[0]


def cube_elasticity_case(coords: torch.Tensor, total_force: float = -1e6):
    """Benchmark load case: z=0 face fixed, `total_force` N in z spread over the z=1 face.
    Returns (F [N,3], fixed node ids)."""
    fixed = face_nodes(coords, 2, 0.0)
    top = face_nodes(coords, 2, 1.0)
    F = torch.zeros((coords.shape[0], 3), dtype=coords.dtype, device=coords.device)
    F[top, 2] = total_force / top.numel()
    return F, fixed


def cube_poisson_case(coords: torch.Tensor):
    """Scalar benchmark case: z=0 face Dirichlet u=0, unit nodal source f=1 elsewhere."""
    fixed = face_nodes(coords, 2, 0.0)
    f = torch.ones((coords.shape[0], 1), dtype=coords.dtype, device=coords.device)
    f[fixed] = 0.0
    return f, fixed


def cube_counts(n: int):
    """Closed-form sizes of the Kuhn cube: tets, nodes, scalar nnz = N + 2*edges."""
    m = n + 1
    edges = 3 * n * m * m + 3 * n * n * m + n ** 3
    return 6 * n ** 3, m ** 3, m ** 3 + 2 * edges
