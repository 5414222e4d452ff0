"""CPU restatement of fem355's reverse Cuthill-McKee renumbering (csrc/reorder.hip) -- TEST INFRASTRUCTURE ONLY.

The reference has no node renumbering (it keeps the file order of `vtk_loader_to_torch`, `solver/element.py:39-90`),
so this is a specification of fem355's own opt-in step, not a reference restatement: parity of the device result
with this oracle is exact (same permutation); its quality is pinned against scipy's `reverse_cuthill_mckee`
(bandwidth) in tests/test_reorder_cpu.py. Only tests/ import it.

Rule (deterministic): level-synchronous Cuthill-McKee over the node graph; a next-level node's parent is its
neighbour in the current level with the smallest CM index; nodes are numbered parent by parent in CM order, a
parent's children in ascending node id. Start: the lowest-(degree, id) node (a boundary node). A finished
component is followed by the lowest-id unvisited node that has neighbours; nodes without any (no element) come last
in id order. The CM order of the swept nodes is reversed."""
import numpy as np


def _sweep(rowptr, colidx, order, level, cm, start, n_done):
    """CM sweep of the component of `start`; appends to `order`."""
    order.append(start)
    cm[start] = n_done
    level[start] = 0
    b, e, L = n_done, n_done + 1, 0
    while b < e:
        par = {}
        for p in range(b, e):
            u = order[p]
            for v in colidx[rowptr[u]:rowptr[u + 1]]:
                v = int(v)
                if level[v] == -1 or level[v] == L + 1:
                    level[v] = L + 1
                    par[v] = min(par.get(v, p), p)
        k = e
        for p in range(b, e):
            u = order[p]
            for v in colidx[rowptr[u]:rowptr[u + 1]]:
                v = int(v)
                if level[v] == L + 1 and par.get(v) == p:
                    order.append(v)
                    cm[v] = k
                    k += 1
        b, e, L = e, k, L + 1


def rcm(rowptr, colidx, n):
    """(perm, inv) int64 numpy: new node k = old node perm[k]; old node v -> inv[v]."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    colidx = np.asarray(colidx, dtype=np.int64)
    deg = rowptr[1:] - rowptr[:-1]
    live = np.nonzero(deg > 0)[0]
    perm = np.empty(n, dtype=np.int64)
    inv = np.empty(n, dtype=np.int64)
    order = []
    if live.size:
        key = deg[live] * (1 << 32) + live
        r0 = int(live[np.argmin(key)])
        level = np.full(n, -1, dtype=np.int64)
        cm = np.full(n, -1, dtype=np.int64)
        _sweep(rowptr, colidx, order, level, cm, r0, 0)
        cursor = 0
        while True:
            cand = np.nonzero((level[cursor:] == -1) & (deg[cursor:] > 0))[0]
            if cand.size == 0:
                break
            r = cursor + int(cand[0])
            cursor = r + 1
            _sweep(rowptr, colidx, order, level, cm, r, len(order))
    ncm = len(order)
    for i, v in enumerate(order):
        perm[ncm - 1 - i] = v
        inv[v] = ncm - 1 - i
    iso = np.nonzero(deg == 0)[0]
    perm[ncm:] = iso
    inv[iso] = np.arange(ncm, n)
    return perm, inv


def bandwidth(rowptr, colidx):
    """max |col - row| of a CSR pattern."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    rows = np.repeat(np.arange(rowptr.size - 1), rowptr[1:] - rowptr[:-1])
    return int(np.abs(np.asarray(colidx, dtype=np.int64) - rows).max()) if rows.size else 0
