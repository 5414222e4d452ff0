"""ORACLE — test infrastructure only. Element-partitioned Jacobi-PCG on the CPU over torch.distributed (gloo).

Restates the distributed algorithm of csrc/pcg.hip (distributed phases) with the oracle's EBE operator
(`compute_nodal_forces`, `solver/element.py:429-464`) and the reference PCG (`solver/solver.py:766-812`):
each rank applies only its own elements, the interface rows of A p are summed over the ranks through the compact
interface vector (all_reduce), and dot products run over owned rows plus a scalar all_reduce. The partition and
halo maps come from the product module (fem355.dist, pure index bookkeeping), so this checks them against the
serial oracle solve without a GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ref_cpu as R

F64 = torch.float64


def halo_sum(v, rm, bs):
    """v [n_local*bs]: interface rows <- sum over ranks."""
    nI = rm.n_iface
    if nI == 0:
        return v
    vv = v.view(-1, bs)
    buf = torch.zeros((nI, bs), dtype=F64)
    has = rm.imap >= 0
    buf[has] = vv[rm.imap[has].long()]
    dist.all_reduce(buf)
    isif = rm.ipos >= 0
    vv[isif] = buf[rm.ipos[isif].long()]
    return v


def gdot(a, b, own_rows):
    t = torch.tensor([float(torch.dot(a[own_rows], b[own_rows]))], dtype=F64)
    dist.all_reduce(t)
    return t[0]


def _setup(coords, rm, f, fixed, kind, E, nu, operator="ebe"):
    """Local operator (halo-summed), Jacobi inverse of the assembled diagonal, local rhs and owned-dof mask.
    operator "ebe": the rank's element matrices and the reference's EBE product; "matfree": the closed-form element
    vectors of the rank's elements formed in every application (the element-chunk operator's algebra, no K_e)."""
    lc = coords[rm.nodes]
    bs = 1 if kind == "poisson" else 3
    n_loc = rm.nodes.numel()
    if operator == "matfree":
        def A(v):
            return halo_sum(R.tet4_forces_matfree(lc, rm.conn, v, kind, E, nu), rm, bs)

        diag = halo_sum(R.tet4_diag_matfree(lc, rm.conn, kind, E, nu), rm, bs)
    else:
        K = E * R.tet4_poisson_K(lc, rm.conn) if kind == "poisson" else R.tet4_K(lc, rm.conn, E, nu)

        def A(v):
            y = R.nodal_forces(K, rm.conn, v.view(n_loc, bs)).reshape(-1)
            return halo_sum(y, rm, bs)

        dofs = (rm.conn.unsqueeze(-1) * bs + torch.arange(bs)).reshape(-1)
        diag = torch.zeros(n_loc * bs, dtype=F64).index_add_(0, dofs, torch.diagonal(K, dim1=1, dim2=2).reshape(-1))
        diag = halo_sum(diag, rm, bs)
    Minv = 1.0 / diag
    Minv[Minv == float("inf")] = 0.0
    gfix = torch.zeros(coords.shape[0], dtype=torch.bool)
    gfix[fixed] = True
    Minv.view(-1, bs)[gfix[rm.nodes]] = 0.0
    b = f.reshape(-1, bs)[rm.nodes].reshape(-1).to(F64)
    own = rm.own.bool().repeat_interleave(bs)
    return A, Minv, b, own


def dist_pcg(coords, elements, f, fixed, rm, kind="poisson", E=1.0, nu=0.0, tol=1e-8, max_iter=1000):
    """One rank's share of the partitioned PCG. Returns (x_local, iterations, status)."""
    A, Minv, b, own = _setup(coords, rm, f, fixed, kind, E, nu)
    x = torch.zeros_like(b)
    r = b - A(x)
    z = Minv * r
    p = z.clone()
    rz = gdot(r, z, own)
    for i in range(max_iter):
        q = A(p)
        alpha = rz / gdot(p, q, own)
        x += alpha * p
        r -= alpha * q
        z = Minv * r
        rz_new = gdot(r, z, own)
        if torch.sqrt(rz_new) < tol:
            return x, i + 1, "converged"
        p = z + (rz_new / rz) * p
        rz = rz_new
    return x, max_iter, "max_iter"


def dist_pcg_single(coords, elements, f, fixed, rm, kind="poisson", E=1.0, nu=0.0, tol=1e-8, max_iter=1000,
                    operator="ebe"):
    """The single-reduction (Chronopoulos-Gear) form of the same PCG, as csrc/pcg.hip k_cg1_* runs it on N>1 GPUs:
    u = M r and v = A u carried alongside r, beta = g/g_prev, p.Ap = d - beta g/alpha_prev, alpha = g/p.Ap with
    g = r.u and d = u.v; p = u + beta p, s = v + beta s, x += alpha p, r -= alpha s. Stop test sqrt(r.z) < tol as
    `solver/solver.py:805`, evaluated at the top of the next pass. operator "matfree": the form the N > 1 element-chunk
    path runs (k_cg1_mf_*). Returns (x_local, iterations, status)."""
    A, Minv, b, own = _setup(coords, rm, f, fixed, kind, E, nu, operator)
    x = torch.zeros_like(b)
    r = b - A(x)
    u = Minv * r
    v = A(u)
    g, d = gdot(r, u, own), gdot(u, v, own)
    p = torch.zeros_like(b)
    s = torch.zeros_like(b)
    g_prev = alpha_prev = None
    for i in range(max_iter + 1):
        beta = 0.0
        if i > 0:
            if torch.sqrt(g) < tol:
                return x, i, "converged"
            beta = g / g_prev
        if i == max_iter:
            break
        pq = d if i == 0 else d - beta * g / alpha_prev
        alpha = g / pq
        p = u + beta * p
        s = v + beta * s
        x += alpha * p
        r -= alpha * s
        u = Minv * r
        v = A(u)
        g_prev, alpha_prev = g, alpha
        g, d = gdot(r, u, own), gdot(u, v, own)
    return x, max_iter, "max_iter"
