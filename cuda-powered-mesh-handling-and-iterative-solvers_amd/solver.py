"""Reference-compatible solver API (`solver/solver.py` of sml2004/CUDA-powered-mesh-handling-and-Iterative-
solvers @ 2025-04-18), executed on the MI355X.

Like the reference, this module re-exports the element API (`from element import *`, `solver/solver.py:1-2`),
so `solver.compute_nodal_forces(...)` etc. resolve exactly as in the notebooks.

The solvers take the reference's hand-off object (element matrices K [M, d, d] + connectivity), assemble them
once on the device into a SELL-64 global matrix (deterministic row-gather, `system.py`) and run the whole
(P)CG iteration on the device (`csrc/pcg.hip`). They print the reference's messages and never raise on
breakdown or non-convergence (`solver/solver.py:187-227,805-811`).
"""
from __future__ import annotations

import torch

try:
    from . import _capi as C
    from . import system as _sys
    from .element import *  # noqa: F401,F403  (the reference's `from element import *`)
    from .element import _dev, _key, cached_incidence, compute_c3d4_K_matrix, compute_c3d6_K_matrix, \
        compute_c3d8_K_matrix
    from .constraints import *  # noqa: F401,F403
    from .constraints import ConstraintSet
except ImportError:  # pragma: no cover - flat import from the package directory
    import _capi as C  # type: ignore
    import system as _sys  # type: ignore
    from element import *  # type: ignore # noqa
    from element import _dev, _key, cached_incidence, compute_c3d4_K_matrix, compute_c3d6_K_matrix, \
        compute_c3d8_K_matrix  # type: ignore
    from constraints import *  # type: ignore # noqa
    from constraints import ConstraintSet  # type: ignore

from collections import OrderedDict

F64 = torch.float64
LONG = torch.long

_GRAPH_CACHE: "OrderedDict[tuple, tuple]" = OrderedDict()


def cached_graph(elements: torch.Tensor, n_nodes: int) -> "_sys.Graph":
    """Pattern of `elements` kept across calls (keyed on pointer + version + shape, like a plan cache)."""
    k = _key(elements, n_nodes)
    hit = _GRAPH_CACHE.get(k)
    if hit is not None:
        _GRAPH_CACHE.move_to_end(k)
        return hit[1]
    g = _sys.build_graph(elements, n_nodes)
    _GRAPH_CACHE[k] = (elements, g)
    while len(_GRAPH_CACHE) > 4:
        _GRAPH_CACHE.popitem(last=False)
    return g


def assemble(K, elements, n_nodes, device="cuda:0"):
    """Global operator of one element family: SELL-64 with dpn x dpn blocks (dpn = d / npe)."""
    dev = _dev(device)
    elements = elements.to(device=dev, dtype=LONG).contiguous()
    K = K.to(device=dev, dtype=F64).contiguous()
    dpn = K.shape[-1] // elements.shape[1]
    g = cached_graph(elements, n_nodes)
    return _sys.SellMatrix(g, dpn).add_element_matrices(K, elements)


def _cg_messages(res, style):
    """The reference's prints for each stop (`solver/solver.py:96-133` static, `:187-227` stable CG)."""
    lead = ("\n",) if style == "static" else ()
    if res.status == C.PCG_CONVERGED:
        print(*lead, f"Converged after {res.iterations} iterations. Residual norm: {res.rz:.3e}")
    elif res.status == C.PCG_BREAKDOWN:
        print(*lead, f"Terminating early at iteration {res.iterations}: p^T K p = {res.pq:.3e}, "
              "which is invalid for SPD systems.")
    elif res.status == C.PCG_ALPHA_NAN:
        print(*lead, f"Terminating at iteration {res.iterations}: alpha is NaN or Inf.")
    elif res.status == C.PCG_BETA_NAN:
        print(*lead, f"Terminating at iteration {res.iterations}: beta is NaN or Inf.")
    else:
        print(*lead, "CG did not converge within the maximum number of iterations.")


def _free_mask(n_nodes, dpn, fixed, dev):
    w = torch.ones((n_nodes, dpn), dtype=F64, device=dev)
    if fixed is not None:
        w[torch.as_tensor(fixed).to(device=dev, dtype=LONG)] = 0.0
    return w.view(-1)


# ============================================================================ CG (`solver/solver.py:144-229`)
def stable_conjugate_gradient_solver(K, elements, F, rbe2, u_init=None, tol=1e-10, max_iter=1000, device="cuda:0",
                                     dtype=torch.float64, eps=1e-30, return_info=False):
    """CG on K u = F with the nodes `rbe2` held at zero (u, r, p zeroed there); alpha = rs/(pAp+eps),
    beta = rs_new/(rs_old+eps); stop when sqrt(r.r) < tol (absolute). Returns u [N, dpn]."""
    dev = _dev(device)
    N = F.shape[0]
    A = assemble(K, elements, N, dev)
    w = _free_mask(N, A.bs, rbe2, dev)
    b = F.to(device=dev, dtype=F64).reshape(-1)
    res = A.pcg(b, u_init, w=w, mode=C.MODE_CG_STABLE, tol=tol, max_iter=max_iter, eps=eps)
    _cg_messages(res, "stable")
    u = res.x.view(N, A.bs).to(device=torch.device(device), dtype=dtype)
    return (u, res) if return_info else u


# ============================================================================ final_solver (`solver/solver.py:231-295`)
def final_solver(K, elements, F, rbe2, u_init=None, tol=1e-10, max_iter=1000, device="cuda:0", dtype=torch.float64,
                 eps=1e-30, return_info=False):
    """The reference's out-of-place CG: the iteration of `stable_conjugate_gradient_solver` (the nodes `rbe2` held
    at zero through a 0/1 mask, alpha = rs/(pAp+eps), beta = rs_new/(rs_old+eps), stop when sqrt(r.r) < tol), the
    same early-stop prints, and no message when max_iter is reached (`:231-295` has no for-else). Runs the same
    device CG (mode CG_STABLE). The reference builds u with requires_grad for autograd through its torch ops; the
    device solve returns a plain tensor."""
    dev = _dev(device)
    N = F.shape[0]
    A = assemble(K, elements, N, dev)
    w = _free_mask(N, A.bs, rbe2, dev)
    b = F.to(device=dev, dtype=F64).reshape(-1)
    res = A.pcg(b, u_init, w=w, mode=C.MODE_CG_STABLE, tol=tol, max_iter=max_iter, eps=eps)
    if res.status != C.PCG_MAXITER:
        _cg_messages(res, "stable")
    u = res.x.view(N, A.bs).to(device=torch.device(device), dtype=dtype)
    return (u, res) if return_info else u


# ============================================================================ constrained CG (`solver/solver.py:394-759`)
def _constrained_messages(res):
    """`solver/solver.py:566-598` / `:735-757`."""
    if res.status == C.PCG_CONVERGED:
        print(f"[CG] Converged @ iter {res.iterations}, residual norm = {res.rz:.3e}")
    elif res.status == C.PCG_BREAKDOWN:
        print(f"[CG] Early terminate @ iter {res.iterations}: p^T K p = {res.pq:.3e}, not valid for SPD.")
    elif res.status == C.PCG_ALPHA_NAN:
        print(f"[CG] Terminate @ iter {res.iterations}: alpha is NaN/Inf.")
    elif res.status == C.PCG_BETA_NAN:
        print(f"[CG] Terminate @ iter {res.iterations}: beta is NaN/Inf.")
    else:
        print("[CG] Did not converge within max_iter.")


def _constrained_solve(K, elements, F, cons_args, order, u_init, tol, max_iter, device, dtype, eps, return_info):
    dev = _dev(device)
    N = F.shape[0]
    A = assemble(K, elements, N, dev)
    if F.shape[1] != A.bs:
        raise ValueError(f"F is [N, {F.shape[1]}] but the element matrices have {A.bs} dofs per node")
    cs = ConstraintSet(N, A.bs, dev, *cons_args, order=order)
    b = F.to(device=dev, dtype=F64).reshape(-1)
    res = A.pcg(b, u_init, w=cs.mask(), mode=C.MODE_CG_CONSTRAINED, tol=tol, max_iter=max_iter, eps=eps,
                schedule=_sys.SCHED_THREE, constraints=cs)
    _constrained_messages(res)
    u = res.x.view(N, A.bs).to(device=torch.device(device), dtype=dtype)
    return (u, res) if return_info else u


def constrained_conjugate_gradient_solver(K, elements, F, rbe2_list, spc_list, u_init=None, tol=1e-10, max_iter=1000,
                                          device="cuda:0", dtype=torch.float64, eps=1e-30, return_info=False):
    """CG on the assembled K with RBE2 (slave dofs follow the master) and SPC (prescribed values) enforced after
    every update, residual zeroed on those dofs; r0 = F - K u0 is formed before the first projection, like the
    reference (`solver/solver.py:512-600`). Stop when sqrt(r.r) < tol. Returns u [N, dpn] (fp64 arithmetic)."""
    cons = (parse_spc_list(spc_list, "cpu"), parse_rbe2_list(rbe2_list, "cpu"))  # noqa: F405
    return _constrained_solve(K, elements, F, cons, 0, u_init, tol, max_iter, device, dtype, eps, return_info)


def new_constrained_conjugate_gradient_solver(K, elements, N, rbe2_list, rbe3_list, spc_list, load_list, u_init=None,
                                              tol=1e-10, max_iter=1000, device="cuda:0", dtype=torch.float64,
                                              eps=1e-30, return_info=False):
    """F [N, 3] from the nodal loads, then the constrained CG with SPC, RBE2 and RBE3 (master = weighted mean of
    its slaves per dof) enforced after every update (`solver/solver.py:702-759`)."""
    F = torch.zeros((N, 3), dtype=F64)
    apply_loads_to_F(F, load_list)  # noqa: F405
    cons = (parse_spc_list(spc_list, "cpu"), parse_rbe2_list(rbe2_list, "cpu"),  # noqa: F405
            parse_rbe3_list(rbe3_list, "cpu"))  # noqa: F405
    return _constrained_solve(K, elements, F, cons, 1, u_init, tol, max_iter, device, dtype, eps, return_info)


# ============================================================================ PCG (`solver/solver.py:766-833`)
def preconditioned_conjugate_gradient_solver(K, elements, F, M_inv, u_init=None, tol=1e-8, max_iter=1000,
                                             device="cuda:0", dtype=torch.float32, return_info=False):
    """Jacobi-PCG: z = M_inv r, stop when sqrt(r.z) < tol (absolute), no eps and no breakdown guards; fixed DOFs
    are handled only through zeros in M_inv, as in the reference. Returns u [N, dpn].
    Arithmetic is fp64 whatever `dtype` (the reference's default fp32 only sets the output dtype here)."""
    dev = _dev(device)
    N = F.shape[0]
    A = assemble(K, elements, N, dev)
    w = M_inv.to(device=dev, dtype=F64).reshape(-1)
    b = F.to(device=dev, dtype=F64).reshape(-1)
    res = A.pcg(b, u_init, w=w, mode=C.MODE_PCG, tol=tol, max_iter=max_iter)
    if res.status == C.PCG_CONVERGED:
        print(f"Converged after {res.iterations} iterations.")
    else:
        print("Preconditioned CG did not converge within the maximum number of iterations.")
    u = res.x.view(N, A.bs).to(device=torch.device(device), dtype=dtype)
    return (u, res) if return_info else u


def compute_diagonal_preconditioner(K, elements, N, device="cuda:0", dtype=torch.float32, exact_diagonal=False):
    """M_inv [N, dpn] of `solver/solver.py:814-833`, inf -> 0.

    By default this reproduces the reference bit for bit, including its slice bug (quirk Q1: `K.view(-1, d)
    [:, ::d+1]` picks column 0 of every element row, `:828`). exact_diagonal=True gives 1/diag(K), the
    function's documented intent (what `solve_tet4` and bench.py use)."""
    lib = C.lib()
    dev = _dev(device)
    elements = elements.to(device=dev, dtype=LONG).contiguous()
    Kd = K.to(device=dev, dtype=F64).contiguous()
    npe = elements.shape[1]
    dpn = Kd.shape[-1] // npe
    inc_ptr, inc = cached_incidence(elements, N)
    diag = torch.empty(N * dpn, dtype=F64, device=dev)
    C.check(lib.fem_ebe_diag(C.ptr(Kd), C.ptr(elements), npe, dpn, C.ptr(inc_ptr), C.ptr(inc), N,
                             0 if exact_diagonal else 1, C.ptr(diag), C.stream(dev)), "fem_ebe_diag")
    minv = torch.empty_like(diag)
    C.check(lib.fem_invert_diag(C.ptr(diag), N * dpn, C.ptr(minv), C.stream(dev)), "fem_invert_diag")
    return minv.view(N, dpn).to(device=torch.device(device), dtype=dtype)


# ============================================================================ static solve (`solver/solver.py:11-135`)
def static_structure_solver(coords, force, fixed, c3d4=None, c3d6=None, c3d8=None, s3=None, s4=None, material=None,
                            u_init=None, tol=1e-10, max_iter=1000, device="cuda:0", dtype=torch.float64, eps=1e-30,
                            return_info=False):
    """Mixed solid mesh: assemble c3d4 (`compute_c3d4_K_matrix`), c3d8 (8-point rule) and c3d6 (single point)
    into one global operator, then stable CG with `fixed` nodes held at zero. u, force are [N, 6]; solids use
    columns 0-2. Shells (s3/s4) are out of scope of this build."""
    if s3 is not None or s4 is not None:
        raise NotImplementedError("static_structure_solver: shell elements (s3/s4) are out of scope of fem355")
    dev = _dev(device)
    coords = coords.to(device=dev, dtype=F64).contiguous()
    force = force.to(device=dev, dtype=F64)
    N = coords.shape[0]
    if force.shape[1] > 3 and bool((force[:, 3:] != 0).any()):
        raise ValueError("static_structure_solver: rotational loads need shell elements (out of scope)")
    fams = []
    E, nu = material["E"], material["nu"]
    if c3d4 is not None:
        el = c3d4.to(device=dev, dtype=LONG).contiguous()
        fams.append((compute_c3d4_K_matrix(coords, el, E, nu, device=dev, dtype=F64), el))
    if c3d8 is not None:
        el = c3d8.to(device=dev, dtype=LONG).contiguous()
        fams.append((compute_c3d8_K_matrix(coords, el, E, nu, device=dev, dtype=F64), el))
    if c3d6 is not None:
        el = c3d6.to(device=dev, dtype=LONG).contiguous()
        fams.append((compute_c3d6_K_matrix(coords, el, E, nu, device=dev, dtype=F64), el))
    print("Preprocessing done.")
    npe_max = max(el.shape[1] for _, el in fams)
    g = _sys.build_graph(_sys.pad_connectivity([el for _, el in fams], npe_max), N)
    A = _sys.SellMatrix(g, 3)
    for Ke, el in fams:
        A.add_element_matrices(Ke, el, inc=_sys.incidence(el, N))
    u0 = None
    if u_init is not None:
        u0 = u_init.to(device=dev, dtype=F64)[:, :3].contiguous()
    w = _free_mask(N, 3, fixed, dev)
    res = A.pcg(force[:, :3].contiguous(), u0, w=w, mode=C.MODE_CG_STABLE, tol=tol, max_iter=max_iter, eps=eps)
    _cg_messages(res, "static")
    u = torch.zeros((N, 6), dtype=F64, device=dev)
    if u_init is not None:
        u[:, 3:] = u_init.to(device=dev, dtype=F64)[:, 3:]
    u[:, :3] = res.x.view(N, 3)
    u[torch.as_tensor(fixed).to(device=dev, dtype=LONG)] = 0.0
    u = u.to(device=torch.device(device), dtype=dtype)
    return (u, res) if return_info else u


# ============================================================================ fused mesh -> solution pipeline
def solve_tet4(coords, elements, f, fixed, kind="poisson", E=1.0, nu=0.0, tol=1e-8, max_iter=10000, device="cuda:0",
               rtol=None, reorder=None, operator="assembled"):
    """Assembly + Jacobi-PCG straight from the mesh (the benchmark pipeline; no element matrices stored):
    c3d4 Poisson (dpn 1, kappa = E) or elasticity (dpn 3), Dirichlet zero on `fixed` nodes via zeros in the
    exact Jacobi M_inv, reference PCG semantics (absolute tol on sqrt(r.z); `rtol` scales it by sqrt(r0.z0)).
    reorder="rcm": solve on the reverse Cuthill-McKee renumbering of the nodes (system.rcm_order; for meshes in
    file order) and return u in the caller's numbering (the returned SellMatrix is the renumbered one).
    Returns (u [N, dpn], PcgResult, SellMatrix)."""
    dev = _dev(device)
    coords = coords.to(device=dev, dtype=F64).contiguous()
    elements = elements.to(device=dev, dtype=LONG).contiguous()
    N = coords.shape[0]
    dpn = 1 if kind == "poisson" else 3
    fixed_mask = torch.zeros(N, dtype=torch.bool, device=dev)
    fixed_mask[torch.as_tensor(fixed).to(device=dev)] = True
    b = f.to(device=dev, dtype=F64).reshape(N, dpn)
    inv = None
    if reorder is not None:
        if reorder != "rcm":
            raise ValueError(f"unknown reorder {reorder!r} (supported: 'rcm')")
        perm, inv = _sys.rcm_order(elements, N)
        coords, elements = _sys.renumber(coords, elements, perm, inv)
        fixed_mask, b = fixed_mask[perm], b[perm]
    if operator == "matfree":
        A = _sys.MatFreeOperator(coords, elements, kind, E, nu)
    else:
        A = _sys.assemble_tet4_system(coords, elements, kind, E, nu)
    A.check_singular()
    mask = torch.zeros((N, A.bs), dtype=torch.uint8, device=dev)
    mask[fixed_mask] = 1
    w = A.jacobi(mask.view(-1))
    b = b.reshape(-1).contiguous().clone()
    if rtol is not None:
        tol = float(rtol) * float(torch.sqrt(torch.dot(b, w * b)))
    res = A.pcg(b, None, w=w, mode=C.MODE_PCG, tol=tol, max_iter=max_iter)
    u = res.x.view(N, A.bs)
    if inv is not None:
        u = u[inv]
    return u, res, A

# every public function runs in the scope of the device its `device` argument names (_capi.on_device)
C.scope_module(globals())
