"""Constraint-aware CG (`solver/solver.py:394-759` of the reference): SPC, RBE2 and RBE3 in the reference's dict
formats, parsed once into flat device index arrays and enforced by the device CG itself (`k_constraints` in
`csrc/pcg.hip`, launched after every x update; the residual masking is the CG's 0/1 weight vector).

Reference-named entry points (re-exported by `solver.py`): parse_spc_list, parse_rbe2_list, parse_rbe3_list,
apply_loads_to_F, enforce_constraints, new_enforce_constraints. The two solvers live in `solver.py`.

Index semantics follow torch indexing as the reference uses it: node indices in [-N, N) (negative ones wrap),
dof indices in [-dpn, dpn); anything else raises IndexError before any device work.
"""
from __future__ import annotations

import torch

try:
    from . import _capi as C
except ImportError:  # pragma: no cover - flat import from the package directory
    import _capi as C  # type: ignore

F64 = torch.float64
LONG = torch.long


def _dev(device):
    C.lib()   # fails loudly without a HIP device (no CPU fallback)
    return C.compute_device(device)


# ---------------------------------------------------------------- the reference's parsers (`:396-476`, `:603-650`)
def parse_spc_list(spc_list, device="cuda:0", dtype=torch.float64):
    """[{'node', 'dofs', 'value'}] -> (spc_nodes int32 [S], spc_dofs int32 [S], spc_values [S]); spc -> dof order."""
    rows = [(c["node"], d, c["value"]) for c in spc_list for d in c["dofs"]]
    n, d, v = zip(*rows) if rows else ((), (), ())
    return (torch.tensor(n, device=device, dtype=torch.int32), torch.tensor(d, device=device, dtype=torch.int32),
            torch.tensor(v, device=device, dtype=dtype))


def parse_rbe2_list(rbe2_list, device="cuda:0"):
    """[{'master', 'slaves', 'dofs'}] -> (rbe2_slaves, rbe2_masters, rbe2_dofs) int32 [R]; rbe2 -> slave -> dof."""
    rows = [(s, c["master"], d) for c in rbe2_list for s in c["slaves"] for d in c["dofs"]]
    s, m, d = zip(*rows) if rows else ((), (), ())
    return tuple(torch.tensor(x, device=device, dtype=torch.int32) for x in (s, m, d))


def parse_rbe3_list(rbe3_list, device="cuda:0", dtype=torch.float64):
    """[{'master', 'slaves', 'dofs', 'weights'}] -> (rbe3_master, rbe3_slaves, rbe3_dofs int32 [E], rbe3_wts [E],
    rbe3_inds int64 [num+1] running offsets, weight_sums [num]); rbe3 -> slave -> dof."""
    m, s, d, w, sums, inds = [], [], [], [], [], [0]
    for c in rbe3_list:
        for k, sl in enumerate(c["slaves"]):
            for dof in c["dofs"]:
                m.append(c["master"])
                s.append(sl)
                d.append(dof)
                w.append(c["weights"][k])
        inds.append(inds[-1] + len(c["slaves"]) * len(c["dofs"]))
        sums.append(sum(c["weights"]))
    i32 = dict(device=device, dtype=torch.int32)
    return (torch.tensor(m, **i32), torch.tensor(s, **i32), torch.tensor(d, **i32),
            torch.tensor(w, device=device, dtype=dtype), torch.tensor(inds, device=device, dtype=torch.int64),
            torch.tensor(sums, device=device, dtype=dtype))


def apply_loads_to_F(F, load_list):
    """F[node, 0:3] += force for every {'node', 'force'} in order, in place (`:653-663`). The adds are done in
    F's dtype in list order (a handful of scalars; set-up, not the solve)."""
    if not load_list:
        return
    Fh = F.detach().cpu().clone()
    for ld in load_list:
        fx, fy, fz = ld["force"]
        Fh[ld["node"], 0] += fx
        Fh[ld["node"], 1] += fy
        Fh[ld["node"], 2] += fz
    F.copy_(Fh)


# ---------------------------------------------------------------- device constraint set
def _flat(nodes, dofs, N, dpn, what):
    """torch-indexing semantics of u[nodes, dofs] on a [N, dpn] array -> flat int64 dofs (host list)."""
    out = []
    for n, d in zip(nodes, dofs):
        n, d = int(n), int(d)
        if not (-N <= n < N) or not (-dpn <= d < dpn):
            raise IndexError(f"{what}: index ({n}, {d}) is out of bounds for a [{N}, {dpn}] displacement array")
        out.append((n % N) * dpn + (d % dpn))
    return out


def _tolist(t):
    return t.tolist() if torch.is_tensor(t) else list(t)


class ConstraintSet:
    """One constraint configuration as flat device arrays (fem_pcg_set_constraints / fem_enforce_constraints).

    order 0 = `enforce_constraints` (RBE2 then SPC), order 1 = `new_enforce_constraints` (SPC, RBE2, RBE3). RBE3
    sets become one group per (set, distinct dof) in ascending dof order (`:685-698`)."""

    def __init__(self, N, dpn, device, spc, rbe2, rbe3=None, order=0):
        self.N, self.dpn, self.order = int(N), int(dpn), int(order)
        self.n = self.N * self.dpn
        dev = _dev(device)
        self.device = dev
        sn, sd, sv = (_tolist(x) for x in spc)
        r2s, r2m, r2d = (_tolist(x) for x in rbe2)
        self.spc_dof = torch.tensor(_flat(sn, sd, N, dpn, "SPC"), dtype=LONG, device=dev)
        self.spc_val = torch.tensor([float(v) for v in sv], dtype=F64, device=dev)
        self.rbe2_slave = torch.tensor(_flat(r2s, r2d, N, dpn, "RBE2 slave"), dtype=LONG, device=dev)
        self.rbe2_master = torch.tensor(_flat(r2m, r2d, N, dpn, "RBE2 master"), dtype=LONG, device=dev)
        ptr, gm, gw, es, ew = [0], [], [], [], []
        if rbe3 is not None:
            m3, s3, d3, w3, inds, sums = (_tolist(x) for x in rbe3)
            for i in range(len(inds) - 1):
                a, b = int(inds[i]), int(inds[i + 1])
                if a == b:
                    continue
                for dval in sorted(set(int(d) for d in d3[a:b])):
                    sel = [e for e in range(a, b) if int(d3[e]) == dval]
                    es += _flat([s3[e] for e in sel], [dval] * len(sel), N, dpn, "RBE3 slave")
                    ew += [float(w3[e]) for e in sel]
                    gm += _flat([m3[a]], [dval], N, dpn, "RBE3 master")
                    gw.append(float(sums[i]))
                    ptr.append(len(es))
        self.G = len(gm)
        self.r3_ptr = torch.tensor(ptr, dtype=LONG, device=dev)
        self.r3_master = torch.tensor(gm, dtype=LONG, device=dev)
        self.r3_wsum = torch.tensor(gw, dtype=F64, device=dev)
        self.r3_slave = torch.tensor(es, dtype=LONG, device=dev)
        self.r3_w = torch.tensor(ew, dtype=F64, device=dev)

    def args(self):
        """fem_pcg_set_constraints arguments after the context handle."""
        return (self.order, self.rbe2_slave.numel(), C.ptr(self.rbe2_slave), C.ptr(self.rbe2_master),
                self.spc_dof.numel(), C.ptr(self.spc_dof), C.ptr(self.spc_val), self.G, C.ptr(self.r3_ptr),
                C.ptr(self.r3_master), C.ptr(self.r3_wsum), C.ptr(self.r3_slave), C.ptr(self.r3_w))

    def mask(self):
        """The CG weight vector: 0 where the reference zeroes r (SPC dofs, RBE2 slaves), 1 elsewhere."""
        w = torch.ones(self.n, dtype=F64, device=self.device)
        w[self.spc_dof] = 0.0
        w[self.rbe2_slave] = 0.0
        return w

    def enforce(self, u, r=None):
        """Project u (and zero r) in place on the device; u, r: [N, dpn] tensors of any dtype / device."""
        lib = C.lib()
        if tuple(u.shape) != (self.N, self.dpn) or (r is not None and tuple(r.shape) != (self.N, self.dpn)):
            raise ValueError(f"enforce: u / r must be [{self.N}, {self.dpn}]")

        def work(t):
            direct = t.device == self.device and t.dtype == F64 and t.is_contiguous()
            return t if direct else t.detach().to(device=self.device, dtype=F64).contiguous()

        uw = work(u)
        rw = work(r) if r is not None else None
        C.check(lib.fem_enforce_constraints(C.ptr(uw), C.ptr(rw) if rw is not None else None, self.n,
                                            *self.args(), C.stream(self.device)), "fem_enforce_constraints")
        if uw is not u:
            u.copy_(uw)
        if rw is not None and rw is not r:
            r.copy_(rw)


def enforce_constraints(u, r, spc_nodes, spc_dofs, spc_values, rbe2_slaves, rbe2_masters, rbe2_dofs):
    """RBE2 (u[slave, d] = u[master, d], gathered before written; r = 0) then SPC (u = value; r = 0), in place
    (`solver/solver.py:478-510`)."""
    N, dpn = u.shape
    ConstraintSet(N, dpn, u.device, (spc_nodes, spc_dofs, spc_values), (rbe2_slaves, rbe2_masters, rbe2_dofs),
                  order=0).enforce(u, r)


def new_enforce_constraints(u, r, spc_nodes, spc_dofs, spc_values, rbe2_slaves, rbe2_masters, rbe2_dofs,
                            rbe3_master, rbe3_slaves, rbe3_dofs, rbe3_weights, rbe3_inds, weight_sums):
    """SPC, then RBE2, then every RBE3 set in order: u[master, d] = sum w u[slave, d] / (sum w + 1e-30) per
    distinct dof ascending; r is not touched by RBE3 (`solver/solver.py:665-700`)."""
    N, dpn = u.shape
    ConstraintSet(N, dpn, u.device, (spc_nodes, spc_dofs, spc_values), (rbe2_slaves, rbe2_masters, rbe2_dofs),
                  (rbe3_master, rbe3_slaves, rbe3_dofs, rbe3_weights, rbe3_inds, weight_sums), order=1).enforce(u, r)


__all__ = ["parse_spc_list", "parse_rbe2_list", "parse_rbe3_list", "apply_loads_to_F", "enforce_constraints",
           "new_enforce_constraints", "ConstraintSet"]

# every public function runs in the scope of the device its `device` argument names (_capi.on_device)
C.scope_module(globals())
