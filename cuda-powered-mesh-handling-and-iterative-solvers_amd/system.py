"""Device-resident global operator: pattern build, assembly into SELL-64, SpMV and the (P)CG driver.

This is the host runtime around the HIP kernels: it allocates device buffers with torch (plumbing only),
calls the C-ABI on the current HIP stream, and owns nothing the kernels compute. The reference has no
assembled operator (it is element-by-element, `solver/element.py:429-464`); the assembled matrix here is
the coalesced COO of `subdivision.ipynb:118-139`, so `A @ p == compute_nodal_forces(K, elements, p)`.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

from . import _capi as C

I32, I64, F64 = torch.int32, torch.int64, torch.float64


def _scoped(cls):
    """Class decorator: every public method (and __init__) runs with the current HIP device set to the object's
    device (`self.device`, or for __init__ the device of the first tensor argument's matrix), so the library's
    allocations and null-stream launches land where the tensors live (`_capi.device_scope`)."""
    import functools

    def wrap(fn):
        @functools.wraps(fn)
        def w(self, *args, **kwargs):
            dev = getattr(self, "device", None)
            if dev is None:   # __init__: SellMatrix(graph, bs) / PcgRunner(A, ...)
                a0 = args[0] if args else None
                dev = getattr(a0, "device", None) or getattr(getattr(a0, "cols", None), "device", None)
            if dev is None or not torch.cuda.is_available():
                return fn(self, *args, **kwargs)
            with C.device_scope(dev):
                return fn(self, *args, **kwargs)
        return w

    for name, fn in list(vars(cls).items()):
        if callable(fn) and (name == "__init__" or not name.startswith("_")) and not isinstance(fn, (staticmethod,
                                                                                                    classmethod, property)):
            setattr(cls, name, wrap(fn))
    return cls


def _dev_scalar(dev, dtype, value):
    return torch.full((1,), value, dtype=dtype, device=dev)


# (P)CG kernel schedules (csrc/pcg.hip): 0 = three kernels with in-kernel grid reductions, 1 = fused (p formed
# inside the SpMV), 2 = deferred (partials summed by the next kernel, no grid atomics), 3 = persistent (one
# cooperative launch per chunk of single-reduction iterations, csrc/pcg_persist.hpp; falls back to 2 where its
# prerequisites do not hold)
SCHED_THREE, SCHED_FUSED, SCHED_DEFERRED, SCHED_PERSIST, SCHED_AUTO = 0, 1, 2, 3, 4
# measured on MI355X (10M-tet cube, 16-bit columns, paired layout; tools/persist_check.py, tools/spmv_tune.py):
# scalar Poisson 44.0 us/it persistent vs 79.4 deferred; 3x3 elasticity: the bs = 3 persistent kernel while the state
# fits on chip (1.2M tets: 43.8 vs 63.2 us three-kernel), the three-kernel schedule past that (10M: 436 vs 633 us for
# the overflow build) -- SCHED_AUTO picks per matrix
DEFAULT_SCHEDULE = {1: SCHED_PERSIST, 3: SCHED_AUTO}


def _schedule(fused, schedule, bs=1):
    if schedule is not None:
        return int(schedule)
    return SCHED_FUSED if fused else DEFAULT_SCHEDULE.get(bs, SCHED_THREE)


@dataclass
class PcgResult:
    x: torch.Tensor
    iterations: int      # the reference's reported count (i+1 at the stop)
    status: int          # _capi.PCG_*
    rz: float            # last r.z (r.r in CG mode) — the "Residual norm" the reference prints (squared)
    pq: float            # last p.Ap (printed on breakdown)
    history: torch.Tensor = None
    schedule: int = -1   # the kernel schedule the solve ran (SCHED_*; after any fallback)


@dataclass
class Graph:
    """Node graph of a mesh: incidence + CSR pattern + SELL-64 pattern, all on one device."""
    n_nodes: int
    npe: int
    inc_ptr: torch.Tensor
    inc: torch.Tensor
    rowptr: torch.Tensor
    colidx: torch.Tensor
    diagpos: torch.Tensor
    slice_ptr: torch.Tensor
    cols: torch.Tensor
    c2s: torch.Tensor = None     # CSR -> SELL entry map, formed on first use (csr2sell)
    dcols: torch.Tensor = None   # int16 col - row deltas, or None when the bandwidth exceeds 32767
    max_width: int = 0           # widest SELL slice in columns (0: unknown)

    @property
    def csr2sell(self):
        """CSR position -> SELL entry (int64 [nnz]). The fused pattern pass skips it (the c3d4 assembly, Jacobi and
        the solvers address SELL through the slice pointer); the stored-K_e assembly and the CSR export form it
        here on first use, on the graph's device and current stream."""
        if self.c2s is None:
            with C.device_scope(self.rowptr.device):
                c2s = torch.empty(max(self.nnz, 1), dtype=I64, device=self.rowptr.device)
                C.check(C.lib().fem_sell_csr2sell(C.ptr(self.rowptr), self.n_nodes, C.ptr(self.slice_ptr),
                                                  C.ptr(c2s), C.stream(self.rowptr.device)), "fem_sell_csr2sell")
                self.c2s = c2s
        return self.c2s

    def solver_layout(self):
        """The bs = 1 solver layout of this pattern (include/fem355.h fem_sell_sl_pattern): lane-paired deltas,
        slice-uniform delta lists, and the persistent schedule's gather windows for this device's grid -- formed once
        per pattern, on first use (or by build_graph(..., solver_layout=True) in its fill pass). None without 16-bit
        deltas."""
        if self.dcols is None:
            return None
        sl = getattr(self, "_sl", None)
        if sl is None:
            dev = self.rowptr.device
            with C.device_scope(dev):
                sl = _solver_layout_arrays(dev, self.sell_entries, self.n_nodes)
                C.check(C.lib().fem_sell_sl_pattern(self.n_nodes, C.ptr(self.slice_ptr), C.ptr(self.dcols), sl.G,
                                                    C.ptr(sl.pcols), C.ptr(sl.ucol), C.ptr(sl.uoff), C.ptr(sl.win),
                                                    C.stream(dev)), "fem_sell_sl_pattern")
            self._sl = sl
        return sl

    @property
    def nnz(self):
        return int(self.colidx.numel())

    @property
    def sell_entries(self):
        return int(self.cols.numel())


@dataclass
class SolverLayout:
    """Solver layout of a bs = 1 pattern (Graph.solver_layout): paired deltas, uniform lists, gather windows."""
    pcols: torch.Tensor
    ucol: torch.Tensor
    uoff: torch.Tensor
    win: torch.Tensor
    G: int


_NCU = {}


def _cu_count(dev):
    """Compute units of `dev` (cached: this sits between the pattern build's one sync and its next launch)."""
    k = dev.index if dev.index is not None else torch.cuda.current_device()
    if k not in _NCU:
        _NCU[k] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _NCU[k]


def _solver_layout_arrays(dev, ent, n_nodes):
    """Uninitialised SolverLayout arrays of a pattern with `ent` SELL entries (G: the persistent grid of `dev`)."""
    ncu = _cu_count(dev)
    G = (ncu // 8) * 8
    ns = (n_nodes + 63) // 64
    return SolverLayout(torch.empty(max(ent, 1), dtype=torch.int16, device=dev),
                        torch.empty(2 * (ent // 64) + 2, dtype=torch.int16, device=dev),
                        torch.empty(max(ns, 1), dtype=I32, device=dev),
                        torch.empty(max(2 * G, 1), dtype=I32, device=dev), G)


def check_connectivity(elements: torch.Tensor, n_nodes: int):
    """IndexError for a node index outside [0, n_nodes) (the kernels gather without bounds checks; the
    reference's torch indexing raises IndexError on such input). One device reduction + sync."""
    if elements.numel() == 0:
        return
    lo, hi = (int(v) for v in torch.stack(torch.aminmax(elements)).cpu())   # one device-to-host copy
    if lo < 0 or hi >= n_nodes:
        raise IndexError(f"element connectivity references node {lo if lo < 0 else hi}, outside [0, {n_nodes})")


def incidence(elements: torch.Tensor, n_nodes: int, checked: bool = False):
    """Deterministic node -> (element, local) incidence of a connectivity block [M, npe] (int64, device)."""
    with C.device_scope(elements.device):
        return _incidence(elements, n_nodes, checked)


def _incidence(elements, n_nodes, checked):
    lib = C.lib()
    if not checked:
        check_connectivity(elements, n_nodes)
    dev = elements.device
    M, npe = elements.shape
    inc_ptr = torch.empty(n_nodes + 1, dtype=I32, device=dev)
    inc = torch.empty(M * npe, dtype=I32, device=dev)
    # workspace from torch's caching allocator: it is reused by the pattern arrays allocated right after
    work = torch.empty(max(int(lib.fem_incidence_work_bytes(M * npe, n_nodes)), 1), dtype=torch.uint8, device=dev)
    C.check(lib.fem_incidence(C.ptr(elements), M, npe, n_nodes, C.ptr(inc_ptr), C.ptr(inc), C.ptr(work),
                              C.stream(dev)), "fem_incidence")
    return inc_ptr, inc


def build_graph(elements: torch.Tensor, n_nodes: int, compress: bool = True, solver_layout: bool = False) -> Graph:
    """Node-graph CSR + SELL-64 pattern of `elements` (one element family, int64 [M, npe] on the device).
    The rows are the coalesced pattern of the reference's COO assembly (`subdivision.ipynb:118-139`).
    compress: also derive 16-bit column deltas (used by the SpMV when every |col - row| <= 32767).
    solver_layout: with the deltas, also form the bs = 1 solver layout (Graph.solver_layout) in the same fill pass."""
    with C.device_scope(elements.device):
        return _build_graph(elements, n_nodes, compress, solver_layout)


def _build_graph(elements, n_nodes, compress, solver_layout=False):
    lib = C.lib()
    dev = elements.device
    elements = elements.contiguous()
    M, npe = elements.shape
    st = C.stream(dev)
    # the connectivity check rides on the incidence's count pass (out-of-range slots are left out; the kernels
    # below only compare node ids, never index by them) and is read back with the sizes in the one sync below
    inc_ptr = torch.empty(n_nodes + 1, dtype=I32, device=dev)
    inc = torch.empty(M * npe, dtype=I32, device=dev)
    bad = torch.empty(1, dtype=I32, device=dev)
    work = torch.empty(max(int(lib.fem_incidence_work_bytes(M * npe, n_nodes)), 1), dtype=torch.uint8, device=dev)
    C.check(lib.fem_incidence_checked(C.ptr(elements), M, npe, n_nodes, C.ptr(inc_ptr), C.ptr(inc), C.ptr(work),
                                      C.ptr(bad), st), "fem_incidence_checked")
    del work
    row_len = torch.empty(n_nodes, dtype=I32, device=dev)
    tmp = torch.empty(max(int(lib.fem_graph_tmp_len(n_nodes)), 1), dtype=I32, device=dev)
    ovf = torch.empty(1, dtype=I32, device=dev)   # 1: some neighbour is > 32767 rows away (no 16-bit deltas)
    C.check(lib.fem_graph_count2(C.ptr(elements), npe, C.ptr(inc_ptr), C.ptr(inc), n_nodes, C.ptr(row_len),
                                 C.ptr(tmp), C.ptr(ovf), st), "fem_graph_count2")
    rowptr = torch.empty(n_nodes + 1, dtype=I32, device=dev)
    work = torch.empty(int(lib.fem_scan_work_len(n_nodes)) + 1, dtype=I32, device=dev)
    C.check(lib.fem_scan_i32(C.ptr(row_len), n_nodes, C.ptr(rowptr), C.ptr(work), st), "fem_scan_i32")
    # the SELL slice widths need only the row lengths: both sizes come back in ONE device-to-host copy
    ns = (n_nodes + 63) // 64
    width = torch.empty(ns, dtype=I64, device=dev)
    C.check(lib.fem_sell_widths(C.ptr(rowptr), n_nodes, C.ptr(width), st), "fem_sell_widths")
    slice_ptr = torch.empty(ns + 1, dtype=I64, device=dev)
    work64 = torch.empty(int(lib.fem_scan_work_len(ns)) + 1, dtype=I64, device=dev)
    C.check(lib.fem_scan_i64(C.ptr(width), ns, C.ptr(slice_ptr), C.ptr(work64), st), "fem_scan_i64")
    sizes = torch.empty(5, dtype=I64, device=dev)   # {nnz, entries, bad, far, widest slice}: one launch
    C.check(lib.fem_graph_sizes(C.ptr(rowptr), C.ptr(slice_ptr), C.ptr(width), n_nodes, C.ptr(bad), C.ptr(ovf),
                                C.ptr(sizes), st), "fem_graph_sizes")
    nnz, ent, nbad, far, maxw = (int(v) for v in sizes.cpu())
    if nbad:   # the sync of the build; the message names the offending node like check_connectivity
        check_connectivity(elements, n_nodes)
    # int32 row pointers / column slots: the int32 scan would wrap past 2^31 entries; the int64 slice scan cannot
    # (per-row lengths stay exact under wrap-around), and nnz <= ent
    if ent >= 2**31:
        raise ValueError(f"fem355: {ent} SELL entries (>= node-graph entries) exceed the int32 pattern "
                         "(split the mesh over GPUs)")
    colidx = torch.empty(nnz, dtype=I32, device=dev)
    diagpos = torch.empty(n_nodes, dtype=I32, device=dev)
    cols = torch.empty(ent, dtype=I32, device=dev)
    dcols = torch.empty(max(ent, 1), dtype=torch.int16, device=dev) if compress and not far else None
    sl = None
    if dcols is not None and solver_layout and os.environ.get("FEM355_SL_SEPARATE") is None:
        sl = _solver_layout_arrays(dev, ent, n_nodes)
        C.check(lib.fem_graph_sell_fill_sl(C.ptr(elements), npe, C.ptr(inc_ptr), C.ptr(inc), n_nodes, C.ptr(rowptr),
                                           C.ptr(tmp), C.ptr(slice_ptr), C.ptr(colidx), C.ptr(diagpos), C.ptr(cols),
                                           C.ptr(dcols), sl.G, C.ptr(sl.pcols), C.ptr(sl.ucol), C.ptr(sl.uoff),
                                           C.ptr(sl.win), st), "fem_graph_sell_fill_sl")
    else:
        C.check(lib.fem_graph_sell_fill(C.ptr(elements), npe, C.ptr(inc_ptr), C.ptr(inc), n_nodes, C.ptr(rowptr),
                                        C.ptr(tmp), C.ptr(slice_ptr), C.ptr(colidx), C.ptr(diagpos), C.ptr(cols),
                                        C.ptr(dcols), None, None, st), "fem_graph_sell_fill")
    del tmp
    g = Graph(n_nodes, npe, inc_ptr, inc, rowptr, colidx, diagpos, slice_ptr, cols)
    if sl is not None:
        g._sl = sl
    g.dcols = dcols
    g.max_width = maxw // 64 if ns > 0 else 0   # widest slice, in columns (the value kernels' window choice)
    return g


def rcm_order(elements: torch.Tensor, n_nodes: int, graph: Graph = None):
    """Reverse Cuthill-McKee renumbering of the mesh nodes, computed on the device (csrc/reorder.hip) ->
    (perm, inv), int64 on the elements' device: new node k is old node perm[k], old node v becomes inv[v].
    Opt-in: meshes read in file order (`vtk_loader_to_torch`, `solver/element.py:39-90`) scatter the SELL slices'
    gathers and can need int32 columns; the renumbered mesh's operator is the same matrix under a symmetric
    permutation, so solutions map back exactly up to summation order."""
    with C.device_scope(elements.device):
        lib = C.lib()
        g = graph if graph is not None else build_graph(elements, n_nodes, compress=False)
        dev = elements.device
        perm = torch.empty(n_nodes, dtype=I32, device=dev)
        inv = torch.empty(n_nodes, dtype=I32, device=dev)
        work = torch.empty(max(int(lib.fem_rcm_work_len(n_nodes)), 1), dtype=I32, device=dev)
        lv = ctypes.c_int(0)
        C.check(lib.fem_rcm(C.ptr(g.rowptr), C.ptr(g.colidx), n_nodes, C.ptr(perm), C.ptr(inv), C.ptr(work),
                            ctypes.byref(lv), C.stream(dev)), "fem_rcm")
        return perm.long(), inv.long()


def renumber(coords: torch.Tensor, elements: torch.Tensor, perm: torch.Tensor, inv: torch.Tensor):
    """The mesh under a node renumbering (rcm_order): coordinates in the new order, connectivity in new ids."""
    return coords[perm], inv[elements]


def pad_connectivity(blocks, npe_max):
    """Concatenate element families into one [sum M, npe_max] block for the pattern (padding repeats node 0
    of the element; duplicates vanish in the unique-neighbour pass)."""
    out = []
    for el in blocks:
        if el.shape[1] < npe_max:
            el = torch.cat([el, el[:, :1].expand(-1, npe_max - el.shape[1])], dim=1)
        out.append(el)
    return torch.cat(out, 0).contiguous()


def uniform_slices(lib, h, s_begin=0, s_end=-1):
    """fem_pcg_uniform_slices of a solver context handle: (uniform slices, slices, column-index bytes per SpMV)."""
    u, n, ib = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    C.check(lib.fem_pcg_uniform_slices(h, int(s_begin), int(s_end), ctypes.byref(u), ctypes.byref(n),
                                       ctypes.byref(ib)), "fem_pcg_uniform_slices")
    return u.value, n.value, ib.value


@_scoped
class SellMatrix:
    """Assembled global operator in SELL-64 with bs x bs blocks (bs = dofs per node)."""

    def __init__(self, graph: Graph, bs: int):
        self.g = graph
        self.bs = bs
        self.device = graph.cols.device
        # values are zeroed lazily: the first add_element_matrices of a fresh matrix STORES every value (padding
        # included) instead of adding onto a zeroed buffer -- one memset and one read of the matrix fewer
        self._vals = None            # plain SELL values, allocated on first use
        self._svals = None           # solver layout values (include/fem355.h fem_assemble_tet4_sl)
        self._plain_ok = False       # which of the two holds the current values
        self._sl_ok = False
        self._fresh = True
        self.use16 = graph.dcols is not None   # 16-bit column deltas in every SpMV of this matrix

    def _plain_buf(self):
        if self._vals is None:
            self._vals = torch.empty(max(self.g.sell_entries, 1) * self.bs * self.bs, dtype=F64, device=self.device)
        return self._vals

    @property
    def solver_layout(self):
        """True while the values live in the solver layout (the default of a fresh matrix's assembly: the PCG reads
        them as they are, no per-solve conversion, one resident copy); `vals` then forms the plain copy on demand."""
        return self._sl_ok

    @property
    def vals(self):
        """SELL values [entries * bs * bs] (plane layout); zero until something was added. The caller may edit them in
        place: once handed out, the plain values are the matrix (a solver-layout copy is dropped, so later matvec /
        jacobi / pcg read the edited values; the next solve converts them at its start)."""
        v = self.plain_values()
        self._sl_ok = False
        return v

    def plain_values(self):
        """The plain SELL values for READING (kernels, exports): formed from the solver layout when only it holds the
        values, which stays the matrix -- edits through this tensor are not seen by solves (use `vals` to edit)."""
        if self._fresh:
            self._plain_buf().zero_()
            self._fresh = False
            self._plain_ok = True
        elif not self._plain_ok and self._sl_ok:   # plain copy of a solver-layout matrix
            sl = self.g.solver_layout()
            C.check(C.lib().fem_sell_sl_unpair(self.g.n_nodes, self.bs, C.ptr(self.g.slice_ptr), C.ptr(self.g.dcols),
                                               C.ptr(sl.uoff), C.ptr(sl.ucol), C.ptr(self.g.rowptr),
                                               C.ptr(self._svals), C.ptr(self._plain_buf()), C.stream(self.device)),
                    "fem_sell_sl_unpair")
            self._plain_ok = True
        return self._vals

    def _sl_target(self):
        """True when the next assembly writes the solver layout: 16-bit deltas, a fresh matrix or one held only there
        (FEM355_SL=0 keeps the plain layout)."""
        return (self.use16 and self.bs in (1, 3) and os.environ.get("FEM355_SL", "1") != "0"
                and (self._fresh or (self._sl_ok and not self._plain_ok)))

    def _svals_buf(self):
        if self._svals is None:
            self._svals = torch.empty(max(self.g.sell_entries, 1) * self.bs * self.bs, dtype=F64, device=self.device)
        return self._svals

    def _modify_plain(self):
        """The plain values about to change: current (or fresh), and the solver layout stale afterwards."""
        if not self._fresh:
            self.plain_values()   # forms the plain copy when only the solver layout holds the values
        self._plain_buf()
        self._sl_ok = False

    @property
    def n_rows(self):
        return self.g.n_nodes

    @property
    def n(self):
        return self.g.n_nodes * self.bs

    # ---------------------------------------------------------------- assembly
    def add_element_matrices(self, Ke: torch.Tensor, elements: torch.Tensor, inc=None):
        """vals += coalesce(P_e^T K_e P_e) of one element family (deterministic row-gather)."""
        lib = C.lib()
        elements = elements.contiguous()
        Ke = Ke.to(F64).contiguous()
        npe = elements.shape[1]
        if Ke.shape[-1] != npe * self.bs:
            raise ValueError(f"element matrix size {Ke.shape[-1]} != {npe}*{self.bs}")
        inc_ptr, inc_ = inc if inc is not None else (
            (self.g.inc_ptr, self.g.inc) if npe == self.g.npe and elements.shape[0] * npe == self.g.inc.numel()
            else incidence(elements, self.g.n_nodes))
        # bs = 3 with the pattern's widest slice known: the tile form writes the SELL planes directly (csr2sell unused)
        tiled = self.bs == 3 and self.g.max_width > 0 and not os.environ.get("FEM355_KE_ROWS") \
            and not os.environ.get("FEM355_KE_COLS") and not os.environ.get("FEM355_KE_DIRECT")
        if tiled and npe in (4, 6, 8, 10) and self._sl_target():   # straight into the solver layout (layout A)
            store = self._fresh
            self._fresh = False
            C.check(lib.fem_assemble_from_ke_sl(C.ptr(Ke), C.ptr(elements), npe, C.ptr(inc_ptr), C.ptr(inc_),
                                                self.g.n_nodes, C.ptr(self.g.rowptr), C.ptr(self.g.colidx),
                                                C.ptr(self.g.slice_ptr), 1 if store else 0, self.g.max_width,
                                                C.ptr(self._svals_buf()), C.stream(self.device)),
                    "fem_assemble_from_ke_sl")
            self._sl_ok, self._plain_ok = True, False
            return self
        # bs = 1: the tile form as well (k_assemble_ke_tile1: no csr2sell map, no memset)
        tiled = tiled or (self.bs == 1 and self.g.max_width > 0 and npe in (4, 6, 8, 10)
                          and not os.environ.get("FEM355_KE_ROWS"))
        self._modify_plain()
        store = self._fresh
        self._fresh = False
        self._plain_ok = True
        C.check(lib.fem_assemble_from_ke_ex2(C.ptr(Ke), C.ptr(elements), npe, self.bs, C.ptr(inc_ptr), C.ptr(inc_),
                                             self.g.n_nodes, C.ptr(self.g.rowptr), C.ptr(self.g.colidx),
                                             None if tiled else C.ptr(self.g.csr2sell), C.ptr(self.g.slice_ptr),
                                             self.g.nnz, self.g.sell_entries, 1 if store else 0,
                                             self.g.max_width if tiled else 0, C.ptr(self._vals),
                                             C.stream(self.device)), "fem_assemble_from_ke_ex2")
        return self

    def add_stiffness_and_mass(self, Ke: torch.Tensor, Me: torch.Tensor, elements: torch.Tensor, mass: "SellMatrix"):
        """This bs = 3 matrix += coalesce(P_e^T K_e P_e) and the bs = 1 `mass` (same pattern object) += coalesce(P_e^T
        Me_e P_e) in ONE pass (include/fem355.h fem_assemble_from_ke_mass_sl: one column search and one incidence walk
        for both). Me is the scalar [M, npe, npe] of `compute_M_matrix(..., scalar=True)`. Both results are bit-identical
        to `add_element_matrices(Ke, ...)` and `mass.add_element_matrices(Me, ...)`; where the fused form does not apply
        (plain layout wanted, a non-fresh pair in different states, another pattern) the two separate calls run."""
        lib = C.lib()
        elements = elements.contiguous()
        npe = elements.shape[1]
        Ke = Ke.to(F64).contiguous()
        Me = Me.to(F64).contiguous()
        if Me.shape[-1] != npe or Ke.shape[-1] != 3 * npe:
            raise ValueError(f"element matrix sizes {Ke.shape[-1]} / {Me.shape[-1]} != 3*{npe} / {npe}")
        fused = (self.bs == 3 and mass.bs == 1 and mass.g is self.g and self.g.max_width > 0
                 and npe in (4, 6, 8, 10) and npe == self.g.npe and elements.shape[0] * npe == self.g.inc.numel()
                 and self._sl_target() and self._fresh == mass._fresh
                 and not any(os.environ.get(k) for k in ("FEM355_KE_ROWS", "FEM355_KE_COLS", "FEM355_KE_DIRECT",
                                                         "FEM355_KM_SPLIT")))
        if not fused:
            self.add_element_matrices(Ke, elements)
            mass.add_element_matrices(Me, elements)
            return self
        store = self._fresh
        self._fresh = False
        mass._modify_plain()
        mass._fresh = False
        C.check(lib.fem_assemble_from_ke_mass_sl(C.ptr(Ke), C.ptr(Me), C.ptr(elements), npe, C.ptr(self.g.inc_ptr),
                                                 C.ptr(self.g.inc), self.g.n_nodes, C.ptr(self.g.rowptr),
                                                 C.ptr(self.g.colidx), C.ptr(self.g.slice_ptr), 1 if store else 0,
                                                 self.g.max_width, C.ptr(self._svals_buf()), C.ptr(mass._vals),
                                                 C.stream(self.device)), "fem_assemble_from_ke_mass_sl")
        self._sl_ok, self._plain_ok = True, False
        mass._plain_ok = True
        return self

    def add_element_matrices_sym(self, Kp: torch.Tensor, elements: torch.Tensor, inc=None):
        """vals += coalesce(P_e^T K_e P_e) from the packed symmetric K_e of `element._solid_ke_sym` (bs = 3: upper
        blocks only, the lower ones read as their transposes; include/fem355.h fem_assemble_from_ke_sym) -- the
        configs[4] internal path: about half the element-matrix bytes written and read. Same sums in the same order
        as `add_element_matrices` of the full K_e whose lower blocks mirror its upper ones."""
        lib = C.lib()
        if self.bs != 3 or self.g.max_width <= 0:
            raise ValueError("packed K_e assembly: bs = 3 with the pattern's slice width (tile form)")
        elements = elements.contiguous()
        npe = elements.shape[1]
        if Kp.dtype != F64 or Kp.dim() != 2 or Kp.shape[1] != int(lib.fem_ke_sym_stride(npe)):
            raise ValueError(f"packed K_e must be fp64 [M, {int(lib.fem_ke_sym_stride(npe))}]")
        Kp = Kp.contiguous()
        inc_ptr, inc_ = inc if inc is not None else (
            (self.g.inc_ptr, self.g.inc) if npe == self.g.npe and elements.shape[0] * npe == self.g.inc.numel()
            else incidence(elements, self.g.n_nodes))
        if self._sl_target():
            store = self._fresh
            self._fresh = False
            out, la = self._svals_buf(), 1
            self._sl_ok, self._plain_ok = True, False
        else:
            self._modify_plain()
            store = self._fresh
            self._fresh = False
            self._plain_ok = True
            out, la = self._vals, 0
        C.check(lib.fem_assemble_from_ke_sym(C.ptr(Kp), C.ptr(elements), npe, C.ptr(inc_ptr), C.ptr(inc_),
                                             self.g.n_nodes, C.ptr(self.g.rowptr), C.ptr(self.g.colidx),
                                             C.ptr(self.g.slice_ptr), 1 if store else 0, self.g.max_width, la,
                                             C.ptr(out), C.stream(self.device)), "fem_assemble_from_ke_sym")
        return self

    def add_tet4(self, coords: torch.Tensor, elements: torch.Tensor, E: float, nu: float = 0.0):
        """vals += the c3d4 operator computed on the fly (bs=3: elasticity E, nu; bs=1: Poisson, kappa=E)."""
        lib = C.lib()
        bad = _dev_scalar(self.device, I64, elements.shape[0])
        self._bad = (bad, elements.shape[0])
        # 16-bit deltas: straight into the solver layout (fresh matrix, or one already held there)
        if self._sl_target() and not os.environ.get("FEM355_ASM_ROWS"):
            sl = self.g.solver_layout() if self.bs == 1 else None
            store = self._fresh
            self._fresh = False
            C.check(lib.fem_assemble_tet4_sl(C.ptr(coords), C.ptr(elements), float(E), float(nu), self.bs,
                                             C.ptr(self.g.inc_ptr), C.ptr(self.g.inc), self.g.n_nodes,
                                             C.ptr(self.g.rowptr), C.ptr(self.g.colidx), C.ptr(self.g.slice_ptr),
                                             C.ptr(sl.uoff) if sl else None, C.ptr(sl.ucol) if sl else None,
                                             1 if store else 0, self.g.max_width, C.ptr(self._svals_buf()), C.ptr(bad),
                                             C.stream(self.device)), "fem_assemble_tet4_sl")
            self._sl_ok, self._plain_ok = True, False
            return self
        self._modify_plain()
        store = self._fresh   # a fresh matrix is stored whole (padding zeroed): no memset, no read of the values
        self._fresh = False
        self._plain_ok = True
        C.check(lib.fem_assemble_tet4_ex2(C.ptr(coords), C.ptr(elements), float(E), float(nu), self.bs,
                                          C.ptr(self.g.inc_ptr), C.ptr(self.g.inc), self.g.n_nodes,
                                          C.ptr(self.g.rowptr), C.ptr(self.g.colidx),
                                          C.ptr(self.g.csr2sell) if os.environ.get("FEM355_ASM_ROWS") else None,
                                          C.ptr(self.g.slice_ptr), 1 if store else 0, self.g.max_width,
                                          C.ptr(self._vals), C.ptr(bad), C.stream(self.device)),
                "fem_assemble_tet4_ex2")
        return self

    def check_singular(self):
        bad = getattr(self, "_bad", None)
        if bad is not None and int(bad[0].item()) < bad[1]:
            raise ValueError("Singular matrix encountered while computing B matrix.")

    # ---------------------------------------------------------------- operators
    def matvec(self, x: torch.Tensor, out: torch.Tensor = None):
        lib = C.lib()
        x = x.to(F64).contiguous()
        y = out if out is not None else torch.empty(self.n, dtype=F64, device=self.device)
        if self._sl_ok:
            if self.bs == 1:
                sl = self.g.solver_layout()
                pc, uo, uc = C.ptr(sl.pcols), C.ptr(sl.uoff), C.ptr(sl.ucol)
            else:   # layout A: plain deltas
                pc, uo, uc = C.ptr(self.g.dcols), None, None
            C.check(lib.fem_spmv_sl(self.g.n_nodes, self.bs, C.ptr(self.g.slice_ptr), pc, C.ptr(self._svals), uo, uc,
                                    C.ptr(x), C.ptr(y), C.stream(self.device)), "fem_spmv_sl")
        elif self.use16:
            C.check(lib.fem_spmv16(self.g.n_nodes, self.bs, C.ptr(self.g.slice_ptr), C.ptr(self.g.dcols),
                                   C.ptr(self.plain_values()), C.ptr(x), C.ptr(y), C.stream(self.device)), "fem_spmv16")
        else:
            C.check(lib.fem_spmv(self.g.n_nodes, self.bs, C.ptr(self.g.slice_ptr), C.ptr(self.g.cols),
                                 C.ptr(self.plain_values()), C.ptr(x), C.ptr(y), C.stream(self.device)), "fem_spmv")
        return y

    def attach_cols16(self, h):
        """Point a (P)CG context at the 16-bit column deltas when this matrix uses them."""
        if self.use16:
            C.check(C.lib().fem_pcg_set_cols16(h, C.ptr(self.g.dcols)), "fem_pcg_set_cols16")

    def solver_vals_ptr(self, fused=False):
        """The values pointer a (P)CG context is created with: the solver layout's when it holds the values (the
        context then reads them through attach_layout), else the plain values."""
        if self._sl_ok and not fused:
            return C.ptr(self._svals)
        return C.ptr(self.plain_values())

    def attach_layout(self, h, fused=False):
        """Hand a context the solver-layout values (+ the bs = 1 pattern, the gather windows) (fem_pcg_set_layout):
        no conversion at start."""
        if self._sl_ok and not fused:
            sl = self.g.solver_layout()
            one = self.bs == 1
            C.check(C.lib().fem_pcg_set_layout(h, C.ptr(self._svals), C.ptr(sl.pcols) if one else None,
                                               C.ptr(sl.uoff) if one else None, C.ptr(sl.ucol) if one else None,
                                               C.ptr(sl.win), sl.G), "fem_pcg_set_layout")

    def jacobi(self, fixed_mask: torch.Tensor = None):
        """w = 1/diag(A) (inf -> 0), zero on fixed DOFs (uint8 mask [n])."""
        lib = C.lib()
        w = torch.empty(self.n, dtype=F64, device=self.device)
        if self._sl_ok:
            sl = self.g.solver_layout() if self.bs == 1 else None
            C.check(lib.fem_jacobi_sl(C.ptr(self._svals), self.bs, C.ptr(self.g.rowptr), C.ptr(self.g.diagpos),
                                      C.ptr(self.g.slice_ptr), C.ptr(sl.uoff) if sl else None,
                                      C.ptr(sl.ucol) if sl else None, self.g.n_nodes,
                                      C.ptr(fixed_mask), C.ptr(w), C.stream(self.device)), "fem_jacobi_sl")
            return w
        C.check(lib.fem_jacobi(C.ptr(self.plain_values()), self.bs, C.ptr(self.g.rowptr), C.ptr(self.g.diagpos),
                               None, C.ptr(self.g.slice_ptr), self.g.n_nodes,
                               C.ptr(fixed_mask), C.ptr(w), C.stream(self.device)), "fem_jacobi")
        return w

    def csr(self):
        """(rowptr, colidx, vals[nnz, bs, bs]) in block-CSR (export / testing)."""
        lib = C.lib()
        out = torch.empty(max(self.g.nnz, 1) * self.bs * self.bs, dtype=F64, device=self.device)
        C.check(lib.fem_sell_to_csr_vals(C.ptr(self.plain_values()), self.bs, C.ptr(self.g.rowptr), self.g.n_nodes,
                                         C.ptr(self.g.csr2sell), C.ptr(self.g.slice_ptr), C.ptr(out),
                                         C.stream(self.device)), "fem_sell_to_csr_vals")
        return self.g.rowptr, self.g.colidx, out[: self.g.nnz * self.bs * self.bs].view(-1, self.bs, self.bs)

    def algorithmic_bytes_spmv(self, index_bytes=None, index_total=None):
        """HBM bytes one SpMV must move: (8 bs^2 + idx) nnzb + 4 (nb+1) + 16 n, fp64 values;
        idx = 4 for int32 columns (the survey's 12 nnz + 4(n+1) + 16 n for bs=1), 2 for 16-bit deltas.
        index_total: the column-index bytes of the stored format instead of idx nnzb (slice-uniform deltas:
        PcgRunner.uniform_slices())."""
        idx = index_bytes if index_bytes is not None else (2 if self.use16 else 4)
        nnzb, nb = self.g.nnz, self.g.n_nodes
        ib = idx * nnzb if index_total is None else int(index_total)
        return 8 * self.bs * self.bs * nnzb + ib + 4 * (nb + 1) + 16 * nb * self.bs

    # ---------------------------------------------------------------- solver
    def pcg(self, b, x0=None, w=None, mode=C.MODE_PCG, tol=1e-8, max_iter=1000, eps=1e-30, history=False,
            chunk=32, fused=False, schedule=None, constraints=None, tune=None):
        """Run the device (P)CG; returns a PcgResult. `constraints` (a constraints.ConstraintSet, mode
        CG_CONSTRAINED, 3-kernel schedule) is projected onto x at start and after every x update. `tune`: the
        context's FEM_TUNE_* flags instead of the library default (A/B checks)."""
        lib = C.lib()
        b = b.to(device=self.device, dtype=F64).contiguous().view(-1)
        x = (torch.zeros(self.n, dtype=F64, device=self.device) if x0 is None
             else x0.to(device=self.device, dtype=F64).clone().contiguous().view(-1))
        w = w.to(device=self.device, dtype=F64).contiguous().view(-1)
        hist = torch.full((max(max_iter, 1),), float("nan"), dtype=F64, device=self.device) if history else None
        h = ctypes.c_void_p()
        sched = _schedule(fused, schedule, self.bs)
        # the solver layout is read by the paired schedules (FEM_TUNE_PAIR = 2); fused / constrained contexts: plain
        plain = sched == SCHED_FUSED or constraints is not None or (tune is not None and not (int(tune) & 2))
        args = (self.g.n_nodes, self.bs, C.ptr(self.g.slice_ptr), C.ptr(self.g.cols), self.solver_vals_ptr(plain),
                C.ptr(b),
                C.ptr(x), C.ptr(w), mode, float(tol), float(eps), C.ptr(hist), hist.numel() if hist is not None else 0,
                C.stream(self.device), ctypes.byref(h))
        rc = lib.fem_pcg_create(*args)
        if rc == C.FEM_EHIP:   # out of memory: hand the library's recycled buffers and torch's cache back, retry once
            C.release_cache()
            torch.cuda.empty_cache()
            rc = lib.fem_pcg_create(*args)
        C.check(rc, "fem_pcg_create")
        try:
            C.check(lib.fem_pcg_set_schedule(h, sched), "fem_pcg_set_schedule")
            if tune is not None:
                C.check(lib.fem_pcg_set_tuning(h, int(tune)), "fem_pcg_set_tuning")
            C.check(lib.fem_pcg_set_entries(h, self.g.sell_entries), "fem_pcg_set_entries")
            self.attach_cols16(h)
            self.attach_layout(h, plain)
            if constraints is not None:
                C.check(lib.fem_pcg_set_constraints(h, *constraints.args()), "fem_pcg_set_constraints")
            it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
            C.check(lib.fem_pcg_solve(h, int(max_iter), int(chunk), ctypes.byref(it), ctypes.byref(stt),
                                      ctypes.byref(rz)), "fem_pcg_solve")
            sc = (ctypes.c_double * 6)()
            C.check(lib.fem_pcg_scalars(h, sc), "fem_pcg_scalars")
            ran = int(lib.fem_pcg_get_schedule(h))
            _check_sync(stt.value)
        finally:
            lib.fem_pcg_destroy(h)
        if hist is not None:
            hist = hist[: min(it.value, hist.numel())]
        return PcgResult(x, it.value, stt.value, rz.value, sc[1], hist, ran)


@_scoped
class MatFreeOperator:
    """Element-chunk c3d4 operator (include/fem355.h fem_mf_*, csrc/matfree.hip): y = K x formed from the vertex
    coordinates in every application -- the reference's element-by-element product (`compute_nodal_forces`,
    `solver/element.py:429-464`) of the c3d4 stiffness (`compute_c3d4_K_matrix`, `:883-903`; kind "elastic", 3 dofs
    per node) or the P1 Laplacian (kind "poisson", kappa = E), no matrix in memory. Same interface as SellMatrix for
    what the solvers use (n, bs, matvec, diag, jacobi, pcg, PcgRunner)."""

    is_matfree = True

    def __init__(self, coords: torch.Tensor, elements: torch.Tensor, kind="elastic", E=1.0, nu=0.0):
        lib = C.lib()
        self.device = coords.device
        self.coords = coords.to(F64).contiguous()
        self.elements = elements.to(torch.int64).contiguous()
        self.kind = kind
        self.bs = 1 if kind == "poisson" else 3
        self.n_nodes = self.coords.shape[0]
        self.n = self.n_nodes * self.bs
        self.M = self.elements.shape[0]
        self.h = ctypes.c_void_p()
        bad = ctypes.c_int64(-1)
        k = C.KIND_POISSON if kind == "poisson" else C.KIND_ELASTIC
        C.check(lib.fem_mf_create(C.ptr(self.coords), C.ptr(self.elements), self.M, self.n_nodes, k, float(E),
                                  float(nu), ctypes.byref(bad), C.stream(self.device), ctypes.byref(self.h)),
                "fem_mf_create")

    def info(self):
        """{chunks, slots, bs, static bytes one application streams, M, N}"""
        out = (ctypes.c_int64 * 6)()
        C.check(C.lib().fem_mf_info(self.h, out), "fem_mf_info")
        keys = ("chunks", "slots", "bs", "static_bytes", "elements", "nodes")
        return dict(zip(keys, list(out)))

    def layout(self):
        """(Morton element order [M], chunk element offsets, chunk slot offsets, slot nodes) as device int32."""
        i = self.info()
        z = lambda k: torch.empty(max(k, 1), dtype=torch.int32, device=self.device)
        eo, cp, sb, cn = z(self.M), z(i["chunks"] + 1), z(i["chunks"] + 1), z(i["slots"])
        C.check(C.lib().fem_mf_order(self.h, C.ptr(eo), C.ptr(cp), C.ptr(sb), C.ptr(cn), C.stream(self.device)),
                "fem_mf_order")
        return eo[: self.M], cp[: i["chunks"] + 1], sb[: i["chunks"] + 1], cn[: i["slots"]]

    def algorithmic_bytes(self):
        """HBM bytes one application must move at least: the static layout streams + the coordinates, x and y once."""
        return self.info()["static_bytes"] + 24 * self.n_nodes + 16 * self.n

    def matvec(self, x: torch.Tensor, out: torch.Tensor = None):
        x = x.to(device=self.device, dtype=F64).contiguous().view(-1)
        y = out if out is not None else torch.empty(self.n, dtype=F64, device=self.device)
        C.check(C.lib().fem_mf_apply(self.h, C.ptr(x), C.ptr(y), C.stream(self.device)), "fem_mf_apply")
        return y

    def diag(self):
        d = torch.empty(self.n, dtype=F64, device=self.device)
        C.check(C.lib().fem_mf_diag(self.h, C.ptr(d), C.stream(self.device)), "fem_mf_diag")
        return d

    def jacobi(self, fixed_mask: torch.Tensor = None):
        """w = 1/diag(K) (inf -> 0), zero on fixed DOFs (uint8 mask [n])."""
        d = self.diag()
        w = torch.empty_like(d)
        C.check(C.lib().fem_jacobi_from_diag(C.ptr(d), self.n, C.ptr(fixed_mask), C.ptr(w), C.stream(self.device)),
                "fem_jacobi_from_diag")
        return w

    def check_singular(self):
        return None   # fem_mf_create already raised for a singular element

    def create_context(self, b, x, w, mode, tol, eps, hist, hist_len, stream, h):
        lib = C.lib()
        if mode == C.MODE_CG_CONSTRAINED:
            raise ValueError("the element-chunk operator has no constrained CG (SPC / RBE2 / RBE3 projections need "
                             "the assembled matrix: SellMatrix.pcg(..., constraints=...))")
        C.check(lib.fem_pcg_create(self.n_nodes, self.bs, None, None, None, C.ptr(b), C.ptr(x), C.ptr(w), mode,
                                   float(tol), float(eps), C.ptr(hist), hist_len, stream, ctypes.byref(h)),
                "fem_pcg_create")
        rc = lib.fem_pcg_set_operator_mf(h, self.h)
        if rc != C.FEM_OK:
            lib.fem_pcg_destroy(h)
            C.check(rc, "fem_pcg_set_operator_mf")

    def pcg(self, b, x0=None, w=None, mode=C.MODE_PCG, tol=1e-8, max_iter=1000, eps=1e-30, history=False, chunk=32):
        """Device (P)CG on this operator (3-kernel schedule with the merged update); returns a PcgResult."""
        lib = C.lib()
        b = b.to(device=self.device, dtype=F64).contiguous().view(-1)
        x = (torch.zeros(self.n, dtype=F64, device=self.device) if x0 is None
             else x0.to(device=self.device, dtype=F64).clone().contiguous().view(-1))
        w = w.to(device=self.device, dtype=F64).contiguous().view(-1)
        hist = torch.full((max(max_iter, 1),), float("nan"), dtype=F64, device=self.device) if history else None
        h = ctypes.c_void_p()
        self.create_context(b, x, w, mode, tol, eps, hist, hist.numel() if hist is not None else 0,
                            C.stream(self.device), h)
        try:
            it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
            C.check(lib.fem_pcg_solve(h, int(max_iter), int(chunk), ctypes.byref(it), ctypes.byref(stt),
                                      ctypes.byref(rz)), "fem_pcg_solve")
            sc = (ctypes.c_double * 6)()
            C.check(lib.fem_pcg_scalars(h, sc), "fem_pcg_scalars")
            ran = int(lib.fem_pcg_get_schedule(h))
            _check_sync(stt.value)
        finally:
            lib.fem_pcg_destroy(h)
        if hist is not None:
            hist = hist[: min(it.value, hist.numel())]
        return PcgResult(x, it.value, stt.value, rz.value, sc[1], hist, ran)

    def close(self):
        if getattr(self, "h", None):
            C.lib().fem_mf_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _check_sync(status):
    if status == C.PCG_SYNC_TIMEOUT:
        raise RuntimeError("persistent PCG: an in-launch wait gave up (grid synchronisation timed out); "
                           "the iterate is not meaningful")


class _DistMarker:
    """Mixin marking distributed runners (they run the 3-kernel schedule)."""


@_scoped
class PcgRunner:
    """Persistent (P)CG context for fixed-iteration timing (bench.py): start once, iterate k, poll."""

    def __init__(self, A: SellMatrix, b, w, x0=None, mode=C.MODE_PCG, tol=0.0, eps=1e-30, fused=False,
                 schedule=None, constraints=None, tune=None):
        """tune: the context's FEM_TUNE_* flags instead of the library default (e.g. TUNE_DEFAULT | TUNE_PK_GV)."""
        self.lib = C.lib()
        self.A = A
        self.device = A.device
        self.b = b.to(device=A.device, dtype=F64).contiguous().view(-1)
        self.w = w.to(device=A.device, dtype=F64).contiguous().view(-1)
        self.x = (torch.zeros(A.n, dtype=F64, device=A.device) if x0 is None
                  else x0.to(device=A.device, dtype=F64).clone().contiguous().view(-1))
        # a dedicated stream: hipGraph capture is not allowed on the legacy default stream
        self.stream = torch.cuda.Stream(device=A.device)
        self.stream.wait_stream(torch.cuda.current_stream(A.device))
        self.h = ctypes.c_void_p()
        if getattr(A, "is_matfree", False):   # one form only: refuse what it would otherwise ignore
            if constraints is not None:
                raise ValueError("the element-chunk operator has no constrained CG (constraints= needs a SellMatrix)")
            if fused or (schedule is not None and int(schedule) not in (SCHED_THREE, SCHED_AUTO)):
                raise ValueError("the element-chunk operator runs the three-kernel schedule (no fused / deferred / "
                                 "persistent form)")
        self.schedule = (0 if isinstance(self, _DistMarker) or getattr(A, "is_matfree", False)
                         else _schedule(fused, schedule, A.bs))
        self.constraints = constraints   # keeps the device arrays alive with the context
        self._mode, self._tol, self._eps = mode, float(tol), float(eps)
        # solver-layout values (bs = 1) unless the context must read the plain ones (distributed, fused, constrained)
        self._create(isinstance(self, _DistMarker) or self.schedule == SCHED_FUSED or constraints is not None)
        if tune is not None:
            self.set_tuning(tune)

    def _create(self, plain):
        A = self.A
        if getattr(A, "is_matfree", False):
            A.create_context(self.b, self.x, self.w, self._mode, self._tol, self._eps, None, 0,
                             ctypes.c_void_p(self.stream.cuda_stream), self.h)
            self._sl = False
            self.stream.wait_stream(torch.cuda.current_stream(A.device))
            return
        C.check(self.lib.fem_pcg_create(A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols),
                                        A.solver_vals_ptr(plain), C.ptr(self.b), C.ptr(self.x), C.ptr(self.w),
                                        self._mode, self._tol, self._eps, None, 0,
                                        ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(self.h)),
                "fem_pcg_create")
        C.check(self.lib.fem_pcg_set_schedule(self.h, self.schedule), "fem_pcg_set_schedule")
        C.check(self.lib.fem_pcg_set_entries(self.h, A.g.sell_entries), "fem_pcg_set_entries")
        A.attach_cols16(self.h)
        A.attach_layout(self.h, plain)
        self._sl = A.solver_layout and not plain
        if self.constraints is not None:
            C.check(self.lib.fem_pcg_set_constraints(self.h, *self.constraints.args()), "fem_pcg_set_constraints")
        # the setup above may enqueue work on the current stream that this context's stream reads: the solver
        # layout formed on first use (paired deltas, uniform lists, gather windows), the plain values formed back
        self.stream.wait_stream(torch.cuda.current_stream(A.device))

    def set_tuning(self, flags):
        if self._sl and not (int(flags) & 2):   # no FEM_TUNE_PAIR: a context over the plain values instead
            self.lib.fem_pcg_destroy(self.h)
            self.h = ctypes.c_void_p()
            self._create(True)
        C.check(self.lib.fem_pcg_set_tuning(self.h, int(flags)), "fem_pcg_set_tuning")

    def finish(self):
        C.check(self.lib.fem_pcg_finish(self.h), "fem_pcg_finish")

    def start(self):
        C.check(self.lib.fem_pcg_start(self.h), "fem_pcg_start")

    def use_graph(self, k):
        C.check(self.lib.fem_pcg_use_graph(self.h, int(k)), "fem_pcg_use_graph")

    def iterate(self, k):
        C.check(self.lib.fem_pcg_iterate(self.h, int(k)), "fem_pcg_iterate")

    def poll(self):
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        C.check(self.lib.fem_pcg_poll(self.h, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)), "fem_pcg_poll")
        _check_sync(stt.value)
        return it.value, stt.value, rz.value

    def debug_window(self, L, lo, hi):
        """Test-only fault injection: overwrite logical workgroup L's gather window (after start())."""
        C.check(self.lib.fem_pcg_debug_window(self.h, int(L), int(lo), int(hi)), "fem_pcg_debug_window")

    def effective_schedule(self):
        """The schedule the context runs (after start(): SCHED_PERSIST may have fallen back to SCHED_DEFERRED)."""
        return int(self.lib.fem_pcg_get_schedule(self.h))

    def uniform_slices(self, s_begin=0, s_end=-1):
        """(slices stored with slice-uniform deltas, slices, column-index bytes per SpMV) over the slices
        [s_begin, s_end) of the context's matrix copy (after start())."""
        return uniform_slices(self.lib, self.h, s_begin, s_end)

    def pipelined(self):
        """True when the started context runs the pipelined persistent iteration (tune |= TUNE_PK_GV; bs = 1, single
        GPU, PCG mode, at most 2 slices per wave -- include/fem355.h FEM_TUNE_PK_GV)."""
        on = ctypes.c_int()
        C.check(self.lib.fem_pcg_pipelined(self.h, ctypes.byref(on)), "fem_pcg_pipelined")
        return bool(on.value)

    def persist_build(self):
        """(register slots per wave, overflow build, packed slices per wave) of the persistent launches (after
        start(); zeros when the context does not run schedule 3)."""
        sl, ov, pk = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        C.check(self.lib.fem_pcg_persist_build(self.h, ctypes.byref(sl), ctypes.byref(ov), ctypes.byref(pk)),
                "fem_pcg_persist_build")
        return sl.value, ov.value, pk.value

    def profile(self, k, every=1):
        """k iterations with hip events around the kernels of every `every`-th one -> (ms sums, counts)."""
        ms = (ctypes.c_double * 3)()
        n = (ctypes.c_int * 3)()
        C.check(self.lib.fem_pcg_profile(self.h, int(k), int(every), ms, n), "fem_pcg_profile")
        return list(ms), list(n)

    def close(self):
        if self.h:
            self.lib.fem_pcg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def assemble_tet4_system(coords, elements, kind="poisson", E=1.0, nu=0.0, graph=None):
    """Mesh -> assembled device operator in one pass (pattern + values; element matrices never stored).
    kind: "poisson" (bs=1, kappa=E) or "elastic" (bs=3)."""
    n_nodes = coords.shape[0]
    bs = 1 if kind == "poisson" else 3
    # bs = 1: the solver layout formed in the pattern's fill pass (the value kernel writes it straight away)
    g = graph if graph is not None else build_graph(elements, n_nodes, solver_layout=bs == 1)
    A = SellMatrix(g, bs).add_tet4(coords.to(F64).contiguous(), elements.contiguous(), E, nu)
    return A


def stream_ceiling(dev, gib=2.0, reps=5):
    """Measured HBM ceilings on this box (report the fraction of the measured STREAM ceiling too):
    16-byte-per-lane read-only sweep and copy over buffers far larger than the 256 MB memory-side cache, best of
    `reps`, timed with hip events on the stream the probes run on."""
    lib = C.lib()
    n = int(gib * (1 << 30) / 8)
    src = torch.ones(n, dtype=torch.float64, device=dev)
    dst = torch.empty(n // 2, dtype=torch.float64, device=dev)
    out = torch.zeros(1, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    res = {}
    for name, fn, nbytes in (("read", lambda: lib.fem_stream_read(C.ptr(src), C.ptr(out), n, 4096, C.stream(dev)), n * 8),
                             ("copy", lambda: lib.fem_stream_copy(C.ptr(src), C.ptr(dst), n // 2, 4096, C.stream(dev)), n * 8)):
        best = None
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            C.check(fn(), "stream probe")
            e1.record(st)
            e1.synchronize()
            t = e0.elapsed_time(e1) * 1e-3
            best = t if best is None else min(best, t)
        res[name] = nbytes / best / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return res
