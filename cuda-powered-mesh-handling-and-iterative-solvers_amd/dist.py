"""Multi-GPU path: element partition across the GPUs of one node, RCCL halo all-reduce inside each PCG iteration.

The reference has no multi-device code; its only decomposition is the single-GPU, randomly seeded region growing
of `subdivision.ipynb:194-297` (global->local node maps by `torch.unique`, `:254-259`). Here:
  * partition: recursive coordinate bisection of element centroids (deterministic: every rank computes the same
    split independently, no communication), RCB splits the longest axis at the element-count median;
  * every rank keeps the GLOBAL node ids of its elements (`torch.unique`, sorted, as `subdivision.ipynb:254-259`),
    assembles the SELL matrix of its own elements over them (unassembled at shared nodes), and knows the global
    interface list (nodes touched by several ranks) and which rows it owns (lowest rank touching the node);
  * per iteration: ONE all-reduce of [interface rows of A p | p.q partial] (each rank's p . q_rank over all its
    local rows: the rank sum is p.q) and one scalar all-reduce of r.z over owned rows (csrc/pcg.hip, distributed
    phases). All ranks hold bit-identical copies of shared dofs.

The partition/halo bookkeeping is plain torch index work run on the mesh's device; it is also exercised on CPU by
tests/test_dist_cpu.py (gloo, world size 2) against the oracle. The RCCL communicator is created in the C-ABI
(fem_comm_init) from a unique id broadcast over torch.distributed.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
from dataclasses import dataclass

import torch

from . import _capi as C
from . import mesh as _mesh
from . import system as _sys

F64, I32, LONG = torch.float64, torch.int32, torch.long
# distributed iteration: 0 = two reductions (halo + p.q, then r.z), 1 = single reduction (Chronopoulos-Gear form,
# one all-reduce of [interface rows of A u | r.z | u.Au] per iteration; csrc/pcg.hip k_cg1_*)
VARIANT_TWO, VARIANT_SINGLE = 0, 1
# exchange of the single-reduction variant: the all-reduce over the GLOBAL interface vector, or grouped
# ncclSend/ncclRecv of [g, d | rows shared with that rank] with every other rank + a fixed-rank-order sum
EXCHANGE_ALLREDUCE, EXCHANGE_P2P = "allreduce", "p2p"
# tuning flags of the distributed contexts (include/fem355.h FEM_TUNE_*): the single-GPU defaults, plus FEM_TUNE_C1F
# for the fused one-launch iteration (k_cg1_fused)
TUNE_DEFAULT, TUNE_C1F = 1 | 2 | 4 | 8, 16


# ============================================================================ partition (host logic, any device)
def element_centroids(coords, elements):
    return coords[elements].mean(dim=1)


def rcb_partition(centroids: torch.Tensor, nparts: int) -> torch.Tensor:
    """Recursive coordinate bisection -> part id [M] (int64). Deterministic: stable sorts, ties by element id."""
    M = centroids.shape[0]
    part = torch.empty(M, dtype=LONG, device=centroids.device)

    def split(ids, k, base):
        if k == 1:
            part[ids] = base
            return
        c = centroids[ids]
        ext = c.amax(0) - c.amin(0)
        axis = int(torch.argmax(ext))          # first maximal axis on ties
        order = torch.sort(c[:, axis], stable=True).indices
        kl = k // 2
        nl = (ids.numel() * kl + k // 2) // k
        left = torch.sort(ids[order[:nl]]).values
        right = torch.sort(ids[order[nl:]]).values
        split(left, kl, base)
        split(right, k - kl, base + kl)

    split(torch.arange(M, device=centroids.device), nparts, 0)
    return part


@dataclass
class RankMesh:
    rank: int
    nparts: int
    elem_ids: torch.Tensor    # global element ids of this rank
    nodes: torch.Tensor       # global node ids of the local rows (sorted)
    conn: torch.Tensor        # local connectivity [M_r, npe]
    imap: torch.Tensor        # [nI] int32 local row of interface node j, -1 if absent
    ipos: torch.Tensor        # [n_local] int32 interface index, -1 interior
    own: torch.Tensor         # [n_local] uint8
    n_iface: int


def node_sharing(elements, part, nparts, n_nodes, touch=None):
    """(number of ranks touching each node, lowest rank touching it); from the touch masks when given."""
    t = touch if touch is not None else touch_masks(elements, part, nparts, n_nodes)
    count = t.sum(0, dtype=I32)
    owner = torch.where(t.any(0), t.to(torch.uint8).argmax(0), torch.full_like(count, nparts, dtype=LONG))
    return count, owner.to(LONG)


def touch_masks(elements, part, nparts, n_nodes):
    """[nparts, n_nodes] bool: rank r has an element on the node."""
    dev = elements.device
    t = torch.zeros((nparts, n_nodes), dtype=torch.bool, device=dev)
    for r in range(nparts):
        t[r, elements[part == r].reshape(-1)] = True
    return t


@dataclass
class P2PMaps:
    """Neighbour-exchange maps of one rank (fem_pcg_set_p2p): messages to/from every other rank, ascending."""
    nranks: int
    peer_rank: list
    peer_cnt: list            # doubles per message: 2 + bs * shared nodes
    csrc: torch.Tensor        # int32 [nI, nranks] slot offset of node J's component 0 for rank r (-1 own, -2 absent)
    ssrc: torch.Tensor        # int32 [nranks] slot offset of rank r's [g, d] (-1 own)


def p2p_maps(rm: RankMesh, touch: torch.Tensor, bs: int) -> P2PMaps:
    """Messages of rank rm.rank to/from each other rank b: [g, d] then bs values per node shared by both, nodes in
    ascending global interface index J (the same order on both sides, so one slot layout serves sending and
    receiving). For every J this rank holds: the slot offset of each other rank that also holds it (rank order is
    the summation order on every rank: shared dofs stay bit-identical)."""
    a, P = rm.rank, rm.nparts
    dev = touch.device
    iface = torch.nonzero(touch.sum(0) > 1, as_tuple=True)[0]          # global interface nodes, J order
    tif = touch[:, iface]                                               # [P, nI]
    nI = int(iface.numel())
    peers = [b for b in range(P) if b != a]
    csrc = torch.full((nI, P), -2, dtype=LONG, device=dev)
    csrc[tif[a], a] = -1
    ssrc = torch.full((P,), -1, dtype=LONG, device=dev)
    cnt = []
    tot = 0
    for b in peers:
        S = torch.nonzero(tif[a] & tif[b], as_tuple=True)[0]           # J, ascending
        csrc[S, b] = tot + 2 + bs * torch.arange(S.numel(), device=dev)
        ssrc[b] = tot
        cnt.append(2 + bs * int(S.numel()))
        tot += cnt[-1]
    if tot >= 2 ** 31:
        raise ValueError("neighbour exchange: message offsets overflow int32")
    return P2PMaps(P, peers, cnt, csrc.to(I32).contiguous(), ssrc.to(I32).contiguous())


def rank_mesh(elements, part, rank, nparts, n_nodes, sharing=None) -> RankMesh:
    count, owner = sharing if sharing is not None else node_sharing(elements, part, nparts, n_nodes)
    ids = torch.nonzero(part == rank, as_tuple=True)[0]
    el = elements[ids]
    nodes, inv = torch.unique(el, return_inverse=True)         # `subdivision.ipynb:254-259`
    conn = inv.reshape(el.shape).contiguous()
    iface = torch.nonzero(count > 1, as_tuple=True)[0]          # sorted global interface node ids
    pos_in_local = torch.searchsorted(nodes, iface)
    present = (pos_in_local < nodes.numel())
    present &= nodes[pos_in_local.clamp(max=max(nodes.numel() - 1, 0))] == iface
    imap = torch.where(present, pos_in_local, torch.full_like(pos_in_local, -1)).to(I32)
    is_if = count[nodes] > 1
    ipos = torch.where(is_if, torch.searchsorted(iface, nodes), torch.full_like(nodes, -1)).to(I32)
    own = (owner[nodes] == rank).to(torch.uint8)
    return RankMesh(rank, nparts, ids, nodes, conn, imap.contiguous(), ipos.contiguous(), own.contiguous(),
                    int(iface.numel()))


# ============================================================================ device side
OPERATORS = ("assembled", "matfree")


class DistSystem:
    """One rank's share: local operator + halo maps. `comm` = RCCL communicator (None: phase-driven).
    operator "assembled": the rank's elements assembled into a local SELL matrix (unassembled at shared nodes);
    "matfree": the element-chunk operator over the rank's own elements (system.MatFreeOperator, csrc/matfree.hpp) --
    the reference's element-by-element product (`solver/element.py:429-464`) restricted to the partition, formed from
    the coordinates in every application; single-reduction iteration only."""

    def __init__(self, coords, elements, part, rank, nparts, kind="poisson", E=1.0, nu=0.0, comm=None,
                 sharing=None, touch=None, operator="assembled"):
        if operator not in OPERATORS:
            raise ValueError(f"unknown operator {operator!r} (one of {OPERATORS})")
        self.lib = C.lib()
        self.dev = coords.device
        self.rm = rank_mesh(elements, part, rank, nparts, coords.shape[0], sharing)
        self._touch = touch
        self._elements, self._part, self._n_nodes = elements, part, coords.shape[0]
        self._p2p = None
        self.comm = comm
        self.operator = operator
        lc = coords[self.rm.nodes].to(F64).contiguous()
        self.n_nodes = lc.shape[0]
        if operator == "matfree":
            self._lc = lc   # the operator reads the local coordinates and connectivity in every application
            self.A = _sys.MatFreeOperator(lc, self.rm.conn, "poisson" if kind == "poisson" else "elastic", E, nu)
        else:
            self.A = _sys.assemble_tet4_system(lc, self.rm.conn, kind, E, nu)
        self.bs = self.A.bs
        self.hbuf = torch.empty(max(self.rm.n_iface, 1) * self.bs, dtype=F64, device=self.dev)

    @property
    def n(self):
        return self.A.n

    def local(self, v_global):
        """Restrict a global nodal field [N, bs] to this rank's rows (nodal values, not partial sums)."""
        return v_global.reshape(-1, self.bs)[self.rm.nodes].reshape(-1).to(F64).contiguous()

    def diag_local(self):
        if self.operator == "matfree":
            return self.A.diag()
        d = torch.empty(self.n, dtype=F64, device=self.dev)
        g = self.A.g
        C.check(self.lib.fem_sell_diag(C.ptr(self.A.plain_values()), self.bs, C.ptr(g.diagpos), C.ptr(g.csr2sell),
                                       g.n_nodes, C.ptr(d), C.stream(self.dev)), "fem_sell_diag")
        return d

    def halo_pack(self, v):
        C.check(self.lib.fem_halo_pack(C.ptr(v), self.bs, C.ptr(self.rm.imap), self.rm.n_iface, C.ptr(self.hbuf),
                                       C.stream(self.dev)), "fem_halo_pack")

    def halo_unpack(self, v):
        C.check(self.lib.fem_halo_unpack(C.ptr(v), self.bs, C.ptr(self.rm.ipos), self.n_nodes, C.ptr(self.hbuf),
                                         C.stream(self.dev)), "fem_halo_unpack")

    def jacobi_from(self, dsum, fixed_mask_local):
        w = torch.empty(self.n, dtype=F64, device=self.dev)
        C.check(self.lib.fem_jacobi_from_diag(C.ptr(dsum), self.n, C.ptr(fixed_mask_local), C.ptr(w),
                                              C.stream(self.dev)), "fem_jacobi_from_diag")
        return w

    def jacobi(self, fixed_mask_local):
        """M_inv of the ASSEMBLED global matrix: the local diagonals are halo-summed first (RCCL)."""
        d = self.diag_local()
        C.check(self.lib.fem_halo_sum(self.comm, C.ptr(d), self.bs, C.ptr(self.rm.imap), self.rm.n_iface,
                                      C.ptr(self.rm.ipos), self.n_nodes, C.ptr(self.hbuf), C.stream(self.dev)),
                "fem_halo_sum")
        return self.jacobi_from(d, fixed_mask_local)

    def p2p(self):
        """Neighbour-exchange maps of this rank (built once; device int32 tensors kept alive here)."""
        if self._p2p is None:
            t = self._touch if self._touch is not None else touch_masks(self._elements, self._part, self.rm.nparts,
                                                                        self._n_nodes)
            self._p2p = p2p_maps(self.rm, t, self.bs)
        return self._p2p

    def runner(self, b, w, tol=0.0, mode=C.MODE_PCG, hist_len=0, variant=VARIANT_SINGLE, exchange=EXCHANGE_ALLREDUCE,
               fused=False):
        return DistRunner(self, b, w, tol, mode, hist_len, variant, exchange, fused)

    def check_variant(self, variant, fused=False):
        if self.operator == "matfree" and (int(variant) != VARIANT_SINGLE or fused):
            raise ValueError("the element-chunk operator runs the single-reduction distributed iteration (variant 1, "
                             "two kernels)")


class DistRunner(_sys._DistMarker, _sys.PcgRunner):
    """(P)CG context of one rank in distributed mode."""

    def __init__(self, ds: DistSystem, b, w, tol, mode, hist_len=0, variant=None, exchange=EXCHANGE_ALLREDUCE,
                 fused=False):
        ds.check_variant(VARIANT_SINGLE if variant is None else variant, fused)
        super().__init__(ds.A, b, w, mode=mode, tol=tol)
        self.ds = ds
        self.hist = torch.full((max(hist_len, 1),), float("nan"), dtype=F64, device=ds.dev) if hist_len else None
        C.check(self.lib.fem_pcg_set_dist(self.h, 1, ds.comm, ds.rm.n_iface, C.ptr(ds.rm.imap), C.ptr(ds.rm.ipos),
                                          C.ptr(ds.rm.own)), "fem_pcg_set_dist")
        self.variant = VARIANT_SINGLE if variant is None else int(variant)
        C.check(self.lib.fem_pcg_set_dist_variant(self.h, self.variant), "fem_pcg_set_dist_variant")
        self.exchange = exchange
        if exchange == EXCHANGE_P2P:
            if self.variant != VARIANT_SINGLE:
                raise ValueError("the neighbour exchange needs the single-reduction variant")
            set_p2p(self.lib, self.h, ds.p2p())
        if fused:
            C.check(self.lib.fem_pcg_set_tuning(self.h, TUNE_DEFAULT | TUNE_C1F), "fem_pcg_set_tuning")

    def phase(self, k):
        C.check(self.lib.fem_pcg_dist_phase(self.h, int(k)), "fem_pcg_dist_phase")

    def buffer(self, k):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(self.lib.fem_pcg_dist_buffer(self.h, int(k), ctypes.byref(p), ctypes.byref(n)), "fem_pcg_dist_buffer")
        return p.value, n.value


# ============================================================================ single-process, multi-partition driver
class PartitionGroup:
    """All P partitions in ONE process on ONE GPU, exchanges summed by a group kernel in rank order: exercises the
    distributed kernels, halo maps and ownership without RCCL (which refuses two ranks per device)."""

    def __init__(self, coords, elements, nparts, kind="poisson", E=1.0, nu=0.0, operator="assembled"):
        self.lib = C.lib()
        part = rcb_partition(element_centroids(coords, elements), nparts)
        touch = touch_masks(elements, part, nparts, coords.shape[0])
        sharing = node_sharing(elements, part, nparts, coords.shape[0], touch)
        self.part = part
        self.ranks = [DistSystem(coords, elements, part, r, nparts, kind, E, nu, None, sharing, touch, operator)
                      for r in range(nparts)]
        self.dev = coords.device

    def group_sum(self, ptrs, n):
        arr = torch.tensor(ptrs, dtype=torch.int64, device=self.dev)
        C.check(self.lib.fem_group_allreduce(C.ptr(arr), len(ptrs), int(n), C.stream(self.dev)), "fem_group_allreduce")
        torch.cuda.current_stream(self.dev).synchronize()   # keep `arr` alive until the kernel ran

    def jacobi(self, fixed_masks):
        ds = [r.diag_local() for r in self.ranks]
        for r, d in zip(self.ranks, ds):
            r.halo_pack(d)
        self.group_sum([r.hbuf.data_ptr() for r in self.ranks], self.ranks[0].hbuf.numel())
        out = []
        for r, d, m in zip(self.ranks, ds, fixed_masks):
            r.halo_unpack(d)
            out.append(r.jacobi_from(d, m))
        return out

    def deliver(self, runs):
        """Neighbour exchange without RCCL: every rank's message to b lands in b's receive slot for it."""
        arr = (ctypes.c_void_p * len(runs))(*[run.h.value for run in runs])
        C.check(self.lib.fem_p2p_deliver(arr, len(runs), C.stream(self.dev)), "fem_p2p_deliver")

    def solve(self, bs_local, ws, tol, max_iter, mode=C.MODE_PCG, variant=None, exchange=EXCHANGE_ALLREDUCE,
              fused=False, fixed=False):
        """Phase-driven (P)CG over the P partitions; returns (per-rank x, iterations, status).
        fixed: exactly `max_iter` iteration passes (x_k after k iterations; no stop-test pass after the last)."""
        # every context on the current stream: the phases of all ranks and the group sums serialise in order
        variant = VARIANT_SINGLE if variant is None else int(variant)
        runs = [_GroupRunner(r, b, w, tol, mode, variant, exchange, fused)
                for r, b, w in zip(self.ranks, bs_local, ws)]
        for run in runs:
            run.start_state()
        p2p = exchange == EXCHANGE_P2P

        def step(ph):
            for run in runs:
                run.phase(ph)
            if p2p and ph in (4, 20):
                self.deliver(runs)
                return
            p0, n0 = runs[0].buffer(ph)
            if n0:
                self.group_sum([run.buffer(ph)[0] for run in runs], n0)

        start, iteration = ((10, 20), (4,)) if variant == VARIANT_SINGLE else ((10, 11, 12), (0, 1, 2, 3))
        for ph in start:
            step(ph)
        it = 0
        # the single-reduction form tests convergence at the start of the next iteration: one extra pass
        for it in range(max_iter + (1 if variant == VARIANT_SINGLE and not fixed else 0)):
            for ph in iteration:
                step(ph)
            if not fixed and (it + 1) % 16 == 0:
                i_, s_, _ = runs[0].poll()
                if s_ != C.PCG_RUNNING:
                    break
        polls = [run.poll() for run in runs]
        xs = [run.x for run in runs]
        for run in runs:
            run.close()
        its = {p[0] for p in polls}
        sts = {p[1] for p in polls}
        assert len(its) == 1 and len(sts) == 1, f"ranks disagree: {polls}"
        return xs, polls[0][0], polls[0][1]


class _GroupRunner:
    """Distributed (P)CG context on the current stream, driven phase by phase by PartitionGroup."""

    def __init__(self, ds: DistSystem, b, w, tol, mode, variant=0, exchange=EXCHANGE_ALLREDUCE, fused=False):
        self.lib = C.lib()
        ds.check_variant(variant, fused)
        A = ds.A
        self.b = b.to(F64).contiguous()
        self.w = w.to(F64).contiguous()
        self.x = torch.zeros(A.n, dtype=F64, device=A.device)
        self.h = ctypes.c_void_p()
        if ds.operator == "matfree":
            A.create_context(self.b, self.x, self.w, mode, float(tol), 1e-30, None, 0, C.stream(A.device), self.h)
        else:
            C.check(self.lib.fem_pcg_create(A.g.n_nodes, A.bs, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols),
                                            C.ptr(A.plain_values()), C.ptr(self.b), C.ptr(self.x), C.ptr(self.w), mode, float(tol), 1e-30, None,
                                            0, C.stream(A.device), ctypes.byref(self.h)), "fem_pcg_create")
            C.check(self.lib.fem_pcg_set_schedule(self.h, 0), "fem_pcg_set_schedule")
            C.check(self.lib.fem_pcg_set_entries(self.h, A.g.sell_entries), "fem_pcg_set_entries")
            A.attach_cols16(self.h)
        C.check(self.lib.fem_pcg_set_dist(self.h, 1, None, ds.rm.n_iface, C.ptr(ds.rm.imap), C.ptr(ds.rm.ipos),
                                          C.ptr(ds.rm.own)), "fem_pcg_set_dist")
        C.check(self.lib.fem_pcg_set_dist_variant(self.h, int(variant)), "fem_pcg_set_dist_variant")
        if exchange == EXCHANGE_P2P:
            set_p2p(self.lib, self.h, ds.p2p())
        if fused:
            C.check(self.lib.fem_pcg_set_tuning(self.h, TUNE_DEFAULT | TUNE_C1F), "fem_pcg_set_tuning")

    def start_state(self):
        C.check(self.lib.fem_pcg_start(self.h), "fem_pcg_start")   # state only (phases do the work)

    def phase(self, k):
        C.check(self.lib.fem_pcg_dist_phase(self.h, int(k)), "fem_pcg_dist_phase")

    def buffer(self, k):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(self.lib.fem_pcg_dist_buffer(self.h, int(k), ctypes.byref(p), ctypes.byref(n)), "fem_pcg_dist_buffer")
        return p.value, n.value

    def poll(self):
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        C.check(self.lib.fem_pcg_poll(self.h, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)), "fem_pcg_poll")
        return it.value, stt.value, rz.value

    def close(self):
        if self.h:
            self.lib.fem_pcg_destroy(self.h)
            self.h = ctypes.c_void_p()


def set_p2p(lib, h, m: P2PMaps):
    npeer = len(m.peer_rank)
    ranks = (ctypes.c_int * max(npeer, 1))(*m.peer_rank)
    cnts = (ctypes.c_int64 * max(npeer, 1))(*m.peer_cnt)
    C.check(lib.fem_pcg_set_p2p(h, m.nranks, npeer, ranks, cnts, C.ptr(m.csrc), C.ptr(m.ssrc)), "fem_pcg_set_p2p")


def gather_solution(ranks, xs, n_nodes, bs):
    """Assemble the global solution from the ranks' copies (owned rows)."""
    dev = xs[0].device
    out = torch.zeros(n_nodes * bs, dtype=F64, device=dev)
    for r, x in zip(ranks, xs):
        own = r.rm.own.bool()
        rows = r.rm.nodes[own]
        out.view(-1, bs)[rows] = x.view(-1, bs)[own]
    return out.view(n_nodes, bs)


# ============================================================================ RCCL bootstrap + bench
def init_comm(rank, world):
    """RCCL communicator for this rank on the current HIP device; the 128-byte id travels over torch.distributed."""
    import torch.distributed as tdist
    lib = C.lib()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        C.check(lib.fem_comm_unique_id(buf), "fem_comm_unique_id")
    obj = [bytes(buf.raw) if rank == 0 else None]
    tdist.broadcast_object_list(obj, src=0)
    comm = ctypes.c_void_p()
    C.check(lib.fem_comm_init(world, rank, obj[0], ctypes.byref(comm)), "fem_comm_init")
    return comm


COMPANION_DROP = ("metric", "n_gpus", "higher_is_better", "scaling", "vs_baseline", "dtype", "data")


class CompanionGuard:
    """A companion measurement inside the ONE bench JSON line, under a watchdog that stays armed until `close()`
    (after the line is printed and, at N > 1, after the final barrier). `run(fn)` stores fn() minus the line-level
    keys under out[key] (an exception as {"error": ...}); `emit()` prints the line once (rank 0). If the watchdog
    fires first -- a collective that never completes, in the companion or in the teardown after it -- rank 0 prints
    the line as it stands (the metric measured before the companion; key = {"error": "timed out ..."}) unless it was
    printed already, and the process exits with status 0: the companion can never cost the metric line."""

    def __init__(self, out, key, rank=0, timeout=240.0):
        import threading
        self.out, self.key, self.rank, self.timeout = out, key, rank, timeout
        self._lock = threading.Lock()
        self._printed = False
        self._timer = threading.Timer(timeout, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def _fire(self):
        with self._lock:
            if self.rank == 0 and self.out is not None and not self._printed:
                if not isinstance(self.out.get(self.key), dict):
                    self.out[self.key] = {"error": f"timed out after {self.timeout:.0f} s"}
                print(json.dumps(self.out), flush=True)
                self._printed = True
            sys.stderr.write(f"[rank {self.rank}] {self.key} companion watchdog fired after {self.timeout:.0f} s\n")
            sys.stderr.flush()
            os._exit(0)

    def run(self, fn):
        try:
            d = fn()
            sub = None if d is None else {k: v for k, v in d.items() if k not in COMPANION_DROP}
        except Exception as e:   # noqa: BLE001 -- reported in the line; the metric above it stands
            sub = {"error": f"{type(e).__name__}: {e}"}
            sys.stderr.write(f"[rank {self.rank}] {self.key} companion failed: {sub['error']}\n")
        if self.out is not None:
            self.out[self.key] = sub
        return self.out

    def emit(self):
        with self._lock:
            if self.rank == 0 and self.out is not None and not self._printed:
                print(json.dumps(self.out), flush=True)
            self._printed = True

    def close(self):
        self._timer.cancel()


def run_chain(path, same_gpu, persist_fn, rccl_fn, rank=0, log=None):
    """The N > 1 measurement decision (bench.py): returns (bench dict or None, "persist" | "rccl").
    path "auto": the persistent multi-GPU schedule (`persist_fn() -> (ok, out)`, raising C.FemError on every rank
    alike when it does not apply), the RCCL element partition (`rccl_fn() -> out`) when it raised or returned not ok;
    "persist": the persistent schedule or a RuntimeError; "rccl": RCCL only. same_gpu (all ranks on one GPU, a
    validation mode): RCCL refuses two ranks per GPU, so a failed persistent schedule is a RuntimeError there too."""
    log = log or (lambda m: print(f"[rank {rank}] {m}", file=sys.stderr, flush=True))
    if path in ("auto", "persist"):
        try:
            ok, out = persist_fn()
        except C.FemError as e:
            log(f"persistent multi-GPU schedule unavailable: {e}")
            ok, out = False, None
        if ok:
            return out, "persist"
        if same_gpu or path == "persist":
            raise RuntimeError("persistent multi-GPU schedule failed (no RCCL fallback "
                               + ("possible: all ranks on one GPU)" if same_gpu else "requested)"))
        log("falling back to the RCCL element partition")
    return rccl_fn(), "rccl"


def bench_main(a, metric):
    """bench.py for N > 1 ranks (one per GPU), strong scaling of the 10M-tet system: Poisson on the persistent
    multi-GPU schedule (rows partitioned, in-kernel hand-offs; RCCL element partition if its self-check fails),
    elasticity on the RCCL element partition; value = CG iterations/s of the global system, max time over ranks.
    Poisson runs also measure the elasticity system (BASELINE configs[3]) under "elasticity" in the same line."""
    import torch.distributed as tdist
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # FEM355_DIST_SAME_GPU=1: every rank on GPU 0, each on its own CU share (validates the multi-process path of
    # the persistent schedule on a one-GPU box; RCCL refuses two ranks per GPU, so there is no RCCL fallback then)
    same_gpu = os.environ.get("FEM355_DIST_SAME_GPU", "0") == "1"
    if same_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    C.lib()
    path = getattr(a, "dist_path", "auto")
    comm = None

    def rccl(kind, operator="assembled"):
        nonlocal comm
        if comm is None:
            comm = init_comm(rank, world)
        return rccl_measure(a, kind, comm, rank, world, dev, tdist, metric, operator)

    def persist(kind):
        from . import dist_persist
        return dist_persist.bench_persist(a, metric, rank, world, dev, tdist, same_gpu=same_gpu, kind=kind)

    # Poisson: the persistent multi-GPU schedule first (rows partitioned, in-kernel hand-offs), RCCL if it does not
    # apply or fails its checks. The elasticity companion the same way: the bs = 3 DIST build where every rank's
    # slices fit on chip (N >= 4 at 10M tets), else the RCCL element partition (BASELINE configs[3])
    if a.kind == "poisson":
        out, _ = run_chain(path, same_gpu, lambda: persist("poisson"), lambda: rccl("poisson"), rank)
    else:
        out = rccl(a.kind)
    drop = os.environ.get("FEM355_DIST_DROP_RANK", "")
    if drop and rank == 0 and isinstance(out, dict):   # a fault-injected run is labelled as such in its line
        out.setdefault("config", {})["fault_injection"] = f"FEM355_DIST_DROP_RANK={drop}"
    guard = None
    if a.kind == "poisson" and getattr(a, "elastic", 0):
        def companion():
            out_e, how = run_chain(path, same_gpu, lambda: persist("elastic"), lambda: rccl("elastic"), rank)
            # BASELINE configs[3] as north_star states it -- element partitions, RCCL exchange of the halo-DOF
            # partials inside every iteration -- measured on every N > 1 run next to the schedule above, with the
            # assembled local operator and with the element-chunk (matrix-free) one. RCCL refuses two ranks on one
            # GPU, so the same-GPU rehearsal skips it.
            if same_gpu:
                er = {"skipped": "all ranks on one GPU (RCCL refuses two ranks per device)"}
            else:
                er = {"assembled": out_e if how == "rccl" else element_rccl(lambda: rccl("elastic", "assembled"))}
                er["matfree"] = element_rccl(lambda: rccl("elastic", "matfree"))
            if rank == 0 and isinstance(out_e, dict):
                out_e = dict(out_e)
                out_e["element_rccl"] = er
            return out_e
        guard = CompanionGuard(out, "elasticity", rank=rank, timeout=float(getattr(a, "elastic_timeout", 240.0)))
        out = guard.run(companion)
        guard.emit()
    elif rank == 0:
        print(json.dumps(out), flush=True)
    # teardown under the same watchdog: a rank stuck in the companion must not hold the others in this barrier
    if comm is not None:
        C.check(C.lib().fem_comm_destroy(comm), "fem_comm_destroy")
    tdist.barrier()
    tdist.destroy_process_group()
    if guard is not None:
        guard.close()


def element_rccl(fn):
    """One element-partition measurement for the "element_rccl" block: its bench dict minus the line-level keys, or
    {"error": ...} (raised on every rank alike: the setup and the checks are collective)."""
    try:
        d = fn()
        return None if d is None else {k: v for k, v in d.items() if k not in COMPANION_DROP + ("cpu_baseline",)}
    except Exception as e:   # noqa: BLE001 -- reported in the line
        sys.stderr.write(f"element_rccl measurement failed: {type(e).__name__}: {e}\n")
        return {"error": f"{type(e).__name__}: {e}"}


def rccl_measure(a, kind, comm, rank, world, dev, tdist, metric, operator="assembled"):
    """The RCCL element-partition measurement of `kind` on the n-cube (every rank calls it); returns the bench
    dict on rank 0, None elsewhere. operator "matfree": every rank applies the element-chunk operator of its own
    elements (no matrix), single-reduction iteration with the configured exchange."""
    def barrier_sync():
        torch.cuda.synchronize()
        tdist.barrier()

    def tmax(v):
        t = torch.tensor([v], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return float(t[0])

    coords, tets = _mesh.kuhn_cube(a.n, device=dev)
    N = coords.shape[0]
    if kind == "poisson":
        f, fixed = _mesh.cube_poisson_case(coords)
        E, nu = 1.0, 0.0
    else:
        f, fixed = _mesh.cube_elasticity_case(coords)
        E, nu = 113.8e9, 0.342
    # warm the kernels (HIP modules and the torch ops of the setup load lazily on first use) and the RCCL
    # connections (set up on the first collective) with the whole setup on a small cube
    c0, t0_ = _mesh.kuhn_cube(8, device=dev)
    p0 = rcb_partition(element_centroids(c0, t0_), world)
    d0 = DistSystem(c0, t0_, p0, rank, world, kind, E, nu, comm, operator=operator)
    d0.jacobi(torch.zeros(d0.n, dtype=torch.uint8, device=dev))
    wbuf = torch.ones(1 << 16, dtype=F64, device=dev)
    C.check(C.lib().fem_allreduce_sum(comm, C.ptr(wbuf), wbuf.numel(), C.stream(dev)), "fem_allreduce_sum")
    del d0, p0
    barrier_sync()

    stages = {}
    t0 = time.perf_counter()
    part = rcb_partition(element_centroids(coords, tets), world)
    touch = touch_masks(tets, part, world, N)
    sharing = node_sharing(tets, part, world, N, touch)
    torch.cuda.synchronize()
    stages["partition_ms"] = (time.perf_counter() - t0) * 1e3
    ds = DistSystem(coords, tets, part, rank, world, kind, E, nu, comm, sharing, touch, operator)
    torch.cuda.synchronize()
    stages["rank_mesh_assembly_ms"] = (time.perf_counter() - t0) * 1e3 - stages["partition_ms"]
    bs = ds.bs
    gmask = torch.zeros((N, bs), dtype=torch.uint8, device=dev)
    gmask[fixed] = 1
    mask = gmask[ds.rm.nodes].reshape(-1).contiguous()
    w = ds.jacobi(mask)
    barrier_sync()
    t_asm = tmax(time.perf_counter() - t0)
    b = ds.local(f)
    # global tolerance: rtol * sqrt(b.Minv b) over owned rows
    own = ds.rm.own.bool().repeat_interleave(bs)
    bz = torch.tensor([float(torch.dot(b[own], (w * b)[own]))], dtype=torch.float64)
    tdist.all_reduce(bz)
    tol = a.rtol * float(bz[0]) ** 0.5

    # hipGraph-captured iterations (RCCL collectives captured with the kernels): at N = 8 the host cost of ~8
    # launches + 2 collectives per iteration would otherwise exceed the device time of an iteration
    gk = int(getattr(a, "dist_graph", 0) or 0)

    def use_graph(r, k):
        if k <= 0:
            return 0
        try:
            r.use_graph(k)
            return k
        except C.FemError as e:   # capture unsupported: plain launches, reported in the JSON
            print(f"[rank {rank}] graph capture failed, plain launches: {e}", file=sys.stderr, flush=True)
            return 0

    mf = operator == "matfree"
    variant = VARIANT_SINGLE if mf else int(getattr(a, "dist_variant", VARIANT_SINGLE))
    exchange = getattr(a, "dist_exchange", EXCHANGE_ALLREDUCE) if variant == VARIANT_SINGLE else EXCHANGE_ALLREDUCE
    fused = bool(getattr(a, "dist_fused", 0)) and variant == VARIANT_SINGLE and not mf

    def solve_to_tol():
        run = ds.runner(b, w, tol=tol, variant=variant, exchange=exchange, fused=fused)
        barrier_sync()
        t0 = time.perf_counter()
        run.start()
        chunk = use_graph(run, gk) or 64
        done, it, stt = 0, 0, C.PCG_RUNNING
        while done < 20000:
            run.iterate(chunk)
            done += chunk
            it, stt, _ = run.poll()
            if stt != C.PCG_RUNNING:
                break
        barrier_sync()
        t = tmax(time.perf_counter() - t0)
        run.close()
        return t, it, stt

    t_solve, it, stt = solve_to_tol()
    fallback = None
    # self-check of the neighbour exchange on the real transport: every rank must converge (the status is global,
    # so a broken exchange shows on all ranks alike); otherwise the all-reduce exchange is measured and reported
    if exchange == EXCHANGE_P2P and tmax(0.0 if stt == C.PCG_CONVERGED else 1.0) > 0.0:
        fallback = f"neighbour exchange solve ended with status {stt} after {it} iterations; all-reduce used"
        print(f"[rank {rank}] {fallback}", file=sys.stderr, flush=True)
        exchange = EXCHANGE_ALLREDUCE
        t_solve, it, stt = solve_to_tol()

    run = ds.runner(b, w, tol=0.0, variant=variant, exchange=exchange, fused=fused)
    run.start()
    import math
    graph_k = use_graph(run, math.gcd(math.gcd(gk, a.steps), a.warmup) if gk > 0 else 0)
    run.iterate(a.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    if graph_k:
        run.iterate(a.steps)
    else:
        ms, cnt = run.profile(a.steps, every=a.sample_every)
    barrier_sync()
    dt = tmax(time.perf_counter() - t0)
    it2, _, _ = run.poll()
    if graph_k:   # kernel times sampled after the timed region (event brackets cannot sit inside a graph)
        run.use_graph(0)
        ms, cnt = run.profile(max(a.sample_every, 20), every=1)
    run.close()
    spmv_ms = tmax(ms[0] / max(cnt[0], 1))
    alg = ds.A.algorithmic_bytes() if mf else ds.A.algorithmic_bytes_spmv()
    alg_total = torch.tensor([float(alg)], dtype=torch.float64)
    tdist.all_reduce(alg_total)
    nI = ds.rm.n_iface
    if rank == 0:
        achieved = alg / (spmv_ms * 1e-3) / 1e9
        ceiling = _sys.stream_ceiling(dev)   # after the timed region, rank 0's GPU only
        out = {
            "metric": metric, "value": a.steps / dt, "unit": "CG iterations/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{tets.shape[0]:,}-tet P1 {kind} Kuhn cube n={a.n}, Jacobi-PCG fixed "
                                   f"iterations, element-partitioned (RCB) over {world} GPUs, "
                                   + ("element-chunk (matrix-free) operator of each rank's own elements, " if mf
                                      else "assembled local SELL operator, ")
                                   + ("RCCL neighbour send/recv of [r.z, u.Au | shared rows] with every other rank"
                                      " (single reduction: one grouped exchange per iteration)"
                                      if variant and exchange == EXCHANGE_P2P else
                                      "RCCL halo all-reduce (single reduction: one all-reduce per iteration)"
                                      if variant else "RCCL halo all-reduce + r.z all-reduce"),
                       "tets": int(tets.shape[0]), "dofs": N * bs, "interface_nodes": nI,
                       "parallelism": f"element partition x{world}", "graph_iterations": graph_k,
                       "operator": operator,
                       "dist_variant": "single-reduction" if variant else "two-reduction",
                       "dist_exchange": exchange, "dist_fused_iteration": fused,
                       "dist_exchange_fallback": fallback},
            "dofs_per_s": N * bs / (t_asm + t_solve), "assembly_ms": t_asm * 1e3, "solve_ms": t_solve * 1e3,
            "assembly_stages_rank0": stages,
            "solve_iters": it, "solve_status": stt,
            "kernel_ms": ({"spmv_local_max": spmv_ms, "exchange": ms[1] / max(cnt[1], 1),
                           "step_update": ms[2] / max(cnt[2], 1)} if variant else
                          {"spmv_local_max": spmv_ms, "exchange_update": ms[1] / max(cnt[1], 1),
                           "pupdate": ms[2] / max(cnt[2], 1)}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8000.0, "traffic": None,
                         "kernel": ("k_cg1_mf_slots + k_cg1_mf_gather" if mf else
                                    "k_cg1_spmv" if variant else "k_pcg_spmv_dot") + " (rank 0 local)",
                         "algorithmic_bytes": alg, "stream_ceiling_GBps": ceiling,
                         "frac_of_stream_read": achieved / ceiling["read"]},
            "cpu_baseline": None,
        }
        return out
    return None
