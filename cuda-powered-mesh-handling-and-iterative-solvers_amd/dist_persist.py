"""Multi-GPU persistent Jacobi-PCG: the single-GPU persistent schedule (csrc/pcg_persist.hpp) spread over ranks by
ROWS, with every per-iteration exchange done inside the running kernels (no collective library call per iteration).

The reference has no multi-device code (its only decomposition is the single-GPU region growing of
`subdivision.ipynb:194-297`); this is the MI355X-native counterpart of DESIGN.md §6's element-partitioned RCCL path
for the bs = 1 (Poisson) system, designed for the strong-scaling target of SURVEY §8(e):
  * partition: the global SELL-64 slices split into `nranks` contiguous ranges of (nearly) equal size; rank r owns
    the rows of its slices. The ordering of the rows (lexicographic on the Kuhn cube, RCM-like on meshes from
    `mesh.py`) keeps the rows a rank gathers from others within a band next to its range;
  * each rank assembles the GLOBAL rows it owns from the elements touching them (global node ids, rows of other
    ranks left partial and never read), so the matrix rows, the Jacobi weights and every per-row operation are
    those of the single-GPU system;
  * every rank's comm block (u, per-workgroup epoch flags, rank sums) is mapped into every other rank through
    hipIpc handles; a workgroup whose rows another rank gathers stores them into that rank's u with system-scope
    stores, releases, and raises its flag there; the grid barrier of every iteration is followed by a rank-level
    exchange of the two sums, summed in rank order on every rank (identical scalars everywhere, deterministic);
  * one process per GPU (bench.py N > 1), or - for validation on one GPU - several ranks as contexts of one process
    on separate streams sharing the CUs (`EmulatedGroup`), or several processes on one GPU (`FEM355_DIST_SAME_GPU`).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _capi as C
from . import system as _sys

F64, I64 = torch.float64, torch.int64


def slice_split(n_rows: int, nranks: int):
    """Global slice bounds [nranks + 1] of the row partition (contiguous, sizes within one slice of each other)."""
    ns = (n_rows + 63) // 64
    if ns < nranks:
        raise ValueError(f"{n_rows} rows ({ns} slices) cannot be split over {nranks} ranks")
    return [r * ns // nranks for r in range(nranks + 1)]


def rank_rows(n_rows: int, split, rank: int):
    return split[rank] * 64, min(split[rank + 1] * 64, n_rows)


def rank_elements(elements: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    """Elements with at least one node among the rows [lo, hi) (their global connectivity)."""
    return elements[((elements >= lo) & (elements < hi)).any(dim=1)].contiguous()


@dataclass
class RankSetup:
    A: "_sys.SellMatrix"
    w: torch.Tensor
    lo: int
    hi: int


def assemble_rank(coords, elements, split, rank, kind="poisson", E=1.0, nu=0.0, fixed_mask=None) -> RankSetup:
    """The global rows [lo, hi) of rank `rank`: pattern + values from the elements touching them, Jacobi weights
    (zero on fixed dofs, uint8 mask over the global rows)."""
    if kind != "poisson":
        raise ValueError("the distributed persistent schedule is bs = 1 (Poisson); elasticity uses dist.py")
    N = coords.shape[0]
    lo, hi = rank_rows(N, split, rank)
    el = rank_elements(elements, lo, hi)
    A = _sys.assemble_tet4_system(coords, el, kind, E, nu)
    if A.g.dcols is None:
        raise ValueError("the distributed persistent schedule needs 16-bit column deltas (banded rows)")
    w = A.jacobi(fixed_mask)
    return RankSetup(A, w, lo, hi)


class RankRunner:
    """One rank's persistent PCG context over its rows of the global system (vectors global-length)."""

    def __init__(self, rs: RankSetup, b, split, rank, nranks, tol=0.0, mode=C.MODE_PCG, eps=1e-30, grid=0,
                 stream=None, x0=None):
        self.lib = C.lib()
        A = rs.A
        self.A, self.rs, self.rank, self.nranks = A, rs, rank, nranks
        self.device = A.device
        self.b = b.to(device=A.device, dtype=F64).contiguous().view(-1)
        self.w = rs.w
        self.x = (torch.zeros(A.n, dtype=F64, device=A.device) if x0 is None
                  else x0.to(device=A.device, dtype=F64).clone().contiguous().view(-1))
        self.stream = stream if stream is not None else torch.cuda.Stream(device=A.device)
        self.stream.wait_stream(torch.cuda.current_stream(A.device))
        self.h = ctypes.c_void_p()
        with C.device_scope(A.device):
            C.check(self.lib.fem_pcg_create(A.g.n_nodes, 1, C.ptr(A.g.slice_ptr), C.ptr(A.g.cols), C.ptr(A.vals),
                                            C.ptr(self.b), C.ptr(self.x), C.ptr(self.w), mode, float(tol), float(eps),
                                            None, 0, ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(self.h)),
                    "fem_pcg_create")
            A.attach_cols16(self.h)
            sp = (ctypes.c_int64 * (nranks + 1))(*split)
            C.check(self.lib.fem_pcg_set_rows(self.h, nranks, rank, sp, int(grid)), "fem_pcg_set_rows")
            base, nbytes = ctypes.c_void_p(), ctypes.c_int64()
            C.check(self.lib.fem_pcg_comm_block(self.h, ctypes.byref(base), ctypes.byref(nbytes)), "fem_pcg_comm_block")
            self.block = base.value
            self.block_bytes = nbytes.value
            lo, hi = ctypes.c_int64(), ctypes.c_int64()
            C.check(self.lib.fem_pcg_col_window(self.h, ctypes.byref(lo), ctypes.byref(hi)), "fem_pcg_col_window")
            self.col_window = (lo.value, hi.value)

    def ipc_handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        C.check(self.lib.fem_ipc_handle(ctypes.c_void_p(self.block), buf), "fem_ipc_handle")
        return bytes(buf.raw)

    def set_peers(self, bases, windows):
        n = self.nranks
        arr = (ctypes.c_void_p * n)(*[ctypes.c_void_p(b) if b else None for b in bases])
        los = (ctypes.c_int64 * n)(*[w[0] for w in windows])
        his = (ctypes.c_int64 * n)(*[w[1] for w in windows])
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_set_peers(self.h, arr, los, his), "fem_pcg_set_peers")

    def start(self):
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_start(self.h), "fem_pcg_start")

    def iterate(self, k):
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_iterate(self.h, int(k)), "fem_pcg_iterate")

    def profile(self, k):
        """k iterations as one launch, hip events around it on the solver stream -> device ms."""
        ms = (ctypes.c_double * 3)()
        cnt = (ctypes.c_int * 3)()
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_profile(self.h, int(k), int(k), ms, cnt), "fem_pcg_profile")
        return ms[0]

    def poll(self):
        it, stt, rz = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_poll(self.h, ctypes.byref(it), ctypes.byref(stt), ctypes.byref(rz)),
                    "fem_pcg_poll")
        return it.value, stt.value, rz.value

    def effective_schedule(self):
        return int(self.lib.fem_pcg_get_schedule(self.h))

    def debug(self, which, n):
        buf = (ctypes.c_int32 * n)()
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_dist_debug(self.h, int(which), buf, int(n)), "fem_pcg_dist_debug")
        return list(buf)

    def set_prof(self, buf):
        with C.device_scope(self.device):
            C.check(self.lib.fem_pcg_set_prof(self.h, C.ptr(buf)), "fem_pcg_set_prof")

    def own_x(self):
        lo, hi = self.rs.lo, self.rs.hi
        return self.x[lo:hi]

    def close(self):
        if self.h:
            self.lib.fem_pcg_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EmulatedGroup:
    """`nranks` ranks as contexts of ONE process on ONE GPU (validation of the distributed kernel without a
    multi-GPU box): each rank gets grid = CUs / nranks workgroups and its own stream, so the ranks' persistent
    launches run concurrently; the comm blocks are plain device pointers (no IPC)."""

    def __init__(self, coords, elements, nranks, b, fixed_mask=None, kind="poisson", E=1.0, nu=0.0, tol=0.0,
                 mode=C.MODE_PCG, x0=None):
        dev = coords.device
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        # a multiple of 8 workgroups per rank within its CU-mask share (at 3+ ranks leave headroom: the masks are
        # laid over the CU numbering, which need not split evenly into usable CUs)
        grid = (ncu // nranks) // 8 * 8 if nranks <= 2 else int(ncu / nranks * 0.85) // 8 * 8
        N = coords.shape[0]
        self.split = slice_split(N, nranks)
        self.ranks = []
        self._raw_streams = []
        lib = C.lib()
        for r in range(nranks):
            # a CU-masked stream per rank: its own hardware queue and its own CUs, so the ranks' launches run side by
            # side (plain streams may share a queue and then serialise: the first rank would wait for the second)
            raw = ctypes.c_void_p()
            with C.device_scope(dev):
                C.check(lib.fem_stream_create_cu(r, nranks, ctypes.byref(raw)), "fem_stream_create_cu")
            self._raw_streams.append(raw.value)
            st = torch.cuda.ExternalStream(raw.value, device=dev)
            rs = assemble_rank(coords, elements, self.split, r, kind, E, nu, fixed_mask)
            self.ranks.append(RankRunner(rs, b, self.split, r, nranks, tol=tol, mode=mode, grid=grid, x0=x0,
                                         stream=st))
        torch.cuda.synchronize(dev)
        bases = [rr.block for rr in self.ranks]
        windows = [rr.col_window for rr in self.ranks]
        for rr in self.ranks:
            rr.set_peers(bases, windows)
        self.n = N

    def start(self):
        for rr in self.ranks:
            rr.start()
        torch.cuda.synchronize()   # the host barrier between every rank's start and any rank's launch

    def iterate(self, k):
        for rr in self.ranks:   # one launch per rank, each on its own stream: they run concurrently
            rr.iterate(k)
        torch.cuda.synchronize()

    def poll(self):
        polls = [rr.poll() for rr in self.ranks]
        its = {p[0] for p in polls}
        sts = {p[1] for p in polls}
        assert len(its) == 1 and len(sts) == 1, f"ranks disagree: {polls}"
        return polls[0]

    def solve(self, max_iter=20000, chunk=512):
        self.start()
        done, it, stt = 0, 0, C.PCG_RUNNING
        while done < max_iter:
            k = min(chunk, max_iter - done)
            self.iterate(k)
            done += k
            it, stt, _ = self.poll()
            if stt != C.PCG_RUNNING:
                break
        return it, stt

    def x(self):
        out = torch.empty(self.n, dtype=F64, device=self.ranks[0].x.device)
        for rr in self.ranks:
            out[rr.rs.lo:rr.rs.hi] = rr.own_x()
        return out

    def close(self):
        for rr in self.ranks:
            rr.close()
        torch.cuda.synchronize()
        for raw in self._raw_streams:
            C.lib().fem_stream_destroy(ctypes.c_void_p(raw))
        self._raw_streams = []
