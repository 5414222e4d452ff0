#!/usr/bin/env python3
"""Symmetric-storage SpMV probe (GPU box): can a bs = 1 matrix stored as its upper triangle only (col >= row), with
every lower entry re-read from the upper storage of the row it mirrors, beat the full-matrix SpMV in the persistent
geometry (one 1024-thread workgroup per CU, waves owning contiguous slice ranges)? The re-read only pays if it is
served by the XCD's L2 (written / read moments apart by the neighbouring waves) instead of HBM / memory-side cache.

    python tools/sym_probe.py [--n 119] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fem355  # noqa: E402
from fem355 import _capi as C, mesh, system  # noqa: E402
import lab as lab_lib  # noqa: E402  (tools/lab: probe kernels, not part of libfem355)

I32, I64, F64 = torch.int32, torch.int64, torch.float64


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


def build_sym(rowptr, colidx, vals, N, dev):
    """Upper-triangle plain SELL-64 with per-slice delta lists + the lower re-read tables (see k_spmv_sym_lab)."""
    S = (N + 63) // 64
    r = torch.repeat_interleave(torch.arange(N, device=dev), (rowptr[1:] - rowptr[:-1]).to(I64))
    c = colidx.to(I64)
    d = c - r
    s = r // 64
    lane = r % 64
    up = d >= 0
    # upper lists: unique (slice, delta) keys, sorted -> per-slice lists in ascending delta
    ku = s[up] * 65536 + d[up]
    uk, uinv = torch.unique(ku, return_inverse=True)
    us = uk // 65536
    wU = torch.bincount(us, minlength=S)
    ulist = torch.zeros(S + 1, dtype=I64, device=dev)
    ulist[1:] = torch.cumsum(wU, 0)
    kpos = torch.arange(uk.numel(), device=dev) - ulist[us]        # index of the delta within its slice list
    uptr = ulist * 64
    uvals = torch.zeros(int(uptr[-1]), dtype=F64, device=dev)
    uvals[uptr[s[up]] + 64 * kpos[uinv] + lane[up]] = vals[up]
    udel = (uk % 65536).to(torch.int16)
    # lower lists
    lo = ~up
    kl = s[lo] * 65536 + (-d[lo])
    lk = torch.unique(kl)
    ls = lk // 65536
    dd = lk % 65536
    wL = torch.bincount(ls, minlength=S)
    lptr = torch.zeros(S + 1, dtype=I64, device=dev)
    lptr[1:] = torch.cumsum(wL, 0)
    q, rr = dd // 64, dd % 64

    def base(sp):
        key = sp * 65536 + dd
        i = torch.searchsorted(uk, key).clamp(max=uk.numel() - 1)
        ok = (sp >= 0) & (uk[i] == key)
        return torch.where(ok, uptr[sp.clamp(min=0)] + 64 * kpos[i], torch.full_like(sp, -1))

    ba, bb = base(ls - q), base(ls - q - 1)
    lbase = torch.stack([ba, bb], 1).reshape(-1)
    assert int(uptr[-1]) < 2**31
    return {"uptr": uptr, "ulist": ulist.to(I32), "udel": udel, "lptr": lptr.to(I32), "ldel": dd.to(I32),
            "lbase": lbase.to(I32), "uvals": uvals, "upper_entries": int(uptr[-1]), "lower_lists": int(lk.numel())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=119)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    lib = C.lib()
    lab = lab_lib.load()
    dev = torch.device("cuda", 0)
    st = C.stream(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    coords, tets = mesh.kuhn_cube(a.n, device=dev)
    A = system.assemble_tet4_system(coords, tets, "poisson", 1.0, 0.0)
    g = A.g
    N = A.n
    rowptr, colidx, vals = A.csr()
    vals = vals.reshape(-1)
    PAD = 40000
    xb = torch.zeros(N + 2 * PAD, dtype=F64, device=dev)
    xb[PAD:PAD + N] = torch.randn(N, dtype=F64, device=dev)
    x = xb[PAD:PAD + N]
    y = torch.zeros(N + 64, dtype=F64, device=dev)
    # production format: paired + slice-uniform
    ent = g.sell_entries
    pv = torch.empty(ent, dtype=F64, device=dev)
    pc = torch.empty(ent, dtype=torch.int16, device=dev)
    ucol = torch.zeros(2 * (ent // 64) + 2, dtype=torch.int16, device=dev)
    uoff = torch.empty((N + 63) // 64, dtype=I32, device=dev)
    C.check(lab.fem_lab_sell_uniform(N, C.ptr(g.slice_ptr), C.ptr(A.vals), C.ptr(g.dcols), C.ptr(pv), C.ptr(pc),
                                     C.ptr(ucol), C.ptr(uoff), st), "uniform")
    ref = A.matvec(x)
    lds = 96 << 10

    def full():
        C.check(lab.fem_lab_spmv_persist_uni(ncu, lds, N, C.ptr(g.slice_ptr), C.ptr(pc), C.ptr(pv), C.ptr(uoff),
                                             C.ptr(ucol), C.ptr(x), C.ptr(y), st), "full")
    full()
    torch.cuda.synchronize()
    out = {"n": a.n, "rows": N, "nnz": g.nnz, "uniform_slices": int((uoff >= 0).sum()),
           "full_err": float((y[:N] - ref).abs().max() / ref.abs().max())}
    out["full_us"] = timed(full, a.reps) * 1e3
    for mode in (1, 2):   # gather-volume probe (wrong results by design): half the gathers / none
        def gth(mode=mode):
            C.check(lab.fem_lab_spmv_gather(mode, ncu, lds, N, C.ptr(g.slice_ptr), C.ptr(pv), C.ptr(uoff), C.ptr(ucol),
                                            C.ptr(x), C.ptr(y), st), "gather")
        gth()
        out[f"gather_mode{mode}_us"] = timed(gth, a.reps) * 1e3
    sym = build_sym(rowptr, colidx, vals, N, dev)
    out["upper_entries"] = sym["upper_entries"]

    def symm():
        C.check(lab.fem_lab_spmv_sym(ncu, lds, N, C.ptr(sym["uptr"]), C.ptr(sym["ulist"]), C.ptr(sym["udel"]),
                                     C.ptr(sym["lptr"]), C.ptr(sym["ldel"]), C.ptr(sym["lbase"]), C.ptr(sym["uvals"]),
                                     C.ptr(x), C.ptr(y), st), "sym")
    y.zero_()
    symm()
    torch.cuda.synchronize()
    out["sym_err"] = float((y[:N] - ref).abs().max() / ref.abs().max())
    out["sym_us"] = timed(symm, a.reps) * 1e3
    full_bytes = 8 * ent + 2 * 64 * 0 + 16 * N
    out["full_GBps_values"] = full_bytes / (out["full_us"] * 1e-6) / 1e9
    out["sym_GBps_upper"] = (8 * sym["upper_entries"] + 16 * N) / (out["sym_us"] * 1e-6) / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
