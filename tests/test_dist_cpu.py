"""N>1 path on the CPU: world-size-2 gloo run of the element-partitioned PCG (oracle/dist_ref.py) on the product's
RCB partition and halo maps (fem355.dist), against the serial oracle solve."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, out_path, variant):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fem355  # noqa: F401
    from fem355 import dist as fd, mesh
    from oracle import dist_ref
    coords, tets = mesh.kuhn_cube(5, jitter=0.1)
    if kind == "poisson":
        f, fixed = mesh.cube_poisson_case(coords)
        E, nu = 1.0, 0.0
    else:
        f, fixed = mesh.cube_elasticity_case(coords)
        E, nu = 113.8e9, 0.342
    part = fd.rcb_partition(fd.element_centroids(coords, tets), world)
    rm = fd.rank_mesh(tets, part, rank, world, coords.shape[0])
    if variant == "matfree":   # the N > 1 element-chunk form: single reduction, element vectors formed every application
        x, it, st = dist_ref.dist_pcg_single(coords, tets, f, fixed, rm, kind, E, nu, tol=1e-9, max_iter=2000,
                                             operator="matfree")
    else:
        solve = dist_ref.dist_pcg_single if variant == "single" else dist_ref.dist_pcg
        x, it, st = solve(coords, tets, f, fixed, rm, kind, E, nu, tol=1e-9, max_iter=2000)
    torch.save({"nodes": rm.nodes, "own": rm.own, "x": x, "it": it, "st": st, "nI": rm.n_iface},
               f"{out_path}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["two", "single", "matfree"])
@pytest.mark.parametrize("kind", ["poisson", "elastic"])
def test_partitioned_pcg_matches_serial(tmp_path, kind, variant):
    """Both distributed forms: two reductions per iteration, and the single-reduction (Chronopoulos-Gear) form --
    the latter also on the element-vector operator without stored K_e (the N > 1 element-chunk path's algebra)."""
    from fem355 import mesh
    from oracle import ref_cpu as R
    world = 2
    out = str(tmp_path / "res")
    mp.spawn(_worker, args=(world, _free_port(), kind, out, variant), nprocs=world, join=True)
    res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    coords, tets = mesh.kuhn_cube(5, jitter=0.1)
    N = coords.shape[0]
    if kind == "poisson":
        f, fixed = mesh.cube_poisson_case(coords)
        K, bs = R.tet4_poisson_K(coords, tets), 1
    else:
        f, fixed = mesh.cube_elasticity_case(coords)
        K, bs = R.tet4_K(coords, tets, 113.8e9, 0.342), 3
    Minv = R.diag_preconditioner(K, tets, N, dpn=bs)
    Minv[fixed] = 0.0
    u, it, st = R.pcg(K, tets, f.view(N, bs), Minv, tol=1e-9, max_iter=2000)
    assert st == "converged"
    assert all(r["st"] == "converged" for r in res)
    assert abs(res[0]["it"] - it) <= 2 and res[0]["it"] == res[1]["it"]
    assert res[0]["nI"] > 0
    glob = torch.zeros(N, bs, dtype=torch.float64)
    owned = torch.zeros(N, dtype=torch.int32)
    for r in res:
        o = r["own"].bool()
        glob[r["nodes"][o]] = r["x"].view(-1, bs)[o]
        owned[r["nodes"][o]] += 1
    assert bool((owned == 1).all())                     # every node owned exactly once
    assert float((glob - u).abs().max() / u.abs().max()) < 1e-10
    # shared copies agree across ranks
    common, i0, i1 = (lambda a, b: (lambda c: (c, torch.searchsorted(a, c), torch.searchsorted(b, c)))(
        a[torch.isin(a, b)]))(res[0]["nodes"], res[1]["nodes"])
    assert common.numel() > 0
    assert torch.equal(res[0]["x"].view(-1, bs)[i0], res[1]["x"].view(-1, bs)[i1])


def test_rcb_partition_properties():
    from fem355 import dist as fd, mesh
    coords, tets = mesh.kuhn_cube(8)
    for P in (2, 3, 4, 8):
        part = fd.rcb_partition(fd.element_centroids(coords, tets), P)
        counts = torch.bincount(part, minlength=P)
        assert int(counts.sum()) == tets.shape[0] and int(counts.min()) > 0
        assert int(counts.max() - counts.min()) <= 1
        # deterministic
        assert torch.equal(part, fd.rcb_partition(fd.element_centroids(coords, tets), P))
    part = fd.rcb_partition(fd.element_centroids(coords, tets), 8)
    cnt, owner = fd.node_sharing(tets, part, 8, coords.shape[0])
    rms = [fd.rank_mesh(tets, part, r, 8, coords.shape[0], (cnt, owner)) for r in range(8)]
    nI = rms[0].n_iface
    assert all(rm.n_iface == nI for rm in rms)
    # each interface node is present on >= 2 ranks, its ipos/imap are mutually consistent
    pres = torch.zeros(nI, dtype=torch.int32)
    for rm in rms:
        has = rm.imap >= 0
        pres += has.int()
        loc = rm.imap[has].long()
        assert torch.equal(rm.ipos[loc].long(), torch.nonzero(has, as_tuple=True)[0])
    assert bool((pres >= 2).all())


@pytest.mark.parametrize("P,bs", [(2, 1), (3, 3), (8, 1)])
def test_p2p_maps_sum_like_the_allreduce(P, bs):
    """Neighbour-exchange maps (fem355.dist.p2p_maps) on CPU, with the kernels' rules: the SpMV scatters each
    interface row into every peer slot of csrc (>= 0) and the [g, d] pair into ssrc; the slots are delivered;
    the update sums in rank order (-1: own row, -2: skip). Every rank's sum of a shared row equals the rank-ordered
    sum of all holders' partials bit for bit (so copies agree across ranks), and [g, d] the rank-ordered sum."""
    from fem355 import dist as fd, mesh
    coords, tets = mesh.kuhn_cube(6, jitter=0.1)
    N = coords.shape[0]
    part = fd.rcb_partition(fd.element_centroids(coords, tets), P)
    touch = fd.touch_masks(tets, part, P, N)
    sharing = fd.node_sharing(tets, part, P, N)
    rms = [fd.rank_mesh(tets, part, r, P, N, sharing) for r in range(P)]
    maps = [fd.p2p_maps(rm, touch, bs) for rm in rms]
    nI = rms[0].n_iface
    iface = torch.nonzero(sharing[0] > 1, as_tuple=True)[0]
    g = torch.Generator().manual_seed(7)
    part_rows = torch.randn(P, nI, bs, generator=g, dtype=torch.float64)   # rank r's partial of node J
    pairs = torch.randn(P, 2, generator=g, dtype=torch.float64)
    psend = []
    for a, m in enumerate(maps):
        buf = torch.full((sum(m.peer_cnt),), float("nan"), dtype=torch.float64)
        for J in range(nI):
            for r in range(P):
                dst = int(m.csrc[J, r])
                if dst >= 0:
                    buf[dst:dst + bs] = part_rows[a, J]
        for r in range(P):
            dst = int(m.ssrc[r])
            if dst >= 0:
                buf[dst:dst + 2] = pairs[a]
        psend.append(buf)
    assert all(not bool(torch.isnan(b).any()) for b in psend)   # every slot element written
    offs = [[sum(m.peer_cnt[:i]) for i in range(len(m.peer_cnt))] for m in maps]
    precv = [torch.zeros_like(b) for b in psend]
    for a, m in enumerate(maps):
        for i, b in enumerate(m.peer_rank):
            j = maps[b].peer_rank.index(a)
            assert maps[b].peer_cnt[j] == m.peer_cnt[i]
            precv[b][offs[b][j]: offs[b][j] + m.peer_cnt[i]] = psend[a][offs[a][i]: offs[a][i] + m.peer_cnt[i]]
    for a, m in enumerate(maps):
        held = touch[a, iface]
        for J in range(nI):
            if not bool(held[J]):
                assert bool((m.csrc[J] == -2).all())
                continue
            for c in range(bs):
                acc, ref = 0.0, 0.0
                for r in range(P):
                    src = int(m.csrc[J, r])
                    if src == -1:
                        acc += float(part_rows[a, J, c])
                    elif src >= 0:
                        acc += float(precv[a][src + c])
                    if bool(touch[r, iface[J]]):
                        ref += float(part_rows[r, J, c])
                assert acc == ref, (a, J, c)
        for c in range(2):
            acc = 0.0
            for r in range(P):
                src = int(m.ssrc[r])
                acc += float(pairs[a, c]) if src < 0 else float(precv[a][src + c])
            ref = 0.0
            for r in range(P):
                ref += float(pairs[r, c])
            assert acc == ref


def test_row_partition_helpers():
    """dist_persist's row partition (host logic): contiguous slice ranges within one slice of each other, covering
    every row once; a rank's elements are exactly those touching its rows."""
    import torch
    from fem355 import dist_persist as DP, mesh
    for n_rows, P in ((1000, 2), (64 * 27000, 8), (65, 1), (64 * 8 + 3, 8)):
        sp = DP.slice_split(n_rows, P)
        assert sp[0] == 0 and sp[-1] == (n_rows + 63) // 64 and len(sp) == P + 1
        sizes = [sp[i + 1] - sp[i] for i in range(P)]
        assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
        rows = [DP.rank_rows(n_rows, sp, r) for r in range(P)]
        assert rows[0][0] == 0 and rows[-1][1] == n_rows
        assert all(rows[i][1] == rows[i + 1][0] for i in range(P - 1))
    c, t = mesh.kuhn_cube(5)
    sp = DP.slice_split(c.shape[0], 2)
    lo, hi = DP.rank_rows(c.shape[0], sp, 1)
    el = DP.rank_elements(t, lo, hi)
    touch = ((t >= lo) & (t < hi)).any(1)
    assert el.shape[0] == int(touch.sum()) and torch.equal(el, t[touch])
