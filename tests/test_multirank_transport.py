"""Rank mode (one process per shard) driven through the library's multi-process code paths on one GPU.

RCCL refuses two ranks on one device, so the driver's 8-GPU run is the only place its send/recv can
execute.  Here two processes share device 0 and the library's exchanges go through a host transport
(jg_ctx_create_rank_transport, gloo underneath): the same rank-mode build (each process builds only
its shard), halo-plan count check, pack kernels, segment placement, reverse exchange and all-reduces
as with RCCL, checked against the oracle: PageRank, CC, single-source DO-BFS, the 8-source bit-parallel
BFS, weighted shortest distance, and jg_graph_neighbors' entry counts (bench.py's source pick).  Per-vertex outputs hold each rank's own vertices; rank 0
combines them.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _combine(dist, world, a, fill):
    """Every rank's array element-wise: each vertex is filled by exactly one rank."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    out = np.array(a, copy=True)
    owned = np.zeros(len(a), np.int32)
    for p in parts:
        p = p.numpy()
        mine = ~np.isnan(p) if np.issubdtype(p.dtype, np.floating) else p != fill
        out[mine] = p[mine]
        owned += mine
    return out, owned


def _worker(rank, world, port, halo, errfile):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import janusgraph_amd as jg
        from janusgraph_amd import _lib
        from janusgraph_amd.transport import GlooTransport
        from oracle import oracle as o
        _lib.tune_set("halo", halo)
        scale = 12
        n = 1 << scale
        s, d = o.rmat_edges(scale, 16, 7)
        vid = (np.arange(n, dtype=np.int64) + 1) << 8
        ctx = jg.Context((0,), rank=rank, nranks=world, transport=GlooTransport(dist, world))
        w = (np.arange(len(s)) % 5 + 1).astype(np.int32)
        g = ctx.build(vid, vid[s], vid[d], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
        assert g.info()["num_shards"] == world
        pr, _ = g.pagerank(0.85, n, 12)
        pr, own_pr = _combine(dist, world, pr, None)
        comp, it = g.connected_components()
        comp, own_cc = _combine(dist, world, comp, np.iinfo(np.int64).max)
        src = int(s[0])
        depth = g.bfs([vid[src]], jg.DIR_BOTH)[0]
        depth, own_d = _combine(dist, world, depth, np.iinfo(np.int32).min)
        msrc = [int(x) for x in s[:8]]
        ms = g.bfs(vid[msrc], jg.DIR_BOTH, max_depth=5).ravel()  # the sharded bit-parallel pull (rank mode)
        ms, own_ms = _combine(dist, world, ms, np.iinfo(np.int32).min)
        import torch
        deg = torch.from_numpy(g.degrees(jg.DIR_BOTH))  # rank mode: own rows' entry counts, 0 for the others
        dist.all_reduce(deg)
        deg = deg.numpy()
        sd = own_sd = None
        if halo:  # sharded shortest distance runs over the halo plan only
            sd = g.shortest_distance(vid[src], 6)
            sd, own_sd = _combine(dist, world, sd, np.iinfo(np.int64).max)
        if rank == 0:
            assert (own_pr == 1).all() and (own_cc == 1).all() and (own_d == 1).all(), "every vertex owned once"
            ds, dd = s.astype(np.int32), d.astype(np.int32)
            ref, _ = o.pagerank(n, ds, dd, 0.85, n, 12)
            rel = np.abs(pr - ref) / np.abs(ref)
            assert rel.max() <= 1e-9, f"PageRank parity {rel.max()}"
            cref, cit = o.connected_components(n, ds, dd, vid)
            np.testing.assert_array_equal(comp, cref)
            assert it == cit, (it, cit)
            np.testing.assert_array_equal(depth, o.bfs(n, ds, dd, src, o.DIR_BOTH))
            assert (own_ms == 1).all()
            for k, sv in enumerate(msrc):
                np.testing.assert_array_equal(ms[k * n:(k + 1) * n], o.bfs(n, ds, dd, sv, o.DIR_BOTH, 5))
            np.testing.assert_array_equal(deg, np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n))
            if sd is not None:
                assert (own_sd == 1).all()
                np.testing.assert_array_equal(sd, o.shortest_distance(n, ds, dd, src, 6, w))
        g.close()
        ctx.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        with open(errfile, "a") as f:
            f.write(f"rank {rank}:\n" + traceback.format_exc())
        raise


def _worker_msbfs(rank, world, port, errfile):
    """64 sources, unbounded, rank mode (the driver's N-GPU bench runs this path): top-down levels with the
    sparse pair exchange, pull levels after the frontier's peak, the last levels top-down again; every row
    against the oracle, and the level count."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import janusgraph_amd as jg
        from janusgraph_amd.transport import GlooTransport
        from oracle import oracle as o
        scale = 14
        n = 1 << scale
        s, d = o.rmat_edges(scale, 16, 0x5EED + scale)
        ds, dd = s.astype(np.int32), d.astype(np.int32)
        vid = (np.arange(n, dtype=np.int64) + 1) << 8
        ctx = jg.Context((0,), rank=rank, nranks=world, transport=GlooTransport(dist, world))
        g = ctx.build(vid, vid[s], vid[d], flags=jg.ADJ_BOTH)
        deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
        # 62 sources with an edge, an isolated vertex and a hub
        srcs = np.concatenate([np.random.default_rng(14).choice(np.flatnonzero(deg > 0), 62, replace=False),
                               [np.flatnonzero(deg == 0)[0], int(np.argmax(deg))]]).astype(np.int64)
        for max_depth in (-1, 2):
            got = g.bfs(vid[srcs], jg.DIR_BOTH, max_depth=max_depth)
            levels = ctx.stats()["levels"]
            got, own = _combine(dist, world, got.ravel(), np.iinfo(np.int32).min)
            if rank == 0:
                assert (own == 1).all(), "every (source, vertex) owned once"
                got = got.reshape(len(srcs), n)
                ptr, adj = o.csr_unordered(n, ds, dd, both=True)
                want = o.msbfs_csr(n, ptr, adj, srcs, max_depth)
                for k in range(len(srcs)):
                    np.testing.assert_array_equal(got[k], want[k], err_msg=f"source {k}, max_depth {max_depth}")
                deepest = int(want.max())
                assert levels == (deepest + 1 if max_depth < 0 else min(deepest + 1, max_depth)), (levels, deepest)
        g.close()
        ctx.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        with open(errfile, "a") as f:
            f.write(f"rank {rank}:\n" + traceback.format_exc())
        raise


def _worker_cc(rank, world, port, errfile, logfile):
    """Sharded CC in rank mode on a graph of many cross-shard chains (many label rounds, few labels moving
    in each after the first): the sparse pair rounds over the host transport (the library's JG_DEBUG_CC
    log must show a sparse forward) and the dense rounds (cc_sparse 0), both against the oracle."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["JG_DEBUG_CC"] = "1"
        fd = os.open(f"{logfile}.{rank}", os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
        os.dup2(fd, 2)  # the library's per-round log
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import janusgraph_amd as jg
        from janusgraph_amd import _lib
        from janusgraph_amd.transport import GlooTransport
        from oracle import oracle as o
        rng = np.random.default_rng(5)
        n, plen = 4000, 40
        perm = rng.permutation(n)
        s, d = [], []
        for c0 in range(0, 3200, plen):  # 80 chains of 40 vertices with scattered ids
            ch = perm[c0:c0 + plen]
            s += list(ch[:-1])
            d += list(ch[1:])
        s += list(rng.integers(3200, n, 900))  # a random part: small components and a few larger ones
        d += list(rng.integers(3200, n, 900))
        s, d = np.array(s, np.int32), np.array(d, np.int32)
        vid = (np.arange(n, dtype=np.int64) + 3) * 7
        ctx = jg.Context((0,), rank=rank, nranks=world, transport=GlooTransport(dist, world))
        g = ctx.build(vid, vid[s], vid[d], flags=jg.ADJ_BOTH)
        out = []
        for sparse in (1, 0):
            _lib.tune_set("cc_sparse", sparse)
            comp, it = g.connected_components()
            comp, own = _combine(dist, world, comp, np.iinfo(np.int64).max)
            out.append((comp, it, own))
        _lib.tune_set("cc_sparse", 1)
        if rank == 0:
            cref, cit = o.connected_components(n, s, d, vid)
            for comp, it, own in out:
                assert (own == 1).all()
                np.testing.assert_array_equal(comp, cref)
                assert it == cit, (it, cit)
        g.close()
        ctx.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        with open(errfile, "a") as f:
            f.write(f"rank {rank}:\n" + traceback.format_exc())
        raise


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world,halo", [(2, 1), (2, 0), (3, 1)])
def test_ranks_over_host_transport(tmp_path, world, halo):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    errfile = str(tmp_path / "err.txt")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, halo, errfile)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    err = open(errfile).read() if os.path.exists(errfile) else ""
    assert all(p.exitcode == 0 for p in procs), f"exit codes {[p.exitcode for p in procs]}\n{err}"


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_msbfs64_unbounded_ranks_over_host_transport(tmp_path, world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    errfile = str(tmp_path / "err.txt")
    port = _free_port()
    procs = [ctx.Process(target=_worker_msbfs, args=(r, world, port, errfile)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    err = open(errfile).read() if os.path.exists(errfile) else ""
    assert all(p.exitcode == 0 for p in procs), f"exit codes {[p.exitcode for p in procs]}\n{err}"


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_cc_sparse_rounds_ranks_over_host_transport(tmp_path, world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    errfile = str(tmp_path / "err.txt")
    logfile = str(tmp_path / "cc.log")
    port = _free_port()
    procs = [ctx.Process(target=_worker_cc, args=(r, world, port, errfile, logfile)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    err = open(errfile).read() if os.path.exists(errfile) else ""
    assert all(p.exitcode == 0 for p in procs), f"exit codes {[p.exitcode for p in procs]}\n{err}"
    log = open(f"{logfile}.0").read()
    assert "forward sparse" in log, log[-2000:]
