"""Multi-rank path on CPU: world_size 2 over gloo (no GPU).

1. bench.py's control plane (RCCL unique-id broadcast, barriers, max-over-ranks timing) across ranks.
2. The 1D vertex partition and exchange algebra of the sharded supersteps, modelled on the CPU:
   degree-sorted vertices dealt round-robin to P shards (jg_build.hip padded_ids_kernel:
   g = (k % P) * S + k / P), every rank folds only its own rows, then the owned slices of the
   full-length vector are allgathered (the RCCL in-place allgather of jg_api.cpp exchange_allgather).
   The sharded result must equal the single-rank oracle bit for bit (same fold order per row).
3. The sparse halo exchange (jg_halo.hip) with world_size 3 over gloo point-to-point: segmented
   compact vectors, per-peer send lists, receive in place; parity with the oracle and matching
   per-peer counts.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def padded_layout(degree, P):
    """Model of the device relabel: sort by degree desc (id asc), deal round-robin, pad to S."""
    n = len(degree)
    order = np.lexsort((np.arange(n), -degree))  # rank k -> vertex
    S = (n + P - 1) // P
    k = np.arange(n)
    padded = np.empty(n, np.int64)
    padded[order] = (k % P) * S + k // P
    return padded, S


def _worker(rank, ws, port, out_q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    import torch
    import torch.distributed as dist

    import bench
    from oracle import oracle as o

    ctl = bench.Control(ws, rank)
    uid = ctl.bcast_bytes(bytes(range(128)) if rank == 0 else None)
    ok_uid = uid == bytes(range(128))
    ctl.barrier()
    mx = ctl.max(float(rank + 1))
    sm = ctl.sum(1.0)

    # sharded PageRank supersteps over gloo allgather
    scale, n = 11, 1 << 11
    s, t = o.rmat_edges(scale, 16, 5)
    s, t = s.astype(np.int32), t.astype(np.int32)
    indeg = np.bincount(t, minlength=n)
    outdeg = np.bincount(s, minlength=n).astype(np.float64)
    padded, S = padded_layout(indeg, ws)
    dense_of_padded = np.full(ws * S, -1, np.int64)
    dense_of_padded[padded] = np.arange(n)
    gs, gt = padded[s], padded[t]
    mine = (gt // S) == rank
    # in-CSR over this rank's rows, entries sorted by global column id (device CSR order)
    rows = gt[mine] - rank * S
    cols = gs[mine]
    key = np.lexsort((cols, rows))
    rows, cols = rows[key], cols[key]
    ptr = np.searchsorted(rows, np.arange(S + 1))
    od = np.zeros(ws * S)
    od[padded] = outdeg
    contrib = np.zeros(ws * S)
    contrib[padded] = (1.0 / n) / outdeg
    iters = 12
    rank_local = np.full(S, 1.0 / n)
    for _ in range(iters - 1):
        nxt = np.zeros(S)
        for r in range(S):
            acc = 0.0
            for j in range(ptr[r], ptr[r + 1]):
                acc = acc + contrib[cols[j]]
            rank_local[r] = 0.85 * acc + 0.15 / n
            g = rank * S + r
            nxt[r] = rank_local[r] / od[g] if dense_of_padded[g] >= 0 else 0.0
        parts = [torch.zeros(S, dtype=torch.float64) for _ in range(ws)]
        dist.all_gather(parts, torch.from_numpy(nxt))  # the exchange step
        contrib = torch.cat(parts).numpy()
    ranks_all = [None] * ws
    dist.all_gather_object(ranks_all, (rank, rank_local.tolist()))
    full = np.zeros(ws * S)
    for r, vals in ranks_all:
        full[r * S:(r + 1) * S] = vals
    got = full[padded]
    if rank == 0:
        ref, _ = o.pagerank(n, s, t, 0.85, n, iters)
        rel = float(np.max(np.abs(got - ref) / ref))
        out_q.put(("rank0", ok_uid, mx, sm, rel, int(S), int(mine.sum())))
    else:
        out_q.put(("rank1", ok_uid, mx, sm, None, int(S), int(mine.sum())))
    ctl.close()


@pytest.mark.timeout(300)
def test_two_rank_gloo_partition_and_exchange(oracle_lib):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, uid0, mx0, sm0, rel, S0, e0), (_, uid1, mx1, sm1, _, S1, e1) = res
    assert uid0 and uid1  # the RCCL unique id reaches every rank
    assert mx0 == mx1 == 2.0 and sm0 == sm1 == 2.0
    assert S0 == S1 == 1024
    assert e0 + e1 == 16 << 11  # every edge is owned by exactly one shard
    assert abs(e0 - e1) < 0.05 * (e0 + e1)  # degree-sorted round-robin balances entries
    assert rel <= 1e-12


def _halo_worker(rank, ws, port, out_q):
    """The sparse halo exchange of jg_halo.hip, modelled rank by rank over gloo point-to-point:
    need / send bitmaps from the full edge list, the segmented compact vector (own rows, then one
    segment of stride T per peer, peer order q < r ? q + 1 : q), columns remapped to compact ids, and
    per superstep: pack the own values each peer reads, send/recv per peer straight into the peer's
    segment (ncclSend/ncclRecv in exchange_halo)."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    import torch
    import torch.distributed as dist

    from oracle import oracle as o

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    scale, n = 10, 1 << 10
    s, t = o.rmat_edges(scale, 16, 9)
    s, t = s.astype(np.int32), t.astype(np.int32)
    indeg = np.bincount(t, minlength=n)
    outdeg = np.bincount(s, minlength=n).astype(np.float64)
    padded, S = padded_layout(indeg, ws)
    gs, gt = padded[s], padded[t]
    P, r = ws, rank
    # halo_mark_kernel (IN adjacency: row = target, col = source)
    rq, cq = gt // S, gs // S
    need = np.zeros(P * S, bool)
    need[gs[(rq == r) & (cq != r)]] = True
    send = np.zeros(P * S, bool)
    sel = (cq == r) & (rq != r)
    send[rq[sel] * S + gs[sel] % S] = True
    recv_cnt = [int(need[q * S:(q + 1) * S].sum()) if q != r else 0 for q in range(P)]
    send_lists = [np.flatnonzero(send[q * S:(q + 1) * S]) if q != r else np.zeros(0, np.int64) for q in range(P)]
    rows_own = int(min(S, (n - r + P - 1) // P))
    T = 1 << 13
    while T < max([rows_own, 8192] + recv_cnt):
        T <<= 1
    seg = lambda q: q + 1 if q < r else q  # noqa: E731
    prefix = np.concatenate([[0], np.cumsum(need)])

    def compact(g):
        q, l = g // S, g % S
        rk = prefix[g] - prefix[q * S]
        return np.where(q == r, l, np.where(q < r, q + 1, q) * T + rk)

    mine = rq == r
    rows = gt[mine] - r * S
    cols = compact(gs[mine])
    key = np.lexsort((cols, rows))
    rows, cols = rows[key], cols[key]
    ptr = np.searchsorted(rows, np.arange(S + 1))
    dense_of_padded = np.full(P * S, -1, np.int64)
    dense_of_padded[padded] = np.arange(n)
    od = np.zeros(P * S)
    od[padded] = outdeg
    vec = np.zeros(P * T)  # the shard's gathered vector
    own_g = r * S + np.arange(S)
    valid = dense_of_padded[own_g] >= 0
    vec[:S][valid] = (1.0 / n) / od[own_g][valid]

    def exchange():
        reqs, bufs = [], {}
        for q in range(P):
            if q == r:
                continue
            if len(send_lists[q]):
                reqs.append(dist.isend(torch.from_numpy(vec[send_lists[q]].copy()), q))
            if recv_cnt[q]:
                bufs[q] = torch.zeros(recv_cnt[q], dtype=torch.float64)
                reqs.append(dist.irecv(bufs[q], q))
        for rq_ in reqs:
            rq_.wait()
        for q, b in bufs.items():
            vec[seg(q) * T:seg(q) * T + recv_cnt[q]] = b.numpy()

    exchange()
    iters = 10
    rank_local = np.full(S, 1.0 / n)
    for _ in range(iters - 1):
        nxt = np.zeros(S)
        for row in range(S):
            acc = 0.0
            for j in range(ptr[row], ptr[row + 1]):
                acc = acc + vec[cols[j]]
            rank_local[row] = 0.85 * acc + 0.15 / n
            g = r * S + row
            nxt[row] = rank_local[row] / od[g] if dense_of_padded[g] >= 0 else 0.0
        vec[:S] = nxt
        exchange()
    # every peer sends exactly what each receiver expects (check_halo_counts)
    counts = [None] * ws
    dist.all_gather_object(counts, (r, [len(x) for x in send_lists], recv_cnt))
    ok_counts = all(counts[q][1][p] == counts[p][2][q] for p in range(P) for q in range(P) if p != q)
    vol = sum(recv_cnt)
    ranks_all = [None] * ws
    dist.all_gather_object(ranks_all, (r, rank_local.tolist()))
    full = np.zeros(ws * S)
    for rr, vals in ranks_all:
        full[rr * S:(rr + 1) * S] = vals
    got = full[padded]
    rel = None
    if rank == 0:
        ref, _ = o.pagerank(n, s, t, 0.85, n, iters)
        rel = float(np.max(np.abs(got - ref) / ref))
    out_q.put((rank, ok_counts, vol, (P - 1) * S, rel))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_three_rank_gloo_halo_exchange(oracle_lib):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_counts, vol, dense, _ in res:
        assert ok_counts
        assert 0 < vol < dense  # the halo is a strict subset of the dense allgather
    assert res[0][4] <= 1e-12


def _sd_worker(rank, ws, port, out_q):
    """Sharded ShortestDistanceVertexProgram (jg_traverse.hip shortest_distance_sharded) modelled rank
    by rank over gloo: the IN adjacency's halo layout as in _halo_worker; per superstep each rank
    pushes min(msg[w] + weight) from its frontier rows into own rows and halo slots, the REVERSE
    halo exchange (exchange_halo_reverse: segment for peer q goes back to q, landing at q's send-list
    positions) hands remote candidates to their owners, owners take the min and apply; frontier
    sizes are summed over ranks (allreduce_sum_i64)."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    import torch
    import torch.distributed as dist

    from oracle import oracle as o

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    scale, n = 9, 1 << 9
    s, t = o.rmat_edges(scale, 8, 3)
    s, t = s.astype(np.int32), t.astype(np.int32)
    wt = (np.arange(len(s)) % 3 + 1).astype(np.int64)
    indeg = np.bincount(t, minlength=n)
    padded, S = padded_layout(indeg, ws)
    gs, gt = padded[s], padded[t]
    P, r = ws, rank
    rq, cq = gt // S, gs // S
    need = np.zeros(P * S, bool)
    need[gs[(rq == r) & (cq != r)]] = True
    send = np.zeros(P * S, bool)
    sel = (cq == r) & (rq != r)
    send[rq[sel] * S + gs[sel] % S] = True
    recv_cnt = [int(need[q * S:(q + 1) * S].sum()) if q != r else 0 for q in range(P)]
    send_lists = [np.flatnonzero(send[q * S:(q + 1) * S]) if q != r else np.zeros(0, np.int64) for q in range(P)]
    T = 1 << 12
    seg = lambda q: q + 1 if q < r else q  # noqa: E731
    prefix = np.concatenate([[0], np.cumsum(need)])

    def compact(g):
        q, l = g // S, g % S
        rk = prefix[g] - prefix[q * S]
        return np.where(q == r, l, np.where(q < r, q + 1, q) * T + rk)

    mine = rq == r
    rows, cols, ws_ = gt[mine] - r * S, compact(gs[mine]), wt[mine]
    key = np.lexsort((cols, rows))
    rows, cols, ws_ = rows[key], cols[key], ws_[key]
    ptr = np.searchsorted(rows, np.arange(S + 1))
    INF, ABSENT = np.iinfo(np.int64).max, np.iinfo(np.int64).min
    seed_dense, max_depth = int(t[0]), 5
    seed_g = int(padded[seed_dense])
    best = np.full(P * T, INF, np.int64)
    dist_ = np.full(S, ABSENT, np.int64)
    msg = np.zeros(S, np.int64)
    frontier = []
    if seed_g // S == r:
        dist_[seed_g % S] = 0
        frontier = [seed_g % S]
    total = torch.tensor([len(frontier)], dtype=torch.int64)
    dist.all_reduce(total)
    for _ in range(max_depth):
        if int(total) == 0:
            break
        for w in frontier:  # ssd_push_kernel
            for j in range(ptr[w], ptr[w + 1]):
                best[cols[j]] = min(best[cols[j]], msg[w] + ws_[j])
        reqs, bufs = [], {}  # exchange_halo_reverse
        for q in range(P):
            if q == r:
                continue
            if recv_cnt[q]:
                reqs.append(dist.isend(torch.from_numpy(best[seg(q) * T:seg(q) * T + recv_cnt[q]].copy()), q))
            if len(send_lists[q]):
                bufs[q] = torch.zeros(len(send_lists[q]), dtype=torch.int64)
                reqs.append(dist.irecv(bufs[q], q))
        for x in reqs:
            x.wait()
        for q, b in bufs.items():  # ssd_recv_kernel
            np.minimum.at(best, send_lists[q], b.numpy())
        for q in range(P):
            if q != r:
                best[seg(q) * T:seg(q) * T + recv_cnt[q]] = INF
        nxt = []  # sd_apply_kernel
        for u in np.flatnonzero(best[:S] != INF):
            b = best[u]
            best[u] = INF
            if dist_[u] == ABSENT or dist_[u] > b:
                dist_[u] = b
                msg[u] = b
                nxt.append(int(u))
        frontier = nxt
        total = torch.tensor([len(frontier)], dtype=torch.int64)
        dist.all_reduce(total)
    parts = [None] * ws
    dist.all_gather_object(parts, (r, dist_.tolist()))
    full = np.zeros(ws * S, np.int64)
    for rr, vals in parts:
        full[rr * S:(rr + 1) * S] = vals
    got = full[padded]  # ABSENT == the oracle's DIST_ABSENT
    ok = None
    if rank == 0:
        ref = o.shortest_distance(n, s, t, seed_dense, max_depth, wt.astype(np.int32))
        ok = bool(np.array_equal(got, ref)) and int((ref >= 0).sum()) > 1
    out_q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_sharded_shortest_distance(oracle_lib):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sd_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] is True
