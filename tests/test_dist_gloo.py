"""Multi-rank path on CPU: world_size 2 over gloo (no GPU).

1. bench.py's control plane (RCCL unique-id broadcast, barriers, max-over-ranks timing) across ranks.
2. The 1D vertex partition and exchange algebra of the sharded supersteps, modelled on the CPU:
   degree-sorted vertices dealt round-robin to P shards (jg_build.hip padded_ids_kernel:
   g = (k % P) * S + k / P), every rank folds only its own rows, then the owned slices of the
   full-length vector are allgathered (the RCCL in-place allgather of jg_api.cpp exchange_allgather).
   The sharded result must equal the single-rank oracle bit for bit (same fold order per row).
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
