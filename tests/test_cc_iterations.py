"""The identity the one-shard connected-components path relies on (jg_cc.hip cc_union_find), checked
on the oracle's restatement of the superstep loop (oracle jo_connected_components,
ConnectedComponentVertexProgram as Fulgora runs it):

    labels     = the minimum String-order id of each vertex's component
    iterations = D + 1 if any vertex has an edge, else 0,  D = max_v dist(v, c(v)),
                 c(v) the minimum-rank vertex of v's component (hop distance over BOTH edges)

as long as D + 1 stays below the 100-iteration cap (beyond it the GPU runs the propagation itself).
Random graphs with isolated vertices, self-loops, multi-edges, paths and stars; pure Python BFS.
"""
from collections import deque

import numpy as np
import pytest


def predicted(n, src, dst, vid, rank):
    adj = [[] for _ in range(n)]
    for a, b in zip(src.tolist(), dst.tolist()):
        adj[a].append(b)
        adj[b].append(a)
    comp = [-1] * n
    label = [0] * n
    far = -1
    for s in range(n):
        if comp[s] >= 0:
            continue
        members, q = [s], deque([s])
        comp[s] = s
        while q:
            u = q.popleft()
            for w in adj[u]:
                if comp[w] < 0:
                    comp[w] = s
                    members.append(w)
                    q.append(w)
        c = min(members, key=lambda x: rank[x])
        dist = {c: 0}
        q = deque([c])
        while q:
            u = q.popleft()
            for w in adj[u]:
                if w not in dist:
                    dist[w] = dist[u] + 1
                    q.append(w)
        for x in members:
            label[x] = int(vid[c])
        if any(adj[x] for x in members):
            far = max(far, max(dist.values()))
    iterations = far + 1 if len(src) else 0
    return np.array(label, np.int64), iterations


def graphs():
    rng = np.random.default_rng(3)
    for n, m in ((1, 0), (5, 0), (40, 30), (200, 150), (300, 900), (500, 400)):
        yield n, rng.integers(0, n, m), rng.integers(0, n, m)
    n = 60  # self-loops only, and a path, and a star
    yield n, np.arange(10), np.arange(10)
    yield n, np.arange(n - 1), np.arange(1, n)
    yield n, np.zeros(n - 1, np.int64), np.arange(1, n)


@pytest.mark.parametrize("case", list(range(9)))
def test_iterations_are_the_root_eccentricity_plus_one(oracle_lib, case):
    n, src, dst = list(graphs())[case]
    rng = np.random.default_rng(case)
    vid = rng.choice(np.arange(1, 10 * n + 2), n, replace=False).astype(np.int64) * 7
    rank = oracle_lib.lex_rank(vid)
    want_label, want_it = predicted(n, np.asarray(src), np.asarray(dst), vid, rank)
    assert want_it <= 98
    label, it = oracle_lib.connected_components(n, src, dst, vid)
    assert it == want_it
    np.testing.assert_array_equal(label, want_label)


def test_long_path_reaches_the_cap(oracle_lib):
    """A 150-vertex path whose minimum sits at one end: D = 149, so Fulgora stops at 99 supersteps
    with labels still in flight (the GPU's one-shard path hands this case to the propagation)."""
    n = 150
    vid = np.arange(10, 10 + n, dtype=np.int64)  # all 2-digit then 3-digit: "10" is the minimum, at vertex 0
    src, dst = np.arange(n - 1), np.arange(1, n)
    rank = oracle_lib.lex_rank(vid)
    _, pred_it = predicted(n, src, dst, vid, rank)
    label, it = oracle_lib.connected_components(n, src, dst, vid)
    assert pred_it > 99 and it == 99
    assert len(set(label.tolist())) > 1  # not converged
