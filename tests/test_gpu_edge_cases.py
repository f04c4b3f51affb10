"""GPU edge cases of the programs, each against the oracle (the restatement of the reference's
semantics) on the same graph:
  * PageRank with vertexCount at its default of 1 and with vertexCount != |V|
    (PageRankVertexProgram.java:64-69: N is the user's parameter, not the measured count), and
    K = 0 / 1 / 2 supersteps (:107-110: K - 1 power steps; K = 0 writes no property);
  * ShortestDistance with maxDepth = 0 (ShortestDistanceVertexProgram.java:144-146: only the seed);
  * CC, BFS, PageRank and ShortestDistance on an edgeless graph and on a graph whose every edge is a
    ghost edge (VertexJobConverter.java:126-129).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PR_RTOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    import janusgraph_amd as jg
    c = jg.Context((0,))
    yield c
    c.close()


@pytest.fixture(scope="module")
def rmat12(oracle_lib):
    o = oracle_lib
    n = 1 << 12
    s, t = o.rmat_edges(12, 16, 21)
    vid = (np.random.default_rng(3).permutation(n).astype(np.int64) + 1) << 8
    return n, vid, s.astype(np.int32), t.astype(np.int32)


def assert_pr(got, want):
    nan = np.isnan(want)
    assert (np.isnan(got) == nan).all()
    rel = np.abs(got[~nan] - want[~nan]) / np.maximum(np.abs(want[~nan]), 1e-300)
    assert rel.max(initial=0.0) <= PR_RTOL, f"max rel err {rel.max()}"


@pytest.mark.parametrize("vertex_count,iterations", [(1, 10), (1, 0), (1, 1), (1, 2), (7, 30), ("n+1000", 12),
                                                     ("n", 0), ("n", 1), ("n", 2)])
def test_pagerank_vertex_count_and_iterations(ctx, oracle_lib, rmat12, vertex_count, iterations):
    import janusgraph_amd as jg
    n, vid, s, t = rmat12
    N = {"n": n, "n+1000": n + 1000}.get(vertex_count, vertex_count)
    g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_IN)
    rank, ec = g.pagerank(0.85, N, iterations)
    want, ec_want = oracle_lib.pagerank(n, s, t, 0.85, N, iterations)
    assert_pr(rank, want)
    assert_pr(ec, ec_want)
    assert ctx.stats()["supersteps"] == iterations
    g.close()


@pytest.mark.parametrize("max_depth", [0, 1])
def test_shortest_distance_max_depth_small(ctx, oracle_lib, rmat12, max_depth):
    import janusgraph_amd as jg
    n, vid, s, t = rmat12
    w = (np.arange(len(s)) % 3 + 1).astype(np.int32)
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    seed = int(t[0])
    got = g.shortest_distance(vid[seed], max_depth)
    want = oracle_lib.shortest_distance(n, s, t, seed, max_depth, w)
    np.testing.assert_array_equal(got, want)
    assert got[seed] == 0
    if max_depth == 0:
        assert (got >= 0).sum() == 1
    g.close()


@pytest.mark.parametrize("case", ["edgeless", "all_ghost"])
def test_programs_without_edges(ctx, oracle_lib, case):
    import janusgraph_amd as jg
    o = oracle_lib
    n = 37
    vid = ((np.arange(n, dtype=np.int64) * 7 + 3) << 8)
    if case == "edgeless":
        src = dst = np.zeros(0, np.int64)
    else:  # every edge has an endpoint the scan did not return (ghost): all dropped
        src = vid[:10]
        dst = np.full(10, (1 << 40) << 8, np.int64)
    g = ctx.build(vid, src, dst, flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    info = g.info()
    assert info["num_edges"] == 0 and info["num_vertices"] == n
    empty = np.zeros(0, np.int32)
    comp, it = g.connected_components()
    want, it_want = o.connected_components(n, empty, empty, vid)
    np.testing.assert_array_equal(comp, want)
    np.testing.assert_array_equal(comp, vid)  # every vertex is its own component
    assert it == it_want
    rank, ec = g.pagerank(0.85, n, 10)
    r_want, ec_want = o.pagerank(n, empty, empty, 0.85, n, 10)
    assert_pr(rank, r_want)
    assert_pr(ec, ec_want)
    depth = g.bfs([vid[5]], jg.DIR_BOTH)[0]
    np.testing.assert_array_equal(depth, o.bfs(n, empty, empty, 5, o.DIR_BOTH))
    dist = g.shortest_distance(vid[5], 10)
    np.testing.assert_array_equal(dist, o.shortest_distance(n, empty, empty, 5, 10))
    g.close()


@pytest.mark.parametrize("shards", [1, 3])
def test_shortest_distance_negative_and_absent_weights(oracle_lib, rmat12, shards):
    """Negative Integer weights give negative distances (reported, not confused with "absent", which
    is JG_DIST_ABSENT); an edge without the weight property (JG_WEIGHT_ABSENT) fails the run only
    when a message crosses it (ShortestDistanceVertexProgram.java:69, VertexMemoryHandler.java:136-138)."""
    import janusgraph_amd as jg
    o = oracle_lib
    n, vid, s, t = rmat12
    rng = np.random.default_rng(9)
    w = rng.integers(-3, 6, len(s)).astype(np.int32)
    ctx = jg.Context((0,) * shards)
    seed = int(t[0])
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    got = g.shortest_distance(vid[seed], 5)
    want = o.shortest_distance(n, s, t, seed, 5, w)
    np.testing.assert_array_equal(got, want)
    assert ((got < 0) & (got != jg.DIST_ABSENT)).any()  # real negative distances exist
    g.close()
    # an unweighted edge into the seed's in-neighbourhood is crossed at superstep 1
    crossed = w.copy()
    crossed[np.flatnonzero(t == seed)[0]] = jg.WEIGHT_ABSENT
    with pytest.raises(ValueError):
        o.shortest_distance(n, s, t, seed, 5, crossed)
    g = ctx.build(vid, vid[s], vid[t], weight=crossed, flags=jg.ADJ_IN | jg.ADJ_OUT)
    with pytest.raises(jg.JanusGpuError) as e:
        g.shortest_distance(vid[seed], 5)
    assert "weight property" in str(e.value)
    g.close()
    # an unweighted edge out of a vertex nothing reaches is never crossed
    reach = o.shortest_distance(n, s, t, seed, 5, w)
    far = np.flatnonzero(reach[t] == jg.DIST_ABSENT)
    if len(far):
        harmless = w.copy()
        harmless[far[0]] = jg.WEIGHT_ABSENT
        g = ctx.build(vid, vid[s], vid[t], weight=harmless, flags=jg.ADJ_IN | jg.ADJ_OUT)
        np.testing.assert_array_equal(g.shortest_distance(vid[seed], 5), o.shortest_distance(n, s, t, seed, 5, harmless))
        g.close()
    ctx.close()


@pytest.mark.parametrize("uf", [1, 0])
def test_connected_components_union_find_and_propagation(ctx, oracle_lib, uf):
    """One shard: union-find labels + BFS superstep count (cc_uf=1), or the propagation (cc_uf=0), on
    a graph with components of every kind, a path at the cap (150 vertices, minimum at one end: Fulgora
    stops at 99 supersteps unconverged, and the union-find path hands it to the propagation) and
    without it."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    rng = np.random.default_rng(11)
    cases = []
    n = 400
    s, d = rng.integers(0, n, 300), rng.integers(0, n, 300)
    s[:5] = d[:5] = 7  # self-loops
    cases.append((n, s, d))
    n = 150
    cases.append((n, np.arange(n - 1), np.arange(1, n)))  # a path past the cap
    cases.append((60, np.arange(59), np.arange(1, 60)))     # a path below it
    try:
        _lib.tune_set("cc_uf", uf)
        for n, s, d in cases:
            vid = np.arange(10, 10 + n, dtype=np.int64)
            g = ctx.build(vid, vid[s], vid[d], flags=jg.ADJ_BOTH)
            comp, it = g.connected_components()
            want, want_it = oracle_lib.connected_components(n, s, d, vid)
            assert it == want_it
            np.testing.assert_array_equal(comp, want)
            g.close()
    finally:
        _lib.tune_set("cc_uf", 1)


@pytest.mark.parametrize("shards", [1, 2])
def test_multi_source_bfs_past_255_levels(oracle_lib, shards):
    """The bit-parallel BFS keeps depths in byte planes for levels 0..254 and widens them to int32 when a
    traversal reaches level 255: a 700-vertex path (plus a few chords and an isolated vertex) from 5
    sources, unbounded and bounded at 300, on 1 and 2 shards, every depth row against the oracle."""
    import janusgraph_amd as jg
    n = 702
    s = list(range(699)) + [10, 400, 650]
    t = list(range(1, 700)) + [12, 405, 651]
    s, t = np.array(s, np.int32), np.array(t, np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    c = jg.Context((0,) * shards)
    g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_BOTH)
    srcs = [0, 3, 350, 699, 701]
    for max_depth in (-1, 300):
        got = g.bfs(vid[srcs], jg.DIR_BOTH, max_depth=max_depth)
        for k, sv in enumerate(srcs):
            np.testing.assert_array_equal(got[k], oracle_lib.bfs(n, s, t, sv, oracle_lib.DIR_BOTH, max_depth),
                                          err_msg=f"shards {shards} max_depth {max_depth} source {sv}")
        assert got[0].max() > 255
    g.close()
    c.close()


@pytest.mark.parametrize("shards,exit_mode", [(1, 1), (1, 2), (1, 0), (3, 1), (3, 2)])
def test_multi_source_bfs_hubs_and_tails(oracle_lib, shards, exit_mode):
    """The 64-source BFS's early-exit rows (msbfs_exit; the split's hub bands scanned row by row) on a
    graph made for it: four hubs of 300-900 leaves joined in a ring, leaves cross-linked to each other's
    hubs, a 150-vertex tail hanging off one leaf, a small separate component and an isolated vertex.  Hub
    rows then need every live source at once while some sources sit at the end of the tail, so some
    levels exit and others must scan whole rows.  All 64 depth rows against the oracle, unbounded and
    bounded, with the adaptive rule (1), the exit forced on every pull level (2) and off (0), on 1 and 3
    shards.  The traversal's level count is the deepest source's depth + 1 (the level that finds nothing
    new), capped by max_depth: an isolated source's level-0 word must not survive into a later frontier
    (ADVICE r04)."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    rng = np.random.default_rng(5)
    src, dst = [], []
    hubs = [0, 1, 2, 3]
    nxt = 4
    leaves = []
    for h, k in zip(hubs, (300, 500, 700, 900)):
        for _ in range(k):
            src.append(h); dst.append(nxt); leaves.append(nxt); nxt += 1
    for a, b in zip(hubs, hubs[1:] + hubs[:1]):
        src.append(a); dst.append(b)
    leaves = np.array(leaves)
    for _ in range(2000):  # leaves linked to other hubs and to each other
        a, b = rng.choice(leaves, 2)
        src.append(int(a)); dst.append(int(rng.choice(hubs)) if rng.random() < 0.5 else int(b))
    prev = int(leaves[7])
    for _ in range(150):  # the tail
        src.append(prev); dst.append(nxt); prev = nxt; nxt += 1
    tail_end = prev
    for a, b in ((nxt, nxt + 1), (nxt + 1, nxt + 2)):  # a small component
        src.append(a); dst.append(b)
    small = nxt
    n = nxt + 4  # + an isolated vertex
    s, t = np.array(src, np.int32), np.array(dst, np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    try:
        _lib.tune_set("msbfs_exit", exit_mode)
        c = jg.Context((0,) * shards)
        g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_BOTH)
        srcs = np.concatenate([[0, 3, tail_end, small, n - 1], rng.choice(leaves, 59, replace=False)])
        for max_depth in (-1, 3):
            got = g.bfs(vid[srcs], jg.DIR_BOTH, max_depth=max_depth)
            levels = c.stats()["levels"]
            deepest = 0
            for k, sv in enumerate(srcs):
                want = oracle_lib.bfs(n, s, t, int(sv), oracle_lib.DIR_BOTH, max_depth)
                np.testing.assert_array_equal(got[k], want,
                                              err_msg=f"shards {shards} exit {exit_mode} max_depth {max_depth} source {sv}")
                deepest = max(deepest, int(want.max()))
            assert levels == (deepest + 1 if max_depth < 0 else min(deepest + 1, max_depth)), (levels, deepest)
        g.close()
        c.close()
    finally:
        _lib.tune_set("msbfs_exit", 1)


def test_vertex_id_remap_arbitrary_ids(ctx, oracle_lib, rmat12):
    """The device id table (jg_build.hip remap_ids_device): arbitrary int64 ids (negative, huge, clustered
    in a few high-bit groups like JanusGraph's partitioned ids), ghost endpoints among them, a duplicate
    id and the reserved INT64_MIN rejected with JG_ERR_ARG."""
    import janusgraph_amd as jg
    o = oracle_lib
    n, _, s, t = rmat12
    rng = np.random.default_rng(17)
    vid = rng.choice(np.iinfo(np.int64).max, n, replace=False).astype(np.int64)
    vid[: n // 4] = -vid[: n // 4]                            # negative ids
    vid[n // 4: n // 2] = (np.arange(n // 4, dtype=np.int64) << 8) | (3 << 60)  # a dense high-bit cluster
    assert len(np.unique(vid)) == n
    assert 12345 not in set(vid.tolist())
    src = vid[s].copy()
    dst = vid[t].copy()
    dst[np.arange(len(dst)) % 97 == 0] = 12345                # edges to an id outside vid: ghosts, dropped
    keep = dst != 12345
    g = ctx.build(vid, src, dst, flags=jg.ADJ_BOTH)
    assert g.info()["ghost_edges"] == int((~keep).sum())
    sv = int(s[0])
    np.testing.assert_array_equal(g.bfs([vid[sv]], jg.DIR_BOTH)[0],
                                  o.bfs(n, s[keep], t[keep], sv, o.DIR_BOTH))
    g.close()
    dup = vid.copy()
    dup[7] = dup[3]
    with pytest.raises(jg.JanusGpuError) as e:
        ctx.build(dup, src, dst, flags=jg.ADJ_BOTH)
    assert e.value.code == -1 and "duplicate" in str(e.value)
    bad = vid.copy()
    bad[5] = np.iinfo(np.int64).min
    with pytest.raises(jg.JanusGpuError) as e:
        ctx.build(bad, src, dst, flags=jg.ADJ_BOTH)
    assert e.value.code == -1
