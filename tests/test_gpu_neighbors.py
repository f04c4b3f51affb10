"""jg_graph_neighbors: a vertex's adjacency handed back in the caller's vertex order (the host copy of the
snapshot the ShortestPath walk-back reads, where Fulgora re-reads the preloaded BOTH slice:
VertexProgramScanJob.java:113-135).  Checked as multisets against the edge list on 1 shard and on 3
logical shards with the halo layout (compact column ids mapped back through the peers' send lists) and
the dense one, for BOTH (self-loops twice), OUT and IN, with sparse JanusGraph ids, ghost edges and
multi-edges."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def graph_edges(oracle_lib, scale=11, seed=3):
    s, t = oracle_lib.rmat_edges(scale, 8, seed)
    n = 1 << scale
    s = np.concatenate([s, [5, 5, 7]]).astype(np.int64)  # a self-loop and a repeated edge
    t = np.concatenate([t, [5, 9, 7]]).astype(np.int64)
    vid = (np.random.default_rng(seed).permutation(n).astype(np.int64) + 1) << 8
    return n, vid, s, t


def want_rows(n, s, t, direction):
    import janusgraph_amd as jg
    rows = [[] for _ in range(n)]
    for a, b in zip(s.tolist(), t.tolist()):
        if direction in (jg.DIR_OUT, jg.DIR_BOTH):
            rows[a].append(b)
        if direction in (jg.DIR_IN, jg.DIR_BOTH):
            rows[b].append(a)
    return rows


@pytest.mark.parametrize("shards,halo", [(1, 1), (3, 1), (3, 0)])
def test_neighbors_match_edge_list(oracle_lib, shards, halo):
    import janusgraph_amd as jg
    n, vid, s, t = graph_edges(oracle_lib)
    ghost = np.int64(((1 << 33) + 3) << 8)  # an endpoint the scan never returned: dropped
    src = np.concatenate([vid[s], [vid[1]]])
    dst = np.concatenate([vid[t], [ghost]])
    jg._lib.tune_set("halo", halo)
    try:
        ctx = jg.Context((0,) * shards)
        g = ctx.build(vid, src, dst, flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    finally:
        jg._lib.tune_set("halo", 1)
    rng = np.random.default_rng(shards)
    rows = np.concatenate([[5, 7, 1], rng.choice(n, 300, replace=False)]).astype(np.int64)
    for direction in (jg.DIR_BOTH, jg.DIR_OUT, jg.DIR_IN):
        want = want_rows(n, s, t, direction)
        off, nbr = g.neighbors(rows, direction)
        assert len(off) == len(rows) + 1 and off[-1] == len(nbr)
        for i, v in enumerate(rows.tolist()):
            np.testing.assert_array_equal(np.sort(nbr[off[i]:off[i + 1]]), np.sort(want[v]),
                                          err_msg=f"shards {shards} halo {halo} dir {direction} vertex {v}")
    off, _ = g.neighbors(np.array([5]), jg.DIR_BOTH)
    assert off[1] == len(want_rows(n, s, t, jg.DIR_BOTH)[5])  # the self-loop counts twice
    g.close()
    ctx.close()


def test_neighbors_errors(oracle_lib):
    import janusgraph_amd as jg
    n, vid, s, t = graph_edges(oracle_lib, scale=8)
    ctx = jg.Context((0,))
    g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_BOTH)
    with pytest.raises(jg.JanusGpuError) as e:
        g.neighbors(np.array([0]), jg.DIR_OUT)  # OUT adjacency not built
    assert e.value.code == jg._lib.JG_ERR_UNSUPPORTED
    with pytest.raises(jg.JanusGpuError) as e:
        g.neighbors(np.array([n]), jg.DIR_BOTH)
    assert e.value.code == jg._lib.JG_ERR_ARG
    off, nbr = g.neighbors(np.array([], np.int64), jg.DIR_BOTH)
    assert list(off) == [0] and len(nbr) == 0
    g.close()
    ctx.close()


def test_bfs_rows_equal_bfs(oracle_lib):
    """jg_bfs_rows writes the same depths as jg_bfs, row by row, and skips NULL rows."""
    import janusgraph_amd as jg
    n, vid, s, t = graph_edges(oracle_lib, scale=12, seed=9)
    for shards in (1, 2):
        ctx = jg.Context((0,) * shards)
        g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_BOTH)
        for srcs in ([vid[3]], list(vid[:70])):
            full = g.bfs(srcs, jg.DIR_BOTH, max_depth=4)
            want = [k % 3 != 1 for k in range(len(srcs))]
            rows = g.bfs_rows(srcs, jg.DIR_BOTH, 4, want=want)
            for k, r in enumerate(rows):
                if want[k]:
                    np.testing.assert_array_equal(r, full[k])
                else:
                    assert r is None
        g.close()
        ctx.close()


def test_bfs_keep_rows_equal_bfs(oracle_lib):
    """jg_bfs_keep + jg_bfs_kept_row (ShortestPaths' bounded direct memory): every kept row equals jg_bfs's,
    on the single-source, sharded single-source and bit-parallel paths; a later keep replaces the rows,
    release (and a bad index) fails the row read with JG_ERR_ARG."""
    import janusgraph_amd as jg
    n, vid, s, t = graph_edges(oracle_lib, scale=12, seed=9)
    for shards in (1, 3):
        ctx = jg.Context((0,) * shards)
        g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_BOTH)
        for srcs, depth in (([vid[3]], -1), (list(vid[:64]), 4), ([vid[7]], 2), (list(vid[5:10]), -1)):
            full = g.bfs(srcs, jg.DIR_BOTH, max_depth=depth)
            g.bfs_keep(srcs, jg.DIR_BOTH, depth)
            out = np.empty(n, np.int32)
            for k in range(len(srcs)):
                np.testing.assert_array_equal(g.bfs_kept_row(k, out), full[k], err_msg=f"{shards} shards, row {k}")
            with pytest.raises(jg.JanusGpuError) as e:
                g.bfs_kept_row(len(srcs))
            assert e.value.code == jg._lib.JG_ERR_ARG
        g.bfs_kept_release()
        with pytest.raises(jg.JanusGpuError):
            g.bfs_kept_row(0)
        with pytest.raises(jg.JanusGpuError):
            g.bfs_keep(list(vid[:65]), jg.DIR_BOTH)  # one bit-parallel batch at most
        g.close()
        ctx.trim()
        ctx.close()
