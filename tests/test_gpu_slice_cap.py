"""Fulgora-exact snapshots under the 100000-entry slice cap (jg_builder_set_query_limit), checked
against the oracle's restatement (oracle.edgestore_snapshot(query_limit=...), pinned on hand-built
rows in tests/test_slice_cap.py).

Fulgora reads an untyped OUT/IN edge scope from each row's first `limit` EDGE-slice entries
(olap/QueryContainer.java:42,121-146).  A receiver reads its own row, so under the cap:
  PageRank gathers over the IN entries within the cap of the receiver's row, divided by the sender's
  edgeCount = its OUT entries within the cap (PageRankVertexProgram.java:90-103);
  ShortestDistance relaxes along the receiver's OUT entries within the cap;
  combiners over IN / OUT read the receiver's IN / OUT entries within the cap;
  CC and ShortestPath scopes are BOTH (fitted, never capped).
Small limits (3..25) exercise the rule on the RMAT-like edgestore fixture; one hub crosses the real
limit of 100000.
"""
import numpy as np
import pytest

from test_edgestore import make_edgestore
from test_gpu_builder import row_chunks
from test_slice_cap import LABEL_A, LABEL_B, Rows

pytestmark = pytest.mark.gpu


def capped_reference(oracle_lib, store, limit, entry_weight=None):
    """The oracle's capped snapshot as dense lists: vid order, OUT list (with weights), IN list."""
    keys, roff, data, off, vpos, tids, tmult = store
    ov, s, d, ent, cap = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult,
                                                       return_entries=True, query_limit=limit)
    index = {int(v): i for i, v in enumerate(ov)}

    def dense(a, b, keep):
        ia = np.array([index.get(int(x), -1) for x in a], np.int64)
        ib = np.array([index.get(int(x), -1) for x in b], np.int64)
        ok = keep & (ia >= 0) & (ib >= 0)
        return ia[ok].astype(np.int32), ib[ok].astype(np.int32), ok

    os_, od, ok = dense(s, d, cap["out_keep"])
    ow = None if entry_weight is None else np.asarray(entry_weight, np.int32)[ent][ok]
    is_, id_, _ = dense(cap["in_src"], cap["in_dst"], np.ones(len(cap["in_src"]), bool))
    return ov, (os_, od, ow), (is_, id_), cap["truncated_rows"]


def gpu_graph(store, limit, flags, in_entries, nchunks=3, entry_weight=None):
    import janusgraph_amd as jg
    keys, roff, data, off, vpos, tids, tmult = store
    ctx = jg.Context((0,))
    b = ctx.builder()
    b.set_schema(tids, tmult, 5)
    b.set_query_limit(limit, in_entries)
    bounds = np.linspace(0, len(keys), nchunks + 1).astype(int)
    for ck, cro, cdata, coff, cvpos in row_chunks(store, bounds):
        cw = None
        if entry_weight is not None:
            e0 = int(roff[np.searchsorted(keys, ck[0])]) if len(ck) else 0
            cw = entry_weight[e0:e0 + len(cvpos)]
        b.add_rows(ck, cro, cdata, coff, cvpos, entry_weight=cw)
    g = b.finish(flags)
    b.close()
    return ctx, g


def pagerank_ref(oracle_lib, n, out_list, in_list, iterations=10):
    ptr, col = oracle_lib.build_in_csr(n, in_list[0], in_list[1])
    edge_count = np.bincount(out_list[0], minlength=n)[:n].astype(np.float64)
    return oracle_lib.pagerank_csr(n, ptr, col, edge_count, 0.85, 1, iterations), edge_count


@pytest.mark.parametrize("limit", [3, 8, 25])
def test_pagerank_under_the_cap(oracle_lib, limit):
    import janusgraph_amd as jg
    store, _, _ = make_edgestore(n=700, m=6000, seed=limit)
    ov, out_list, in_list, trunc = capped_reference(oracle_lib, store, limit)
    ctx, g = gpu_graph(store, limit, jg.ADJ_IN, jg.DIR_IN)
    assert np.array_equal(g.vertex_ids(), ov)
    assert g.info()["truncated_vertices"] == trunc > 0
    rank, ec = g.pagerank(0.85, 1, 10)
    want, want_ec = pagerank_ref(oracle_lib, len(ov), out_list, in_list)
    np.testing.assert_array_equal(ec, want_ec)
    np.testing.assert_allclose(rank, want, rtol=1e-9, atol=0)  # +inf where a sender's edgeCount is 0
    g.close()
    ctx.close()


def test_limit_above_every_row_equals_the_untruncated_graph(oracle_lib):
    import janusgraph_amd as jg
    store, _, _ = make_edgestore(n=700, m=6000, seed=2)
    ctx, g = gpu_graph(store, 10 ** 6, jg.ADJ_IN, jg.DIR_IN)
    keys, roff, data, off, vpos, tids, tmult = store
    g0, _ = ctx.build_edgestore(keys, roff, data, off, vpos, tids, tmult, flags=jg.ADJ_IN)
    assert g.info()["truncated_vertices"] == 0
    r1, e1 = g.pagerank(0.85, 1, 10)
    r0, e0 = g0.pagerank(0.85, 1, 10)
    np.testing.assert_array_equal(e1, e0)
    np.testing.assert_allclose(r1, r0, rtol=1e-12, atol=0)
    g.close()
    g0.close()
    ctx.close()


@pytest.mark.parametrize("limit", [4, 12])
def test_combiners_read_their_own_capped_entries(oracle_lib, limit):
    import janusgraph_amd as jg
    store, _, _ = make_edgestore(n=500, m=4000, seed=40 + limit)
    ov, out_list, in_list, _ = capped_reference(oracle_lib, store, limit)
    n = len(ov)
    ctx, g = gpu_graph(store, limit, jg.ADJ_IN | jg.ADJ_OUT, jg.DIR_IN)
    init = np.arange(1, n + 1, dtype=np.int64)
    for direction, (a, b) in ((jg.DIR_OUT, out_list[:2]), (jg.DIR_IN, in_list)):
        for comb in (jg.COMBINE_SUM, jg.COMBINE_MIN):
            x, rec = g.combine_steps(direction, comb, 2, init)
            wx, wrec = oracle_lib.combine_steps(n, a, b, direction, comb, 2, init)
            np.testing.assert_array_equal(rec, wrec)
            np.testing.assert_array_equal(x[rec], wx[wrec])
    g.close()
    ctx.close()


@pytest.mark.parametrize("weighted", [False, True])
def test_shortest_distance_reads_capped_out_entries(oracle_lib, weighted):
    import janusgraph_amd as jg
    limit = 6
    store, _, _ = make_edgestore(n=600, m=5000, seed=77)
    keys, roff, data, off, vpos, tids, tmult = store
    ew = None
    if weighted:
        ew = np.random.default_rng(3).integers(-2, 9, len(vpos)).astype(np.int32)
    ov, out_list, _, _ = capped_reference(oracle_lib, store, limit, ew)
    ctx, g = gpu_graph(store, limit, jg.ADJ_IN | jg.ADJ_OUT, jg.DIR_OUT, entry_weight=ew)
    n = len(ov)
    for seed in (0, 9, 311):
        dist = g.shortest_distance(int(ov[seed]), 5)
        want = oracle_lib.shortest_distance(n, out_list[0], out_list[1], seed, 5, out_list[2])
        np.testing.assert_array_equal(dist, want)
    g.close()
    ctx.close()


def test_both_adjacency_is_never_capped(oracle_lib):
    """ConnectedComponent / ShortestPath scopes load BOTH: a fitted query, no hard limit."""
    import janusgraph_amd as jg
    store, _, _ = make_edgestore(n=600, m=5000, seed=5)
    keys, roff, data, off, vpos, tids, tmult = store
    ctx, g = gpu_graph(store, 3, jg.ADJ_BOTH, jg.DIR_IN)
    g0, _ = ctx.build_edgestore(keys, roff, data, off, vpos, tids, tmult, flags=jg.ADJ_BOTH)
    c1, i1 = g.connected_components()
    c0, i0 = g0.connected_components()
    np.testing.assert_array_equal(c1, c0)
    assert i1 == i0
    src = g.vertex_ids()[:5]
    np.testing.assert_array_equal(g.bfs(src, jg.DIR_BOTH), g0.bfs(src, jg.DIR_BOTH))
    g.close()
    g0.close()
    ctx.close()


def test_sender_with_no_out_entry_in_its_slice_sends_infinity(oracle_lib):
    """The hub's IN entries of label A fill its slice before its OUT entries of label B: its edgeCount
    is 0, Fulgora sends rank / 0 = +Infinity and the hub's out-neighbours, whose own slices hold the
    edge, read it."""
    import janusgraph_amd as jg
    g = Rows(8)
    for j in (1, 2, 3, 4):
        g.edge(j, 0, LABEL_A)
    for j in (5, 6, 7):
        g.edge(0, j, LABEL_B)
    store = g.store()
    ov, out_list, in_list, trunc = capped_reference(oracle_lib, store, 3)
    ctx, gg = gpu_graph(store, 3, jg.ADJ_IN, jg.DIR_IN, nchunks=1)
    rank, ec = gg.pagerank(0.85, 1, 4)
    want, want_ec = pagerank_ref(oracle_lib, len(ov), out_list, in_list, 4)
    hub = int(np.flatnonzero(ov == g.vid[0])[0])
    assert ec[hub] == 0 and want_ec[hub] == 0
    assert np.isinf(want).sum() >= 3
    np.testing.assert_array_equal(ec, want_ec)
    np.testing.assert_allclose(rank, want, rtol=1e-9, atol=0)
    gg.close()
    ctx.close()


def test_hub_past_fulgora_hard_limit(oracle_lib):
    """One hub with 70000 out-edges and 70000 in-edges (multi-edges to 3000 leaves): at the real
    limit of 100000 it reads every OUT entry and the first 30000 IN entries in column order."""
    import janusgraph_amd as jg
    from oracle import edgecodec as ec
    nleaf = 3000
    g = Rows(1 + nleaf)
    rng = np.random.default_rng(100)
    hub = g.vid[0]
    rel = 10 ** 6
    for k in range(70000):  # written directly: the Rows helper is per edge and slower
        a = g.vid[1 + int(rng.integers(0, nleaf))]
        g.rows[hub].append(ec.encode_edge(LABEL_A, ec.OUT, a, rel))
        g.rows[a].append(ec.encode_edge(LABEL_A, ec.IN, hub, rel))
        rel += 1
        b = g.vid[1 + int(rng.integers(0, nleaf))]
        g.rows[b].append(ec.encode_edge(LABEL_A, ec.OUT, hub, rel))
        g.rows[hub].append(ec.encode_edge(LABEL_A, ec.IN, b, rel))
        rel += 1
    for j in range(1, nleaf):  # a ring among the leaves
        g.edge(j, j + 1)
    store = g.store()
    limit = jg.FULGORA_HARD_QUERY_LIMIT
    ov, out_list, in_list, trunc = capped_reference(oracle_lib, store, limit)
    assert trunc == 1
    h = int(np.flatnonzero(ov == hub)[0])
    assert np.sum(in_list[1] == h) == limit - 70000
    ctx, gg = gpu_graph(store, limit, jg.ADJ_IN, jg.DIR_IN)
    assert gg.info()["truncated_vertices"] == 1
    rank, ecount = gg.pagerank(0.85, 1, 10)
    want, want_ec = pagerank_ref(oracle_lib, len(ov), out_list, in_list)
    np.testing.assert_array_equal(ecount, want_ec)
    np.testing.assert_allclose(rank, want, rtol=1e-9, atol=0)
    gg.close()
    ctx.close()


def test_query_limit_errors():
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    store, _, _ = make_edgestore(n=50, m=200, seed=1)
    keys, roff, data, off, vpos, tids, tmult = store
    ctx = jg.Context((0,))
    b = ctx.builder()
    with pytest.raises(jg.JanusGpuError):
        b.set_query_limit(-1)
    with pytest.raises(jg.JanusGpuError):
        b.set_query_limit(10, jg.DIR_BOTH)
    b.set_schema(tids, tmult, 5)
    b.add_rows(keys, roff, data, off, vpos)
    with pytest.raises(jg.JanusGpuError):  # after the first chunk
        b.set_query_limit(10)
    b.close()
    b = ctx.builder()
    b.add_vertices(np.array([256], np.int64))
    with pytest.raises(jg.JanusGpuError):  # ids have no slices
        b.set_query_limit(10)
    b.close()
    b = ctx.builder()  # weights are OUT-entry weights: the IN adjacency must come from OUT entries
    b.set_schema(tids, tmult, 5)
    b.set_query_limit(10, jg.DIR_IN)
    b.add_rows(keys, roff, data, off, vpos, entry_weight=np.ones(len(vpos), np.int32))
    with pytest.raises(jg.JanusGpuError) as e:
        b.finish(jg.ADJ_IN)
    assert e.value.code == _lib.JG_ERR_ARG
    b.close()
    ctx.close()
