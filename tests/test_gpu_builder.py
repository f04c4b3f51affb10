"""The chunked snapshot (jg_builder_*): the call sequence the Java GpuGraphComputer makes over JNI
(java/org/janusgraph/graphdb/olap/gpu/GpuGraphComputer.java, Snapshot), replayed through ctypes.

* rows mode: jg_builder_set_schema, jg_builder_add_rows per scan chunk (rows never split), finish ->
  the same graph as jg_graph_build_edgestore on the whole store and as the oracle's restatement
  (oracle.edgestore_snapshot), vertex order included; vertex-cut representatives land in different
  chunks.
* ids mode: jg_builder_add_vertices / add_edges chunks (the weighted-ShortestDistance snapshot) ->
  the same results as jg_graph_build on the concatenation; at RMAT-24 the 268 M edges (2 GiB per id
  array, past Java's 2 GiB direct-buffer limit) go through in chunks.
* state and argument errors are status codes.
"""
import numpy as np
import pytest

from test_edgestore import _dense, make_edgestore

pytestmark = pytest.mark.gpu


def row_chunks(store, bounds):
    """Split a store into chunks of whole rows [r0, r1), each with chunk-local offsets."""
    keys, roff, data, off, vpos, _, _ = store
    out = []
    for r0, r1 in zip(bounds[:-1], bounds[1:]):
        e0, e1 = int(roff[r0]), int(roff[r1])
        b0, b1 = int(off[e0]), int(off[e1])
        out.append((keys[r0:r1], roff[r0:r1 + 1] - e0, data[b0:b1], off[e0:e1 + 1] - b0, vpos[e0:e1]))
    return out


@pytest.mark.parametrize("nchunks", [1, 3, 7])
def test_builder_rows_equal_one_shot_and_oracle(oracle_lib, nchunks):
    import janusgraph_amd as jg
    store, (v, s, t), ghost_out = make_edgestore(n=600, m=5000, seed=nchunks)
    keys, roff, data, off, vpos, tids, tmult = store
    ov, os_, ot = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
    ctx = jg.Context((0,))
    b = ctx.builder()
    b.set_schema(tids, tmult, 5)
    bounds = np.linspace(0, len(keys), nchunks + 1).astype(int)
    for ch in row_chunks(store, bounds):
        b.add_rows(*ch)
    g = b.finish(jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    b.close()
    st = ctx.stats()
    assert st["kernel_launches"] == nchunks and st["kernel_ms_total"] > 0
    vid = g.vertex_ids()
    assert np.array_equal(vid, ov) and np.array_equal(vid, v)
    info = g.info()
    assert info["num_edges"] == len(s) and info["ghost_edges"] == ghost_out
    g1, vid1 = ctx.build_edgestore(keys, roff, data, off, vpos, tids, tmult)
    assert np.array_equal(vid1, vid)
    n = len(v)
    ds, dd = _dense(ov, os_, ot)
    rank, ecount = g.pagerank(0.85, n, 10)
    rank1, _ = g1.pagerank(0.85, n, 10)
    np.testing.assert_array_equal(rank, rank1)
    ref, ref_e = oracle_lib.pagerank(n, ds, dd, 0.85, n, 10)
    assert np.max(np.abs(rank - ref) / np.abs(ref)) <= 1e-9
    np.testing.assert_array_equal(ecount, ref_e)
    comp, _ = g.connected_components()
    np.testing.assert_array_equal(comp, oracle_lib.connected_components(n, ds, dd, vid)[0])
    g.close()
    g1.close()
    ctx.close()


def test_builder_ids_weighted_equal_one_shot(oracle_lib):
    import janusgraph_amd as jg
    o = oracle_lib
    n = 1 << 11
    s, t = o.rmat_edges(11, 16, 4)
    vid = (np.random.default_rng(2).permutation(n).astype(np.int64) + 1) << 8
    w = (np.arange(len(s)) % 5 + 1).astype(np.int32)
    ghost = np.int64(((1 << 35) + 1) << 8)  # an endpoint the scan never returned
    src = np.concatenate([vid[s], [vid[3]]])
    dst = np.concatenate([vid[t], [ghost]])
    ww = np.concatenate([w, [1]]).astype(np.int32)
    ctx = jg.Context((0,))
    b = ctx.builder()
    for part in np.array_split(np.arange(n), 3):
        b.add_vertices(vid[part])
    for part in np.array_split(np.arange(len(src)), 5):
        b.add_edges(src[part], dst[part], ww[part])
    g = b.finish(jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    assert np.array_equal(g.vertex_ids(), vid)
    assert g.info()["ghost_edges"] == 1
    seed = int(t[0])
    got = g.shortest_distance(vid[seed], 12)
    np.testing.assert_array_equal(got, o.shortest_distance(n, s, t, seed, 12, w))
    g1 = ctx.build(vid, src, dst, weight=ww)
    np.testing.assert_array_equal(got, g1.shortest_distance(vid[seed], 12))
    r, _ = g.pagerank(0.85, n, 8)
    r1, _ = g1.pagerank(0.85, n, 8)
    np.testing.assert_array_equal(r, r1)
    g.close()
    g1.close()
    ctx.close()


def test_builder_errors():
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    b = ctx.builder()
    b.add_vertices(np.array([256, 512], np.int64))
    b.add_edges(np.array([256]), np.array([512]), np.array([3], np.int32))
    with pytest.raises(jg.JanusGpuError):  # weights on some chunks only
        b.add_edges(np.array([512]), np.array([256]))
    with pytest.raises(jg.JanusGpuError):  # rows cannot be mixed into an ids snapshot
        b.add_rows(np.zeros(0, np.uint64), [0], b"", [0], [])
    with pytest.raises(jg.JanusGpuError):  # the schema must come first
        b.set_schema()
    g = b.finish(jg.ADJ_IN)
    with pytest.raises(jg.JanusGpuError):  # single use
        b.finish(jg.ADJ_IN)
    with pytest.raises(jg.JanusGpuError):
        b.add_vertices(np.array([1024], np.int64))
    b.close()
    with pytest.raises(jg.JanusGpuError):
        g.vertex_ids(1, 5)
    g.close()
    b2 = ctx.builder()
    b2.add_vertices(np.array([5, 5], np.int64))
    with pytest.raises(jg.JanusGpuError) as e:
        b2.finish(jg.ADJ_IN)
    assert "duplicate" in str(e.value)
    b2.close()
    ctx.close()


def test_builder_ids_past_2gib_rmat24(oracle_lib):
    """268 M edges (2 GiB per int64 id array) in 8 chunks == the device-generated RMAT-24 graph."""
    import janusgraph_amd as jg
    o = oracle_lib
    scale = 24
    n, m = 1 << scale, 16 << scale
    seed = 0x5EED + scale
    ctx = jg.Context((0,))
    b = ctx.builder()
    b.add_vertices(np.arange(n, dtype=np.int64))
    step = m // 8
    for e0 in range(0, m, step):
        s, d = o.rmat_edges(scale, 16, seed, e0, step)
        b.add_edges(s, d)
        del s, d
    g = b.finish(jg.ADJ_IN)
    b.close()
    assert g.info()["num_edges"] == m
    r, ec = g.pagerank(0.85, n, 6)
    g.close()
    g2 = ctx.build_rmat(scale, 16, seed, flags=jg.ADJ_IN)
    r2, ec2 = g2.pagerank(0.85, n, 6)
    g2.close()
    ctx.close()
    np.testing.assert_array_equal(ec, ec2)
    np.testing.assert_array_equal(r, r2)


def test_builder_wide_and_narrow_chunks(oracle_lib):
    """A chunk holding an entry of 256 bytes or more is staged with int64 offsets; the others with
    1-byte lengths and value positions.  Both decode to the oracle's snapshot."""
    import janusgraph_amd as jg
    from oracle import edgecodec as ec
    from test_slice_cap import Rows
    rng = np.random.default_rng(8)
    g = Rows(300)
    for _ in range(2500):
        g.edge(int(rng.integers(0, 300)), int(rng.integers(0, 300)))
    g.rows[g.vid[150]].append(ec.encode_property(ec.schema_id(5, "user_key"), 77, bytes(range(256)) * 2))
    store = g.store()
    keys, roff, data, off, vpos, tids, tmult = store
    assert np.max(np.diff(off)) >= 256
    ov, os_, ot = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
    ds, dd = _dense(ov, os_, ot)
    n = len(ov)
    ref, ref_e = oracle_lib.pagerank(n, ds, dd, 0.85, n, 10)
    ctx = jg.Context((0,))
    for nchunks in (1, 4):
        b = ctx.builder()
        b.set_schema(tids, tmult, 5)
        for ch in row_chunks(store, np.linspace(0, len(keys), nchunks + 1).astype(int)):
            b.add_rows(*ch)
        gg = b.finish(jg.ADJ_IN)
        b.close()
        st = ctx.stats()
        assert st["exchange_ms"] > 0 and st["kernel_ms_total"] >= st["exchange_ms"]
        assert np.array_equal(gg.vertex_ids(), ov)
        rank, ecount = gg.pagerank(0.85, n, 10)
        assert np.max(np.abs(rank - ref) / np.abs(ref)) <= 1e-9
        np.testing.assert_array_equal(ecount, ref_e)
        gg.close()
    ctx.close()
