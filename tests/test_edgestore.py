"""CSR snapshot straight from edgestore rows (jg_graph_build_edgestore).

A random graph is written the way JanusGraph lays it out in the edgestore (test-side writer:
oracle/edgecodec.py, EdgeSerializer.writeRelation; row keys: IDManager.getKey): one row per vertex
key, the VertexExists property first, user properties, every edge twice (OUT on the source row, IN
on the target row; a self-loop both on one row), plus the things the scan must skip: ghost rows
(edges but no VertexExists: VertexJobConverter.isGhostVertex), schema rows with odd keys
(getKeyFilter), system and invisible edges.  The ground truth is known by construction; the oracle's
restatement (oracle.edgestore_snapshot) is pinned against it on the CPU, and the GPU snapshot is
checked against both (vertex order, edge multiset through the graph info, and program results).
"""
import numpy as np
import pytest

from janusgraph_amd.idmanager import IDManager
from oracle import edgecodec as ec


def make_edgestore(n=300, m=2000, seed=0, ghosts=0.08, partition_bits=5, partitioned=4):
    """Returns (store arrays, (V, src, dst) by construction, OUT entries on live rows to ghosts)."""
    from oracle.oracle import canonical_vertex_id
    rng = np.random.default_rng(seed)
    idm = IDManager(partition_bits)
    vids = []
    seen = set()
    while len(vids) < n:  # normal and unmodifiable vertices over every partition
        count = int(rng.integers(1, 1 << 30))
        part = int(rng.integers(0, 1 << partition_bits))
        suffix = 0b100 if rng.integers(0, 8) == 0 else 0b000
        v = (((count << partition_bits) + part) << 3) | suffix
        if v not in seen:
            seen.add(v)
            vids.append(v)
    # vertex-cut vertices: the last `partitioned` indices get canonical ids and 3 representative rows
    reps = {}
    for i in range(n - partitioned, n):
        count = int(rng.integers(1, 1 << 30))
        canon = canonical_vertex_id((count << (partition_bits + 3)) | 2, partition_bits)
        others = [(((count << partition_bits) + p) << 3) | 2 for p in range(1 << partition_bits)]
        others = [x for x in others if x != canon]
        pick = [others[int(k)] for k in rng.choice(len(others), 2, replace=False)]
        vids[i] = canon
        reps[i] = [canon] + pick
    ghost = rng.random(n) < ghosts
    ghost[n - partitioned:] = False
    labels = [ec.schema_id(c, "user_edge") for c in (11, 12, 13, 14)]
    mults = [ec.MULTI, ec.SIMPLE, ec.ONE2MANY, ec.MANY2ONE]
    tids = np.array(labels[1:], np.int64)
    tmult = np.array(mults[1:], np.int8)
    name_key = ec.schema_id(5, "user_key")
    sys_edge = ec.schema_id(2, "system_edge")
    s = rng.integers(0, n, m)
    t = rng.integers(0, n, m)
    t[: m // 50] = s[: m // 50]  # self-loops
    s[m // 50: m // 25] = s[0]   # a hub with multi-edges
    t[m // 50: m // 25] = t[0]
    lab = rng.integers(0, len(labels), m)
    rows = {}  # row vertex id -> [(entry bytes, value position)]

    def row_of(i):  # the row an entry of vertex i goes to (any representative of a partitioned one)
        return reps[i][int(rng.integers(0, 3))] if i in reps else vids[i]

    rel = 1000
    for i in range(n):
        for rv in reps.get(i, [vids[i]]):
            rows.setdefault(rv, [])
        if not ghost[i]:  # VertexExists lives on the (canonical) vertex row
            rows[vids[i]].append(ec.encode_property(ec.schema_id(1, "system_key"), rel, b"\x01"))
            rel += 1
        rows[vids[i]].append(ec.encode_property(name_key, rel, b"name%d" % i))
        rel += 1
        if rng.integers(0, 10) == 0:
            rows[vids[i]].append(ec.encode_edge(sys_edge, ec.OUT, vids[int(rng.integers(0, n))], rel))
            rel += 1
        if rng.integers(0, 10) == 0:  # an invisible user edge
            rows[vids[i]].append(ec.encode_edge(labels[0], ec.OUT, vids[int(rng.integers(0, n))], rel,
                                                invisible=True))
            rel += 1
    for e in range(m):
        a, b, L = int(s[e]), int(t[e]), int(lab[e])
        ra, rb = row_of(a), row_of(b)
        rows[ra].append(ec.encode_edge(labels[L], ec.OUT, rb, rel, mults[L]))  # other = a representative id
        rows[rb].append(ec.encode_edge(labels[L], ec.IN, ra, rel, mults[L]))
        rel += 1
    row_ids = list(rows)
    keys = [idm.get_key(v) for v in row_ids]
    ents = [rows[v] for v in row_ids]
    # schema rows (odd keys) holding entries of their own, never decoded
    for c in (3, 7, 9):
        keys.append(ec.schema_id(c, "user_edge"))
        ents.append([(b"\xff\xff\xff", 1)])
        row_ids.append(None)
    order = sorted(range(len(keys)), key=lambda r: keys[r])  # the scan is key-ordered
    data, off, vpos, roff = bytearray(), [0], [], [0]
    for r in order:
        for b, vp in sorted(ents[r], key=lambda ev: ev[0][: ev[1]]):  # columns in byte order
            data += b
            off.append(len(data))
            vpos.append(vp)
        roff.append(len(vpos))
    index = {v: i for i, v in enumerate(vids)}
    live = [row_ids[r] for r in order if row_ids[r] in index and not ghost[index[row_ids[r]]]]
    keep = [(e_s, e_t) for e_s, e_t in zip(s, t) if not ghost[e_s] and not ghost[e_t]]
    truth = (np.array(live, np.int64), np.array([vids[a] for a, _ in keep], np.int64),
             np.array([vids[b] for _, b in keep], np.int64))
    ghost_out = sum(1 for e_s, e_t in zip(s, t) if not ghost[e_s] and ghost[e_t])
    store = (np.array([keys[r] for r in order], np.uint64), np.array(roff, np.int64), bytes(data),
             np.array(off, np.int64), np.array(vpos, np.int32), tids, tmult)
    return store, truth, ghost_out


def _edge_multiset(src, dst):
    return sorted(zip(src.tolist(), dst.tolist()))


def test_oracle_snapshot_matches_construction(oracle_lib):
    for seed in range(3):
        store, (v, s, t), ghost_out = make_edgestore(seed=seed)
        keys, roff, data, off, vpos, tids, tmult = store
        gv, gs, gt = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
        assert np.array_equal(gv, v)
        live = np.isin(gt, gv)  # targets that are ghosts drop at the dense remap (jg_graph_build's rule)
        assert int((~live).sum()) == ghost_out
        assert _edge_multiset(gs[live], gt[live]) == _edge_multiset(s, t)


def test_oracle_key_to_vertex_id_inverts_get_key(oracle_lib):
    idm = IDManager(5)
    vids = [idm.to_vertex_id(i) for i in (1, 2, 99, 1 << 40)] + [(((77 << 5) + 31) << 3) | 4]
    keys = np.array([idm.get_key(v) for v in vids], np.uint64)
    assert oracle_lib.key_to_vertex_id(keys).tolist() == vids
    assert oracle_lib.key_to_vertex_id(np.array([ec.schema_id(3, "user_edge"), 6], np.uint64)).tolist() == [-1, -2]


def _dense(vid, src, dst):
    index = {int(x): i for i, x in enumerate(vid)}
    ds = np.array([index.get(int(a), -1) for a in src], np.int64)
    dd = np.array([index.get(int(b), -1) for b in dst], np.int64)
    ok = (ds >= 0) & (dd >= 0)
    return ds[ok].astype(np.int32), dd[ok].astype(np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_edgestore_snapshot_matches_oracle(seed, oracle_lib):
    import janusgraph_amd as jg
    store, (v, s, t), ghost_out = make_edgestore(n=500, m=4000, seed=seed)
    keys, roff, data, off, vpos, tids, tmult = store
    ov, os_, ot = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
    ctx = jg.Context((0,))
    g, vid = ctx.build_edgestore(keys, roff, data, off, vpos, tids, tmult)
    assert np.array_equal(vid, ov) and np.array_equal(vid, v)
    info = g.info()
    assert info["num_vertices"] == len(v)
    assert info["num_edges"] == len(s)
    assert info["ghost_edges"] == ghost_out  # OUT entries on live rows whose target is a ghost
    n = len(v)
    ds, dd = _dense(ov, os_, ot)
    rank, ecount = g.pagerank(0.85, n, 10)
    ref, ref_e = oracle_lib.pagerank(n, ds, dd, 0.85, n, 10)
    assert np.max(np.abs(rank - ref) / np.abs(ref)) <= 1e-9
    np.testing.assert_array_equal(ecount, ref_e)
    src = int(ds[0])
    depth = g.bfs([vid[src]], jg.DIR_BOTH)[0]
    np.testing.assert_array_equal(depth, oracle_lib.bfs(n, ds, dd, src, oracle_lib.DIR_BOTH))
    comp, _ = g.connected_components()
    cref, _ = oracle_lib.connected_components(n, ds, dd, vid)
    np.testing.assert_array_equal(comp, cref)
    g.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_edgestore_edge_cases():
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    # no rows at all
    g, vid = ctx.build_edgestore(np.zeros(0, np.uint64), [0], b"", [0], [])
    assert len(vid) == 0 and g.info()["num_edges"] == 0
    g.close()
    # a malformed entry on a live row is refused
    idm = IDManager(5)
    exists, vp = ec.encode_property(ec.schema_id(1, "system_key"), 1, b"\x01")
    lab = ec.schema_id(9, "user_edge")
    bad = ec.write_relation_type(lab, True, ec.OUT) + b"\x01\x02"
    v1 = idm.to_vertex_id(1)
    data = exists + bad
    with pytest.raises(jg.JanusGpuError):
        ctx.build_edgestore([idm.get_key(v1)], [0, 2], data, [0, len(exists), len(data)], [vp, len(bad)])
    ctx.close()
