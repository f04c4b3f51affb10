"""Fulgora's per-row slice cap, restated by the oracle (oracle.edgestore_snapshot(query_limit=...)).

Fulgora loads an untyped OUT or IN edge scope (PageRank's outE/inE, ShortestDistance's inE) as the
row's EDGE slice with the hard limit of 100000 entries (olap/QueryContainer.java:42,121-146; the query
is not fitted, query/vertex/BasicVertexCentricQueryBuilder.java:451-456).  The slice holds the visible
user edges of both directions in column order (idhandling/IDHandler.java:172-193), and the in-memory
store stops returning entries at the limit (inmemory/SinglePageEntryBuffer.java:54-77).  These tests
pin the restatement on hand-built rows whose column order is known by construction; the GPU builds
are checked against it in tests/test_gpu_slice_cap.py.
"""
import numpy as np

from janusgraph_amd.idmanager import IDManager
from oracle import edgecodec as ec

LABEL_A = ec.schema_id(11, "user_edge")
LABEL_B = ec.schema_id(12, "user_edge")
VERTEX_EXISTS = ec.schema_id(1, "system_key")


def store_from_rows(rows, partition_bits=5, type_ids=(), type_mult=()):
    """rows: {vertex id: [(entry bytes, value position)]} -> the scan's arrays, rows in key order,
    entries in column order (the edgestore's sort)."""
    idm = IDManager(partition_bits)
    order = sorted(rows, key=idm.get_key)
    data, off, vpos, roff = bytearray(), [0], [], [0]
    for v in order:
        for b, vp in sorted(rows[v], key=lambda ev: ev[0][: ev[1]]):
            data += b
            off.append(len(data))
            vpos.append(vp)
        roff.append(len(vpos))
    return (np.array([idm.get_key(v) for v in order], np.uint64), np.array(roff, np.int64), bytes(data),
            np.array(off, np.int64), np.array(vpos, np.int32), np.array(type_ids, np.int64),
            np.array(type_mult, np.int8))


class Rows:
    """A tiny graph written as JanusGraph lays it out: VertexExists first, every edge OUT on its
    source row and IN on its target row."""

    def __init__(self, nvert, partition_bits=5):
        self.idm = IDManager(partition_bits)
        self.vid = [self.idm.to_vertex_id(i + 1) for i in range(nvert)]
        self.rows = {v: [ec.encode_property(VERTEX_EXISTS, 10 + i, b"\x01")] for i, v in enumerate(self.vid)}
        self.rel = 1000

    def edge(self, a, b, label=LABEL_A):
        va, vb = self.vid[a], self.vid[b]
        self.rows[va].append(ec.encode_edge(label, ec.OUT, vb, self.rel))
        self.rows[vb].append(ec.encode_edge(label, ec.IN, va, self.rel))
        self.rel += 1

    def store(self):
        return store_from_rows(self.rows)


def star(k_out=5, k_in=5):
    """Hub 0 with out-edges to 1..k_out and in-edges from k_out+1..k_out+k_in."""
    g = Rows(1 + k_out + k_in)
    for j in range(1, k_out + 1):
        g.edge(0, j)
    for j in range(k_out + 1, k_out + k_in + 1):
        g.edge(j, 0)
    return g


def test_star_keeps_the_first_entries_in_column_order(oracle_lib):
    """The hub's slice is its 5 OUT entries, then its 5 IN entries (same label: the direction bit is
    the lowest bit of the relation-type header), each group by the other vertex id (same varint
    length: byte order = id order).  A limit of 7 keeps every OUT entry and the IN entries of the
    two smallest sources."""
    g = star()
    keys, roff, data, off, vpos, tids, tmult = g.store()
    v, s, d, cap = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, query_limit=7)
    hub = g.vid[0]
    assert cap["truncated_rows"] == 1
    assert np.all(cap["out_keep"])  # every OUT entry: the hub's 5 are its first 5, the leaves have 1
    ins = sorted(zip(cap["in_src"].tolist(), cap["in_dst"].tolist()))
    want = sorted([(hub, g.vid[j]) for j in range(1, 6)] + [(g.vid[6], hub), (g.vid[7], hub)])
    assert ins == want


def test_in_entries_before_out_entries_of_a_later_label(oracle_lib):
    """Label A sorts before label B, so the hub's IN entries of A come before its OUT entries of B:
    with a limit of 3 the hub reads 3 IN entries and none of its OUT entries (edgeCount 0)."""
    g = Rows(8)
    for j in (1, 2, 3, 4):
        g.edge(j, 0, LABEL_A)
    for j in (5, 6, 7):
        g.edge(0, j, LABEL_B)
    keys, roff, data, off, vpos, tids, tmult = g.store()
    v, s, d, cap = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, query_limit=3)
    hub = g.vid[0]
    keep = cap["out_keep"]
    assert not np.any(keep[s == hub]) and np.all(keep[s != hub])
    assert sorted(cap["in_src"][cap["in_dst"] == hub].tolist()) == [g.vid[1], g.vid[2], g.vid[3]]
    assert cap["truncated_rows"] == 1


def test_limit_above_every_row_changes_nothing(oracle_lib):
    """No row reaches the limit: every OUT entry is kept and the IN entries are the same edges."""
    from test_edgestore import make_edgestore
    store, _, _ = make_edgestore(n=200, m=1500, seed=4)
    keys, roff, data, off, vpos, tids, tmult = store
    v, s, d = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
    v2, s2, d2, cap = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, query_limit=10 ** 6)
    assert np.array_equal(v, v2) and np.array_equal(s, s2) and np.array_equal(d, d2)
    assert np.all(cap["out_keep"]) and cap["truncated_rows"] == 0
    # between live vertices, the IN entries are the OUT entries' edges (a ghost row is never
    # processed, so its entries appear in neither list; edges to or from it drop at the dense remap)
    live = np.isin(d, v)
    ilive = np.isin(cap["in_src"], v)
    assert sorted(zip(cap["in_src"][ilive].tolist(), cap["in_dst"][ilive].tolist())) == \
        sorted(zip(s[live].tolist(), d[live].tolist()))


def test_limit_counts_both_directions_and_skips_other_relations(oracle_lib):
    """Properties, system edges and invisible edges are outside the EDGE slice and take no slot."""
    g = star(k_out=2, k_in=2)
    hub = g.vid[0]
    sys_edge = ec.schema_id(2, "system_edge")
    g.rows[hub].append(ec.encode_property(ec.schema_id(5, "user_key"), 7, b"name"))
    g.rows[hub].append(ec.encode_edge(sys_edge, ec.OUT, g.vid[1], 5000))
    g.rows[hub].append(ec.encode_edge(LABEL_A, ec.OUT, g.vid[2], 5001, invisible=True))
    keys, roff, data, off, vpos, tids, tmult = g.store()
    v, s, d, cap = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, query_limit=3)
    assert np.all(cap["out_keep"])
    assert sorted(cap["in_src"][cap["in_dst"] == hub].tolist()) == [g.vid[3]]
    assert cap["truncated_rows"] == 1
