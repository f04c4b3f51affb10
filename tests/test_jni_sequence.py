"""GpuGraphComputer's JNI call sequences replayed through ctypes (the Java drop-in cannot run here:
no JDK). java/native/janusgpu_jni.c is a pass-through (tests/test_jni_shim.py), so each JanusGpu
native below is the C-ABI call the shim makes, with the buffers GpuSnapshot / GpuGraphComputer build:

  ctxCreate -> builderCreate -> builderSetQueryLimit (100000: Fulgora's slice cap) -> builderSetSchema ->
  builderAddRows (one per scan chunk of whole rows,
  entry weights for ShortestDistance) -> builderFinish -> builderDestroy -> graphInfo ->
  graphVertexIds (chunks) -> pageRank | shortestDistance | connectedComponents | bfs (64 sources per
  call, ShortestPathVertexProgram) -> graphDestroy -> ctxDestroy

Results are checked against the oracle's restatement of the scan (oracle.edgestore_snapshot) and
programs.
"""
import ctypes
from collections import deque

import numpy as np
import pytest

from test_edgestore import _dense, make_edgestore
from test_gpu_builder import row_chunks

pytestmark = pytest.mark.gpu


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _ok(status):
    from janusgraph_amd import _lib
    _lib.check(status)


class JavaRun:
    """GpuSnapshot.scan + GpuSnapshot.vertexIds as the Java code issues them."""

    def __init__(self, store, flags, entry_weight=None, nchunks=4, vid_chunk=97, in_entries=2, limit=100000):
        from janusgraph_amd import _lib
        L = _lib.load()
        self.L = L
        keys, roff, data, off, vpos, tids, tmult = store
        self.ctx = ctypes.c_void_p()
        devs = (ctypes.c_int * 1)(0)
        _ok(L.jg_ctx_create(devs, 1, ctypes.byref(self.ctx)))
        b = ctypes.c_void_p()
        _ok(L.jg_builder_create(self.ctx, ctypes.byref(b)))
        try:
            _ok(L.jg_builder_set_query_limit(b, limit, in_entries))  # GpuGraphComputer.queryLimit(), inEntries()
            _ok(L.jg_builder_set_schema(b, _p(tids), _p(tmult), len(tids), 5))
            bounds = np.linspace(0, len(keys), nchunks + 1).astype(int)
            for ch in row_chunks(store, bounds):
                ck, cro, cdata, coff, cvpos = (np.ascontiguousarray(x) for x in ch)
                cdata = np.frombuffer(bytes(cdata), np.uint8)
                e0 = int(roff[np.searchsorted(keys, ck[0])]) if len(ck) else 0
                cw = None if entry_weight is None else np.ascontiguousarray(entry_weight[e0:e0 + len(cvpos)], np.int32)
                _ok(L.jg_builder_add_rows(b, _p(ck.astype(np.uint64)), len(ck), _p(cro.astype(np.int64)), _p(cdata),
                                          len(cdata), _p(coff.astype(np.int64)), _p(cvpos.astype(np.int32)), _p(cw),
                                          len(cvpos)))
            self.g = ctypes.c_void_p()
            _ok(L.jg_builder_finish(b, flags, ctypes.byref(self.g)))
        finally:
            _ok(L.jg_builder_destroy(b))
        info = _lib.GraphInfo()
        _ok(L.jg_graph_info_get(self.g, ctypes.byref(info)))
        n = info.num_vertices
        self.vid = np.empty(n, np.int64)
        for o in range(0, n, vid_chunk):  # GpuSnapshot.vertexIds reads the ids in chunks
            cnt = min(vid_chunk, n - o)
            part = np.empty(cnt, np.int64)
            _ok(L.jg_graph_vertex_ids(self.g, o, cnt, _p(part)))
            self.vid[o:o + cnt] = part

    def close(self):
        _ok(self.L.jg_graph_destroy(self.g))
        _ok(self.L.jg_ctx_destroy(self.ctx))


@pytest.fixture(scope="module")
def store():
    return make_edgestore(n=700, m=6000, seed=11)


def oracle_graph(oracle_lib, store):
    keys, roff, data, off, vpos, tids, tmult = store[0]
    ov, os_, ot = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult)
    ds, dd = _dense(ov, os_, ot)
    return ov, ds, dd


def test_pagerank_sequence(oracle_lib, store):
    ov, ds, dd = oracle_graph(oracle_lib, store)
    r = JavaRun(store[0], flags=2)  # JanusGpu.ADJ_IN
    n = len(r.vid)
    assert np.array_equal(r.vid, ov)
    rank, count = np.empty(n), np.empty(n)
    _ok(r.L.jg_pagerank(r.g, 0.85, 1, 10, _p(rank), _p(count)))  # vertexCount at its default of 1
    want, ec = oracle_lib.pagerank(n, ds, dd, 0.85, 1, 10)
    assert np.max(np.abs(rank - want) / np.abs(want)) <= 1e-9
    np.testing.assert_array_equal(count, ec)
    r.close()


def test_shortest_distance_sequence_with_entry_weights(oracle_lib, store):
    """GpuSnapshot.WeightReader: every entry's weight read on the host (here: by relation id), sent
    with the rows; the library keeps the weights of the kept OUT edges."""
    from janusgraph_amd import _lib
    keys, roff, data, off, vpos, tids, tmult = store[0]
    t, d, o, rel = oracle_lib.decode_edges(data, off, vpos, tids, tmult)
    weight_of_rel = {int(x): int(x % 7) - 1 for x in np.unique(rel[rel >= 0])}  # -1 .. 5
    missing = [x for x in sorted(weight_of_rel)[::53]]
    for x in missing:  # some edges have no weight property at all
        weight_of_rel[x] = int(_lib.WEIGHT_ABSENT)
    ew = np.array([weight_of_rel.get(int(x), int(_lib.WEIGHT_ABSENT)) if dd == 0 else int(_lib.WEIGHT_ABSENT)
                   for x, dd in zip(rel, d)], np.int32)
    ov, os_, ot, ent = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, return_entries=True)
    r = JavaRun(store[0], flags=2 | 1, entry_weight=ew, in_entries=1)  # ShortestDistance: JanusGpu.DIR_OUT
    n = len(r.vid)
    index = {int(v): i for i, v in enumerate(ov)}
    live = np.array([int(a) in index and int(b) in index for a, b in zip(os_, ot)])
    ds = np.array([index[int(a)] for a in os_[live]], np.int32)
    dd_ = np.array([index[int(b)] for b in ot[live]], np.int32)
    w_live = ew[ent][live]
    for seed in (0, 5, 17):
        dist = np.empty(n, np.int64)
        try:
            want = oracle_lib.shortest_distance(n, ds, dd_, seed, 6, w_live)
        except ValueError:
            assert r.L.jg_shortest_distance(r.g, int(ov[seed]), 6, _p(dist)) == _lib.JG_ERR_ARG
            continue
        _ok(r.L.jg_shortest_distance(r.g, int(ov[seed]), 6, _p(dist)))
        np.testing.assert_array_equal(dist, want)
    r.close()


def test_connected_components_sequence(oracle_lib, store):
    ov, ds, dd = oracle_graph(oracle_lib, store)
    r = JavaRun(store[0], flags=4)  # JanusGpu.ADJ_BOTH
    n = len(r.vid)
    comp = np.empty(n, np.int64)
    it = ctypes.c_int32(0)
    _ok(r.L.jg_connected_components(r.g, _p(comp), ctypes.byref(it)))
    want, want_it = oracle_lib.connected_components(n, ds, dd, ov)
    np.testing.assert_array_equal(comp, want)
    assert it.value == want_it
    r.close()


def all_shortest_paths(adj, s, t):
    """Every shortest s..t path by plain BFS (the check, not the Java walk-back)."""
    dist = {s: 0}
    q = deque([s])
    while q:
        u = q.popleft()
        for w in adj[u]:
            if w not in dist:
                dist[w] = dist[u] + 1
                q.append(w)
    if t not in dist:
        return []
    out = []

    def back(v, suffix):
        if v == s:
            out.append(tuple(reversed(suffix + [v])))
            return
        for u in sorted(set(adj[v])):
            if dist.get(u) == dist[v] - 1:
                back(u, suffix + [v])
    back(t, [])
    return out


def test_shortest_path_sequence_batches_of_64(oracle_lib, store):
    """ShortestPaths.execute: 70 sources -> two jg_bfs calls (64 + 6), DIR_BOTH, maxDistance; paths
    rebuilt by walking back over neighbours one level closer."""
    ov, ds, dd = oracle_graph(oracle_lib, store)
    r = JavaRun(store[0], flags=4)
    n = len(r.vid)
    adj = [[] for _ in range(n)]
    for a, b in zip(ds.tolist(), dd.tolist()):
        adj[a].append(b)
        adj[b].append(a)
    sources = list(range(70))
    targets = set(range(0, n, 9))
    max_distance = 3
    got = set()
    for b0 in range(0, len(sources), 64):
        k = min(64, len(sources) - b0)
        src = np.array([ov[s] for s in sources[b0:b0 + k]], np.int64)
        depth = np.empty(k * n, np.int32)
        _ok(r.L.jg_bfs(r.g, _p(src), k, 3, max_distance, _p(depth)))
        depth = depth.reshape(k, n)
        for j in range(k):
            s = sources[b0 + j]
            for t in range(n):
                if depth[j, t] < 0 or t not in targets:
                    continue

                def walk(v, suffix):
                    suffix = suffix + [v]
                    if v == s:
                        got.add(tuple(reversed(suffix)))
                        return
                    for u in sorted(set(adj[v])):
                        if depth[j, u] == depth[j, v] - 1:
                            walk(u, suffix)
                walk(t, [])
    want = set()
    for s in sources:
        for t in targets:
            for p in all_shortest_paths(adj, s, t):
                if len(p) - 1 <= max_distance:
                    want.add(p)
    assert got == want and len(got) > 70
    r.close()
