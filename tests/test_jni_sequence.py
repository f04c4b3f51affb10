"""GpuGraphComputer's JNI call sequences replayed through ctypes (the Java drop-in cannot run here:
no JDK). java/native/janusgpu_jni.c is a pass-through (tests/test_jni_shim.py), so each JanusGpu
native below is the C-ABI call the shim makes, with the buffers GpuSnapshot / GpuGraphComputer build:

  ctxCreate -> builderCreate -> builderSetQueryLimit (100000: Fulgora's slice cap) -> builderSetSchema ->
  builderAddRows (one per scan chunk of whole rows,
  entry weights for ShortestDistance) -> builderFinish -> builderDestroy -> graphInfo ->
  graphVertexIds (chunks) -> pageRank | shortestDistance | connectedComponents | bfsRows (64 sources
  per call, one 4n-byte buffer per source, ShortestPathVertexProgram) + graphNeighbors (PathDag: the
  size call, then the fill call) -> graphDestroy -> ctxDestroy

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


class DirectMemory:
    """The direct (off-heap) bytes GpuGraphComputer.ShortestPaths holds at once: GpuGraphComputer.direct()
    buffers, released when the Java code drops them (computer.gpu.direct-memory bounds the peak)."""

    def __init__(self):
        self.live = self.peak = 0

    def take(self, nbytes):
        self.live += max(int(nbytes), 8)
        self.peak = max(self.peak, self.live)

    def drop(self, nbytes):
        self.live -= max(int(nbytes), 8)


def jni_kept_rows(L, g, src_vids, n, max_depth, row, mem=None):
    """ShortestPaths.execute's batch: JanusGpu.bfsKeep (the 64 rows stay on the device), then bfsKeptRow
    into ONE reused direct(4L * n) buffer per source; yields that buffer once per source."""
    src = np.ascontiguousarray(src_vids, np.int64)
    _ok(L.jg_bfs_keep(g, _p(src), len(src), 3, max_depth))  # JanusGpu.DIR_BOTH
    for j in range(len(src)):
        _ok(L.jg_bfs_kept_row(g, j, _p(row)))
        yield row


def jni_neighbors(L, g, budget=1 << 62, mem=None):
    """PathDag.neighbors: JanusGpu.graphNeighbors once for the offsets, once more for the neighbours; a batch
    whose buffers would pass the walk-back's budget (computer.gpu.direct-memory / 2) is split in halves."""
    def call(rows):
        r = np.ascontiguousarray(rows, np.int64)
        k = len(r)
        off = np.empty(k + 1, np.int64)
        if mem:
            mem.take(8 * k + 8 * (k + 1))
        _ok(L.jg_graph_neighbors(g, 3, _p(r), k, _p(off), None))
        if 8 * int(off[-1]) + 16 * (k + 1) > budget and k > 1:
            if mem:
                mem.drop(8 * k + 8 * (k + 1))
            mid = k // 2
            oa, na = call(r[:mid])
            ob, nb_ = call(r[mid:])
            return np.concatenate([oa, oa[-1] + ob[1:]]), np.concatenate([na, nb_])
        nbr = np.empty(max(int(off[-1]), 1), np.int64)
        if mem:
            mem.take(8 * int(off[-1]))
        _ok(L.jg_graph_neighbors(g, 3, _p(r), k, _p(off), _p(nbr)))
        if mem:
            mem.drop(8 * int(off[-1]) + 8 * k + 8 * (k + 1))
        return off, nbr[:int(off[-1])]
    return call


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
    """ShortestPaths.execute: 70 sources -> two jg_bfs_keep batches (64 + 6: the bit-parallel and the
    single-source paths), each row read back by jg_bfs_kept_row into one buffer, DIR_BOTH, maxDistance;
    paths rebuilt by PathDag (predecessors read through jg_graph_neighbors, batches split under a tiny
    budget) -> every shortest path."""
    from janusgraph_amd import _lib
    from janusgraph_amd.computer import PathDag
    ov, ds, dd = oracle_graph(oracle_lib, store)
    r = JavaRun(store[0], flags=4)
    n = len(r.vid)
    adj = [[] for _ in range(n)]
    for a, b in zip(ds.tolist(), dd.tolist()):
        adj[a].append(b)
        adj[b].append(a)
    sources = list(range(70))
    target = np.zeros(n, bool)
    target[::9] = True
    max_distance = 3
    dag = PathDag(jni_neighbors(r.L, r.g, budget=1 << 12), n)  # a tiny budget: the batch split runs
    got = set()
    row = np.empty(n, np.int32)
    for b0 in range(0, len(sources), 64):
        batch = sources[b0:b0 + 64]
        for s, depth in zip(batch, jni_kept_rows(r.L, r.g, ov[batch], n, max_distance, row)):
            paths, _ = dag.paths(depth, s, target)
            got |= {tuple(p) for p in paths}
    _ok(r.L.jg_bfs_kept_release(r.g))
    assert r.L.jg_bfs_kept_row(r.g, 0, _p(row)) == _lib.JG_ERR_ARG  # released
    want = set()
    for s in sources:
        for t in np.flatnonzero(target).tolist():
            for p in all_shortest_paths(adj, s, t):
                if len(p) - 1 <= max_distance:
                    want.add(p)
    assert got == want and len(got) > 70
    r.close()


def test_shortest_path_sequence_rmat24(oracle_lib):
    """ShortestPaths.execute at RMAT-24 (n = 2^24) from a snapshot built the GpuSnapshot way (vertex and edge
    ids in chunks under a direct buffer's 2 GiB): a 64-source batch kept on the device and read back one
    row at a time into one 4n-byte buffer, vertex ids read back in GpuSnapshot.vertexIds chunks of 2^24;
    three depth rows against oracle.bfs_csr, and PathDag's predecessor lists and path counts against the
    oracle's CSR."""
    from janusgraph_amd import _lib
    from janusgraph_amd.computer import PathDag
    from test_gpu_configs import host_edges, pick_sources
    o = oracle_lib
    scale = 24
    n = 1 << scale
    s, d = host_edges(o, scale)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8  # graph.set-vertex-id ids (IDManager.toVertexId)
    L = _lib.load()
    ctx = ctypes.c_void_p()
    _ok(L.jg_ctx_create((ctypes.c_int * 1)(0), 1, ctypes.byref(ctx)))
    b = ctypes.c_void_p()
    _ok(L.jg_builder_create(ctx, ctypes.byref(b)))
    _ok(L.jg_builder_add_vertices(b, _p(vid), n))
    step = 1 << 26  # 512 MB int64 chunks: each under a direct buffer's 2 GiB
    for e0 in range(0, len(s), step):
        cs = np.ascontiguousarray(vid[s[e0:e0 + step]])
        cd = np.ascontiguousarray(vid[d[e0:e0 + step]])
        _ok(L.jg_builder_add_edges(b, _p(cs), _p(cd), None, len(cs)))
    g = ctypes.c_void_p()
    _ok(L.jg_builder_finish(b, 4, ctypes.byref(g)))  # JanusGpu.ADJ_BOTH
    _ok(L.jg_builder_destroy(b))
    chunk = 1 << 24
    got_vid = np.empty(n, np.int64)
    for off in range(0, n, chunk):
        _ok(L.jg_graph_vertex_ids(g, off, min(chunk, n - off), _p(got_vid[off:])))
    np.testing.assert_array_equal(got_vid, vid)
    ptr, adj = o.csr_unordered(n, s, d, both=True)
    del s, d
    srcs = pick_sources(ptr, 64, scale)
    row = np.empty(n, np.int32)
    depth = None
    for k, got in enumerate(jni_kept_rows(L, g, vid[srcs], n, -1, row)):
        if k in (0, 31, 63):
            np.testing.assert_array_equal(got, o.bfs_csr(n, ptr, adj, int(srcs[k])))
        if k == 0:
            depth = got.copy()
    rng = np.random.default_rng(5)
    reached = np.flatnonzero(depth >= 1)
    target = np.zeros(n, bool)
    target[rng.choice(reached, 60, replace=False)] = True
    dag = PathDag(jni_neighbors(L, g), n)
    pred, targets, _ = dag.predecessors(depth, target)
    assert len(targets) == 60 and len(pred) >= 60
    for v, p in pred.items():
        nb = adj[ptr[v]:ptr[v + 1]]
        np.testing.assert_array_equal(np.sort(p), np.unique(nb[depth[nb] == depth[v] - 1]))
    # path counts of depth-2 targets: one path per distinct depth-1 neighbour
    near = np.flatnonzero(depth == 2)[:20]
    tmask = np.zeros(n, bool)
    tmask[near] = True
    paths, deepest = dag.paths(depth, int(srcs[0]), tmask)
    assert deepest == 2
    want = sum(len(np.unique(adj[ptr[t]:ptr[t + 1]][depth[adj[ptr[t]:ptr[t + 1]]] == 1])) for t in near.tolist())
    assert len(paths) == want and all(p[0] == srcs[0] and len(p) == 3 for p in paths)
    _ok(L.jg_graph_destroy(g))
    _ok(L.jg_ctx_destroy(ctx))


def test_shortest_path_buffer_plan_rmat26(oracle_lib):
    """ShortestPaths.execute's direct memory at configs[4]'s scale (RMAT-26, n = 2^26).
    The old plan held 64 x direct(4n) = 17.2 GB per batch (an OutOfMemoryError under the JVM's default
    direct-memory limit); now one 268 MB row is reused (the batch stays on the device, jg_bfs_keep) and the
    walk-back's neighbour batches split at computer.gpu.direct-memory / 2.  Replays the batch and one
    source's walk-back with the default 1 GiB budget: peak direct bytes <= 1 GiB (<= 2 GiB asked), three
    kept rows bit-exact against the oracle, predecessors against the oracle's CSR."""
    from janusgraph_amd import _lib
    from janusgraph_amd.computer import PathDag
    from test_gpu_configs import host_edges, pick_sources, seed_of
    o = oracle_lib
    scale = 26
    n = 1 << scale
    budget = 1 << 30  # computer.gpu.direct-memory default
    s, d = host_edges(o, scale)
    ptr, adj = o.csr_unordered(n, s, d, both=True)
    del s, d
    L = _lib.load()
    ctx = ctypes.c_void_p()
    _ok(L.jg_ctx_create((ctypes.c_int * 1)(0), 1, ctypes.byref(ctx)))
    g = ctypes.c_void_p()
    _ok(L.jg_graph_build_rmat(ctx, scale, 16, seed_of(scale), 4, ctypes.byref(g)))  # ADJ_BOTH; vid == index
    mem = DirectMemory()
    assert 4 * n <= budget // 2  # GpuGraphComputer's own precondition
    mem.take(4 * n)  # the reused row
    mem.take(8 * 64)  # the source batch
    row = np.empty(n, np.int32)
    srcs = pick_sources(ptr, 64, scale)
    dag = PathDag(jni_neighbors(L, g, budget // 2, mem), n)
    for k, got in enumerate(jni_kept_rows(L, g, srcs, n, -1, row)):
        if k in (0, 17, 63):
            np.testing.assert_array_equal(got, o.bfs_csr(n, ptr, adj, int(srcs[k])), err_msg=f"kept row {k}")
        if k == 0:  # one source's walk-back: every reached vertex of depth 3 a target (hubs included)
            tmask = np.zeros(n, bool)
            far = np.flatnonzero(got == 3)
            tmask[far[:: max(1, len(far) // 3000)]] = True
            pred, targets, deepest = dag.predecessors(got, tmask)
            assert deepest == 3 and len(targets) > 1000
            for v in list(pred)[:500]:
                nb = adj[ptr[v]:ptr[v + 1]]
                np.testing.assert_array_equal(np.sort(pred[v]), np.unique(nb[got[nb] == got[v] - 1]))
    assert mem.peak <= budget <= 2 << 30, f"peak direct memory {mem.peak} bytes"
    _ok(L.jg_graph_destroy(g))
    _ok(L.jg_ctx_destroy(ctx))


def test_ctx_destroy_before_graph_is_refused(oracle_lib):
    """VERDICT r05 item 3 (the r05f segfault): jg_ctx_destroy while a graph or builder of the context is
    alive returns JG_ERR_STATE and leaves the context usable; the graph still runs, then everything tears
    down in the right order.  (Before: the context destroyed its streams and a later jg_graph_destroy
    synchronised a destroyed stream.)  Error style: FulgoraGraphComputer.java:241-243."""
    from janusgraph_amd import _lib
    o = oracle_lib
    L = _lib.load()
    ctx = ctypes.c_void_p()
    _ok(L.jg_ctx_create((ctypes.c_int * 1)(0), 1, ctypes.byref(ctx)))
    g = ctypes.c_void_p()
    _ok(L.jg_graph_build_rmat(ctx, 10, 16, 7, 2, ctypes.byref(g)))  # ADJ_IN
    b = ctypes.c_void_p()
    _ok(L.jg_builder_create(ctx, ctypes.byref(b)))
    assert L.jg_ctx_destroy(ctx) == _lib.JG_ERR_STATE
    assert b"still alive" in L.jg_last_error()
    _ok(L.jg_builder_destroy(b))
    assert L.jg_ctx_destroy(ctx) == _lib.JG_ERR_STATE  # the graph is still alive
    n = 1 << 10
    rank = np.empty(n, np.float64)
    cnt = np.empty(n, np.float64)
    _ok(L.jg_pagerank(g, ctypes.c_double(0.85), n, 10, _p(rank), _p(cnt)))  # the context still works
    s, t = o.rmat_edges(10, 16, 7)
    ref, _ = o.pagerank(n, s.astype(np.int32), t.astype(np.int32), 0.85, n, 10)
    assert (np.abs(rank - ref) / np.abs(ref)).max() <= 1e-9
    _ok(L.jg_graph_destroy(g))
    _ok(L.jg_ctx_destroy(ctx))
