"""ctypes front-end of the CPU restatement in oracle/jg_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by janusgraph_amd/.  Semantics and reference citations live in jg_oracle.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libjg_oracle.so")
_lib = None

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile libjg_oracle.so (gcc, OpenMP) if missing or stale."""
    src = os.path.join(_HERE, "jg_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.jo_rmat_edges.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p]
        L.jo_rmat_edges.restype = None
        L.jo_remap.argtypes = [_i64p, ctypes.c_int64, _i64p, _i64p, ctypes.c_int64, _i32p, _i32p, _i64p]
        L.jo_remap.restype = ctypes.c_int64
        L.jo_pagerank.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, ctypes.c_double,
                                  ctypes.c_int64, ctypes.c_int, _f64p, _f64p]
        L.jo_pagerank.restype = None
        L.jo_pagerank_superstep_csr.argtypes = [ctypes.c_int64, _i64p, _i32p, _f64p, _f64p, ctypes.c_double,
                                                ctypes.c_int64, _f64p, ctypes.c_void_p]
        L.jo_pagerank_superstep_csr.restype = None
        L.jo_build_in_csr.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, _i64p, _i32p]
        L.jo_build_in_csr.restype = None
        L.jo_shortest_distance.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int, _i64p]
        L.jo_shortest_distance.restype = ctypes.c_int
        L.jo_bfs.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, ctypes.c_int, ctypes.c_int64,
                             ctypes.c_int, _i32p]
        L.jo_bfs.restype = None
        L.jo_lex_rank.argtypes = [_i64p, ctypes.c_int64, _i32p]
        L.jo_lex_rank.restype = None
        L.jo_connected_components.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, _i64p, ctypes.c_int,
                                              _i64p]
        L.jo_connected_components.restype = ctypes.c_int
        L.jo_cc_csr.argtypes = [ctypes.c_int64, _i64p, _i32p, _i32p, ctypes.c_int, _i32p]
        L.jo_cc_csr.restype = ctypes.c_int
        L.jo_csr_unordered.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, ctypes.c_int, _i64p, _i32p]
        L.jo_csr_unordered.restype = None
        L.jo_bfs_csr.argtypes = [ctypes.c_int64, _i64p, _i32p, ctypes.c_int64, ctypes.c_int, _i32p]
        L.jo_bfs_csr.restype = None
        L.jo_lex_rank_iota.argtypes = [ctypes.c_int64, _i32p]
        L.jo_lex_rank_iota.restype = None
        L.jo_bfs_validate.argtypes = [ctypes.c_int64, ctypes.c_int64, _i32p, _i32p, _i32p, ctypes.c_int64,
                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.jo_bfs_validate.restype = ctypes.c_int
        L.jo_pagerank_csr.argtypes = [ctypes.c_int64, _i64p, _i32p, _f64p, ctypes.c_double, ctypes.c_int64,
                                      ctypes.c_int, _f64p]
        L.jo_pagerank_csr.restype = None
        L.jo_msbfs_csr.argtypes = [ctypes.c_int64, _i64p, _i32p, _i64p, ctypes.c_int, ctypes.c_int, _i32p]
        L.jo_msbfs_csr.restype = None
        L.jo_num_threads.argtypes = []
        L.jo_num_threads.restype = ctypes.c_int
        _u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
        _i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
        L.jo_decode_edges.argtypes = [_u8p, _i64p, _i32p, ctypes.c_int64, _i64p, _i8p, ctypes.c_int32, _i64p, _i8p,
                                      _i64p, _i64p]
        L.jo_decode_edges.restype = None
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def num_threads() -> int:
    return int(lib().jo_num_threads())


def rmat_edges(scale: int, edgefactor: int, seed: int, e0: int = 0, count: int | None = None):
    """Graph500 Kronecker edges e0..e0+count of RMAT(scale, seed); dense int64 ids."""
    m = edgefactor << scale
    if count is None:
        count = m - e0
    src = np.empty(count, np.int64)
    dst = np.empty(count, np.int64)
    lib().jo_rmat_edges(scale, seed, e0, count, src, dst)
    return src, dst


def remap(vid, src, dst):
    """Sparse ids -> dense (caller order), ghost edges dropped.  Returns (dsrc, ddst, keep_idx)."""
    vid, src, dst = _i64(vid), _i64(src), _i64(dst)
    m = len(src)
    dsrc = np.empty(max(m, 1), np.int32)
    ddst = np.empty(max(m, 1), np.int32)
    keep = np.empty(max(m, 1), np.int64)
    k = lib().jo_remap(vid, len(vid), src, dst, m, dsrc, ddst, keep)
    if k < 0:
        raise ValueError("duplicate vertex id")
    return dsrc[:k].copy(), ddst[:k].copy(), keep[:k].copy()


def pagerank(n, src, dst, damping=0.85, vertex_count=1, iterations=10):
    src, dst = _i32(src), _i32(dst)
    rank = np.empty(max(n, 1), np.float64)
    ec = np.empty(max(n, 1), np.float64)
    lib().jo_pagerank(n, len(src), src, dst, float(damping), int(vertex_count), int(iterations), rank, ec)
    return rank[:n], ec[:n]


def build_in_csr(n, src, dst):
    src, dst = _i32(src), _i32(dst)
    ptr = np.empty(n + 1, np.int64)
    col = np.empty(max(len(src), 1), np.int32)
    lib().jo_build_in_csr(n, len(src), src, dst, ptr, col)
    return ptr, col[: len(src)]


def pagerank_superstep_csr(n, in_ptr, in_src, contrib_in, edge_count, damping, vertex_count, rank_out=None):
    out = np.empty(n, np.float64)
    rp = None
    if rank_out is not None:
        rp = rank_out.ctypes.data_as(ctypes.c_void_p)
    lib().jo_pagerank_superstep_csr(n, _i64(in_ptr), _i32(in_src), np.ascontiguousarray(contrib_in, np.float64),
                                    np.ascontiguousarray(edge_count, np.float64), float(damping),
                                    int(vertex_count), out, rp)
    return out


DIST_ABSENT = np.iinfo(np.int64).min  # DISTANCE never written (jg_shortest_distance's marker too)
WEIGHT_ABSENT = np.iinfo(np.int32).min  # an edge without the weight property


def shortest_distance(n, src, dst, seed, max_depth, weight=None):
    """dist[v], DIST_ABSENT where the property stays absent; ValueError if a message crosses an edge
    whose weight is WEIGHT_ABSENT (Fulgora: edge.value(weightProperty) throws)."""
    src, dst = _i32(src), _i32(dst)
    dist = np.empty(max(n, 1), np.int64)
    w = None
    if weight is not None:
        weight = _i32(weight)
        w = weight.ctypes.data_as(ctypes.c_void_p)
    if lib().jo_shortest_distance(n, len(src), src, dst, w, int(seed), int(max_depth), dist) != 0:
        raise ValueError("a traversed edge has no weight property")
    return dist[:n]


def golden_distance(d):
    """The golden fixtures write an absent DISTANCE as -1 (their weights are positive)."""
    d = np.asarray(d, np.int64).copy()
    d[d == -1] = DIST_ABSENT
    return d


DIR_OUT, DIR_IN, DIR_BOTH = 1, 2, 3


def bfs(n, src, dst, source, direction=DIR_BOTH, max_depth=-1):
    src, dst = _i32(src), _i32(dst)
    depth = np.empty(max(n, 1), np.int32)
    lib().jo_bfs(n, len(src), src, dst, int(direction), int(source), int(max_depth), depth)
    return depth[:n]


def lex_rank(vid):
    vid = _i64(vid)
    r = np.empty(max(len(vid), 1), np.int32)
    lib().jo_lex_rank(vid, len(vid), r)
    return r[: len(vid)]


def connected_components(n, src, dst, vid, max_iterations=100):
    src, dst, vid = _i32(src), _i32(dst), _i64(vid)
    comp = np.empty(max(n, 1), np.int64)
    it = lib().jo_connected_components(n, len(src), src, dst, vid, int(max_iterations), comp)
    return comp[:n], int(it)


def decode_edges(data, off, vpos, type_ids=(), type_mult=()):
    """Decode edgestore entries (jo_decode_edges): data[off[i]:off[i+1]] is entry i, vpos[i] its value
    position.  Returns (type_id, dir, other, relation_id) arrays; dir 0 OUT, 1 IN, 2 property, 3 system."""
    data = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                                np.uint8)
    off, vpos = _i64(off), _i32(vpos)
    n = len(vpos)
    t, d, o, r = (np.empty(n, np.int64), np.empty(n, np.int8), np.empty(n, np.int64), np.empty(n, np.int64))
    tid = _i64(type_ids) if len(type_ids) else np.zeros(1, np.int64)
    tm = np.ascontiguousarray(type_mult, np.int8) if len(type_mult) else np.zeros(1, np.int8)
    lib().jo_decode_edges(data if len(data) else np.zeros(1, np.uint8), off, vpos, n, tid, tm, len(type_ids), t, d, o, r)
    return t, d, o, r


VERTEX_EXISTS_ID = (1 << 6) | 37  # BaseKey.VertexExists (types/system/BaseKey.java:40-41): SystemPropertyKey count 1


def key_to_vertex_id(keys, partition_bits=5):
    """IDManager.getKeyID (graphdb/idmanagement/IDManager.java:496-506) over uint64 row keys.
    Odd keys (schema / invisible rows) come back as -1, keys with no user vertex type as -2."""
    k = np.asarray(keys, np.uint64)
    poff = 64 - partition_bits
    part = (k >> np.uint64(poff)) if poff < 64 else np.zeros_like(k)
    count = (k >> np.uint64(3)) & np.uint64((1 << (poff - 3)) - 1)
    suffix = k & np.uint64(7)
    vid = ((((count << np.uint64(partition_bits)) + part) << np.uint64(3)) | suffix).astype(np.int64)
    vid[(k & np.uint64(1)) == 1] = -1
    vid[suffix == 6] = -2
    return vid


def canonical_vertex_id(vid, partition_bits=5):
    """IDManager.getCanonicalVertexId (graphdb/idmanagement/IDManager.java:525-547)."""
    count = vid >> (partition_bits + 3)
    h, off = 0, 0
    while off < 64:
        h ^= (count >> off) & ((1 << partition_bits) - 1)
        off += partition_bits
    return (((count << partition_bits) + h) << 3) | 2


def edgestore_snapshot(keys, row_off, data, off, vpos, type_ids=(), type_mult=(), partition_bits=5,
                       return_entries=False, query_limit=0):
    """The scan -> snapshot step restated row by row (the checker of jg_graph_build_edgestore):
    VertexJobConverter.getKeyFilter drops invisible rows (olap/VertexJobConverter.java:174-177);
    process/isGhostVertex keep a row only if its first entry is the VertexExists property (:122-151),
    except a non-canonical representative of a partitioned vertex, which is never a ghost; the rows'
    OUT entries of visible user edges are the edges (each edge is stored OUT on its source row and IN
    on its target row, graphdb/database/StandardJanusGraph.java:617-640).  Partitioned vertices
    (comp/VertexProgramScanJob.java:88-102, FulgoraVertexMemory.getCanonicalId) are one vertex: the
    canonical id, whose edges are the union over its representative rows.
    Returns (vid of kept vertices in row order, src ids, dst ids[, entry index of each edge]); raises
    ValueError where Java throws.

    query_limit > 0 restates Fulgora's slice cap (olap/QueryContainer.java:42,121-146: an untyped OUT/IN
    edge scope is not fitted, BasicVertexCentricQueryBuilder.java:451-456, so each processed row's EDGE
    slice, IDHandler.getBounds(EDGE) = the visible user edges of both directions in column order, is
    read with that limit, SinglePageEntryBuffer.getSlice :54-77) and appends a dict: out_keep[i] = edge
    i's OUT entry is among its row's first query_limit slice entries; in_src/in_dst = the edges whose
    IN entry is (other endpoint -> row vertex); truncated_rows = rows whose slice reached the limit
    (VertexJobConverter.java:139)."""
    data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    off, row_off = _i64(off), _i64(row_off)
    t, d, o, _ = decode_edges(data, off, vpos, type_ids, type_mult)
    vids = key_to_vertex_id(keys, partition_bits)

    def canon(v):
        if v > 0 and v & 7 == 2 and v >> (partition_bits + 3) > 0:
            if partition_bits == 0:
                raise ValueError("no partition bits")
            return canonical_vertex_id(v, partition_bits)
        return v

    keep_v, src, dst, ent = [], [], [], []
    out_keep, in_src, in_dst, truncated = [], [], [], 0
    for r, vid in enumerate(vids):
        vid = int(vid)
        e0, e1 = int(row_off[r]), int(row_off[r + 1])
        if vid == -1:
            continue
        if vid == -2:
            raise ValueError("row key with an unrecognized vertex id type")
        cv = canon(vid)
        if cv == vid:  # a normal vertex, or the canonical representative: the ghost rule
            if e0 == e1:
                continue
            if d[e0] < 0:
                raise ValueError("malformed entry")
            if not (d[e0] == 2 and t[e0] == VERTEX_EXISTS_ID):
                continue  # ghost vertex
            keep_v.append(cv)
        rank = 0  # slice entries of this row so far
        for e in range(e0, e1):
            if d[e] < 0:
                raise ValueError("malformed entry")
            visible = (int(data[off[e]]) >> 6) == 1  # relation-type header prefix >> 1: 1 = user, visible
            in_slice = visible and d[e] in (0, 1)
            within = query_limit <= 0 or rank < query_limit
            rank += in_slice
            if d[e] == 0 and visible:
                src.append(cv)
                dst.append(canon(int(o[e])))
                ent.append(e)
                out_keep.append(within)
            elif d[e] == 1 and visible and within:
                in_src.append(canon(int(o[e])))
                in_dst.append(cv)
        truncated += query_limit > 0 and rank >= query_limit
    out = (np.array(keep_v, np.int64), np.array(src, np.int64), np.array(dst, np.int64))
    if return_entries:
        out = out + (np.array(ent, np.int64),)
    if query_limit > 0:
        out = out + ({"out_keep": np.array(out_keep, bool), "in_src": np.array(in_src, np.int64),
                      "in_dst": np.array(in_dst, np.int64), "truncated_rows": int(truncated)},)
    return out


COMBINE_SUM, COMBINE_MIN, COMBINE_MAX = 0, 1, 2


def combine_steps(n, src, dst, direction, combiner, steps, init=None, int32_wrap=True):
    """Combiner vertex programs restated with numpy (checker of jg_combine_steps): `steps` supersteps
    of x[v] = COMBINE over v's `direction` adjacency entries (v, w) of x[w]; DIR_OUT = v's out-edges
    (messages sent on Local.of(inE), OLAPTest.java:429), BOTH = out- and in-entries (a self-loop
    twice).  SUM of nothing is 0 (reduce(0, +)); MIN/MAX of nothing keeps the identity with
    received = False.  Returns (x, received)."""
    src, dst = np.asarray(src, np.int64), np.asarray(dst, np.int64)
    x = np.ones(n, np.int64) if init is None else np.asarray(init, np.int64).copy()
    if int32_wrap:
        x = x.astype(np.int32).astype(np.int64)
    rows, cols = [], []
    if direction in (DIR_OUT, DIR_BOTH):
        rows.append(src)
        cols.append(dst)
    if direction in (DIR_IN, DIR_BOTH):
        rows.append(dst)
        cols.append(src)
    r = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    c = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    received = np.bincount(r, minlength=n)[:n] > 0 if len(r) else np.zeros(n, bool)
    ident = {COMBINE_SUM: 0, COMBINE_MIN: np.iinfo(np.int64).max, COMBINE_MAX: np.iinfo(np.int64).min}[combiner]
    for _ in range(steps):
        y = np.full(n, ident, np.int64)
        if combiner == COMBINE_SUM:
            np.add.at(y, r, x[c])  # int64 wraps modulo 2^64; truncating to int32 gives the Java int sum
            if int32_wrap:
                y = y.astype(np.int32).astype(np.int64)
        elif combiner == COMBINE_MIN:
            np.minimum.at(y, r, x[c])
        else:
            np.maximum.at(y, r, x[c])
        x = y
    if steps == 0:
        received = np.zeros(n, bool)
    return x, received


# ---- full-size checkers (parallel CSR builds; tests/test_gpu_configs.py) ----

def csr_unordered(n, key, other, both=False):
    """CSR rows = key, entries = other (both: symmetrised, a self-loop twice); entry order inside a
    row unspecified.  Returns (ptr int64[n+1], adj int32)."""
    key, other = _i32(key), _i32(other)
    m = len(key)
    ptr = np.empty(n + 1, np.int64)
    adj = np.empty(max((2 if both else 1) * m, 1), np.int32)
    lib().jo_csr_unordered(n, m, key, other, 1 if both else 0, ptr, adj)
    return ptr, adj[: (2 if both else 1) * m]


def bfs_csr(n, ptr, adj, source, max_depth=-1):
    depth = np.empty(max(n, 1), np.int32)
    lib().jo_bfs_csr(n, _i64(ptr), _i32(adj), int(source), int(max_depth), depth)
    return depth[:n]


def msbfs_csr(n, ptr, adj, sources, max_depth=-1):
    """Bit-parallel hop depth from up to 64 sources (jo_msbfs_csr).  Returns int32 [nsrc, n]."""
    src = _i64(np.atleast_1d(sources))
    depth = np.empty(max(len(src) * n, 1), np.int32)
    lib().jo_msbfs_csr(n, _i64(ptr), _i32(adj), src, len(src), int(max_depth), depth)
    return depth[: len(src) * n].reshape(len(src), n)


def lex_rank_iota(n):
    """jo_lex_rank of vid = 0..n-1 (String order of the decimal ids), in O(n)."""
    r = np.empty(max(n, 1), np.int32)
    lib().jo_lex_rank_iota(n, r)
    return r[:n]


def cc_csr(n, ptr, adj, rank, max_iterations=100):
    """jo_connected_components' superstep loop on a BOTH CSR with given lex ranks.
    Returns (label rank per vertex, iterations)."""
    label = np.empty(max(n, 1), np.int32)
    it = lib().jo_cc_csr(n, _i64(ptr), _i32(adj), _i32(rank), int(max_iterations), label)
    return label[:n], int(it)


def bfs_validate(n, src, dst, depth, source, comp=None):
    """Graph500 validation (jo_bfs_validate).  Returns (error bits, edges with a reached endpoint)."""
    comp_p = None
    if comp is not None:
        comp = _i32(comp)
        comp_p = comp.ctypes.data_as(ctypes.c_void_p)
    edges = ctypes.c_int64(0)
    err = lib().jo_bfs_validate(n, len(src), _i32(src), _i32(dst), _i32(depth), int(source), comp_p,
                                ctypes.byref(edges))
    return int(err), int(edges.value)


def pagerank_csr(n, in_ptr, in_src, edge_count, damping=0.85, vertex_count=1, iterations=10):
    rank = np.empty(max(n, 1), np.float64)
    lib().jo_pagerank_csr(n, _i64(in_ptr), _i32(in_src), np.ascontiguousarray(edge_count, np.float64),
                          float(damping), int(vertex_count), int(iterations), rank)
    return rank[:n]
