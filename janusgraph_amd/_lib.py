"""ctypes binding of libjanusgpu (include/janusgpu.h).

The HIP library is the only compute path: if libjanusgpu.so is missing or fails to load, every
entry point raises — there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes
import weakref
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libjanusgpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "janusgpu.h")

JG_OK = 0
JG_ERR_ARG = -1
JG_ERR_OOM = -2
JG_ERR_HIP = -3
JG_ERR_RCCL = -4
JG_ERR_UNSUPPORTED = -5
JG_ERR_STATE = -6

ADJ_OUT, ADJ_IN, ADJ_BOTH = 1, 2, 4
DIR_OUT, DIR_IN, DIR_BOTH = 1, 2, 3
COMBINE_SUM, COMBINE_MIN, COMBINE_MAX = 0, 1, 2
FULGORA_HARD_QUERY_LIMIT = 100000
DIST_ABSENT = np.iinfo(np.int64).min   # JG_DIST_ABSENT: DISTANCE never written
WEIGHT_ABSENT = np.iinfo(np.int32).min  # JG_WEIGHT_ABSENT: the edge has no weight property
UNIQUE_ID_BYTES = 128

# every function the header declares (checked by tests/test_abi.py against include/janusgpu.h)
EXPORTS = [
    "jg_abi_version", "jg_last_error", "jg_ctx_create", "jg_comm_unique_id", "jg_ctx_create_rank",
    "jg_ctx_create_rank_transport",
    "jg_ctx_destroy", "jg_ctx_last_stats", "jg_ctx_set_profiling", "jg_graph_build", "jg_graph_build_edgestore",
    "jg_graph_build_rmat",
    "jg_graph_info_get", "jg_graph_destroy", "jg_pagerank", "jg_pagerank_begin", "jg_pagerank_step",
    "jg_pagerank_end", "jg_shortest_distance", "jg_bfs", "jg_connected_components", "jg_combine_steps", "jg_decode_edges", "jg_graph_sync",
    "jg_tune_set", "jg_builder_create", "jg_builder_add_vertices", "jg_builder_add_edges", "jg_builder_set_schema",
    "jg_builder_add_rows", "jg_builder_finish", "jg_builder_destroy", "jg_graph_vertex_ids",
    "jg_builder_set_query_limit", "jg_bfs_rows", "jg_graph_neighbors", "jg_builder_set_weight_key",
    "jg_bfs_keep", "jg_bfs_kept_row", "jg_bfs_kept_release", "jg_ctx_trim",
]
# JG_PROP_* property value types (jg_builder_set_weight_key)
PROP_BYTE, PROP_SHORT, PROP_INT, PROP_LONG, PROP_CHAR, PROP_BOOL, PROP_DATE, PROP_FLOAT, PROP_DOUBLE, PROP_UUID, \
    PROP_STRING = range(1, 12)
ABI_VERSION = 3  # JG_ABI_VERSION of include/janusgpu.h this binding's structs follow


class GraphInfo(ctypes.Structure):
    _fields_ = [
        ("num_vertices", ctypes.c_int64), ("num_edges", ctypes.c_int64), ("ghost_edges", ctypes.c_int64),
        ("self_loops", ctypes.c_int64), ("truncated_vertices", ctypes.c_int64),
        ("max_in_degree", ctypes.c_int64), ("max_out_degree", ctypes.c_int64), ("device_bytes", ctypes.c_int64),
        ("num_shards", ctypes.c_int32), ("flags", ctypes.c_uint32), ("exchange_values", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Stats(ctypes.Structure):
    _fields_ = [
        ("supersteps", ctypes.c_int32), ("levels", ctypes.c_int32), ("build_ms", ctypes.c_double),
        ("compute_ms", ctypes.c_double), ("exchange_ms", ctypes.c_double), ("kernel_ms_total", ctypes.c_double),
        ("kernel_launches", ctypes.c_int64), ("algorithmic_bytes", ctypes.c_double),
        ("edges_traversed", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# jg_transport (include/janusgpu.h): a host transport for rank mode without RCCL (tests)
_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p),
                                ctypes.POINTER(ctypes.c_size_t))


class Transport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather", _ALLGATHER_FN), ("exchange", _EXCHANGE_FN)]


def _make_transport(obj):
    """Wrap an object with allgather(data: bytes) -> bytes (every rank's data, rank order) and
    exchange(sends: [(peer, bytes)], recvs: [(peer, nbytes)]) -> [bytes] into a jg_transport.
    Returns (struct, keep-alive references)."""
    import traceback

    def allgather(user, inp, out, nbytes):
        try:
            got = obj.allgather(ctypes.string_at(inp, nbytes) if nbytes else b"")
            if len(got) % max(nbytes, 1) != 0:
                return 2
            ctypes.memmove(out, got, len(got))
            return 0
        except Exception:  # an exception must not cross the C frames
            traceback.print_exc()
            return 1

    def exchange(user, ns, sp, sbuf, sbytes, nr, rp, rbuf, rbytes):
        try:
            sends = [(int(sp[i]), ctypes.string_at(sbuf[i], sbytes[i])) for i in range(ns)]
            recvs = [(int(rp[i]), int(rbytes[i])) for i in range(nr)]
            got = obj.exchange(sends, recvs)
            for i in range(nr):
                if len(got[i]) != rbytes[i]:
                    return 2
                ctypes.memmove(rbuf[i], got[i], rbytes[i])
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    fa, fe = _ALLGATHER_FN(allgather), _EXCHANGE_FN(exchange)
    return Transport(None, fa, fe), (fa, fe, obj)


class JanusGpuError(RuntimeError):
    """A non-zero status from libjanusgpu (the Java side wraps these in JanusGraphException)."""

    def __init__(self, code, message):
        super().__init__(f"libjanusgpu error {code}: {message}")
        self.code = code


_lib = None
_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32


def load():
    """Load libjanusgpu.so (raises if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libjanusgpu.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (hipcc, gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "jg_abi_version": ([], ctypes.c_int),
        "jg_last_error": ([], ctypes.c_char_p),
        "jg_ctx_create": ([ctypes.POINTER(ctypes.c_int), ctypes.c_int, _PP], ctypes.c_int),
        "jg_comm_unique_id": ([_P], ctypes.c_int),
        "jg_ctx_create_rank": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _PP], ctypes.c_int),
        "jg_ctx_create_rank_transport": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Transport), _PP],
                                         ctypes.c_int),
        "jg_ctx_destroy": ([_P], ctypes.c_int),
        "jg_ctx_last_stats": ([_P, ctypes.POINTER(Stats)], ctypes.c_int),
        "jg_ctx_set_profiling": ([_P, ctypes.c_int], ctypes.c_int),
        "jg_graph_build": ([_P, _P, _i64, _P, _P, _P, _i64, ctypes.c_uint32, _PP], ctypes.c_int),
        "jg_graph_build_edgestore": ([_P, _P, _i64, _P, _P, _i64, _P, _P, _i64, _P, _P, _i32, _i32, ctypes.c_uint32,
                                      _P, _P, _PP], ctypes.c_int),
        "jg_graph_build_rmat": ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, _PP],
                                ctypes.c_int),
        "jg_graph_info_get": ([_P, ctypes.POINTER(GraphInfo)], ctypes.c_int),
        "jg_graph_destroy": ([_P], ctypes.c_int),
        "jg_pagerank": ([_P, ctypes.c_double, _i64, _i32, _P, _P], ctypes.c_int),
        "jg_pagerank_begin": ([_P, ctypes.c_double, _i64], ctypes.c_int),
        "jg_pagerank_step": ([_P, _i32], ctypes.c_int),
        "jg_pagerank_end": ([_P, _P, _P], ctypes.c_int),
        "jg_shortest_distance": ([_P, _i64, _i32, _P], ctypes.c_int),
        "jg_bfs": ([_P, _P, _i32, _i32, _i32, _P], ctypes.c_int),
        "jg_connected_components": ([_P, _P, _P], ctypes.c_int),
        "jg_combine_steps": ([_P, _i32, _i32, _i32, _P, _i32, _P, _P], ctypes.c_int),
        "jg_decode_edges": ([_P, _P, _i64, _P, _P, _i64, _P, _P, _i32, _P, _P, _P, _P], ctypes.c_int),
        "jg_graph_sync": ([_P], ctypes.c_int),
        "jg_tune_set": ([ctypes.c_char_p, _i64], ctypes.c_int),
        "jg_builder_create": ([_P, _PP], ctypes.c_int),
        "jg_builder_add_vertices": ([_P, _P, _i64], ctypes.c_int),
        "jg_builder_add_edges": ([_P, _P, _P, _P, _i64], ctypes.c_int),
        "jg_builder_set_schema": ([_P, _P, _P, _i32, _i32], ctypes.c_int),
        "jg_builder_add_rows": ([_P, _P, _i64, _P, _P, _i64, _P, _P, _P, _i64], ctypes.c_int),
        "jg_builder_finish": ([_P, ctypes.c_uint32, _PP], ctypes.c_int),
        "jg_builder_destroy": ([_P], ctypes.c_int),
        "jg_graph_vertex_ids": ([_P, _i64, _i64, _P], ctypes.c_int),
        "jg_builder_set_query_limit": ([_P, _i64, _i32], ctypes.c_int),
        "jg_bfs_rows": ([_P, _P, _i32, _i32, _i32, _P], ctypes.c_int),
        "jg_graph_neighbors": ([_P, _i32, _P, _i64, _P, _P], ctypes.c_int),
        "jg_builder_set_weight_key": ([_P, _i64, _P, _P, _i32], ctypes.c_int),
        "jg_bfs_keep": ([_P, _P, _i32, _i32, _i32], ctypes.c_int),
        "jg_bfs_kept_row": ([_P, _i32, _P], ctypes.c_int),
        "jg_bfs_kept_release": ([_P], ctypes.c_int),
        "jg_ctx_trim": ([_P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.jg_abi_version() != ABI_VERSION:
        raise ImportError(f"libjanusgpu.so has ABI {L.jg_abi_version()}, this binding needs {ABI_VERSION}: rebuild it")
    _lib = L
    # JG_TUNE="key=value,key=value": performance knobs for profiling runs (results are unaffected)
    for item in filter(None, os.environ.get("JG_TUNE", "").split(",")):
        k, v = item.split("=")
        tune_set(k.strip(), int(v))
    return L


def check(status):
    if status != JG_OK:
        msg = load().jg_last_error()
        raise JanusGpuError(status, msg.decode() if msg else "")


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def tune_set(key: str, value: int):
    """Process-wide performance knob (results are unaffected; the list is jg_api.cpp jg_tune_set), e.g.
    msbfs_exit, bfs_narrow, and at graph build time pull_split, band<i>_deg, band<i>_bit, halo (sharded
    graphs: compact vectors + sparse halo exchange instead of the dense allgather)."""
    check(load().jg_tune_set(key.encode(), int(value)))


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    check(load().jg_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw


class Context:
    """jg_ctx: one process driving `devices` (sharded 1D when several), or rank `rank` of `nranks`
    (over RCCL with `unique_id`, or over a host `transport`: see _make_transport).  In rank mode every
    per-vertex output holds this rank's vertices only; the others keep NaN / the integer fill
    (INT32_MIN for depths, INT64_MAX for int64 outputs)."""

    def __init__(self, devices=(0,), rank=None, nranks=1, unique_id=None, transport=None):
        L = load()
        self._h = ctypes.c_void_p()
        self.nranks = int(nranks) if rank is not None else 1
        if transport is not None:
            if rank is None:
                raise ValueError("a transport needs rank and nranks")
            self._tr, self._tr_keep = _make_transport(transport)
            check(L.jg_ctx_create_rank_transport(int(devices[0]), int(nranks), int(rank), ctypes.byref(self._tr),
                                                 ctypes.byref(self._h)))
        elif rank is None:
            devs = (ctypes.c_int * len(devices))(*devices)
            check(L.jg_ctx_create(devs, len(devices), ctypes.byref(self._h)))
        else:
            uid = None
            if unique_id is not None:
                self._uid = ctypes.create_string_buffer(bytes(unique_id), UNIQUE_ID_BYTES)
                uid = ctypes.cast(self._uid, ctypes.c_void_p)
            check(L.jg_ctx_create_rank(int(devices[0]), int(nranks), int(rank), uid, ctypes.byref(self._h)))

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            # the graphs and builders first: they use the context's streams, and jg_ctx_destroy refuses
            # (JG_ERR_STATE) while any is alive
            for g in list(getattr(self, "_graphs", ())):
                g.close()
            for b in list(getattr(self, "_builders", ())):
                b.close()
            check(load().jg_ctx_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_profiling(self, on=True):
        check(load().jg_ctx_set_profiling(self._h, 1 if on else 0))

    def trim(self):
        """jg_ctx_trim: the device memory the library caches goes back to the devices."""
        check(load().jg_ctx_trim(self._h))

    def stats(self) -> dict:
        s = Stats()
        check(load().jg_ctx_last_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def decode_edges(self, data, entry_off, value_pos, type_ids=(), type_mult=()):
        """jg_decode_edges: decode edgestore entries (column + value bytes) on the GPU.
        Returns (type_id, dir, other_vertex_id, relation_id); dir 0 OUT, 1 IN, 2 property, 3 system
        relation, -1 malformed."""
        data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                    np.uint8)
        off = np.ascontiguousarray(entry_off, np.int64)
        vpos = np.ascontiguousarray(value_pos, np.int32)
        n = len(vpos)
        if len(off) != n + 1:
            raise ValueError("entry_off needs n + 1 offsets")
        tid = np.ascontiguousarray(type_ids, np.int64)
        tm = np.ascontiguousarray(type_mult, np.int8)
        if len(tid) != len(tm):
            raise ValueError("type_ids and type_mult differ in length")
        t, d, o, r = (np.empty(max(n, 1), np.int64), np.empty(max(n, 1), np.int8), np.empty(max(n, 1), np.int64),
                      np.empty(max(n, 1), np.int64))
        check(load().jg_decode_edges(self._h, _ptr(data), len(data), _ptr(off), _ptr(vpos), n, _ptr(tid), _ptr(tm),
                                     len(tid), _ptr(t), _ptr(d), _ptr(o), _ptr(r)))
        return t[:n], d[:n], o[:n], r[:n]

    def build(self, vid, src, dst, weight=None, flags=ADJ_IN | ADJ_OUT | ADJ_BOTH) -> "Graph":
        vid = np.ascontiguousarray(vid, np.int64)
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        if len(src) != len(dst):
            raise ValueError("src and dst differ in length")
        w = None if weight is None else np.ascontiguousarray(weight, np.int32)
        if w is not None and len(w) != len(src):
            raise ValueError("weight must have one entry per edge")
        h = ctypes.c_void_p()
        check(load().jg_graph_build(self._h, _ptr(vid), len(vid), _ptr(src), _ptr(dst), _ptr(w), len(src),
                                    flags, ctypes.byref(h)))
        return Graph(self, h, len(vid))

    def build_edgestore(self, row_keys, row_entry_off, data, entry_off, value_pos, type_ids=(), type_mult=(),
                        partition_bits=5, flags=ADJ_IN | ADJ_OUT | ADJ_BOTH):
        """jg_graph_build_edgestore: the CSR snapshot from raw edgestore rows, decoded on the GPU.
        Returns (graph, vid): vid = ids of the non-ghost vertex rows, the order outputs are indexed in."""
        keys = np.ascontiguousarray(row_keys, np.uint64)
        roff = np.ascontiguousarray(row_entry_off, np.int64)
        data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                    np.uint8)
        off = np.ascontiguousarray(entry_off, np.int64)
        vpos = np.ascontiguousarray(value_pos, np.int32)
        if len(roff) != len(keys) + 1 or len(off) != len(vpos) + 1:
            raise ValueError("row_entry_off needs nrows + 1 offsets, entry_off nentries + 1")
        tid = np.ascontiguousarray(type_ids, np.int64)
        tm = np.ascontiguousarray(type_mult, np.int8)
        if len(tid) != len(tm):
            raise ValueError("type_ids and type_mult differ in length")
        vid = np.empty(max(len(keys), 1), np.int64)
        nv = ctypes.c_int64(0)
        h = ctypes.c_void_p()
        check(load().jg_graph_build_edgestore(self._h, _ptr(keys), len(keys), _ptr(roff), _ptr(data), len(data),
                                              _ptr(off), _ptr(vpos), len(vpos), _ptr(tid), _ptr(tm), len(tid),
                                              partition_bits, flags, _ptr(vid), ctypes.byref(nv), ctypes.byref(h)))
        return Graph(self, h, nv.value), vid[:nv.value].copy()

    def builder(self) -> "Builder":
        """jg_builder: the snapshot fed in chunks (ids, or raw edgestore rows decoded as they arrive)."""
        return Builder(self)

    def build_rmat(self, scale, edgefactor=16, seed=1, flags=ADJ_IN) -> "Graph":
        h = ctypes.c_void_p()
        check(load().jg_graph_build_rmat(self._h, scale, edgefactor, seed, flags, ctypes.byref(h)))
        return Graph(self, h, 1 << scale)


class Builder:
    """jg_builder_*: add_vertices / add_edges chunks, or set_schema then add_rows chunks, then finish()."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        check(load().jg_builder_create(ctx.handle, ctypes.byref(self._h)))
        if not hasattr(ctx, "_builders"):
            ctx._builders = weakref.WeakSet()
        ctx._builders.add(self)

    def close(self):
        if self._h:
            check(load().jg_builder_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_vertices(self, vid):
        vid = np.ascontiguousarray(vid, np.int64)
        check(load().jg_builder_add_vertices(self._h, _ptr(vid), len(vid)))

    def add_edges(self, src, dst, weight=None):
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        if len(src) != len(dst):
            raise ValueError("src and dst differ in length")
        w = None if weight is None else np.ascontiguousarray(weight, np.int32)
        if w is not None and len(w) != len(src):
            raise ValueError("weight must have one entry per edge")
        check(load().jg_builder_add_edges(self._h, _ptr(src), _ptr(dst), _ptr(w), len(src)))

    def set_schema(self, type_ids=(), type_mult=(), partition_bits=5):
        tid = np.ascontiguousarray(type_ids, np.int64)
        tm = np.ascontiguousarray(type_mult, np.int8)
        if len(tid) != len(tm):
            raise ValueError("type_ids and type_mult differ in length")
        self._schema = (tid, tm)
        check(load().jg_builder_set_schema(self._h, _ptr(tid), _ptr(tm), len(tid), int(partition_bits)))

    def set_query_limit(self, limit=FULGORA_HARD_QUERY_LIMIT, in_entries=DIR_IN):
        """Fulgora's per-row slice cap (jg_builder_set_query_limit; QueryContainer.java:42,133): the
        directed adjacencies hold only what Fulgora's programs would read.  in_entries=DIR_IN: the IN
        adjacency from the rows' IN entries (PageRank, combiners over IN); DIR_OUT: the transpose of the
        capped OUT entries (ShortestDistance).  Call before the first add_rows."""
        check(load().jg_builder_set_query_limit(self._h, int(limit), int(in_entries)))

    def set_weight_key(self, weight_key, key_ids=(), key_types=()):
        """jg_builder_set_weight_key: the edges' Integer weight decoded on the GPU from their values.
        weight_key / key_ids are inline ids (the key id without its 4 padding bits); key_types JG_PROP_*."""
        ids = np.ascontiguousarray(key_ids, np.int64)
        types = np.ascontiguousarray(key_types, np.int8)
        if len(ids) != len(types):
            raise ValueError("key_ids and key_types differ in length")
        check(load().jg_builder_set_weight_key(self._h, int(weight_key), _ptr(ids), _ptr(types), len(ids)))

    def add_rows(self, row_keys, row_entry_off, data, entry_off, value_pos, entry_weight=None):
        keys = np.ascontiguousarray(row_keys, np.uint64)
        roff = np.ascontiguousarray(row_entry_off, np.int64)
        data = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data,
                                    np.uint8)
        off = np.ascontiguousarray(entry_off, np.int64)
        vpos = np.ascontiguousarray(value_pos, np.int32)
        if len(roff) != len(keys) + 1 or len(off) != len(vpos) + 1:
            raise ValueError("row_entry_off needs nrows + 1 offsets, entry_off nentries + 1")
        w = None if entry_weight is None else np.ascontiguousarray(entry_weight, np.int32)
        if w is not None and len(w) != len(vpos):
            raise ValueError("entry_weight needs one value per entry")
        check(load().jg_builder_add_rows(self._h, _ptr(keys), len(keys), _ptr(roff), _ptr(data), len(data), _ptr(off),
                                         _ptr(vpos), _ptr(w), len(vpos)))

    def finish(self, flags=ADJ_IN | ADJ_OUT | ADJ_BOTH) -> "Graph":
        h = ctypes.c_void_p()
        check(load().jg_builder_finish(self._h, flags, ctypes.byref(h)))
        g = Graph(self.ctx, h, 0)
        g.n = g.info()["num_vertices"]
        return g


class Graph:
    """jg_graph: a device-resident CSR snapshot; outputs are indexed like the vid[] it was built from."""

    def __init__(self, ctx: Context, handle, n):
        self.ctx, self._h, self.n = ctx, handle, n
        if not hasattr(ctx, "_graphs"):
            ctx._graphs = weakref.WeakSet()
        ctx._graphs.add(self)

    def _out(self, size, dtype):
        """An output array; in rank mode pre-filled so the other ranks' vertices are recognisable."""
        if getattr(self.ctx, "nranks", 1) <= 1:
            return np.empty(size, dtype)
        fill = np.nan if np.issubdtype(dtype, np.floating) else (
            np.iinfo(dtype).min if np.dtype(dtype) == np.int32 else np.iinfo(dtype).max)
        return np.full(size, fill, dtype)

    def close(self):
        if self._h:
            check(load().jg_graph_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        i = GraphInfo()
        check(load().jg_graph_info_get(self._h, ctypes.byref(i)))
        return i.as_dict()

    def sync(self):
        check(load().jg_graph_sync(self._h))

    def vertex_ids(self, offset=0, count=None):
        """jg_graph_vertex_ids: the vertex ids in output order."""
        count = self.n - offset if count is None else count
        out = np.empty(max(count, 1), np.int64)
        check(load().jg_graph_vertex_ids(self._h, int(offset), int(count), _ptr(out)))
        return out[:count]

    def pagerank(self, damping=0.85, vertex_count=1, iterations=10):
        rank = self._out(self.n, np.float64)
        ec = self._out(self.n, np.float64)
        check(load().jg_pagerank(self._h, float(damping), int(vertex_count), int(iterations), _ptr(rank), _ptr(ec)))
        return rank, ec

    def pagerank_begin(self, damping=0.85, vertex_count=1):
        check(load().jg_pagerank_begin(self._h, float(damping), int(vertex_count)))

    def pagerank_step(self, nsteps=1):
        check(load().jg_pagerank_step(self._h, int(nsteps)))

    def pagerank_end(self, want=True):
        rank = self._out(self.n, np.float64) if want else None
        ec = self._out(self.n, np.float64) if want else None
        check(load().jg_pagerank_end(self._h, _ptr(rank), _ptr(ec)))
        return rank, ec

    def shortest_distance(self, seed_vid, max_depth):
        dist = self._out(self.n, np.int64)
        check(load().jg_shortest_distance(self._h, int(seed_vid), int(max_depth), _ptr(dist)))
        return dist

    def bfs(self, sources, direction=DIR_BOTH, max_depth=-1, want=True):
        src = np.ascontiguousarray(np.atleast_1d(sources), np.int64)
        depth = self._out(len(src) * self.n, np.int32) if want else None
        check(load().jg_bfs(self._h, _ptr(src), len(src), int(direction), int(max_depth), _ptr(depth)))
        return None if depth is None else depth.reshape(len(src), self.n)

    def bfs_rows(self, sources, direction=DIR_BOTH, max_depth=-1, want=None):
        """jg_bfs_rows: one depth array per source (want[s] False: that row stays on the device)."""
        src = np.ascontiguousarray(np.atleast_1d(sources), np.int64)
        want = [True] * len(src) if want is None else list(want)
        rows = [self._out(self.n, np.int32) if w else None for w in want]
        ptrs = (ctypes.c_void_p * len(src))(*[None if r is None else r.ctypes.data for r in rows])
        check(load().jg_bfs_rows(self._h, _ptr(src), len(src), int(direction), int(max_depth), ptrs))
        return rows

    def bfs_keep(self, sources, direction=DIR_BOTH, max_depth=-1):
        """jg_bfs_keep: the traversal's depth rows (<= 64 sources) stay on the device for bfs_kept_row."""
        src = np.ascontiguousarray(np.atleast_1d(sources), np.int64)
        check(load().jg_bfs_keep(self._h, _ptr(src), len(src), int(direction), int(max_depth)))

    def bfs_kept_row(self, s, out=None):
        """jg_bfs_kept_row: row s of the last bfs_keep, into `out` (n int32) or a new array."""
        if out is not None and not (isinstance(out, np.ndarray) and out.dtype == np.int32 and out.ndim == 1
                                    and out.flags.c_contiguous and out.size >= self.n):
            raise ValueError("out must be a C-contiguous int32 array of at least n elements")  # 
        row = self._out(self.n, np.int32) if out is None else out
        check(load().jg_bfs_kept_row(self._h, int(s), _ptr(row)))
        return row

    def bfs_kept_release(self):
        check(load().jg_bfs_kept_release(self._h))

    def neighbors(self, rows, direction=DIR_BOTH):
        """jg_graph_neighbors: (off, nbr) CSR of the given output-order rows, in output-order indices."""
        r = np.ascontiguousarray(np.atleast_1d(rows), np.int64)
        off = np.empty(len(r) + 1, np.int64)
        check(load().jg_graph_neighbors(self._h, int(direction), _ptr(r), len(r), _ptr(off), None))
        nbr = np.empty(max(int(off[-1]), 1), np.int64)
        check(load().jg_graph_neighbors(self._h, int(direction), _ptr(r), len(r), _ptr(off), _ptr(nbr)))
        return off, nbr[:int(off[-1])]

    def degrees(self, direction=DIR_BOTH, rows=None):
        """Entries per row of the `direction` adjacency (jg_graph_neighbors' offsets only), all rows by default."""
        r = np.arange(self.n, dtype=np.int64) if rows is None else np.ascontiguousarray(rows, np.int64)
        off = np.empty(len(r) + 1, np.int64)
        check(load().jg_graph_neighbors(self._h, int(direction), _ptr(r), len(r), _ptr(off), None))
        return np.diff(off)

    def combine_steps(self, direction, combiner=COMBINE_SUM, steps=1, init=None, int32_wrap=True):
        """jg_combine_steps: `steps` supersteps of x[v] = COMBINE over v's `direction` entries of x[w].
        Returns (x, received) indexed like vid[]."""
        x0 = None if init is None else np.ascontiguousarray(init, np.int64)
        if x0 is not None and len(x0) != self.n:
            raise ValueError("init needs one value per vertex")
        out = np.empty(max(self.n, 1), np.int64)
        rec = np.empty(max(self.n, 1), np.uint8)
        check(load().jg_combine_steps(self._h, int(direction), int(combiner), 1 if int32_wrap else 0, _ptr(x0),
                                      int(steps), _ptr(out), _ptr(rec)))
        return out[:self.n], rec[:self.n].astype(bool)

    def connected_components(self):
        comp = self._out(self.n, np.int64)
        it = ctypes.c_int32(0)
        check(load().jg_connected_components(self._h, _ptr(comp), ctypes.byref(it)))
        return comp, int(it.value)
