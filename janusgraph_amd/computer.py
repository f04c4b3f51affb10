"""GpuGraphComputer — host-side mirror of the TinkerPop GraphComputer API over libjanusgpu.

Mirrors FulgoraGraphComputer (janusgraph-core/src/main/java/org/janusgraph/graphdb/olap/computer/
FulgoraGraphComputer.java):
  vertices/edges (graph filters: stored, unsupported at submit)          :108-118, :522
  result/persist/workers/program/mapReduce (+ JanusGraphComputer.resultMode) :120-152
  submit(): single use, validation, async execution -> Future[ComputerResult] :154-208
  memory().getIteration() == last superstep index, getRuntime() in ms        FulgoraMemory.java:97-101
  map-reduce results under mr.memory_key                                      :288-357
  write-back of computed keys (ORIGINAL -> the graph, NEW -> a result view)   :359-471
The supersteps themselves run in libjanusgpu (HIP, gfx950): this module snapshots the graph once,
calls the C-ABI, and shapes the outputs like Fulgora's.  There is no CPU execution path: programs
the GPU does not run raise ProgramNotSupported (the Java side delegates those to Fulgora).
"""
from __future__ import annotations

import concurrent.futures as cf
import time

import numpy as np

from . import _lib
from .computer_types import (Persist, ProgramNotSupported, ResultGraph, ResultMode, computer_has_already_been_submitted,
                             computer_has_no_vertex_program_nor_map_reducers, graph_filter_not_supported)
from .graph import InMemoryGraph
from .programs import (CombinerVertexProgram, ConnectedComponentVertexProgram, PageRankVertexProgram,
                       ShortestDistanceVertexProgram, ShortestPathVertexProgram)


class Memory:
    """Global memory of a finished computation (FulgoraMemory after complete())."""

    def __init__(self):
        self._map = {}
        self._iteration = 0
        self._runtime = 0

    def get(self, key):
        if key not in self._map:
            raise KeyError(f"The memory does not contain the provided key: {key}")
        return self._map[key]

    def set(self, key, value):
        self._map[key] = value

    def exists(self, key):
        return key in self._map

    def keys(self):
        return set(self._map)

    def getIteration(self):  # noqa: N802
        return self._iteration

    def getRuntime(self):  # noqa: N802
        return self._runtime

    iteration = property(getIteration)
    runtime = property(getRuntime)


class ComputedGraph:
    """ResultGraph.NEW view: the original vertices with the computed keys overlaid."""

    def __init__(self, base: InMemoryGraph, props: dict):
        self.base, self.props = base, props

    def value(self, vid, key):
        return self.props[int(vid)][key]

    def properties(self, vid):
        return self.props.get(int(vid), {})


class ComputerResult:
    def __init__(self, graph, memory: Memory):
        self._graph, self._memory = graph, memory

    def graph(self):
        return self._graph

    def memory(self) -> Memory:
        return self._memory


class GpuGraphComputer:
    """graph.compute(GpuGraphComputer.class) for the programs of programs.RECOGNISED."""

    def __init__(self, graph: InMemoryGraph, devices=(0,), context: _lib.Context | None = None):
        self.graph = graph
        self.devices = tuple(devices)
        self._context = context
        self.vertex_program = None
        self.map_reduces = []
        self.result_graph_mode = None
        self.persist_mode = None
        self.num_threads = 1
        self.vertex_filter = None
        self.edge_filter = None
        self.executed = False

    # ---- GraphComputer builder methods ----
    def vertices(self, vertex_filter):
        self.vertex_filter = vertex_filter
        return self

    def edges(self, edge_filter):
        self.edge_filter = edge_filter
        return self

    def result(self, mode: ResultGraph):
        if mode is None:
            raise ValueError("Need to specify mode")
        self.result_graph_mode = mode
        return self

    def persist(self, mode: Persist):
        if mode is None:
            raise ValueError("Need to specify mode")
        self.persist_mode = mode
        return self

    def resultMode(self, mode: ResultMode):  # noqa: N802 (JanusGraphComputer.resultMode)
        return self.result(mode.result_graph).persist(mode.persist)

    def workers(self, threads: int):
        if threads <= 0:
            raise ValueError(f"Invalid number of threads: {threads}")
        self.num_threads = threads  # GPU parallelism is internal; accepted for API parity
        return self

    def program(self, vertex_program):
        if self.vertex_program is not None:
            raise RuntimeError("A vertex program has already been set")
        self.vertex_program = vertex_program
        return self

    def mapReduce(self, map_reduce):  # noqa: N802
        self.map_reduces.append(map_reduce)
        return self

    @staticmethod
    def features():
        return {"supportsVertexAddition": False, "supportsVertexRemoval": False,
                "supportsVertexPropertyAddition": True, "supportsVertexPropertyRemoval": False,
                "supportsEdgeAddition": False, "supportsEdgeRemoval": False, "supportsEdgePropertyAddition": False,
                "supportsEdgePropertyRemoval": False, "supportsGraphFilter": False}

    # ---- submit ----
    def submit(self) -> cf.Future:
        if self.executed:
            raise computer_has_already_been_submitted()
        self.executed = True
        if self.vertex_program is None and not self.map_reduces:
            raise computer_has_no_vertex_program_nor_map_reducers()
        if self.vertex_filter is not None or self.edge_filter is not None:
            raise graph_filter_not_supported()
        vp = self.vertex_program
        if vp is not None:
            if not isinstance(vp, (PageRankVertexProgram, ShortestDistanceVertexProgram,
                                   ConnectedComponentVertexProgram, ShortestPathVertexProgram,
                                   CombinerVertexProgram)):
                raise ProgramNotSupported(f"{type(vp).__name__} is not run by GpuGraphComputer; "
                                          f"delegate to FulgoraGraphComputer")
            self.map_reduces.extend(vp.get_map_reducers())
        if self.persist_mode is None:
            self.persist_mode = vp.preferred_persist if vp is not None else Persist.NOTHING
        if self.result_graph_mode is None:
            self.result_graph_mode = vp.preferred_result_graph if vp is not None else ResultGraph.ORIGINAL
        pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="GpuGraphComputer")
        fut = pool.submit(self._submit_async)
        pool.shutdown(wait=False)
        return fut

    # ---- execution ----
    def _ctx(self) -> _lib.Context:
        if self._context is None:
            self._context = _lib.Context(self.devices)
        return self._context

    def _submit_async(self) -> ComputerResult:
        t0 = time.perf_counter()
        memory = Memory()
        props = {}
        vids = None
        if self.vertex_program is not None:
            vids, props, iteration, extra = self._execute_vertex_program(self.vertex_program)
            memory._iteration = iteration
            for k, v in extra.items():
                memory.set(k, v)
        for mr in self.map_reduces:
            emitted = []
            for vid in (vids if vids is not None else []):
                mr.map(int(vid), props.get(int(vid), {}), lambda k, v: emitted.append((k, v)))
            final = getattr(mr, "generate_final_result", None)
            memory.set(mr.memory_key, final(emitted) if final else iter(emitted))
        result_graph = self._write_back(props)
        memory._runtime = int(round((time.perf_counter() - t0) * 1000))
        return ComputerResult(result_graph, memory)

    def _execute_vertex_program(self, vp):
        g0 = self.graph
        ctx = self._ctx()
        if isinstance(vp, PageRankVertexProgram):
            vid, src, dst, _ = g0.snapshot()
            if vp.max_iterations == 0:
                return vid, {}, 0, {}
            g = ctx.build(vid, src, dst, flags=_lib.ADJ_IN)
            try:
                rank, ec = g.pagerank(vp.damping_factor, vp.vertex_count, vp.max_iterations)
            finally:
                g.close()
            props = {int(v): {vp.PAGE_RANK: float(r), vp.OUTGOING_EDGE_COUNT: float(c)}
                     for v, r, c in zip(vid, rank, ec)}
            return vid, props, vp.max_iterations, {}
        if isinstance(vp, ShortestDistanceVertexProgram):
            vid, src, dst, w = g0.snapshot(weight_property=vp.weight_property)
            g = ctx.build(vid, src, dst, weight=w, flags=_lib.ADJ_IN | _lib.ADJ_OUT)
            try:
                dist = g.shortest_distance(vp.seed, vp.max_depth)
            finally:
                g.close()
            props = {int(v): {vp.DISTANCE: int(d)} for v, d in zip(vid, dist) if d != _lib.DIST_ABSENT}
            return vid, props, vp.max_depth, {}
        if isinstance(vp, ConnectedComponentVertexProgram):
            vid, src, dst, _ = g0.snapshot()
            g = ctx.build(vid, src, dst, flags=_lib.ADJ_BOTH)
            try:
                comp, it = g.connected_components()
            finally:
                g.close()
            props = {int(v): {vp.property: str(int(c))} for v, c in zip(vid, comp)}
            return vid, props, it, {}
        if isinstance(vp, ShortestPathVertexProgram):
            return self._shortest_paths(ctx, vp)
        if isinstance(vp, CombinerVertexProgram):
            vid, src, dst, _ = g0.snapshot()
            direction = CombinerVertexProgram.SCOPES[vp.scope]
            adj = {_lib.DIR_OUT: _lib.ADJ_OUT, _lib.DIR_IN: _lib.ADJ_IN, _lib.DIR_BOTH: _lib.ADJ_BOTH}[direction]
            g = ctx.build(vid, src, dst, flags=adj)
            try:
                x, received = g.combine_steps(direction, CombinerVertexProgram.COMBINERS.index(vp.combiner), vp.length,
                                              np.full(len(vid), vp.initial_message, np.int64), vp.int32)
            finally:
                g.close()
            # a sum always sets the key (reduce(0, +)); min/max only where a message arrived
            keep = np.ones(len(vid), bool) if vp.combiner == "sum" else received
            props = {int(v): {vp.property_key: int(d)} for v, d, k in zip(vid, x, keep) if k}
            return vid, props, vp.length, {}
        raise ProgramNotSupported(type(vp).__name__)

    def _shortest_paths(self, ctx, vp):
        """ShortestPaths.execute of the Java drop-in: one depth row per source (jg_bfs_rows, 64 sources
        per bit-parallel pass), paths rebuilt by PathDag over the snapshot's BOTH adjacency."""
        vid, src, dst, _ = self.graph.snapshot()
        index = {int(v): i for i, v in enumerate(vid.tolist())}
        sources = [index[s] for s in (vp.sources if vp.sources is not None else vid.tolist()) if s in index]
        target = None
        if vp.targets is not None:
            target = np.zeros(len(vid), bool)
            target[[index[t] for t in vp.targets if t in index]] = True
        g = ctx.build(vid, src, dst, flags=_lib.ADJ_BOTH)
        paths, max_level = [], 0
        try:
            dag = PathDag(g.neighbors, len(vid))
            for b0 in range(0, len(sources), SOURCES_PER_BFS):
                batch = sources[b0:b0 + SOURCES_PER_BFS]
                rows = g.bfs_rows(vid[batch], _lib.DIR_BOTH, -1 if vp.max_distance is None else vp.max_distance)
                for s, depth in zip(batch, rows):
                    got, deepest = dag.paths(depth, s, target)
                    max_level = max(max_level, deepest)
                    paths.extend([int(vid[x]) for x in p] for p in got)
        finally:
            g.close()
        return vid, {}, max_level + 1, {vp.SHORTEST_PATHS: paths}

    def _write_back(self, props):
        if self.persist_mode is Persist.NOTHING:
            return None if self.result_graph_mode is ResultGraph.NEW else self.graph
        if self.result_graph_mode is ResultGraph.ORIGINAL:
            for vid, kv in props.items():
                v = self.graph.vertices.get(vid)
                if v is not None:
                    v.properties.update(kv)
            return self.graph
        return ComputedGraph(self.graph, props)


SOURCES_PER_BFS = 64  # jg_bfs_rows: one bit-parallel pass per 64 sources


class PathDag:
    """Every shortest path from one source to the targets it reaches, rebuilt from its depth row (mirror
    of GpuGraphComputer.PathDag, java/.../GpuGraphComputer.java): the predecessors of a vertex at depth d
    are its BOTH neighbours at depth d - 1, read level by level from the device snapshot
    (jg_graph_neighbors), deepest targets first, so each vertex on some path is expanded once; paths are
    then enumerated from each target (ascending) back to the source.  `neighbors(rows)` -> (off, nbr)."""

    ROWS_PER_CALL = 1 << 14

    def __init__(self, neighbors, n):
        self.neighbors = neighbors
        self.n = n

    def predecessors(self, depth, target=None):
        """{vertex: predecessor array} for every vertex on a shortest path to a target; and the targets."""
        depth = np.asarray(depth)
        reached = depth >= 0
        if target is not None:
            reached &= target
        targets = np.flatnonzero(reached)
        if len(targets) == 0:
            return {}, targets, -1
        deepest = int(depth[targets].max())
        level = [[] for _ in range(deepest + 1)]
        for d in range(deepest + 1):
            level[d] = list(targets[depth[targets] == d])
        queued = np.zeros(self.n, bool)
        queued[targets] = True
        pred = {}
        for d in range(deepest, 0, -1):
            cur = np.asarray(level[d], np.int64)
            for f in range(0, len(cur), self.ROWS_PER_CALL):
                rows = cur[f:f + self.ROWS_PER_CALL]
                off, nbr = self.neighbors(rows)
                for i, v in enumerate(rows.tolist()):
                    nb = nbr[off[i]:off[i + 1]]
                    nb = nb[depth[nb] == d - 1]
                    _, first = np.unique(nb, return_index=True)
                    p = nb[np.sort(first)]  # distinct, in adjacency order
                    pred[v] = p
                    new = p[~queued[p]]
                    queued[new] = True
                    level[d - 1].extend(new.tolist())
        return pred, targets, deepest

    def paths(self, depth, s, target=None):
        """(paths as vertex-index lists, deepest target depth (0 if none))."""
        pred, targets, deepest = self.predecessors(depth, target)
        out = []
        for t in targets.tolist():
            stack = [(t, [t])]
            while stack:
                v, suffix = stack.pop()
                if v == s:
                    out.append(list(reversed(suffix)))
                    continue
                for u in reversed(pred[v].tolist()):  # first predecessor first, as the Java recursion
                    stack.append((u, suffix + [u]))
        return out, max(deepest, 0)
