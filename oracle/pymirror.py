"""Pure-Python vertex-centric mirror of Fulgora's BSP engine — TEST INFRASTRUCTURE ONLY.

A second, independent restatement (the C oracle is the optimised one) that keeps the
reference's structure: per-vertex `execute(vertex, messenger, memory)`, Local message scopes whose
messages are stored on the SENDER and pulled by the receiver over the reverse incident traversal,
previous-superstep-only visibility, and the iteration/terminate bookkeeping of the driver loop.
Pure-Python loops: small graphs only (fixtures, KATs, cross-checks).

Reference (paths under /root/reference/janusgraph-core/src/main/java/org/janusgraph/):
  graphdb/olap/computer/FulgoraGraphComputer.java:210-230   superstep loop / terminate / incrIteration
  graphdb/olap/computer/FulgoraGraphComputer.java:249-253   SPVP scopes forced to {Local(bothE), Global}
  graphdb/olap/computer/VertexMemoryHandler.java:121-165    receiveMessages / sendMessage
  graphdb/olap/computer/VertexState.java:77-138             message slots, combiner, completeIteration
  graphdb/olap/computer/FulgoraMemory.java:97-106           complete() / completeSubRound()
Programs (paths under /root/reference/janusgraph-backend-testutils/src/main/java/org/janusgraph/):
  olap/PageRankVertexProgram.java:89-110, olap/ShortestDistanceVertexProgram.java:112-146,
  olap/ShortestDistanceMessageCombiner.java:29-31; TinkerPop ConnectedComponentVertexProgram
  (3.4.6, not in the container; SURVEY.md A.3 [TP-recall]).
"""
from __future__ import annotations

from dataclasses import dataclass, field

OUT, IN, BOTH = "out", "in", "both"
_REVERSE = {OUT: IN, IN: OUT, BOTH: BOTH}


@dataclass(frozen=True)
class LocalScope:
    """MessageScope.Local.of(__::<direction>E, edgeFunction)."""
    direction: str
    name: str
    edge_fn: object = None  # (msg, edge) -> msg


@dataclass
class Edge:
    src: int
    dst: int
    label: str = "e"
    props: dict = field(default_factory=dict)


class MiniGraph:
    """Vertices (ids) + directed MULTI edges; edges to ids outside `vertices` are ghost edges."""

    def __init__(self, vertices, edges):
        self.vertices = list(vertices)
        self.vset = set(self.vertices)
        self.edges = [e if isinstance(e, Edge) else Edge(*e) for e in edges]
        self.out_adj = {v: [] for v in self.vertices}
        self.in_adj = {v: [] for v in self.vertices}
        for e in self.edges:
            if e.src in self.vset and e.dst in self.vset:  # VertexJobConverter ghost rule
                self.out_adj[e.src].append(e)
                self.in_adj[e.dst].append(e)
        # row order of a single-label JanusGraph row: other vertex id, then relation (insertion) order
        for v in self.vertices:
            self.out_adj[v].sort(key=lambda e: e.dst)
            self.in_adj[v].sort(key=lambda e: e.src)

    def incident(self, v, direction):
        if direction == OUT:
            return [(e, e.dst) for e in self.out_adj[v]]
        if direction == IN:
            return [(e, e.src) for e in self.in_adj[v]]
        return [(e, e.dst) for e in self.out_adj[v]] + [(e, e.src) for e in self.in_adj[v]]


class Memory:
    def __init__(self):
        self.iteration = 0
        self.store = {}

    def is_initial_iteration(self):
        return self.iteration == 0


class Messenger:
    def __init__(self, engine, v):
        self.engine, self.v = engine, v

    def receive_messages(self):
        eng, out = self.engine, []
        for scope in eng.prev_scopes:
            # reverse incident traversal from v, then the other endpoint's stored message
            for e, other in eng.graph.incident(self.v, _REVERSE[scope.direction]):
                msg = eng.prev_msgs.get((other, scope.name))
                if msg is not None:
                    out.append(scope.edge_fn(msg, e) if scope.edge_fn else msg)
        return out

    def send_message(self, scope, m):
        self.engine.cur_msgs[(self.v, scope.name)] = m  # stored on the sender, overwritten


class Engine:
    """executeVertexProgram of FulgoraGraphComputer, one vertex at a time."""

    def __init__(self, graph: MiniGraph):
        self.graph = graph

    def run(self, program):
        g, mem = self.graph, Memory()
        self.props = {v: {} for v in g.vertices}
        self.prev_msgs, self.cur_msgs = {}, {}
        program.setup(mem)
        self.prev_scopes = []
        while True:
            # nextIteration(getMessageScopes(memory)) sets the scopes this superstep SENDS on; messages
            # are received over the previous superstep's (FulgoraVertexMemory.java:101-112)
            cur_scopes = program.message_scopes(mem)
            for v in g.vertices:
                program.execute(v, self.props[v], Messenger(self, v), mem, g)
            self.prev_msgs, self.cur_msgs = self.cur_msgs, {}
            self.prev_scopes = cur_scopes
            if program.terminate(mem):
                break
            mem.iteration += 1
        return self.props, mem.iteration


class PageRankProgram:
    """olap/PageRankVertexProgram.java:89-110."""

    def __init__(self, damping=0.85, iterations=10, vertex_count=1):
        self.d, self.K, self.N = damping, iterations, vertex_count
        self.outE = LocalScope(OUT, "outE")
        self.inE = LocalScope(IN, "inE")

    def setup(self, mem):
        pass

    def message_scopes(self, mem):
        return [self.outE, self.inE]

    def execute(self, v, props, msgr, mem, g):
        if mem.is_initial_iteration():
            msgr.send_message(self.inE, 1.0)
        elif mem.iteration == 1:
            initial = 1.0 / self.N
            edge_count = 0.0
            for m in msgr.receive_messages():
                edge_count = edge_count + m
            props["pageRank"] = initial
            props["edgeCount"] = edge_count
            msgr.send_message(self.outE, initial / edge_count if edge_count else float("inf"))
        else:
            s = 0.0
            for m in msgr.receive_messages():
                s = s + m
            r = (self.d * s) + ((1.0 - self.d) / self.N)
            props["pageRank"] = r
            ec = props["edgeCount"]
            msgr.send_message(self.outE, r / ec if ec else float("inf"))

    def terminate(self, mem):
        return mem.iteration >= self.K


class ShortestDistanceProgram:
    """olap/ShortestDistanceVertexProgram.java:112-146 (weightProperty "distance")."""

    def __init__(self, seed, max_depth, weight_property="distance", unit_weights=False):
        self.seed, self.max_depth = seed, max_depth
        wp = weight_property
        fn = (lambda msg, e: msg + 1) if unit_weights else (lambda msg, e: msg + int(e.props[wp]))
        self.scope = LocalScope(IN, "inE", fn)

    def setup(self, mem):
        pass

    def message_scopes(self, mem):
        return [self.scope]

    def execute(self, v, props, msgr, mem, g):
        if mem.is_initial_iteration():
            if v == self.seed:
                props["distance"] = 0
                msgr.send_message(self.scope, 0)
        else:
            msgs = msgr.receive_messages()
            if not msgs:
                return
            shortest = min(msgs)
            if "distance" not in props or props["distance"] > shortest:
                props["distance"] = shortest
                msgr.send_message(self.scope, shortest)

    def terminate(self, mem):
        return mem.iteration >= self.max_depth


class ConnectedComponentProgram:
    """TinkerPop ConnectedComponentVertexProgram 3.4.6 [TP-recall] over BOTH edges."""

    def __init__(self, max_iterations=100):
        self.max_iterations = max_iterations
        self.scope = LocalScope(BOTH, "bothE")

    def setup(self, mem):
        mem.store["halt"] = True

    def message_scopes(self, mem):
        return [self.scope]

    def execute(self, v, props, msgr, mem, g):
        if mem.is_initial_iteration():
            props["component"] = str(v)
            if g.incident(v, BOTH):
                msgr.send_message(self.scope, str(v))
                mem.store["halt"] = False
        else:
            cur, different = props["component"], False
            for cand in msgr.receive_messages():
                if cand < cur:  # String.compareTo on ASCII digits == Python str order
                    cur, different = cand, True
            if different:
                props["component"] = cur
                msgr.send_message(self.scope, cur)
                mem.store["halt"] = False

    def terminate(self, mem):
        if mem.store["halt"] or mem.iteration >= self.max_iterations - 1:
            return True
        mem.store["halt"] = True
        return False


def bfs_depth(graph: MiniGraph, source, direction=BOTH, max_depth=-1):
    """Hop depth along `direction` (SPVP depth under Fulgora's forced bothE scope when BOTH)."""
    depth = {v: -1 for v in graph.vertices}
    if source not in graph.vset:
        return depth
    depth[source] = 0
    frontier = [source]
    while frontier:
        nxt = []
        for u in frontier:
            if 0 <= max_depth <= depth[u]:
                continue
            for _, w in graph.incident(u, direction):
                if depth[w] < 0:
                    depth[w] = depth[u] + 1
                    nxt.append(w)
        frontier = nxt
    return depth


class DegreeCounterProgram:
    """janusgraph-test/.../olap/OLAPTest.java:424-503 (DegreeCounter): Integer sums, Local.of(inE),
    combiner (a, b) -> a + b.  The general form takes the combiner and scope (CombinerVertexProgram)."""

    def __init__(self, length=1, combine=lambda a, b: a + b, direction=IN, initial=1, key="degree", int32=True):
        self.length, self.combine, self.initial, self.key, self.int32 = length, combine, initial, key, int32
        self.scope = LocalScope(direction, "deg")
        self.sum = combine(2, 3) == 5

    def setup(self, mem):
        pass

    def message_scopes(self, mem):
        return [self.scope] if mem.iteration < self.length else []

    def _int(self, x):
        if not self.int32:
            return x
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >> 31 else x

    def execute(self, v, props, msgr, mem, g):
        if mem.is_initial_iteration():
            msgr.send_message(self.scope, self.initial)
            return
        msgs = msgr.receive_messages()
        if self.sum:
            degree = 0  # IteratorUtils.stream(...).reduce(0, (a, b) -> a + b)
            for m in msgs:
                degree = self._int(degree + m)
        else:
            if not msgs:
                return
            degree = msgs[0]
            for m in msgs[1:]:
                degree = self.combine(degree, m)
        props[self.key] = degree
        if mem.iteration < self.length:
            msgr.send_message(self.scope, degree)

    def terminate(self, mem):
        return mem.iteration >= self.length
