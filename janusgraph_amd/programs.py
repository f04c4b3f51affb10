"""Vertex programs and map-reduces that GpuGraphComputer recognises and runs on the GPU.

Same names, configuration keys, builders and output keys as the reference:
  PageRankVertexProgram / PageRankMapReduce
      janusgraph-backend-testutils/src/main/java/org/janusgraph/olap/PageRankVertexProgram.java:46-166,
      PageRankMapReduce.java:32-67
  ShortestDistanceVertexProgram / ShortestDistanceMapReduce
      janusgraph-backend-testutils/.../olap/ShortestDistanceVertexProgram.java:40-192,
      ShortestDistanceMapReduce.java:29-64
  ConnectedComponentVertexProgram, ShortestPathVertexProgram
      TinkerPop 3.4.6 gremlin-core (third party, not in the container; SURVEY.md A.3/A.4 [TP-recall])
  CombinerVertexProgram / DegreeCounter / DegreeMapper
      a superstep loop with a sum / min / max MessageCombiner over one Local scope, as
      janusgraph-test/src/main/java/org/janusgraph/olap/OLAPTest.java:424-540 (DegreeCounter,
      DegreeMapper) writes it; message combining per VertexState.java:85-114
Any other program is not recognised: the computer refuses it with ProgramNotSupported so that the
caller (the Java GpuGraphComputer) delegates it to FulgoraGraphComputer unchanged.
"""
from __future__ import annotations

from .computer_types import Persist, ResultGraph


class VertexProgram:
    """Configuration-carrying program (storeState/loadState as a dict)."""

    VERTEX_PROGRAM = "gremlin.vertexProgram"
    preferred_result_graph = ResultGraph.ORIGINAL
    preferred_persist = Persist.VERTEX_PROPERTIES
    compute_keys: tuple = ()

    def __init__(self, configuration: dict):
        self.configuration = dict(configuration)
        self.load_state(self.configuration)

    def load_state(self, conf):
        pass

    def store_state(self) -> dict:
        return dict(self.configuration, **{self.VERTEX_PROGRAM: type(self).__name__})

    def get_map_reducers(self):
        return []


class _Builder:
    def __init__(self, cls):
        self.cls = cls
        self.configuration = {}

    def create(self, graph=None):
        return self.cls(self.configuration)


class PageRankVertexProgram(VertexProgram):
    PAGE_RANK = "janusgraph.pageRank.pageRank"
    OUTGOING_EDGE_COUNT = "janusgraph.pageRank.edgeCount"
    DAMPING_FACTOR = "janusgraph.pageRank.dampingFactor"
    MAX_ITERATIONS = "janusgraph.pageRank.maxIterations"
    VERTEX_COUNT = "janusgraph.pageRank.vertexCount"
    compute_keys = (PAGE_RANK, OUTGOING_EDGE_COUNT)

    def load_state(self, conf):  # PageRankVertexProgram.java:64-69
        self.damping_factor = float(conf.get(self.DAMPING_FACTOR, 0.85))
        self.max_iterations = int(conf.get(self.MAX_ITERATIONS, 10))
        self.vertex_count = int(conf.get(self.VERTEX_COUNT, 1))

    class Builder(_Builder):
        def __init__(self):
            super().__init__(PageRankVertexProgram)

        def vertexCount(self, n):  # noqa: N802 (reference names)
            self.configuration[PageRankVertexProgram.VERTEX_COUNT] = int(n)
            return self

        def dampingFactor(self, d):  # noqa: N802
            self.configuration[PageRankVertexProgram.DAMPING_FACTOR] = float(d)
            return self

        def iterations(self, k):
            self.configuration[PageRankVertexProgram.MAX_ITERATIONS] = int(k)
            return self

    @classmethod
    def build(cls):
        return cls.Builder()


class ShortestDistanceVertexProgram(VertexProgram):
    DISTANCE = "janusgraph.shortestDistanceVertexProgram.distance"
    MAX_DEPTH = "janusgraph.shortestDistanceVertexProgram.maxDepth"
    WEIGHT_PROPERTY = "janusgraph.shortestDistanceVertexProgram.weightProperty"
    SEED = "janusgraph.shortestDistanceVertexProgram.seedID"
    compute_keys = (DISTANCE,)

    def load_state(self, conf):  # ShortestDistanceVertexProgram.java:65-71
        if self.MAX_DEPTH not in conf or self.SEED not in conf:
            raise KeyError("maxDepth and seed are required")
        self.max_depth = int(conf[self.MAX_DEPTH])
        self.seed = int(conf[self.SEED])
        self.weight_property = conf.get(self.WEIGHT_PROPERTY, "distance")

    class Builder(_Builder):
        def __init__(self):
            super().__init__(ShortestDistanceVertexProgram)

        def maxDepth(self, d):  # noqa: N802
            self.configuration[ShortestDistanceVertexProgram.MAX_DEPTH] = int(d)
            return self

        def seed(self, vid):
            self.configuration[ShortestDistanceVertexProgram.SEED] = int(vid)
            return self

        def weightProperty(self, key):  # noqa: N802
            self.configuration[ShortestDistanceVertexProgram.WEIGHT_PROPERTY] = key
            return self

    @classmethod
    def build(cls):
        return cls.Builder()


class ConnectedComponentVertexProgram(VertexProgram):
    COMPONENT = "gremlin.connectedComponentVertexProgram.component"
    PROPERTY = "gremlin.connectedComponentVertexProgram.property"
    MAX_ITERATIONS = "gremlin.connectedComponentVertexProgram.maxIterations"
    compute_keys = (COMPONENT,)

    def load_state(self, conf):
        self.property = conf.get(self.PROPERTY, self.COMPONENT)
        self.max_iterations = int(conf.get(self.MAX_ITERATIONS, 100))
        if self.max_iterations != 100:
            raise ValueError("GpuGraphComputer runs ConnectedComponentVertexProgram with maxIterations = 100")

    class Builder(_Builder):
        def __init__(self):
            super().__init__(ConnectedComponentVertexProgram)

        def property(self, key):
            self.configuration[ConnectedComponentVertexProgram.PROPERTY] = key
            return self

    @classmethod
    def build(cls):
        return cls.Builder()


class ShortestPathVertexProgram(VertexProgram):
    """Depth on the GPU (Fulgora forces {Local(bothE), Global}), paths rebuilt on the host."""

    SHORTEST_PATHS = "gremlin.shortestPathVertexProgram.shortestPaths"
    preferred_persist = Persist.NOTHING

    def load_state(self, conf):
        self.sources = conf.get("sources")  # None = every vertex
        self.targets = conf.get("targets")  # None = every vertex
        self.max_distance = conf.get("maxDistance")
        self.include_edges = bool(conf.get("includeEdges", False))
        if self.include_edges:
            raise ValueError("includeEdges is not supported by GpuGraphComputer")

    class Builder(_Builder):
        def __init__(self):
            super().__init__(ShortestPathVertexProgram)

        def source(self, *vids):
            self.configuration["sources"] = [int(v) for v in vids]
            return self

        def target(self, *vids):
            self.configuration["targets"] = [int(v) for v in vids]
            return self

        def maxDistance(self, d):  # noqa: N802
            self.configuration["maxDistance"] = int(d)
            return self

    @classmethod
    def build(cls):
        return cls.Builder()


class CombinerVertexProgram(VertexProgram):
    """A program whose every superstep is x_t[v] = COMBINE of the messages v receives, each neighbour
    sending its x_{t-1}: superstep 0 sends `initial_message`, supersteps 1..length store the combined
    value under `property_key` and send it on while t < length; terminate at iteration >= length.
    `scope` is the send scope's direction: "inE" (DegreeCounter's DEG_MSG, OLAPTest.java:429) reaches
    the sources of a vertex's in-edges, so a vertex receives from its out-neighbours."""

    preferred_result_graph = ResultGraph.NEW
    preferred_persist = Persist.VERTEX_PROPERTIES
    COMBINERS = ("sum", "min", "max")
    SCOPES = {"inE": 1, "outE": 2, "bothE": 3}  # -> the receiver's pull direction (DIR_OUT/IN/BOTH)

    def __init__(self, length=1, property_key="degree", combiner="sum", scope="inE", initial_message=1,
                 int32=True):
        if length <= 0:
            raise ValueError("length must be positive")  # Preconditions.checkArgument(length>0), :438
        if combiner not in self.COMBINERS or scope not in self.SCOPES:
            raise ValueError("unknown combiner or scope")
        self.length, self.property_key, self.combiner, self.scope = length, property_key, combiner, scope
        self.initial_message, self.int32 = initial_message, int32
        self.compute_keys = (property_key,)
        super().__init__({"length": length})


class DegreeCounter(CombinerVertexProgram):
    """OLAPTest.DegreeCounter (OLAPTest.java:424-503): k-hop out-path counts, Integer sums."""

    DEGREE = "degree"

    def __init__(self, length=1):
        super().__init__(length, self.DEGREE, "sum", "inE", 1, True)


class MapReduce:
    memory_key = None

    def map(self, vid, props, emit):
        raise NotImplementedError


class PageRankMapReduce(MapReduce):
    DEFAULT_MEMORY_KEY = "pageRank"

    def __init__(self, memory_key=DEFAULT_MEMORY_KEY):
        self.memory_key = memory_key

    @classmethod
    def build(cls):
        return _MrBuilder(cls)

    def map(self, vid, props, emit):  # PageRankMapReduce.java:62-67
        v = props.get(PageRankVertexProgram.PAGE_RANK)
        if v is not None:
            emit(vid, v)


class ShortestDistanceMapReduce(MapReduce):
    DEFAULT_MEMORY_KEY = "shortestDistance"

    def __init__(self, memory_key=DEFAULT_MEMORY_KEY):
        self.memory_key = memory_key

    @classmethod
    def build(cls):
        return _MrBuilder(cls)

    def map(self, vid, props, emit):  # ShortestDistanceMapReduce.java:59-64
        v = props.get(ShortestDistanceVertexProgram.DISTANCE)
        if v is not None:
            emit(vid, v)


class DegreeMapper(MapReduce):
    """OLAPTest.DegreeMapper (OLAPTest.java:505-540): memory["degrees"] = {vertex id: degree}."""

    DEGREE_RESULT = "degrees"
    memory_key = DEGREE_RESULT

    def map(self, vid, props, emit):
        v = props.get(DegreeCounter.DEGREE)
        if v is not None:
            emit(vid, v)

    def generate_final_result(self, key_values):
        return {k: v for k, v in key_values}


class _MrBuilder:
    def __init__(self, cls):
        self.cls, self.key = cls, cls.DEFAULT_MEMORY_KEY

    def memoryKey(self, key):  # noqa: N802
        self.key = key
        return self

    def create(self):
        return self.cls(self.key)


RECOGNISED = (PageRankVertexProgram, ShortestDistanceVertexProgram, ConnectedComponentVertexProgram,
              ShortestPathVertexProgram, CombinerVertexProgram)
