"""janusgraph_amd — MI355X-native OLAP graph computer for JanusGraph (GpuGraphComputer).

The compute path is libjanusgpu.so (hand-written HIP for gfx950, C-ABI in include/janusgpu.h);
this package is its host-side mirror of the TinkerPop GraphComputer API.
"""
from ._lib import (ADJ_BOTH, ADJ_IN, ADJ_OUT, COMBINE_MAX, COMBINE_MIN, COMBINE_SUM, DIR_BOTH, DIR_IN,  # noqa: F401
                   DIR_OUT, DIST_ABSENT, FULGORA_HARD_QUERY_LIMIT, LIB_PATH, WEIGHT_ABSENT, Builder, Context,
                   Graph, JanusGpuError, load)
from .computer import ComputedGraph, ComputerResult, GpuGraphComputer, Memory  # noqa: F401
from .computer_types import (GraphComputerError, Persist, ProgramNotSupported, ResultGraph,  # noqa: F401
                             ResultMode)
from .graph import InMemoryGraph, load_graph_of_the_gods  # noqa: F401
from .idmanager import IDManager, VertexIDType  # noqa: F401
from .programs import (CombinerVertexProgram, ConnectedComponentVertexProgram, DegreeCounter,  # noqa: F401
                       DegreeMapper, PageRankMapReduce, PageRankVertexProgram, ShortestDistanceMapReduce,
                       ShortestDistanceVertexProgram, ShortestPathVertexProgram)

__all__ = [
    "Context", "Graph", "JanusGpuError", "load", "ADJ_IN", "ADJ_OUT", "ADJ_BOTH", "DIR_IN", "DIR_OUT", "DIR_BOTH",
    "LIB_PATH", "GpuGraphComputer", "ComputerResult", "ComputedGraph", "Memory", "GraphComputerError",
    "ProgramNotSupported", "Persist", "ResultGraph", "ResultMode", "InMemoryGraph", "load_graph_of_the_gods",
    "IDManager", "VertexIDType", "PageRankVertexProgram", "PageRankMapReduce", "ShortestDistanceVertexProgram",
    "ShortestDistanceMapReduce", "ConnectedComponentVertexProgram", "ShortestPathVertexProgram",
    "CombinerVertexProgram", "DegreeCounter", "DegreeMapper", "COMBINE_SUM", "COMBINE_MIN", "COMBINE_MAX",
]
