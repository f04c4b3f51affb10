"""GraphComputer enums and exceptions (TinkerPop GraphComputer / JanusGraphComputer vocabulary).

JanusGraphComputer.ResultMode: janusgraph-core/src/main/java/org/janusgraph/core/JanusGraphComputer.java:29-56.
Exception messages follow TinkerPop's GraphComputer.Exceptions as used by FulgoraGraphComputer
(janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:134-190).
"""
from enum import Enum


class ResultGraph(Enum):
    ORIGINAL = "original"
    NEW = "new"


class Persist(Enum):
    NOTHING = "nothing"
    VERTEX_PROPERTIES = "vertex_properties"
    EDGES = "edges"


class ResultMode(Enum):
    """JanusGraphComputer.ResultMode -> (ResultGraph, Persist)."""
    NONE = (ResultGraph.NEW, Persist.NOTHING)
    PERSIST = (ResultGraph.ORIGINAL, Persist.VERTEX_PROPERTIES)
    LOCALTX = (ResultGraph.NEW, Persist.VERTEX_PROPERTIES)

    @property
    def result_graph(self):
        return self.value[0]

    @property
    def persist(self):
        return self.value[1]


class GraphComputerError(Exception):
    """TinkerPop GraphComputer.Exceptions / IllegalStateException / IllegalArgumentException."""


class ProgramNotSupported(GraphComputerError):
    """Not a program the GPU runs: the Java GpuGraphComputer delegates it to FulgoraGraphComputer."""


def computer_has_already_been_submitted():
    return GraphComputerError("The computer has already been submitted and can only be submitted once")


def computer_has_no_vertex_program_nor_map_reducers():
    return GraphComputerError("The computer has no vertex program or map reducers to execute")


def graph_filter_not_supported():
    return GraphComputerError("The computer does not support graph filtering")
