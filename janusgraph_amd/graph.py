"""A minimal in-memory property graph standing in for a JanusGraph instance on janusgraph-inmemory.

It gives GpuGraphComputer what the reference's snapshot path gives Fulgora:
  * vertex rows keyed by JanusGraph ids (IDManager layout, idmanager.py), ghost rows included
    (VertexJobConverter.isGhostVertex, janusgraph-core/.../olap/VertexJobConverter.java:145-151);
  * adjacency as (src, dst, label, properties) MULTI edges, self-loops allowed;
  * vertex properties that computed keys are written back into (ResultGraph.ORIGINAL /
    Persist.VERTEX_PROPERTIES, janusgraph-core/.../olap/computer/FulgoraGraphComputer.java:359-471).
snapshot() is the once-per-computer edgestore scan (replacing Fulgora's scan per superstep).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .idmanager import IDManager


@dataclass
class Vertex:
    id: int
    label: str = "vertex"
    properties: dict = field(default_factory=dict)
    ghost: bool = False  # row without VertexExists: never executes, never sends

    def value(self, key):
        return self.properties[key]


@dataclass
class Edge:
    out_id: int
    in_id: int
    label: str
    properties: dict = field(default_factory=dict)


class InMemoryGraph:
    def __init__(self, partition_bits: int = 5, set_vertex_id: bool = False):
        self.idm = IDManager(partition_bits)
        self.set_vertex_id = set_vertex_id  # graph.set-vertex-id
        self.vertices: dict[int, Vertex] = {}
        self.edges: list[Edge] = []
        self._count = 0

    # --- mutation (OLTP side, only what the tests need) ---
    def add_vertex(self, label: str = "vertex", id: int | None = None, **props) -> Vertex:  # noqa: A002
        if id is not None:
            if not self.set_vertex_id:
                raise ValueError("vertex ids can only be set with graph.set-vertex-id=true")
            vid = self.idm.to_vertex_id(id)
        else:
            self._count += 1
            vid = self.idm.to_vertex_id(self._count)
        if vid in self.vertices:
            raise ValueError(f"vertex {vid} already exists")
        v = Vertex(vid, label, dict(props))
        self.vertices[vid] = v
        return v

    def add_edge(self, out_v, in_v, label: str = "edge", **props) -> Edge:
        oid = out_v.id if isinstance(out_v, Vertex) else int(out_v)
        iid = in_v.id if isinstance(in_v, Vertex) else int(in_v)
        e = Edge(oid, iid, label, dict(props))
        self.edges.append(e)
        return e

    def make_ghost(self, v):
        """Simulate a partially deleted vertex: its row loses VertexExists, edges stay in other rows."""
        self.vertices[v.id if isinstance(v, Vertex) else int(v)].ghost = True

    def vertex(self, vid) -> Vertex:
        return self.vertices[int(vid)]

    # --- OLAP snapshot ---
    def snapshot(self, weight_property: str | None = None):
        """(vid, src, dst, weight): existing vertices + every stored edge (ghost endpoints included;
        the library drops them).  weight: int32 edge property per edge (WEIGHT_ABSENT where the edge
        has none: Fulgora only fails if a message crosses such an edge), or None."""
        vid = np.fromiter((v.id for v in self.vertices.values() if not v.ghost), dtype=np.int64)
        src = np.fromiter((e.out_id for e in self.edges), dtype=np.int64, count=len(self.edges))
        dst = np.fromiter((e.in_id for e in self.edges), dtype=np.int64, count=len(self.edges))
        weight = None
        if weight_property is not None:
            from ._lib import WEIGHT_ABSENT
            w = [int(e.properties[weight_property]) if weight_property in e.properties else int(WEIGHT_ABSENT)
                 for e in self.edges]
            weight = np.asarray(w, dtype=np.int32)
        return vid, src, dst, weight


def load_graph_of_the_gods(graph: InMemoryGraph) -> dict:
    """GraphOfTheGodsFactory.load (janusgraph-core/.../example/GraphOfTheGodsFactory.java:116-151)."""
    v = {}
    for name, label, props in [
        ("saturn", "titan", {"age": 10000}), ("sky", "location", {}), ("sea", "location", {}),
        ("jupiter", "god", {"age": 5000}), ("neptune", "god", {"age": 4500}), ("hercules", "demigod", {"age": 30}),
        ("alcmene", "human", {"age": 45}), ("pluto", "god", {"age": 4000}), ("nemean", "monster", {}),
        ("hydra", "monster", {}), ("cerberus", "monster", {}), ("tartarus", "location", {}),
    ]:
        v[name] = graph.add_vertex(label, name=name, **props)
    E = graph.add_edge
    E(v["jupiter"], v["saturn"], "father")
    E(v["jupiter"], v["sky"], "lives", reason="loves fresh breezes")
    E(v["jupiter"], v["neptune"], "brother")
    E(v["jupiter"], v["pluto"], "brother")
    E(v["neptune"], v["sea"], "lives", reason="loves waves")
    E(v["neptune"], v["jupiter"], "brother")
    E(v["neptune"], v["pluto"], "brother")
    E(v["hercules"], v["jupiter"], "father")
    E(v["hercules"], v["alcmene"], "mother")
    E(v["hercules"], v["nemean"], "battled", time=1)
    E(v["hercules"], v["hydra"], "battled", time=2)
    E(v["hercules"], v["cerberus"], "battled", time=12)
    E(v["pluto"], v["jupiter"], "brother")
    E(v["pluto"], v["neptune"], "brother")
    E(v["pluto"], v["tartarus"], "lives", reason="no fear of death")
    E(v["pluto"], v["cerberus"], "pet")
    E(v["cerberus"], v["tartarus"], "lives")
    return v
