"""Generate the golden fixtures under tests/golden/ (committed together with this script).

Every fixture re-creates a known-answer test of the reference's own suite as DATA (vertex ids, edge
lists, weights) plus expected outputs, computed by the vertex-centric Python mirror of Fulgora
(oracle/pymirror.py) and, where the reference test states one, by the test's closed form:

  pr_tree        janusgraph-backend-testutils/.../olap/OLAPTest.java:570-655  (testPageRank:
                 branch 6, diameter 5, child->parent "likes", iterations(10), vertexCount(numV),
                 closed form pr[d] = (1-a)/N + a*6*pr[d+1], pr[5] = (1-a)/N)
  sssp_tree      OLAPTest.java:657-714 (testShortestDistance: growVertex maxDepth 16, maxBranch 5,
                 weights 1..3 on "distance", maxDepth+4 supersteps; DISTANCE == stored depth)
  cc_kat         OLAPTest.java:736-778 (testConnectedComponent: 0->1->2 plus an isolated vertex)
  spvp_diamond   OLAPTest.java:716-734 (testShortestPath: v1->{v2,v3}->v4, one path v1..v2 of 2)
  gods           core/example/GraphOfTheGodsFactory.java:116-151 (12 vertices, 17 edges; config #1
                 of BASELINE.json: PageRank 30 iterations)
  random_*       small MULTI graphs with self-loops and ghost edges (mirror outputs)

Vertex ids follow JanusGraph's user-id layout at the default 32 partitions: IDManager.toVertexId(i)
= i << 8 (core/graphdb/idmanagement/IDManager.java:578-582).  Java's Random is re-implemented so the
randomly grown trees follow the same draw sequence shape as the reference (including the
re-evaluated loop bound of growVertex).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pymirror as pm  # noqa: E402


def to_vertex_id(i: int) -> int:
    return i << 8


class JavaRandom:
    """java.util.Random (48-bit LCG) — nextInt(bound) as in the JDK."""

    def __init__(self, seed):
        self.seed = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)

    def _next(self, bits):
        self.seed = (self.seed * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        r = self.seed >> (48 - bits)
        if r & (1 << (bits - 1)):
            r -= 1 << bits
        return r

    def next_int(self, bound):
        r = self._next(31)
        m = bound - 1
        if bound & m == 0:
            return (bound * r) >> 31
        u = r
        while True:
            r = u % bound
            if u - r + m < (1 << 31):
                return r
            u = self._next(31)


def save(name, meta, **arrays):
    np.savez(os.path.join(HERE, f"{name}.npz"), **{k: np.asarray(v) for k, v in arrays.items()})
    with open(os.path.join(HERE, f"{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def arrays_of(graph: pm.MiniGraph):
    vid = np.array(graph.vertices, np.int64)
    src = np.array([e.src for e in graph.edges], np.int64)
    dst = np.array([e.dst for e in graph.edges], np.int64)
    return vid, src, dst


def run_pr(graph, damping, iterations, vertex_count):
    props, it = pm.Engine(graph).run(pm.PageRankProgram(damping, iterations, vertex_count))
    rank = np.array([props[v].get("pageRank", np.nan) for v in graph.vertices], np.float64)
    ec = np.array([props[v].get("edgeCount", np.nan) for v in graph.vertices], np.float64)
    return rank, ec, it


def run_sd(graph, seed, max_depth, unit=False):
    props, it = pm.Engine(graph).run(pm.ShortestDistanceProgram(seed, max_depth, unit_weights=unit))
    return np.array([props[v].get("distance", -1) for v in graph.vertices], np.int64), it


def run_cc(graph):
    props, it = pm.Engine(graph).run(pm.ConnectedComponentProgram())
    return np.array([int(props[v]["component"]) for v in graph.vertices], np.int64), it


def pr_tree():
    branch, diameter, alpha = 6, 5, 0.85
    num_v = (branch ** (diameter + 1) - 1) // (branch - 1)
    vertices, edges, dist = [], [], []

    def add_vertex():
        vertices.append(to_vertex_id(len(vertices) + 1))
        return vertices[-1]

    def expand(v, distance):
        dist.append((v, distance))
        if distance < diameter:
            for _ in range(branch):
                u = add_vertex()
                edges.append((u, v))  # u.addEdge("likes", v)
                expand(u, distance + 1)

    expand(add_vertex(), 0)
    assert len(vertices) == num_v
    depth_of = dict(dist)
    correct = [0.0] * (diameter + 1)
    for i in range(diameter, -1, -1):
        pr = (1.0 - alpha) / num_v
        if i < diameter:
            pr += alpha * branch * correct[i + 1]
        correct[i] = pr
    g = pm.MiniGraph(vertices, edges)
    rank, ec, it = run_pr(g, alpha, 10, num_v)
    depth = np.array([depth_of[v] for v in vertices], np.int32)
    closed = np.array([correct[d] for d in depth], np.float64)
    assert np.allclose(rank, closed, rtol=1e-12, atol=0), "mirror disagrees with the OLAPTest closed form"
    vid, src, dst = arrays_of(g)
    save("pr_tree", {"damping": alpha, "iterations": 10, "vertex_count": num_v, "supersteps": it,
                     "source": "OLAPTest.java:589-655"},
         vid=vid, src=src, dst=dst, depth=depth, rank=rank, edge_count=ec, closed_form=closed)


def sssp_tree(seed=20171):
    rnd = JavaRandom(seed)
    max_depth, max_branch = 16, 5
    vertices, edges, w, dist = [], [], [], []

    def add_vertex():
        vertices.append(to_vertex_id(len(vertices) + 1))
        return vertices[-1]

    def grow(v, depth):
        dist.append((v, depth))
        total = 1
        if depth >= max_depth:
            return total
        i = 0
        while i < rnd.next_int(max_branch) + 1:  # bound re-drawn every iteration, as in Java
            d = rnd.next_int(3) + 1
            n = add_vertex()
            edges.append(pm.Edge(n, v, "connect", {"distance": d}))
            w.append(d)
            total += grow(n, depth + d)
            i += 1
        return total

    root = add_vertex()
    num_v = grow(root, 0)
    assert num_v == len(vertices)
    g = pm.MiniGraph(vertices, edges)
    got, it = run_sd(g, root, max_depth + 4)
    depth_of = dict(dist)
    stored = np.array([depth_of[v] for v in vertices], np.int64)
    assert (got == stored).all(), "mirror disagrees with OLAPTest.testShortestDistance"
    vid, src, dst = arrays_of(g)
    save("sssp_tree", {"seed_vid": int(root), "max_depth": max_depth + 4, "supersteps": it,
                       "source": "OLAPTest.java:657-714", "java_random_seed": seed},
         vid=vid, src=src, dst=dst, weight=np.array(w, np.int32), distance=got)


def cc_kat():
    # v1 -knows-> v2 -knows-> v3, isolated vertex; ids as an allocator might hand them out
    vertices = [to_vertex_id(i) for i in (3, 7, 12, 40)]
    edges = [(vertices[0], vertices[1]), (vertices[1], vertices[2])]
    g = pm.MiniGraph(vertices, edges)
    comp, it = run_cc(g)
    assert comp[3] == vertices[3] and comp[0] == comp[1] == comp[2]
    vid, src, dst = arrays_of(g)
    save("cc_kat", {"supersteps": it, "source": "OLAPTest.java:736-778"}, vid=vid, src=src, dst=dst,
         component=comp)


def spvp_diamond():
    vertices = [to_vertex_id(i) for i in (1, 2, 3, 4)]
    v1, v2, v3, v4 = vertices
    g = pm.MiniGraph(vertices, [(v1, v2), (v1, v3), (v2, v4), (v3, v4)])
    d = pm.bfs_depth(g, v1, pm.BOTH)
    depth = np.array([d[v] for v in vertices], np.int32)
    vid, src, dst = arrays_of(g)
    save("spvp_diamond", {"source_vid": v1, "target_vid": v2, "expected_paths": [[v1, v2]],
                          "source": "OLAPTest.java:716-734"}, vid=vid, src=src, dst=dst, depth=depth)


GODS_VERTICES = ["saturn", "sky", "sea", "jupiter", "neptune", "hercules", "alcmene", "pluto", "nemean",
                 "hydra", "cerberus", "tartarus"]
GODS_EDGES = [("jupiter", "saturn", "father"), ("jupiter", "sky", "lives"), ("jupiter", "neptune", "brother"),
              ("jupiter", "pluto", "brother"), ("neptune", "sea", "lives"), ("neptune", "jupiter", "brother"),
              ("neptune", "pluto", "brother"), ("hercules", "jupiter", "father"), ("hercules", "alcmene", "mother"),
              ("hercules", "nemean", "battled"), ("hercules", "hydra", "battled"), ("hercules", "cerberus", "battled"),
              ("pluto", "jupiter", "brother"), ("pluto", "neptune", "brother"), ("pluto", "tartarus", "lives"),
              ("pluto", "cerberus", "pet"), ("cerberus", "tartarus", "lives")]


def gods():
    vid_of = {name: to_vertex_id(i + 1) for i, name in enumerate(GODS_VERTICES)}
    vertices = [vid_of[n] for n in GODS_VERTICES]
    edges = [pm.Edge(vid_of[a], vid_of[b], lab) for a, b, lab in GODS_EDGES]
    g = pm.MiniGraph(vertices, edges)
    rank, ec, it = run_pr(g, 0.85, 30, 12)
    comp, cc_it = run_cc(g)
    d = pm.bfs_depth(g, vid_of["jupiter"], pm.BOTH)
    depth = np.array([d[v] for v in vertices], np.int32)
    sd, _ = run_sd(g, vid_of["saturn"], 10, unit=True)
    vid, src, dst = arrays_of(g)
    save("gods", {"names": GODS_VERTICES, "damping": 0.85, "iterations": 30, "vertex_count": 12,
                  "pr_supersteps": it, "cc_supersteps": cc_it, "bfs_source": vid_of["jupiter"],
                  "sd_seed": vid_of["saturn"], "sd_max_depth": 10,
                  "source": "GraphOfTheGodsFactory.java:116-151"},
         vid=vid, src=src, dst=dst, rank=rank, edge_count=ec, component=comp, depth=depth, sd_unit=sd)


def random_graph(name, n, m, seed, ghosts=5, loops=4):
    rng = np.random.default_rng(seed)
    ids = np.sort(rng.choice(np.arange(1, 50 * n), size=n, replace=False)).astype(np.int64) << 8
    rng.shuffle(ids)
    src = ids[rng.integers(0, n, m)]
    dst = ids[rng.integers(0, n, m)]
    ls = rng.integers(0, n, loops)
    src = np.concatenate([src, ids[ls], src[:3]])  # self-loops and multi-edges
    dst = np.concatenate([dst, ids[ls], dst[:3]])
    ghost = (np.arange(1, ghosts + 1, dtype=np.int64) * 7 + 50 * n) << 8  # ids not in V
    gsrc = np.concatenate([src, ghost, ids[:ghosts]])
    gdst = np.concatenate([dst, ids[-ghosts:], ghost])
    weight = rng.integers(1, 4, len(gsrc)).astype(np.int32)
    edges = [pm.Edge(int(a), int(b), "e", {"distance": int(w)}) for a, b, w in zip(gsrc, gdst, weight)]
    g = pm.MiniGraph([int(x) for x in ids], edges)
    rank, ec, it = run_pr(g, 0.85, 12, n)
    seed_v = int(ids[0])
    sd, _ = run_sd(g, seed_v, 6)
    comp, cc_it = run_cc(g)
    d = pm.bfs_depth(g, seed_v, pm.BOTH)
    depth = np.array([d[v] for v in g.vertices], np.int32)
    save(name, {"damping": 0.85, "iterations": 12, "vertex_count": n, "pr_supersteps": it, "cc_supersteps": cc_it,
                "seed_vid": seed_v, "sd_max_depth": 6, "ghost_edges": 2 * ghosts},
         vid=ids, src=gsrc, dst=gdst, weight=weight, rank=rank, edge_count=ec, distance=sd, component=comp,
         depth=depth)


def main():
    pr_tree()
    sssp_tree()
    cc_kat()
    spvp_diamond()
    gods()
    random_graph("random_small", 60, 150, 7)
    random_graph("random_medium", 400, 2400, 11)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
