"""OLAPTest re-expressed against GpuGraphComputer (janusgraph-backend-testutils/.../olap/OLAPTest.java).

Same graphs, same programs, same assertions as the reference's tests, through the TinkerPop-style
API; every superstep runs in libjanusgpu on the GPU.
"""
import random

import numpy as np
import pytest

import janusgraph_amd as jg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = jg.Context((0,))
    yield c
    c.close()


def expand(g, v, distance, diameter, branch):  # OLAPTest.java:570-587
    v.properties["distance"] = distance
    if distance < diameter:
        for _ in range(branch):
            u = g.add_vertex()
            g.add_edge(u, v, "likes")
            expand(g, u, distance + 1, diameter, branch)


def test_page_rank(ctx):  # OLAPTest.testPageRank :589-655
    branch, diameter, alpha = 6, 5, 0.85
    num_v = (branch ** (diameter + 1) - 1) // (branch - 1)
    g = jg.InMemoryGraph()
    expand(g, g.add_vertex(), 0, diameter, branch)
    correct = [0.0] * (diameter + 1)
    for i in range(diameter, -1, -1):
        correct[i] = (1.0 - alpha) / num_v + (alpha * branch * correct[i + 1] if i < diameter else 0.0)
    computer = jg.GpuGraphComputer(g, context=ctx).resultMode(jg.ResultMode.NONE).workers(4)
    computer.program(jg.PageRankVertexProgram.build().iterations(10).vertexCount(num_v).dampingFactor(alpha).create(g))
    computer.mapReduce(jg.PageRankMapReduce.build().create())
    result = computer.submit().result()
    ranks = list(result.memory().get(jg.PageRankMapReduce.DEFAULT_MEMORY_KEY))
    assert len(ranks) == num_v and len({k for k, _ in ranks}) == num_v
    computed_sum = correct_sum = 0.0
    for vid, pr in ranks:
        d = g.vertex(vid).value("distance")
        assert abs(pr - correct[d]) <= 1e-9 * correct[d]  # per vertex (the reference asserts the sum)
        computed_sum += pr
        correct_sum += correct[d]
    assert abs(correct_sum - computed_sum) < 0.001
    assert result.memory().getIteration() == 10
    assert result.graph() is None  # ResultMode.NONE -> EmptyGraph


def grow_vertex(g, rnd, vertex, depth, max_depth, max_branch):  # OLAPTest.java:702-714
    vertex.properties["distance"] = depth
    total = 1
    if depth >= max_depth:
        return total
    i = 0
    while i < rnd.randrange(max_branch) + 1:
        dist = rnd.randrange(3) + 1
        n = g.add_vertex()
        g.add_edge(n, vertex, "connect", distance=dist)
        total += grow_vertex(g, rnd, n, depth + dist, max_depth, max_branch)
        i += 1
    return total


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_shortest_distance(ctx, seed):  # OLAPTest.testShortestDistance :657-700
    g = jg.InMemoryGraph()
    max_depth, max_branch = 16, 5
    vertex = g.add_vertex()
    num_v = grow_vertex(g, random.Random(seed), vertex, 0, max_depth, max_branch)
    computer = jg.GpuGraphComputer(g, context=ctx).resultMode(jg.ResultMode.NONE).workers(4)
    computer.program(jg.ShortestDistanceVertexProgram.build().seed(vertex.id).maxDepth(max_depth + 4).create(g))
    computer.mapReduce(jg.ShortestDistanceMapReduce.build().create())
    result = computer.submit().result()
    count = 0
    for vid, dist in result.memory().get(jg.ShortestDistanceMapReduce.DEFAULT_MEMORY_KEY):
        assert 0 <= dist < 2 ** 31 - 1
        assert g.vertex(vid).value("distance") == dist
        count += 1
    assert count == num_v and count > 0
    assert result.memory().getIteration() == max_depth + 4


def test_shortest_path(ctx):  # OLAPTest.testShortestPath :716-734
    g = jg.InMemoryGraph()
    v1, v2, v3, v4 = (g.add_vertex() for _ in range(4))
    g.add_edge(v1, v2, "E")
    g.add_edge(v1, v3, "E")
    g.add_edge(v2, v4, "E")
    g.add_edge(v3, v4, "E")
    vp = jg.ShortestPathVertexProgram.build().source(v1.id).target(v2.id).create(g)
    result = jg.GpuGraphComputer(g, context=ctx).program(vp).submit().result()
    paths = result.memory().get(jg.ShortestPathVertexProgram.SHORTEST_PATHS)
    assert len(paths) == 1 and len(paths[0]) == 2 and paths[0] == [v1.id, v2.id]
    # the diamond has two shortest v1..v4 paths
    vp = jg.ShortestPathVertexProgram.build().source(v1.id).target(v4.id).create(g)
    paths = jg.GpuGraphComputer(g, context=ctx).program(vp).submit().result().memory().get(vp.SHORTEST_PATHS)
    assert sorted(paths) == [[v1.id, v2.id, v4.id], [v1.id, v3.id, v4.id]]


def test_connected_component(ctx):  # OLAPTest.testConnectedComponent :736-778
    g = jg.InMemoryGraph()
    a, b, c = (g.add_vertex(id_prop=i) for i in range(3))
    g.add_edge(a, b, "knows")
    g.add_edge(b, c, "knows")
    isolated = g.add_vertex(id_prop=-1)
    vp = jg.ConnectedComponentVertexProgram.build().create(g)
    result = jg.GpuGraphComputer(g, context=ctx).program(vp).resultMode(jg.ResultMode.LOCALTX).submit().result()
    view = result.graph()
    key = jg.ConnectedComponentVertexProgram.COMPONENT
    assert view.value(isolated.id, key) == str(isolated.id)
    comps = [view.value(v.id, key) for v in (a, b, c)]
    assert comps[0] == comps[1] == comps[2] == min((str(v.id) for v in (a, b, c)))


def test_page_rank_persist_original(ctx):
    """ResultGraph.ORIGINAL + Persist.VERTEX_PROPERTIES writes the computed keys back (Fulgora :359-471)."""
    g = jg.InMemoryGraph()
    gods = jg.load_graph_of_the_gods(g)
    vp = jg.PageRankVertexProgram.build().iterations(30).vertexCount(12).create(g)
    result = jg.GpuGraphComputer(g, context=ctx).program(vp).resultMode(jg.ResultMode.PERSIST).submit().result()
    assert result.graph() is g
    assert gods["hercules"].value(jg.PageRankVertexProgram.OUTGOING_EDGE_COUNT) == 5.0
    assert gods["saturn"].value(jg.PageRankVertexProgram.PAGE_RANK) > gods["hercules"].value(
        jg.PageRankVertexProgram.PAGE_RANK)
    assert result.memory().getIteration() == 30 and result.memory().getRuntime() >= 0


def test_ghost_vertices_do_not_count(ctx):
    """A ghost row never executes; edges to it are not counted (VertexJobConverter.java:126-129)."""
    g = jg.InMemoryGraph()
    a, b, ghost = g.add_vertex(), g.add_vertex(), g.add_vertex()
    g.add_edge(a, b)
    g.add_edge(a, ghost)
    g.make_ghost(ghost)
    vp = jg.PageRankVertexProgram.build().iterations(3).vertexCount(2).create(g)
    view = jg.GpuGraphComputer(g, context=ctx).program(vp).resultMode(jg.ResultMode.LOCALTX).submit().result().graph()
    assert view.value(a.id, vp.OUTGOING_EDGE_COUNT) == 1.0
    assert ghost.id not in view.props


def test_exception_propagates_to_caller(ctx):  # OLAPTest.vertexProgramExceptionPropagatesToCaller :312-329
    """A message crossing an edge without the weight property fails the run through the Future, as
    edge.value(weightProperty) throws in Fulgora (ShortestDistanceVertexProgram.java:69); an edge no
    message crosses is harmless (VertexMemoryHandler.java:136-138 applies the edge function to
    present messages only)."""
    g = jg.InMemoryGraph()
    a, b, c = g.add_vertex(), g.add_vertex(), g.add_vertex()
    g.add_edge(a, b)               # never crossed: a pulls over a->b, b never sends
    g.add_edge(c, a, distance=-4)  # a negative distance is a distance, not "absent"
    vp = jg.ShortestDistanceVertexProgram.build().seed(a.id).maxDepth(3).create(g)
    view = jg.GpuGraphComputer(g, context=ctx).program(vp).resultMode(jg.ResultMode.LOCALTX).submit().result().graph()
    assert view.value(a.id, vp.DISTANCE) == 0 and view.value(c.id, vp.DISTANCE) == -4
    assert vp.DISTANCE not in view.properties(b.id)
    g.add_edge(b, a)               # crossed at superstep 1: b pulls a's message over b->a
    vp = jg.ShortestDistanceVertexProgram.build().seed(a.id).maxDepth(3).create(g)
    fut = jg.GpuGraphComputer(g, context=ctx).program(vp).submit()
    with pytest.raises(jg.JanusGpuError) as e:
        fut.result()
    assert "weight property" in str(e.value)


def test_rmat_pagerank_through_computer(ctx, oracle_lib):
    n = 1 << 12
    s, t = oracle_lib.rmat_edges(12, 16, 3)
    g = jg.InMemoryGraph(set_vertex_id=True)
    vs = [g.add_vertex(id=i + 1) for i in range(n)]
    for a, b in zip(s.tolist(), t.tolist()):
        g.add_edge(vs[a], vs[b])
    vp = jg.PageRankVertexProgram.build().iterations(20).vertexCount(n).create(g)
    view = jg.GpuGraphComputer(g, context=ctx).program(vp).resultMode(jg.ResultMode.LOCALTX).submit().result().graph()
    ref, _ = oracle_lib.pagerank(n, s.astype(np.int32), t.astype(np.int32), 0.85, n, 20)
    got = np.array([view.value(v.id, vp.PAGE_RANK) for v in vs])
    assert (np.abs(got - ref) / ref).max() <= 1e-9
