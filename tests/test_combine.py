"""Combiner vertex programs: OLAPTest.DegreeCounter / DegreeMapper and the sum/min/max family
(jg_combine_steps).

Reference: janusgraph-test/src/main/java/org/janusgraph/olap/OLAPTest.java
  generateRandomGraph :114-140 (vertex i gets i+1 random out-edges "knows"), degreeCounting :283-310
  (DegreeCounter(1) + DegreeMapper: degree == uid, total numV(numV+1)/2, getIteration() == 1),
  degreeCountingDistance :331-369 (DegreeCounter(2) under every ResultMode: the sum over out-neighbours
  of their out-degree, getIteration() == 2), DegreeCounter :424-503, DegreeMapper :505-540.
Oracles: oracle/pymirror.py DegreeCounterProgram (the vertex-centric engine, pinned here against the
reference's own assertions) and oracle.combine_steps (numpy; pinned against the mirror).
"""
import random

import numpy as np
import pytest

from oracle import pymirror as pm


def random_graph(num_v, seed=0):
    """generateRandomGraph: vertex i (uid i+1) gets i+1 out-edges to uniformly random vertices."""
    rnd = random.Random(seed)
    edges = []
    for i in range(num_v):
        for _ in range(i + 1):
            edges.append((i, rnd.randrange(num_v)))
    return edges


def test_mirror_degree_counter_matches_reference_assertions():
    num_v = 60
    edges = random_graph(num_v, 3)
    g = pm.MiniGraph(range(num_v), edges)
    props, it = pm.Engine(g).run(pm.DegreeCounterProgram(1))
    assert it == 1
    assert [props[v]["degree"] for v in range(num_v)] == [v + 1 for v in range(num_v)]
    assert sum(props[v]["degree"] for v in range(num_v)) == num_v * (num_v + 1) // 2
    props2, it2 = pm.Engine(g).run(pm.DegreeCounterProgram(2))
    assert it2 == 2
    out = {v: [b for a, b in edges if a == v] for v in range(num_v)}
    for v in range(num_v):  # degreeCountingDistance's actualDegree2
        assert props2[v]["degree"] == sum(len(out[w]) for w in out[v])


def _mixed_graph(n, m, seed):
    rng = np.random.default_rng(seed)
    s = rng.integers(0, n, m)
    t = rng.integers(0, n, m)
    t[: m // 20] = s[: m // 20]  # self-loops
    return s, t


@pytest.mark.parametrize("direction,scope", [(1, pm.IN), (2, pm.OUT), (3, pm.BOTH)])
@pytest.mark.parametrize("combiner", [0, 1, 2])
def test_numpy_oracle_matches_mirror(oracle_lib, direction, scope, combiner):
    n, m = 40, 150
    s, t = _mixed_graph(n, m, direction * 3 + combiner)
    init = np.random.default_rng(combiner).integers(-1000, 1000, n)
    fn = {0: lambda a, b: a + b, 1: min, 2: max}[combiner]
    steps = 3
    g = pm.MiniGraph(range(n), list(zip(s.tolist(), t.tolist())))
    prog = pm.DegreeCounterProgram(steps, fn, scope, 0)
    prog.initial = None
    # per-vertex initial messages: superstep 0 sends init[v]
    base_exec = prog.execute

    def execute(v, props, msgr, mem, gg):
        if mem.is_initial_iteration():
            msgr.send_message(prog.scope, int(init[v]))
        else:
            base_exec(v, props, msgr, mem, gg)
    prog.execute = execute
    props, _ = pm.Engine(g).run(prog)
    x, rec = oracle_lib.combine_steps(n, s, t, direction, combiner, steps, init)
    for v in range(n):
        if combiner == 0:  # a sum always sets the key (reduce(0, +))
            assert x[v] == props[v]["degree"], v
        elif "degree" in props[v]:
            assert rec[v] and x[v] == props[v]["degree"], v
        else:
            assert not rec[v]


def test_numpy_oracle_int32_wraps(oracle_lib):
    # one hub with 4 out-edges to vertices sending 2^30: the Java int sum wraps to 0
    x, _ = oracle_lib.combine_steps(5, [0, 0, 0, 0], [1, 2, 3, 4], 1, 0, 1, [0, 1 << 30, 1 << 30, 1 << 30, 1 << 30])
    assert x[0] == 0
    x, _ = oracle_lib.combine_steps(5, [0, 0, 0, 0], [1, 2, 3, 4], 1, 0, 1, [0, 1 << 30, 1 << 30, 1 << 30, 1 << 30],
                                    int32_wrap=False)
    assert x[0] == 1 << 32


def test_computer_refuses_without_gpu_only_on_submit():
    """DegreeCounter is recognised (no ProgramNotSupported at submit validation); length must be > 0."""
    import janusgraph_amd as jg
    with pytest.raises(ValueError):
        jg.DegreeCounter(0)
    assert isinstance(jg.DegreeCounter(2), jg.CombinerVertexProgram)


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [1, 2, 3])
@pytest.mark.parametrize("combiner", [0, 1, 2])
def test_gpu_combine_matches_oracle(oracle_lib, direction, combiner):
    import janusgraph_amd as jg
    scale = 12
    n = 1 << scale
    s, t = oracle_lib.rmat_edges(scale, 16, 5 + direction)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    rng = np.random.default_rng(combiner)
    init = rng.integers(-(1 << 31), 1 << 31, n)
    ctx = jg.Context((0,))
    g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    for steps, wrap in ((1, True), (3, True), (2, False)):
        x, rec = g.combine_steps(direction, combiner, steps, init, wrap)
        ref, rref = oracle_lib.combine_steps(n, s, t, direction, combiner, steps, init, wrap)
        np.testing.assert_array_equal(x, ref)
        np.testing.assert_array_equal(rec, rref)
    g.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_degree_counting():  # OLAPTest.degreeCounting :283-310
    import janusgraph_amd as jg
    num_v = 200
    g = jg.InMemoryGraph()
    vs = [g.add_vertex(uid=i + 1) for i in range(num_v)]
    for i, b in random_graph(num_v, 11):
        g.add_edge(vs[i], vs[b], "knows")
    computer = jg.GpuGraphComputer(g).resultMode(jg.ResultMode.NONE).workers(4)
    computer.program(jg.DegreeCounter())
    computer.mapReduce(jg.DegreeMapper())
    result = computer.submit().result()
    degrees = result.memory().get(jg.DegreeMapper.DEGREE_RESULT)
    assert len(degrees) == num_v
    total = 0
    for vid, degree in degrees.items():
        assert g.vertex(vid).value("uid") == degree
        total += degree
    assert total == num_v * (num_v + 1) // 2
    assert result.memory().getIteration() == 1


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["LOCALTX", "PERSIST", "NONE"])
def test_gpu_degree_counting_distance(mode):  # OLAPTest.degreeCountingDistance :331-369
    import janusgraph_amd as jg
    num_v = 100
    g = jg.InMemoryGraph()
    vs = [g.add_vertex(uid=i + 1) for i in range(num_v)]
    edges = random_graph(num_v, 5)
    for i, b in edges:
        g.add_edge(vs[i], vs[b], "knows")
    result = jg.GpuGraphComputer(g).resultMode(getattr(jg.ResultMode, mode)).workers(1).program(
        jg.DegreeCounter(2)).submit().result()
    assert result.memory().getIteration() == 2
    out = {v: [b for a, b in edges if a == v] for v in range(num_v)}
    if mode == "NONE":
        return
    view = result.graph()
    for i in range(num_v):
        want = sum(len(out[w]) for w in out[i])
        got = view.value(vs[i].id, "degree") if mode == "LOCALTX" else g.vertex(vs[i].id).value("degree")
        assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("shards,halo", [(2, 1), (3, 1), (8, 1), (3, 0)])
def test_gpu_combine_logical_shards(oracle_lib, shards, halo):
    """Sharded combiner supersteps (IN / BOTH through the halo exchange or the dense allgather, OUT
    through the allgather of owned slices) == the oracle."""
    import janusgraph_amd as jg
    scale = 12
    n = 1 << scale
    s, t = oracle_lib.rmat_edges(scale, 16, 21)
    vid = (np.random.default_rng(4).permutation(n).astype(np.int64) + 1) << 8
    init = np.random.default_rng(9).integers(-(1 << 31), 1 << 31, n)
    ctx = jg.Context((0,) * shards)
    jg._lib.tune_set("halo", halo)
    try:
        g = ctx.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
    finally:
        jg._lib.tune_set("halo", 1)
    for direction in (1, 2, 3):
        for combiner in (0, 1):
            x, rec = g.combine_steps(direction, combiner, 3, init, True)
            ref, rref = oracle_lib.combine_steps(n, s, t, direction, combiner, 3, init, True)
            np.testing.assert_array_equal(x, ref)
            np.testing.assert_array_equal(rec, rref)
    g.close()
    ctx.close()
