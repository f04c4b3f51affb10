"""GPU parity of the narrow bit-parallel BFS (jg_narrow.hip: 2..8 sources on one shard, one frontier byte
per row, each source choosing its own direction every level) against the oracle's single-source BFS
(oracle/jg_oracle.c jo_bfs, restating ShortestPathVertexProgram's hop depths under Fulgora's forced BOTH
scope, FulgoraGraphComputer.java:249-253).  Bit-exact depths for every source row.

Paths covered: pure top-down levels, pure bottom-up levels, mixed levels (some sources pushed, some
pulled), the queue rebuilt by a scan when a source changes direction, pass B of the bottom-up rows
(wave per row), sources that are isolated / in a small component / duplicated / not vertices, hub
sources (bottom-up from level 0), directed OUT and IN traversals, depth bounds, deep traversals past the
preallocated level arrays, jg_bfs_keep, and the engine off (bfs_narrow 0: the 64-source engine) for
the same stats of depths.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def graph_case(o, scale, seed=7):
    """RMAT-`scale` with sparse JanusGraph-style ids, plus an isolated vertex and a two-vertex component."""
    s0, t0 = o.rmat_edges(scale, 16, seed)
    n0 = 1 << scale
    n = n0 + 3
    rng = np.random.default_rng(scale)
    vid = np.concatenate([(rng.permutation(n0).astype(np.int64) + 1) << 8,
                          (np.arange(3, dtype=np.int64) + n0 + 1) << 8 | 7])
    ds = np.concatenate([s0, np.array([n0 + 1], s0.dtype)])
    dd = np.concatenate([t0, np.array([n0 + 2], t0.dtype)])
    return n, n0, vid, ds, dd


def knobs(pairs):
    from janusgraph_amd import _lib
    for k, v in pairs:
        _lib.tune_set(k, v)


DEFAULTS = [("bfs_narrow", 1), ("nb_alpha", 30), ("nb_first", 16), ("bfs_beta", 24)]


@pytest.fixture(scope="module")
def case15(oracle_lib):
    import janusgraph_amd as jg
    n, n0, vid, ds, dd = graph_case(oracle_lib, 15)
    ctx = jg.Context((0,))
    g = ctx.build(vid, vid[ds], vid[dd], flags=1 | 2 | 4)
    deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
    yield dict(n=n, n0=n0, vid=vid, ds=ds, dd=dd, g=g, ctx=ctx, deg=deg)
    g.close()
    ctx.close()


def check_rows(o, c, srcs, direction=3, max_depth=-1):
    g = c["g"]
    got = g.bfs(c["vid"][srcs], direction, max_depth)
    levels = c["ctx"].stats()["levels"]
    deepest = 0
    for k, s in enumerate(srcs):
        want = o.bfs(c["n"], c["ds"], c["dd"], int(s), direction, max_depth)
        np.testing.assert_array_equal(got[k], want,
                                      err_msg=f"source {k} ({s}), direction {direction}, max_depth {max_depth}")
        deepest = max(deepest, int(want.max()))
    # the level that finds nothing new ends the traversal; a bound stops it at max_depth
    assert levels == (deepest + 1 if max_depth < 0 else min(deepest + 1, max_depth)), (levels, deepest)
    return got


@pytest.mark.parametrize("variant", ["default", "all_top_down", "bottom_up_early", "first4", "first64",
                                     "beta_high"])
def test_narrow_sources_vs_oracle(oracle_lib, case15, variant):
    """2..8 sources (giant component, hubs, an isolated vertex, the small component) under knob settings
    that force each level kind: nb_alpha 1e6 keeps every source top-down, nb_alpha 1 turns a source
    bottom-up as soon as its frontier has an entry (hub sources from level 0), nb_first 4 / 64 moves rows
    between the bottom-up passes, bfs_beta 1e6 keeps bottom-up sources bottom-up to the end."""
    c = case15
    pairs = {"default": [], "all_top_down": [("nb_alpha", 1000000)], "bottom_up_early": [("nb_alpha", 1)],
             "first4": [("nb_first", 4)], "first64": [("nb_first", 64)],
             "beta_high": [("bfs_beta", 1000000)]}[variant]
    rng = np.random.default_rng(5)
    conn = np.flatnonzero(c["deg"][:c["n0"]] > 0)
    hubs = np.argsort(-c["deg"][:c["n0"]])[:3]
    try:
        knobs(pairs)
        for ns in range(2, 9):
            srcs = rng.choice(conn, ns, replace=False)
            check_rows(oracle_lib, c, srcs)
        # hubs, the isolated vertex, the small component, a duplicate
        srcs = np.array([hubs[0], c["n0"], c["n0"] + 2, hubs[1], conn[7], conn[7], hubs[2], conn[99]])
        check_rows(oracle_lib, c, srcs)
        for md in (0, 1, 2, 3):
            check_rows(oracle_lib, c, srcs[:5], 3, md)
    finally:
        knobs(DEFAULTS)


@pytest.mark.parametrize("direction", [1, 2])
def test_narrow_directed(oracle_lib, case15, direction):
    """OUT (push over OUT, pull over IN) and IN traversals, default and bottom-up-early settings."""
    c = case15
    srcs = np.unique(c["ds"])[::211][:8]
    try:
        for pairs in ([], [("nb_alpha", 1)], [("nb_alpha", 1000000)]):
            knobs(pairs)
            check_rows(oracle_lib, c, srcs[:6], direction)
            check_rows(oracle_lib, c, srcs, direction, 2)
    finally:
        knobs(DEFAULTS)


def test_narrow_missing_source_and_stats(oracle_lib, case15):
    """A vid that is not a vertex gives an all -1 row; the engine off (the 64-source engine) gives the same
    depths; the stats count levels and examined entries."""
    c = case15
    g, ctx = c["g"], c["ctx"]
    srcs = np.flatnonzero(c["deg"] > 0)[[3, 500, 9000]]
    vids = np.concatenate([c["vid"][srcs], [12345]])
    got = g.bfs(vids, 3)
    st = ctx.stats()
    assert (got[3] == -1).all()
    assert st["levels"] >= 2 and st["edges_traversed"] > 0 and st["algorithmic_bytes"] > 0
    try:
        knobs([("bfs_narrow", 0)])
        ref = g.bfs(vids, 3)
    finally:
        knobs(DEFAULTS)
    np.testing.assert_array_equal(got, ref)


def test_narrow_keep_rows(oracle_lib, case15):
    c = case15
    g = c["g"]
    srcs = np.flatnonzero(c["deg"] > 0)[[1, 77, 1234, 4321]]
    g.bfs_keep(c["vid"][srcs], 3)
    for k, s in enumerate(srcs):
        np.testing.assert_array_equal(g.bfs_kept_row(k), oracle_lib.bfs(c["n"], c["ds"], c["dd"], int(s), 3))
    g.bfs_kept_release()


def test_narrow_deep_path(oracle_lib):
    """A 300-vertex path plus a cycle: ~300 levels, past the 16 preallocated level arrays and the
    first level batches; sources at both ends, in the middle and on the cycle."""
    import janusgraph_amd as jg
    n = 340
    a = np.arange(299)
    cyc = np.arange(300, 340)
    ds = np.concatenate([a, cyc]).astype(np.int32)
    dd = np.concatenate([a + 1, np.roll(cyc, -1)]).astype(np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    ctx = jg.Context((0,))
    try:
        g = ctx.build(vid, vid[ds], vid[dd], flags=1 | 2 | 4)
        for srcs in ([0, 299], [0, 150, 299, 310], [5, 6, 7, 8, 9, 10, 11, 12]):
            for direction, md in ((3, -1), (1, -1), (3, 200)):
                got = g.bfs(vid[srcs], direction, md)
                for k, s in enumerate(srcs):
                    np.testing.assert_array_equal(got[k], oracle_lib.bfs(n, ds, dd, s, direction, md),
                                                  err_msg=f"sources {srcs} source {s} direction {direction}")
        g.close()
    finally:
        ctx.close()


def test_narrow_rmat20_bench_sources(oracle_lib):
    """configs[1]'s graph (RMAT-20 from the device generator) from 8 bench-style sources: every row equal to
    the oracle's bit-parallel checker (jo_msbfs_csr, pinned by tests/test_oracle_fullsize.py)."""
    import janusgraph_amd as jg
    o = oracle_lib
    scale = 20
    n = 1 << scale
    s, d = o.rmat_edges(scale, 16, 0x5EED + scale)
    ptr, adj = o.csr_unordered(n, s.astype(np.int32), d.astype(np.int32), both=True)
    cand = np.flatnonzero(np.diff(ptr) > 0)
    srcs = np.random.default_rng(20).choice(cand, 8, replace=False).astype(np.int64)
    want = o.msbfs_csr(n, ptr, adj, srcs)
    ctx = jg.Context((0,))
    try:
        g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_BOTH)
        for k0, k1 in ((0, 8), (0, 2), (3, 8)):
            got = g.bfs(srcs[k0:k1], jg.DIR_BOTH)
            for k in range(k1 - k0):
                assert np.array_equal(got[k], want[k0 + k]), f"source {k0 + k}"
        g.close()
    finally:
        ctx.close()
