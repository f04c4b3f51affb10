"""Weighted ShortestDistance with an unbounded hop count: near-far delta-stepping (jg_traverse.hip
sd_delta_stepping) against the oracle's superstep restatement
(oracle/jg_oracle.c jo_shortest_distance, ShortestDistanceVertexProgram.java:112-146), bit for bit.

The gate: one shard, maxDepth >= rows - 1 (the hop bound cannot bind) and no negative weight; otherwise
the frontier Bellman-Ford supersteps run (Tune::sd_delta = 0 forces them).  Each test compares both
paths with the oracle on the same graph, and one checks that the delta path really ran (its pass count
with delta = 1 is the number of distinct distances, far above the superstep count).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DEPTH_INF = 2**31 - 1


@pytest.fixture(scope="module")
def ctx():
    import janusgraph_amd as jg
    c = jg.Context((0,))
    yield c
    c.close()


@pytest.fixture(scope="module")
def rmat12(oracle_lib):
    n = 1 << 12
    s, t = oracle_lib.rmat_edges(12, 16, 21)
    vid = (np.random.default_rng(3).permutation(n).astype(np.int64) + 1) << 8
    return n, vid, s.astype(np.int32), t.astype(np.int32)


def run_sd(g, seed_vid, max_depth, delta, dist32=2):
    from janusgraph_amd import _lib
    try:
        _lib.tune_set("sd_delta", delta)
        _lib.tune_set("sd_dist32", dist32)
        return g.shortest_distance(seed_vid, max_depth)
    finally:
        _lib.tune_set("sd_delta", -1)
        _lib.tune_set("sd_dist32", 1)


@pytest.mark.parametrize("delta", [-1, 1, 3, 64, 100000])
def test_delta_stepping_matches_oracle(ctx, oracle_lib, rmat12, delta):
    """Weights 0..39 (zero weights too: rows relaxed again inside their bucket)."""
    import janusgraph_amd as jg
    n, vid, s, t = rmat12
    w = np.random.default_rng(5).integers(0, 40, len(s)).astype(np.int32)
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    seed = int(t[0])
    want = oracle_lib.shortest_distance(n, s, t, seed, DEPTH_INF, w)
    got = run_sd(g, vid[seed], DEPTH_INF, delta)
    np.testing.assert_array_equal(got, want)
    assert (got > 0).sum() > n // 8
    g.close()


def test_delta_path_runs(ctx, oracle_lib, rmat12):
    """delta = 1 with weights >= 1: one pass per distinct distance, many more than the supersteps."""
    import janusgraph_amd as jg
    n, vid, s, t = rmat12
    w = np.random.default_rng(6).integers(1, 30, len(s)).astype(np.int32)
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    seed = int(t[0])
    want = oracle_lib.shortest_distance(n, s, t, seed, DEPTH_INF, w)
    bf = run_sd(g, vid[seed], DEPTH_INF, 0)
    bf_levels = ctx.stats()["levels"]
    ds = run_sd(g, vid[seed], DEPTH_INF, 1)
    ds_passes = ctx.stats()["levels"]
    np.testing.assert_array_equal(bf, want)
    np.testing.assert_array_equal(ds, want)
    distinct = len(np.unique(want[want >= 0]))
    assert ds_passes >= distinct > bf_levels
    assert ctx.stats()["supersteps"] == DEPTH_INF
    g.close()


@pytest.mark.parametrize("slack", [0, 1, 2])
def test_hop_bound_gate(ctx, oracle_lib, slack):
    """A path 0 <- 1 <- ... <- n-1 of weight-1 edges (each edge u -> u-1 carries the seed's distance one
    hop further) plus heavy shortcuts: maxDepth = rows - 1 (delta path) reaches the far end along the
    path, rows - 2 / rows - 3 (supersteps) must take the shortcuts."""
    import janusgraph_amd as jg
    n = 60
    s = list(range(1, n))
    t = list(range(0, n - 1))
    w = [1] * (n - 1)
    for a in range(5, n, 7):  # a -> 0 at weight 1000: one hop from the seed
        s.append(a)
        t.append(0)
        w.append(1000)
    s, t, w = np.array(s, np.int32), np.array(t, np.int32), np.array(w, np.int32)
    vid = (np.arange(n, dtype=np.int64) + 11) << 8
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    md = n - 1 - slack
    want = oracle_lib.shortest_distance(n, s, t, 0, md, w)
    np.testing.assert_array_equal(run_sd(g, vid[0], md, -1), want)
    np.testing.assert_array_equal(run_sd(g, vid[0], md, 0), want)
    if slack == 0:
        np.testing.assert_array_equal(want, np.arange(n))
    else:
        assert want[n - 1] > n - 1  # the bound binds: a shortcut was needed
    g.close()


def test_negative_weights_take_the_supersteps(ctx, oracle_lib):
    """A negative weight closes the gate (delta-stepping needs weights >= 0); on a DAG (edges from a
    higher to a lower index: the supersteps converge) the unbounded result is the oracle's."""
    import janusgraph_amd as jg
    rng = np.random.default_rng(8)
    n, m = 2000, 20000
    a, b = rng.integers(0, n, m), rng.integers(0, n, m)
    s, t = np.maximum(a, b).astype(np.int32), np.minimum(a, b).astype(np.int32)
    keep = s != t
    s, t = s[keep], t[keep]
    w = rng.integers(-4, 9, len(s)).astype(np.int32)
    vid = (rng.permutation(n).astype(np.int64) + 1) << 8
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    got = run_sd(g, vid[0], DEPTH_INF, -1)
    np.testing.assert_array_equal(got, want)
    assert ((got < 0) & (got != jg.DIST_ABSENT)).any()
    g.close()


def test_absent_weights_and_unreached_seed(ctx, oracle_lib, rmat12):
    """An absent weight on an edge the run crosses fails it (ShortestDistanceVertexProgram.java:69),
    one out of an unreached row does not; a seed without in-edges reaches only itself."""
    import janusgraph_amd as jg
    o = oracle_lib
    n, vid, s, t = rmat12
    w = np.random.default_rng(9).integers(0, 7, len(s)).astype(np.int32)
    seed = int(t[0])
    crossed = w.copy()
    crossed[np.flatnonzero(t == seed)[0]] = jg.WEIGHT_ABSENT
    with pytest.raises(ValueError):
        o.shortest_distance(n, s, t, seed, DEPTH_INF, crossed)
    g = ctx.build(vid, vid[s], vid[t], weight=crossed, flags=jg.ADJ_IN | jg.ADJ_OUT)
    with pytest.raises(jg.JanusGpuError) as e:
        run_sd(g, vid[seed], DEPTH_INF, -1)
    assert "weight property" in str(e.value)
    g.close()
    reach = o.shortest_distance(n, s, t, seed, DEPTH_INF, w)
    far = np.flatnonzero(reach[t] == jg.DIST_ABSENT)
    if len(far):
        harmless = w.copy()
        harmless[far[0]] = jg.WEIGHT_ABSENT
        g = ctx.build(vid, vid[s], vid[t], weight=harmless, flags=jg.ADJ_IN | jg.ADJ_OUT)
        np.testing.assert_array_equal(run_sd(g, vid[seed], DEPTH_INF, -1),
                                      o.shortest_distance(n, s, t, seed, DEPTH_INF, harmless))
        g.close()
    lone = int(np.setdiff1d(np.arange(n), t)[0])  # no in-edge: nothing carries its distance on
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    got = run_sd(g, vid[lone], DEPTH_INF, -1)
    np.testing.assert_array_equal(got, o.shortest_distance(n, s, t, lone, DEPTH_INF, w))
    assert (got != jg.DIST_ABSENT).sum() == 1 and got[lone] == 0
    g.close()


def test_delta_stepping_rmat16(ctx, oracle_lib):
    """RMAT-16 with weights 1..255 (Graph500 SSSP style), unbounded: delta path vs oracle."""
    import janusgraph_amd as jg
    n = 1 << 16
    s, t = oracle_lib.rmat_edges(16, 16, 13)
    s, t = s.astype(np.int32), t.astype(np.int32)
    w = np.random.default_rng(10).integers(1, 256, len(s)).astype(np.int32)
    vid = (np.random.default_rng(16).permutation(n).astype(np.int64) + 1) << 8
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN)
    seed = int(np.bincount(t, minlength=n).argmax())
    want = oracle_lib.shortest_distance(n, s, t, seed, DEPTH_INF, w)
    got = run_sd(g, vid[seed], DEPTH_INF, -1)
    np.testing.assert_array_equal(got, want)
    assert (got > 0).sum() > n // 4
    g.close()


@pytest.mark.parametrize("delta,dist32", [(-1, 2), (32, 2), (-1, 0)])
def test_delta_stepping_rmat20_matches_oracle(ctx, oracle_lib, delta, dist32):
    """delta-stepping at RMAT-20 (the smallest size README and tools/sd_bench.py time),
    weights 1..255 (Graph500 SSSP style), unbounded hops, seeded at the row of largest in-degree, against
    the oracle's superstep restatement bit for bit (until now only the GPU superstep path was compared
    at this size: a self-comparison)."""
    import janusgraph_amd as jg
    n = 1 << 20
    s, t = oracle_lib.rmat_edges(20, 16, 0x55D + 20)
    s, t = s.astype(np.int32), t.astype(np.int32)
    w = np.random.default_rng(20).integers(1, 256, len(s)).astype(np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    seed = int(np.bincount(t, minlength=n).argmax())
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN)
    want = oracle_lib.shortest_distance(n, s, t, seed, DEPTH_INF, w)
    got = run_sd(g, vid[seed], DEPTH_INF, delta, dist32)
    np.testing.assert_array_equal(got, want)
    assert (want >= 0).sum() > n // 4  # most of the graph reached
    assert ctx.stats()["levels"] > 1
    g.close()


@pytest.mark.parametrize("wpath", [0, 1, 5])
def test_long_path_crosses_many_batches(ctx, oracle_lib, wpath):
    """A 3000-row path (the hop-gate test's edge direction) in shuffled ids, plus random edges of weight
    0..63 that shorten nothing: thousands of buckets (weight 1, delta 1) or of passes inside one bucket
    (weight 0), so the device-side step rings wrap many times and each call runs many host batches.  The
    delta path (auto delta and delta = 1, 32- and 64-bit distances) and the Bellman-Ford supersteps
    (delta = 0, one superstep per hop: the superstep ring wraps too; also with a hop bound that binds)
    all equal the oracle."""
    import janusgraph_amd as jg
    n = 3000
    rng = np.random.default_rng(40 + wpath)
    a, b = rng.integers(0, n, 400), rng.integers(0, n, 400)
    # the extra edges run from a lower to a higher row: against the path's flow, so they shorten nothing
    s = np.concatenate([np.arange(1, n), np.minimum(a, b)]).astype(np.int32)
    t = np.concatenate([np.arange(0, n - 1), np.maximum(a, b)]).astype(np.int32)
    w = np.concatenate([np.full(n - 1, wpath), rng.integers(0, 64, 400)]).astype(np.int32)
    keep = s != t
    s, t, w = s[keep], t[keep], w[keep]
    vid = (rng.permutation(n).astype(np.int64) + 3) << 8
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    np.testing.assert_array_equal(want, wpath * np.arange(n))
    for delta in (-1, 1, 0):
        np.testing.assert_array_equal(run_sd(g, vid[0], DEPTH_INF, delta), want)
    np.testing.assert_array_equal(run_sd(g, vid[0], DEPTH_INF, 1, 0), want)  # 64-bit distances
    bounded = oracle_lib.shortest_distance(n, s, t, 0, n // 2, w)
    assert (bounded == jg.DIST_ABSENT).sum() == n - 1 - n // 2
    np.testing.assert_array_equal(run_sd(g, vid[0], n // 2, -1), bounded)
    g.close()


@pytest.mark.parametrize("wexp", [28, 30])
def test_distance_width_gate(ctx, oracle_lib, wexp):
    """Tune::sd_dist32 (2: 32 bits at any size when safe, 0: never, 1: from 2^23 rows): 32-bit distances only
    when rows x the largest weight stays below 2^32 - 1.  A
    12-row path of weight-2^wexp edges plus a few edges that shorten nothing: 2^28 keeps 32 bits with distances past
    2^31 (unsigned), 2^30 needs 64 bits (distances past 2^32); both equal the oracle, with 32 bits off too."""
    import janusgraph_amd as jg
    n = 12
    rng = np.random.default_rng(wexp)
    a, b = rng.integers(0, n, 6), rng.integers(0, n, 6)
    s = list(range(1, n)) + list(np.minimum(a, b))  # extra edges from a lower to a higher row: no shortcut
    t = list(range(0, n - 1)) + list(np.maximum(a, b))
    w = [1 << wexp] * (n - 1) + list(rng.integers(1 << (wexp - 1), 1 << wexp, 6))
    s, t, w = np.array(s, np.int32), np.array(t, np.int32), np.array(w, np.int32)
    vid = (np.arange(n, dtype=np.int64) + 5) << 8
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN | jg.ADJ_OUT)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    assert want.max() > (1 << 31)
    for dist32 in (2, 0, 1):
        np.testing.assert_array_equal(run_sd(g, vid[0], DEPTH_INF, -1, dist32), want)
    g.close()
