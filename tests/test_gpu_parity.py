"""GPU parity: libjanusgpu (HIP, gfx950) against the golden fixtures and the CPU oracle.

Bars (BASELINE.json north_star): bit-exact for BFS depths, component labels and integer distances;
per-vertex relative error <= 1e-9 for fp64 PageRank after a fixed iteration count.
"""
import json
import os

import numpy as np
import pytest

from oracle.oracle import golden_distance

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PR_RTOL = 1e-9  # north_star: per-vertex relative error <= 1e-9 (fp64)
ALL = 1 | 2 | 4


def golden(name):
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    return {k: z[k] for k in z.files}, meta


@pytest.fixture(scope="module")
def ctx():
    import janusgraph_amd as jg
    c = jg.Context((0,))
    yield c
    c.close()


def assert_pr_close(got, want):
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape
    nan_w = np.isnan(want)
    assert (np.isnan(got) == nan_w).all()
    g, w = got[~nan_w], want[~nan_w]
    rel = np.abs(g - w) / np.maximum(np.abs(w), 1e-300)
    assert rel.max(initial=0.0) <= PR_RTOL, f"max rel err {rel.max()}"


@pytest.mark.parametrize("name", ["gods", "pr_tree", "random_small", "random_medium"])
def test_pagerank_golden(ctx, name):
    d, meta = golden(name)
    g = ctx.build(d["vid"], d["src"], d["dst"], flags=ALL)
    rank, ec = g.pagerank(meta["damping"], meta["vertex_count"], meta["iterations"])
    assert_pr_close(rank, d["rank"])
    assert_pr_close(ec, d["edge_count"])
    if name == "pr_tree":  # OLAPTest.testPageRank closed form, asserted per vertex
        assert_pr_close(rank, d["closed_form"])
        assert abs(rank.sum() - d["closed_form"].sum()) < 0.001
    st = ctx.stats()
    assert st["supersteps"] == meta["iterations"]


def test_shortest_distance_golden_tree(ctx):
    d, meta = golden("sssp_tree")
    g = ctx.build(d["vid"], d["src"], d["dst"], weight=d["weight"], flags=ALL)
    dist = g.shortest_distance(meta["seed_vid"], meta["max_depth"])
    np.testing.assert_array_equal(dist, golden_distance(d["distance"]))


@pytest.mark.parametrize("name", ["random_small", "random_medium"])
def test_shortest_distance_golden_random(ctx, name):
    d, meta = golden(name)
    g = ctx.build(d["vid"], d["src"], d["dst"], weight=d["weight"], flags=ALL)
    np.testing.assert_array_equal(g.shortest_distance(meta["seed_vid"], meta["sd_max_depth"]), golden_distance(d["distance"]))


def test_shortest_distance_unit_gods(ctx):
    d, meta = golden("gods")
    g = ctx.build(d["vid"], d["src"], d["dst"], flags=ALL)
    np.testing.assert_array_equal(g.shortest_distance(meta["sd_seed"], meta["sd_max_depth"]), golden_distance(d["sd_unit"]))


@pytest.mark.parametrize("name", ["gods", "cc_kat", "random_small", "random_medium"])
def test_connected_components_golden(ctx, name):
    d, meta = golden(name)
    g = ctx.build(d["vid"], d["src"], d["dst"], flags=ALL)
    comp, it = g.connected_components()
    np.testing.assert_array_equal(comp, d["component"])
    key = "supersteps" if "supersteps" in meta else "cc_supersteps"
    assert it == meta[key]


@pytest.mark.parametrize("name,src_key", [("gods", "bfs_source"), ("spvp_diamond", "source_vid"),
                                          ("random_small", "seed_vid"), ("random_medium", "seed_vid")])
def test_bfs_golden(ctx, name, src_key):
    d, meta = golden(name)
    g = ctx.build(d["vid"], d["src"], d["dst"], flags=ALL)
    depth = g.bfs([meta[src_key]], 3)[0]
    np.testing.assert_array_equal(depth, d["depth"])


def rmat_case(oracle_lib, scale, ef=16, seed=7, sparse_ids=True):
    o = oracle_lib
    s, t = o.rmat_edges(scale, ef, seed)
    n = 1 << scale
    if sparse_ids:
        rng = np.random.default_rng(scale)
        vid = (rng.permutation(n).astype(np.int64) + 1) << 8  # IDManager.toVertexId(i) at 32 partitions
        return n, vid, vid[s], vid[t], s, t
    vid = np.arange(n, dtype=np.int64)
    return n, vid, s, t, s, t


def dense_of(vid, ids):
    order = np.argsort(vid)
    return order[np.searchsorted(vid[order], ids)].astype(np.int32)


@pytest.mark.parametrize("scale", [10, 14, 16])
def test_pagerank_rmat_vs_oracle(ctx, oracle_lib, scale):
    n, vid, src, dst, _, _ = rmat_case(oracle_lib, scale)
    g = ctx.build(vid, src, dst, flags=2)
    rank, ec = g.pagerank(0.85, n, 30)
    ds, dd = dense_of(vid, src), dense_of(vid, dst)
    r_ref, ec_ref = oracle_lib.pagerank(n, ds, dd, 0.85, n, 30)
    assert_pr_close(ec, ec_ref)
    # dangling / isolated vertices: rank is still written (1-d)/N etc.
    assert_pr_close(rank, r_ref)


@pytest.mark.parametrize("scale", [12, 16])
def test_rmat_device_generator_matches_oracle(ctx, oracle_lib, scale):
    """jg_graph_build_rmat generates on the device; identical results prove the identical edge list."""
    n = 1 << scale
    g = ctx.build_rmat(scale, 16, 7, flags=2)
    rank, ec = g.pagerank(0.85, n, 12)
    s, t = oracle_lib.rmat_edges(scale, 16, 7)
    r_ref, ec_ref = oracle_lib.pagerank(n, s.astype(np.int32), t.astype(np.int32), 0.85, n, 12)
    np.testing.assert_array_equal(ec, ec_ref)
    assert_pr_close(rank, r_ref)


@pytest.mark.parametrize("scale", [10, 14, 17])
def test_bfs_rmat_vs_oracle(ctx, oracle_lib, scale):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, scale)
    g = ctx.build(vid, src, dst, flags=4)
    deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
    cand = np.nonzero(deg)[0]
    for k in range(3):
        s = int(cand[(k * 7919) % len(cand)])
        depth = g.bfs([vid[s]], 3)[0]
        ref = oracle_lib.bfs(n, ds, dd, s, 3)
        np.testing.assert_array_equal(depth, ref)


def test_bfs_without_depth_output_skips_the_empty_suffix(ctx, oracle_lib):
    """want=False on a BOTH traversal: the init skips the empty suffix's rows (dobfs_single `tail`), which
    the traversal never reads.  Isolated sources (in that suffix) and connected ones alternate, so stale
    depths of an earlier source would show: every want=False run must count the levels and edges of the
    want=True run from the same source, and a later want=True run must still match the oracle."""
    import janusgraph_amd as jg
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 15)
    g = ctx.build(vid, src, dst, flags=ALL)
    deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
    iso = np.flatnonzero(deg == 0)[:3]
    conn = np.flatnonzero(deg > 0)[[0, 11, 257]]
    assert len(iso) == 3
    for s in [int(x) for pair in zip(iso, conn) for x in pair]:
        g.bfs([vid[s]], jg.DIR_BOTH, want=False)
        quiet = (ctx.stats()["levels"], ctx.stats()["edges_traversed"])
        got = g.bfs([vid[s]], jg.DIR_BOTH)[0]
        assert (ctx.stats()["levels"], ctx.stats()["edges_traversed"]) == quiet
        np.testing.assert_array_equal(got, oracle_lib.bfs(n, ds, dd, s, 3))
    # want=True skips the suffix too now, and CC shares the seen bytes; alternate want=False BFS,
    # connected_components and want=True / kept rows from isolated and connected sources
    comp_ref, _ = oracle_lib.connected_components(n, ds, dd, vid)
    for s in [int(x) for pair in zip(conn, iso) for x in pair]:
        g.bfs([vid[s]], jg.DIR_BOTH, want=False)
        comp, _ = g.connected_components()
        np.testing.assert_array_equal(comp, comp_ref)
        np.testing.assert_array_equal(g.bfs([vid[s]], jg.DIR_BOTH)[0], oracle_lib.bfs(n, ds, dd, s, 3))
        g.bfs_keep([vid[s]], jg.DIR_BOTH)
        np.testing.assert_array_equal(g.bfs_kept_row(0), oracle_lib.bfs(n, ds, dd, s, 3))
    g.close()


@pytest.mark.parametrize("mode,split_min", [(0, 65536), (1, 1), (1, 4096), (2, 1)])
def test_bfs_split_top_down_matches_oracle(oracle_lib, mode, split_min):
    """Split top-down levels (owner store + claim launch, Tune::bfs_td_split) against the CAS claims:
    identical depths, edge counts and CC superstep counts (the eccentricity BFS shares the level code),
    for every level split (mode 1) and level 1 only (mode 2)."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    c = jg.Context((0,))
    try:
        _lib.tune_set("bfs_td_split", mode)
        _lib.tune_set("bfs_td_split_min", split_min)
        for scale in (14, 17):
            n, vid, src, dst, ds, dd = rmat_case(oracle_lib, scale)
            g = c.build(vid, src, dst, flags=ALL)
            deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
            cand = np.nonzero(deg)[0]
            for k in range(3):
                s = int(cand[(k * 7919) % len(cand)])
                _lib.tune_set("bfs_td_split", 0)
                g.bfs([vid[s]], 3, want=False)
                edges_cas = c.stats()["edges_traversed"]
                _lib.tune_set("bfs_td_split", mode)
                got = g.bfs([vid[s]], 3)[0]
                np.testing.assert_array_equal(got, oracle_lib.bfs(n, ds, dd, s, 3))
                # each reached vertex claimed exactly once: the same frontier degree sums as the CAS claims
                assert c.stats()["edges_traversed"] == edges_cas
                for direction in (1, 2):
                    np.testing.assert_array_equal(g.bfs([vid[s]], direction)[0],
                                                  oracle_lib.bfs(n, ds, dd, s, direction))
            comp, it = g.connected_components()
            comp_ref, it_ref = oracle_lib.connected_components(n, ds, dd, vid)
            np.testing.assert_array_equal(comp, comp_ref)
            assert it == it_ref
            g.close()
    finally:
        _lib.tune_set("bfs_td_split", 2)
        _lib.tune_set("bfs_td_split_min", 65536)
        c.close()


def test_bfs_isolated_and_missing_source(ctx, oracle_lib):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 10)
    g = ctx.build(vid, src, dst, flags=4)
    deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
    iso = np.nonzero(deg == 0)[0]
    if len(iso):
        depth = g.bfs([vid[iso[0]]], 3)[0]
        assert depth[iso[0]] == 0 and (np.delete(depth, iso[0]) == -1).all()
    depth = g.bfs([12345], 3)[0]  # not a vertex id
    assert (depth == -1).all()


@pytest.mark.parametrize("max_depth", [0, 1, 2, 3])
def test_bfs_max_depth(ctx, oracle_lib, max_depth):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 12)
    g = ctx.build(vid, src, dst, flags=4)
    s = int(ds[0])
    np.testing.assert_array_equal(g.bfs([vid[s]], 3, max_depth)[0], oracle_lib.bfs(n, ds, dd, s, 3, max_depth))


def test_multisource_bfs_rmat(ctx, oracle_lib):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 13)
    g = ctx.build(vid, src, dst, flags=4)
    rng = np.random.default_rng(3)
    srcs = rng.choice(np.unique(ds), 64, replace=False)
    depth = g.bfs(vid[srcs], 3)
    for k in (0, 1, 31, 63):
        np.testing.assert_array_equal(depth[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3))


@pytest.mark.parametrize("mode,shards", [("skip", 1), ("noskip", 1), ("skip_pull_only", 1), ("skip_bands3", 1),
                                         ("skip_wide", 1), ("skip", 3), ("skip", 8), ("skip_sharded_pull_only", 3),
                                         ("skip_dense_reverse", 3), ("skip_dense", 2), ("exit_off", 1),
                                         ("exit_every_bitmapped_level", 1), ("exit_every_level", 1), ("exit_no_skip", 1),
                                         ("td_probe_always", 1), ("td_probe_never", 1), ("td_probe_never", 3),
                                         ("exit_first3", 1), ("exit_first32", 3), ("scan_queue_off", 1),
                                         ("scan_queue_always", 1), ("td_rowapply_off", 1), ("td_rowapply_always", 1)])
def test_msbfs_task_skip_matches_oracle(oracle_lib, mode, shards):
    """The 64-source BFS's pull levels skip merge tasks whose rows can gain no live bit
    (MergeArgs::live): all 64 depth rows equal the oracle's, with sources in the giant component, an
    isolated vertex and a vertex of a small component (their bits never reach the rest, so no row ever
    holds every source), on one shard and on logical shards (halo and dense vectors).  On sharded halo
    plans the small-frontier levels run top-down (own rows pushed, peers' bits returned by the reverse
    halo exchange, sparse (offset, word) pairs when few staging slots are set, the whole segments with
    skip_dense_reverse); skip_sharded_pull_only keeps every sharded level a pull level (msbfs_td 2).
    One shard: levels after the frontier's peak scan every row with early exit (msbfs_exit)."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    knobs = {"skip": [], "noskip": [("msbfs_skip", 0)], "skip_pull_only": [("msbfs_td", 0)],
             "skip_bands3": [("band0_deg", 64), ("band0_bit", 8), ("band1_deg", 16), ("band1_bit", 5),
                             ("band2_deg", 4), ("band2_bit", 3)],
             "skip_wide": [("band0_deg", 2), ("band0_bit", 7), ("band1_deg", 0)],
             "skip_dense": [("halo", 0)], "skip_sharded_pull_only": [("msbfs_td", 2)],
             "skip_dense_reverse": [("msbfs_sparse", 0)],
             # the early exit (msbfs_exit: 1, the default, on levels where few band-0 tasks are live)
             "exit_off": [("msbfs_exit", 0)], "exit_every_bitmapped_level": [("msbfs_exit_live", 1000)],
             "exit_every_level": [("msbfs_exit", 2)],
             # the visited probe of top-down edges (skipped below level msbfs_td_noprobe, 2 by default)
             "td_probe_always": [("msbfs_td_noprobe", 0)], "td_probe_never": [("msbfs_td_noprobe", 1000)],
             # the early exit's lane pass over 3 / 32 entries per row (16 by default)
             "exit_first3": [("msbfs_exit_first", 3), ("msbfs_exit_live", 1000)],
             "exit_first32": [("msbfs_exit_first", 32), ("msbfs_exit_live", 1000)],
             # the next top-down queue built by the frontier scan (msbfs_scan_queue: never / after every probe)
             "scan_queue_off": [("msbfs_scan_queue", 0)], "scan_queue_always": [("msbfs_scan_queue", 1001)],
             # top-down applies in row order (msbfs_td_rowapply: never / every one-shard level)
             "td_rowapply_off": [("msbfs_td_rowapply", 0)], "td_rowapply_always": [("msbfs_td_rowapply", 1024)],
             "exit_no_skip": [("msbfs_exit", 2), ("msbfs_skip", 0)]}[mode]
    n0, vid0, src0, dst0, ds0, dd0 = rmat_case(oracle_lib, 15)
    n = n0 + 3  # + an isolated vertex and a two-vertex component
    vid = np.concatenate([vid0, (np.arange(3, dtype=np.int64) + n0 + 1) << 8 | 7])
    ds = np.concatenate([ds0, np.array([n0 + 1], ds0.dtype)])
    dd = np.concatenate([dd0, np.array([n0 + 2], dd0.dtype)])
    try:
        for k, v in knobs:
            _lib.tune_set(k, v)
        c = jg.Context((0,) * shards)
        g = c.build(vid, vid[ds], vid[dd], flags=2 | 4)
        rng = np.random.default_rng(11)
        srcs = np.concatenate([rng.choice(np.unique(ds0), 62, replace=False), [n0, n0 + 2]])
        depth = g.bfs(vid[srcs], 3)
        for k in range(len(srcs)):
            np.testing.assert_array_equal(depth[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3), err_msg=f"source {k}")
        bounded = g.bfs(vid[srcs[:5]], 3, 3)
        for k in range(5):
            np.testing.assert_array_equal(bounded[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3, 3),
                                          err_msg=f"source {k}, max_depth 3")
        g.close()
        c.close()
    finally:
        _lib.tune_set("msbfs_skip", 1)
        _lib.tune_set("msbfs_td", 1)
        _lib.tune_set("msbfs_sparse", 1)
        _lib.tune_set("msbfs_exit", 1)
        _lib.tune_set("msbfs_exit_live", 950)
        _lib.tune_set("msbfs_td_noprobe", 2)
        _lib.tune_set("msbfs_exit_first", 16)
        _lib.tune_set("msbfs_scan_queue", 50)
        _lib.tune_set("msbfs_td_rowapply", 4)
        _lib.tune_set("halo", 1)
        for k, v in (("band0_deg", 96), ("band0_bit", 0), ("band1_deg", -1), ("band1_bit", 0), ("band2_deg", -1),
                     ("band2_bit", 0), ("band3_deg", 0)):  # the defaults (Tune::band_deg / band_bits)
            _lib.tune_set(k, v)


@pytest.mark.parametrize("direction", [1, 2])
def test_directed_bfs(ctx, oracle_lib, direction):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 12)
    g = ctx.build(vid, src, dst, flags=3)
    s = int(ds[5])
    np.testing.assert_array_equal(g.bfs([vid[s]], direction)[0], oracle_lib.bfs(n, ds, dd, s, direction))


def test_msbfs_rows_past_the_suffix_are_never_read(ctx, oracle_lib, monkeypatch):
    """One shard, BOTH: the 64-source BFS clears its frontier and visited words only before the empty suffix
    (the rows past it are never read after level 0; the source rows among them are stored by the init).
    With JG_MSBFS_POISON those rows hold garbage instead of whatever the allocator left: every depth row
    must still match the oracle, isolated sources (in the suffix) included, and so must the level count."""
    import janusgraph_amd as jg
    monkeypatch.setenv("JG_MSBFS_POISON", "1")
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 15)
    g = ctx.build(vid, src, dst, flags=ALL)
    deg = np.bincount(ds, minlength=n) + np.bincount(dd, minlength=n)
    iso = np.flatnonzero(deg == 0)[:5]
    live = np.flatnonzero(deg > 0)
    conn = live[np.linspace(0, len(live) - 1, 59).astype(np.int64)]
    srcs = np.concatenate([conn[:20], iso, conn[20:]])
    assert len(iso) == 5 and len(srcs) == 64
    depth = g.bfs(vid[srcs], jg.DIR_BOTH)
    deepest = 0
    for k, s0 in enumerate(srcs):
        want = oracle_lib.bfs(n, ds, dd, int(s0), 3)
        np.testing.assert_array_equal(depth[k], want, err_msg=f"source {k}")
        deepest = max(deepest, int(want.max()))
    assert ctx.stats()["levels"] == deepest + 1
    g.close()


@pytest.mark.parametrize("exit_mode", [0, 1, 2])
def test_directed_multi_source_bfs(ctx, oracle_lib, exit_mode):
    """The 64-source BFS along OUT edges (pulling over the IN adjacency, pushing over OUT) with the early
    exit off, adaptive and forced on every pull level: all depth rows against the oracle."""
    from janusgraph_amd import _lib
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 15)
    try:
        _lib.tune_set("msbfs_exit", exit_mode)
        g = ctx.build(vid, src, dst, flags=3)
        srcs = np.unique(ds)[::97][:64]
        depth = g.bfs(vid[srcs], 1)
        levels = ctx.stats()["levels"]
        deepest = 0
        for k in range(len(srcs)):
            want = oracle_lib.bfs(n, ds, dd, int(srcs[k]), 1)
            np.testing.assert_array_equal(depth[k], want, err_msg=f"source {k}")
            deepest = max(deepest, int(want.max()))
        assert levels == deepest + 1  # the level that finds nothing new ends the traversal
        g.close()
    finally:
        _lib.tune_set("msbfs_exit", 1)


@pytest.mark.parametrize("scale", [12, 16])
def test_shortest_distance_rmat(ctx, oracle_lib, scale):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, scale)
    w = (np.arange(len(src)) % 3 + 1).astype(np.int32)
    g = ctx.build(vid, src, dst, weight=w, flags=3)
    seed = int(dd[0])
    np.testing.assert_array_equal(g.shortest_distance(vid[seed], 6), oracle_lib.shortest_distance(n, ds, dd, seed, 6, w))
    gu = ctx.build(vid, src, dst, flags=3)
    np.testing.assert_array_equal(gu.shortest_distance(vid[seed], 4), oracle_lib.shortest_distance(n, ds, dd, seed, 4))


@pytest.mark.parametrize("scale", [10, 15])
def test_connected_components_rmat(ctx, oracle_lib, scale):
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, scale)
    g = ctx.build(vid, src, dst, flags=4)
    comp, it = g.connected_components()
    ref, ref_it = oracle_lib.connected_components(n, ds, dd, vid)
    np.testing.assert_array_equal(comp, ref)
    assert it == ref_it


def test_graph_info_counts(ctx):
    d, meta = golden("random_small")
    g = ctx.build(d["vid"], d["src"], d["dst"], flags=ALL)
    info = g.info()
    assert info["ghost_edges"] == meta["ghost_edges"]
    assert info["num_edges"] == len(d["src"]) - meta["ghost_edges"]
    assert info["self_loops"] >= 4
    assert info["num_shards"] == 1


@pytest.mark.parametrize("shards,scale,halo", [(2, 13, 1), (3, 13, 1), (4, 13, 1), (8, 15, 1),
                                               (2, 13, 0), (3, 13, 0)])
def test_logical_shards_match_single(oracle_lib, shards, scale, halo):
    """P logical shards on one device (exchange by device copies) == 1 shard == oracle; halo = 1 is
    the compact-vector halo exchange, 0 the dense allgather."""
    import janusgraph_amd as jg
    c = jg.Context((0,) * shards)
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, scale)
    jg._lib.tune_set("halo", halo)
    try:
        g = c.build(vid, src, dst, flags=2 | 4)
    finally:
        jg._lib.tune_set("halo", 1)
    rank, _ = g.pagerank(0.85, n, 15)
    r_ref, _ = oracle_lib.pagerank(n, ds, dd, 0.85, n, 15)
    assert_pr_close(rank, r_ref)
    comp, it = g.connected_components()
    ref, ref_it = oracle_lib.connected_components(n, ds, dd, vid)
    np.testing.assert_array_equal(comp, ref)
    assert it == ref_it
    srcs = np.unique(ds)[:5]
    depth = g.bfs(vid[srcs], 3)
    for k in range(len(srcs)):
        np.testing.assert_array_equal(depth[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3))
    depth = g.bfs(vid[srcs], 1)  # OUT traversal: bit-parallel pull over the IN adjacency
    for k in range(len(srcs)):
        np.testing.assert_array_equal(depth[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 1))
    # single source, BOTH: the sharded direction-optimising BFS (halo plans), unbounded and bounded
    for k in range(3):
        for md in (-1, 2):
            d1 = g.bfs(vid[srcs[k:k + 1]], 3, md)[0]
            np.testing.assert_array_equal(d1, oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3, md))
    assert g.info()["num_shards"] == shards
    g.close()
    c.close()


@pytest.mark.parametrize("shards,uf", [(2, 1), (3, 1), (8, 1), (3, 0), (3, "nosearch"), (8, "nosearch"), (3, "dense"),
                                       (8, "dense")])
def test_sharded_connected_components_union_find(oracle_lib, shards, uf):
    """Logical shards over halo plans: local union-finds, tree labels spread over the halo, and one
    sharded BFS from every component's minimum-rank vertex for the superstep count (cc_uf_sharded=1),
    or the label propagation (0); "nosearch" skips the bounded giant-to-giant search, so every peer
    takes the fallback (giant rows link every flagged copy); "dense" moves every label in every label
    round (cc_sparse=0; the default sends only the labels that fell, as pairs).  Components of every kind (isolated vertices, self-loops, small
    components split across shards, an RMAT giant), a path past the 99-superstep cap (handed to the
    propagation) and one below it; labels and superstep counts against the oracle."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    rng = np.random.default_rng(12)
    cases = []
    n = 400
    s, d = rng.integers(0, n, 300), rng.integers(0, n, 300)
    s[:5] = d[:5] = 7  # self-loops
    cases.append((n, s, d, np.arange(10, 10 + n, dtype=np.int64)))
    n = 150
    cases.append((n, np.arange(n - 1), np.arange(1, n), np.arange(10, 10 + n, dtype=np.int64)))  # past the cap
    cases.append((60, np.arange(59), np.arange(1, 60), np.arange(10, 70, dtype=np.int64)))  # below it
    n0, vid0, src0, dst0, ds0, dd0 = rmat_case(oracle_lib, 13)
    n = n0 + 5  # + isolated vertices and a 3-vertex chain whose minimum id sits in the middle
    extra = (np.arange(5, dtype=np.int64) + 7) * 1000003
    ids = np.concatenate([vid0, extra])
    cases.append((n, np.concatenate([ds0, [n0 + 2, n0 + 3]]), np.concatenate([dd0, [n0 + 3, n0 + 4]]), ids))
    try:
        _lib.tune_set("cc_uf_sharded", 0 if uf == 0 else 1)
        _lib.tune_set("cc_uf_search", 0 if uf == "nosearch" else 1)
        _lib.tune_set("cc_sparse", 0 if uf == "dense" else 1)
        c = jg.Context((0,) * shards)
        for n, s, d, vid in cases:
            g = c.build(vid, vid[s], vid[d], flags=jg.ADJ_BOTH)
            comp, it = g.connected_components()
            want, want_it = oracle_lib.connected_components(n, np.asarray(s, np.int32), np.asarray(d, np.int32), vid)
            assert it == want_it, f"{shards} shards, n={n}: {it} supersteps, oracle {want_it}"
            np.testing.assert_array_equal(comp, want)
            g.close()
        c.close()
    finally:
        _lib.tune_set("cc_uf_sharded", 1)
        _lib.tune_set("cc_uf_search", 1)
        _lib.tune_set("cc_sparse", 1)


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_logical_shards_shortest_distance(oracle_lib, shards):
    """Sharded ShortestDistanceVertexProgram (weighted and unit) over the IN halo plan: push into own
    rows and halo slots, reverse halo exchange to the owners == the oracle, for several hop bounds."""
    import janusgraph_amd as jg
    c = jg.Context((0,) * shards)
    n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 13)
    w = (np.arange(len(src)) % 3 + 1).astype(np.int32)
    g = c.build(vid, src, dst, weight=w, flags=2)
    gu = c.build(vid, src, dst, flags=2)
    for seed in (int(dd[0]), int(dd[7])):
        for md in (1, 3, 6, 30):
            np.testing.assert_array_equal(g.shortest_distance(vid[seed], md),
                                          oracle_lib.shortest_distance(n, ds, dd, seed, md, w))
            np.testing.assert_array_equal(gu.shortest_distance(vid[seed], md),
                                          oracle_lib.shortest_distance(n, ds, dd, seed, md))
    g.close()
    gu.close()
    c.close()


def test_hub_rows_chunked(ctx, oracle_lib):
    """A star with hubs above the chunking threshold (8192) in and out."""
    n = 40000
    rng = np.random.default_rng(5)
    hub_in = np.zeros(20000, np.int64)
    src = np.concatenate([rng.integers(1, n, 20000), np.full(15000, 1), rng.integers(0, n, 30000)])
    dst = np.concatenate([hub_in, rng.integers(2, n, 15000), rng.integers(0, n, 30000)])
    vid = np.arange(n, dtype=np.int64) + 1000
    g = ctx.build(vid, src + 1000, dst + 1000, flags=ALL)
    rank, _ = g.pagerank(0.85, n, 20)
    r_ref, _ = oracle_lib.pagerank(n, src.astype(np.int32), dst.astype(np.int32), 0.85, n, 20)
    assert_pr_close(rank, r_ref)
    comp, it = g.connected_components()
    ref, ref_it = oracle_lib.connected_components(n, src.astype(np.int32), dst.astype(np.int32), vid)
    np.testing.assert_array_equal(comp, ref)
    depth = g.bfs([1000], 3)[0]
    np.testing.assert_array_equal(depth, oracle_lib.bfs(n, src.astype(np.int32), dst.astype(np.int32), 0, 3))


def test_errors_are_status_codes(ctx):
    import janusgraph_amd as jg
    with pytest.raises(jg.JanusGpuError) as e:
        ctx.build(np.array([5, 5], np.int64), np.array([5]), np.array([5]))
    assert "duplicate" in str(e.value)
    g = ctx.build(np.array([1, 2], np.int64), np.array([1]), np.array([2]), flags=4)
    with pytest.raises(jg.JanusGpuError):
        g.pagerank(0.85, 2, 5)  # no in-adjacency built
    with pytest.raises(jg.JanusGpuError):
        g.pagerank_step(1)


@pytest.mark.parametrize("mode", ["plain", "split", "split_bands3", "split_wide", "split_sub1", "split_sub2_4",
                                  "split_w24", "split_w32", "split_stage_off", "split_stage512", "cc_first3"])
def test_pull_engine_variants_match_oracle(oracle_lib, mode):
    """Every pull-engine variant (jg_tune_set knobs) gives oracle parity: plain degree classes, the
    XCD-sliced split with its band layouts, entry packings and partial staging windows."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    knobs = {"plain": [("pull_split", 0)],
             "split": [("pull_split", 1)],
             "split_bands3": [("band0_deg", 64), ("band0_bit", 8), ("band1_deg", 16), ("band1_bit", 5),
                              ("band2_deg", 4), ("band2_bit", 3)],
             "split_wide": [("band0_deg", 2), ("band0_bit", 7), ("band1_deg", 0)],
             "split_sub1": [("band1_sub", 1)],
             "split_sub2_4": [("band0_deg", 64), ("band0_sub", 4), ("band1_deg", 16), ("band1_sub", 2),
                              ("band2_deg", 4), ("band2_sub", 1)],
             "split_w24": [("merge_pack", 24)],
             "split_w32": [("merge_pack", 0)],
             "split_stage_off": [("merge_stage0", 0), ("merge_stage1", 0)],
             "split_stage512": [("merge_stage0", 512), ("merge_stage1", 512)],
             "cc_first3": [("cc_first", 3)]}[mode]
    try:
        for k, v in knobs:
            _lib.tune_set(k, v)
        c = jg.Context((0,))
        n, vid, src, dst, ds, dd = rmat_case(oracle_lib, 15)
        g = c.build(vid, src, dst, flags=2 | 4)
        rank, _ = g.pagerank(0.85, n, 12)
        r_ref, _ = oracle_lib.pagerank(n, ds, dd, 0.85, n, 12)
        assert_pr_close(rank, r_ref)
        comp, it = g.connected_components()
        ref, ref_it = oracle_lib.connected_components(n, ds, dd, vid)
        np.testing.assert_array_equal(comp, ref)
        assert it == ref_it
        srcs = np.unique(ds)[:40]
        depth = g.bfs(vid[srcs], 3)
        for k in (0, 17, 39):
            np.testing.assert_array_equal(depth[k], oracle_lib.bfs(n, ds, dd, int(srcs[k]), 3))
        g.close()
        c.close()
    finally:
        _lib.tune_set("pull_split", 1)
        _lib.tune_set("merge_pack", 1)
        _lib.tune_set("merge_stage0", -1)
        _lib.tune_set("merge_stage1", -1)
        _lib.tune_set("cc_first", 1)
        for k, v in (("band0_deg", 96), ("band0_bit", 0), ("band1_deg", -1), ("band1_bit", 0), ("band2_deg", -1),
                     ("band2_bit", 0), ("band3_deg", 0)):
            _lib.tune_set(k, v)


@pytest.mark.gpu
def test_decode_edges_matches_oracle(ctx, oracle_lib):
    """GPU edgestore decode (jg_decode_edges) == the C oracle == the values the restated writer
    encoded, over every entry kind (tests/test_edgecodec.py random_entries)."""
    from test_edgecodec import check_decoded, random_entries
    data, off, vpos, tids, tmult, exp = random_entries(20000, seed=7)
    got = ctx.decode_edges(data, off, vpos, tids, tmult)
    check_decoded(got, exp)
    ref = oracle_lib.decode_edges(data, off, vpos, tids, tmult)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_decode_edges_edge_cases(ctx):
    """Empty input; a truncated varint is reported as malformed (dir -1) without reading past it;
    out-of-range offsets are rejected before any launch."""
    import janusgraph_amd as jg
    from oracle import edgecodec as ec
    t, d, o, r = ctx.decode_edges(b"", [0], [])
    assert len(t) == len(d) == len(o) == len(r) == 0
    lab = ec.schema_id(9, "user_edge")
    good, vp = ec.encode_edge(lab, ec.OUT, 1 << 40, 17)
    hdr = ec.write_relation_type(lab, True, ec.OUT)
    bad = hdr + b"\x01\x02"  # backward varint with no first (stop-marked) byte
    data = good + bad
    t, d, o, r = ctx.decode_edges(data, [0, len(good), len(data)], [vp, len(bad)])
    assert list(d) == [0, -1] and o[0] == 1 << 40 and r[0] == 17 and o[1] == -1
    with pytest.raises(jg.JanusGpuError):
        ctx.decode_edges(data, [0, len(data) + 5], [1])


@pytest.mark.parametrize("tail", [64, 1, 0])
def test_bfs_tail_grid_deeper_than_history(oracle_lib, tail):
    """bfs_tail_grid: launches past the deepest of the last traversals run with a small grid.  Shallow
    traversals first (history of 2-3 levels), then ones that go 40 levels down a path hanging off the
    graph: the levels past the prediction do real work on the small grid (one workgroup with tail 1,
    both directions grid-stride), and every depth still equals the oracle's."""
    import janusgraph_amd as jg
    from janusgraph_amd import _lib
    n0, vid0, src0, dst0, ds0, dd0 = rmat_case(oracle_lib, 12)
    plen = 40
    n = n0 + plen
    vid = np.concatenate([vid0, (np.arange(plen, dtype=np.int64) + n0 + 1) << 8 | 3])
    hub = int(np.bincount(ds0, minlength=n0).argmax())
    ps = np.concatenate([[hub], np.arange(n0, n - 1)]).astype(ds0.dtype)
    pd = np.arange(n0, n).astype(ds0.dtype)
    ds, dd = np.concatenate([ds0, ps]), np.concatenate([dd0, pd])
    try:
        _lib.tune_set("bfs_tail_grid", tail)
        c = jg.Context((0,))
        g = c.build(vid, vid[ds], vid[dd], flags=4)
        for sv in (hub, hub, int(ds0[1])):  # shallow: the history
            np.testing.assert_array_equal(g.bfs([vid[sv]], 3)[0], oracle_lib.bfs(n, ds, dd, sv, 3))
        for sv in (n - 1, n0 + 5, n - 1):  # the path's far end: ~45 levels
            np.testing.assert_array_equal(g.bfs([vid[sv]], 3)[0], oracle_lib.bfs(n, ds, dd, sv, 3),
                                          err_msg=f"tail grid {tail}, source {sv}")
            assert c.stats()["levels"] > 30
        np.testing.assert_array_equal(g.bfs([vid[hub]], 3, 2)[0], oracle_lib.bfs(n, ds, dd, hub, 3, 2))
        g.close()
        c.close()
    finally:
        _lib.tune_set("bfs_tail_grid", 64)
