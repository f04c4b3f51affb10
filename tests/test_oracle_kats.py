"""The CPU oracle pinned against the reference's own known-answer tests (CPU only).

The oracle (oracle/jg_oracle.c) is a restatement of Fulgora's semantics; it is trusted only because
it reproduces, bit for bit or within fp64 rounding, the expectations the reference's OLAPTest states
and the independent vertex-centric mirror (oracle/pymirror.py) computes.
"""
import json
import os

import numpy as np
import pytest

from oracle.oracle import golden_distance

from oracle import pymirror as pm

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    z = np.load(os.path.join(GOLD, f"{name}.npz"))
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    return {k: z[k] for k in z.files}, meta


def test_pr_tree_closed_form(oracle_lib):
    """OLAPTest.testPageRank (OLAPTest.java:589-655): pr[d] = (1-a)/N + a*6*pr[d+1]; sum within 0.001."""
    d, meta = golden("pr_tree")
    assert meta["vertex_count"] == 9331 and meta["iterations"] == 10
    ds, dd, _ = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    rank, ec = oracle_lib.pagerank(len(d["vid"]), ds, dd, meta["damping"], meta["vertex_count"], 10)
    np.testing.assert_allclose(rank, d["closed_form"], rtol=1e-12)
    assert abs(rank.sum() - d["closed_form"].sum()) < 0.001
    # leaves have no in-edges: pr[5] = (1-a)/N; root has no out-edge: edgeCount 0
    assert (ec[d["depth"] == 0] == 0).all() and (ec[d["depth"] > 0] == 1).all()


def test_sssp_tree(oracle_lib):
    """OLAPTest.testShortestDistance (OLAPTest.java:657-714): DISTANCE == stored depth, all reached."""
    d, meta = golden("sssp_tree")
    ds, dd, keep = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    seed = int(np.nonzero(d["vid"] == meta["seed_vid"])[0][0])
    dist = oracle_lib.shortest_distance(len(d["vid"]), ds, dd, seed, meta["max_depth"], d["weight"][keep])
    np.testing.assert_array_equal(dist, golden_distance(d["distance"]))
    assert (dist >= 0).all()


def test_cc_kat(oracle_lib):
    """OLAPTest.testConnectedComponent (OLAPTest.java:736-762): 3 share a label, isolated keeps its id."""
    d, meta = golden("cc_kat")
    ds, dd, _ = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    comp, it = oracle_lib.connected_components(len(d["vid"]), ds, dd, d["vid"])
    np.testing.assert_array_equal(comp, d["component"])
    assert comp[3] == d["vid"][3]
    assert len(set(comp[:3].tolist())) == 1
    assert it == meta["supersteps"]


def test_spvp_diamond(oracle_lib):
    """OLAPTest.testShortestPath (OLAPTest.java:716-734): v1 -> v2 is one hop (one path of 2)."""
    d, meta = golden("spvp_diamond")
    ds, dd, _ = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    depth = oracle_lib.bfs(len(d["vid"]), ds, dd, 0, oracle_lib.DIR_BOTH)
    np.testing.assert_array_equal(depth, d["depth"])
    assert depth[1] == 1


@pytest.mark.parametrize("name", ["gods", "random_small", "random_medium"])
def test_oracle_matches_mirror(oracle_lib, name):
    d, meta = golden(name)
    n = len(d["vid"])
    ds, dd, keep = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    rank, ec = oracle_lib.pagerank(n, ds, dd, meta["damping"], meta["vertex_count"], meta["iterations"])
    np.testing.assert_allclose(rank, d["rank"], rtol=1e-13)
    np.testing.assert_array_equal(ec, d["edge_count"])
    comp, it = oracle_lib.connected_components(n, ds, dd, d["vid"])
    np.testing.assert_array_equal(comp, d["component"])
    assert it == meta["cc_supersteps"]
    src_key = "bfs_source" if name == "gods" else "seed_vid"
    s = int(np.nonzero(d["vid"] == meta[src_key])[0][0])
    np.testing.assert_array_equal(oracle_lib.bfs(n, ds, dd, s, oracle_lib.DIR_BOTH), d["depth"])
    if "distance" in d:
        seed = int(np.nonzero(d["vid"] == meta["seed_vid"])[0][0])
        dist = oracle_lib.shortest_distance(n, ds, dd, seed, meta["sd_max_depth"], d["weight"][keep])
        np.testing.assert_array_equal(dist, golden_distance(d["distance"]))


def test_gods_known_structure(oracle_lib):
    d, meta = golden("gods")
    names = meta["names"]
    ds, dd, _ = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    assert len(ds) == 17 and len(names) == 12
    rank, ec = oracle_lib.pagerank(12, ds, dd, 0.85, 12, 30)
    # out-degree (janusgraph.pageRank.edgeCount) straight from GraphOfTheGodsFactory.java:128-147
    expect = {"jupiter": 4, "neptune": 3, "hercules": 5, "pluto": 4, "cerberus": 1, "saturn": 0, "sky": 0}
    for k, v in expect.items():
        assert ec[names.index(k)] == v
    # every vertex is in one weakly connected component labelled by the String-min id
    comp, _ = oracle_lib.connected_components(12, ds, dd, d["vid"])
    assert len(set(comp.tolist())) == 1
    assert comp[0] == min(d["vid"].tolist(), key=str)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_pagerank_iteration_edge_cases(oracle_lib, k):
    """K = 0: no property written; K = 1: rank = 1/N; K = 2: one power step."""
    d, meta = golden("gods")
    ds, dd, _ = oracle_lib.remap(d["vid"], d["src"], d["dst"])
    rank, ec = oracle_lib.pagerank(12, ds, dd, 0.85, 12, k)
    g = pm.MiniGraph(d["vid"].tolist(), list(zip(d["src"].tolist(), d["dst"].tolist())))
    props, it = pm.Engine(g).run(pm.PageRankProgram(0.85, k, 12))
    assert it == k
    want = np.array([props[v].get("pageRank", np.nan) for v in g.vertices])
    np.testing.assert_array_equal(np.isnan(rank), np.isnan(want))
    np.testing.assert_allclose(rank[~np.isnan(want)], want[~np.isnan(want)], rtol=1e-15)


def test_lex_rank_string_order(oracle_lib):
    ids = np.array([1, 10, 2, 100, 256, 2560, 257, 9, 0, 1000000000000], np.int64)
    r = oracle_lib.lex_rank(ids)
    got = [int(x) for x in ids[np.argsort(r)]]
    assert got == sorted(ids.tolist(), key=str)


def test_remap_ghosts_and_duplicates(oracle_lib):
    vid = np.array([256, 512, 768], np.int64)
    s, t, keep = oracle_lib.remap(vid, np.array([256, 512, 999, 768]), np.array([512, 768, 256, 1]))
    assert s.tolist() == [0, 1] and t.tolist() == [1, 2] and keep.tolist() == [0, 1]
    with pytest.raises(ValueError):
        oracle_lib.remap(np.array([1, 1], np.int64), np.array([1]), np.array([1]))


def test_rmat_generator_properties(oracle_lib):
    s, t = oracle_lib.rmat_edges(14, 16, 99)
    assert len(s) == 16 << 14 and s.min() >= 0 and s.max() < 1 << 14
    s2, t2 = oracle_lib.rmat_edges(14, 16, 99, e0=1000, count=500)
    np.testing.assert_array_equal(s[1000:1500], s2)  # counter-based: any slice regenerates
    np.testing.assert_array_equal(t[1000:1500], t2)
    deg = np.bincount(s, minlength=1 << 14)
    assert deg.max() > 20 * deg.mean()  # power-law skew
    s3, _ = oracle_lib.rmat_edges(14, 16, 100)
    assert not np.array_equal(s, s3)
