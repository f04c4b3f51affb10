"""GPU parity at the BASELINE.json config sizes (configs[1..4]; configs[0], GraphOfTheGods, is
tests/test_gpu_parity.py::test_pagerank_golden[gods]).

Every result is checked against the CPU restatement in oracle/ on the same Graph500 RMAT graph
(the device generator is bit-identical to oracle.rmat_edges):
  configs[1]  SPVP BFS, RMAT-20 ef16, 1 GPU: depths from 3 sources (and depth-bounded) bit-exact.
  configs[2]  PageRank fp64, RMAT-24 ef16, K = 30 (29 power steps), vertexCount = |V|: per-vertex
              relative error <= 1e-9, edgeCount exact; on 1 shard and on 2, 4 and 8 logical shards (the
              1/2/4/8-GPU layouts and halo exchanges on one device).
  configs[3]  ConnectedComponent, RMAT-26 ef16: every String-min label and the iteration count exact, on
              1 shard (union-find + root BFS) and on 2 and 8 logical shards (the label propagation with
              its halo exchange that 2..8 GPUs run), plus the sharded single-source DO-BFS (dobfs_sharded,
              what a BFS on 2..8 GPUs runs) from 3 degree > 0 sources on the same sharded graphs (2, 4
              and 8 shards), and the one-GPU DO-BFS the bench times at this size (3 sources, one
              depth-bounded, Graph500 validation).
  configs[4]  64-source MS-BFS, RMAT-26 ef16 on 8 logical shards (the 8-GPU layout and halo exchange on
              one device): all 64 depth rows bit-exact, plus Graph500 validation of 3 of them.
The oracle side uses the parallel checkers of jg_oracle.c (jo_csr_unordered, jo_bfs_csr,
jo_msbfs_csr, jo_cc_csr, jo_pagerank_csr), pinned to the serial restatements by
tests/test_oracle_fullsize.py.  Host memory: ~45 GB at RMAT-26 (int32 edges, BOTH CSR, 64 depth rows).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PR_RTOL = 1e-9  # north_star: per-vertex relative error <= 1e-9 (fp64)
EF = 16


def seed_of(scale):
    return 0x5EED + scale  # bench.py / tools/big_configs.py


def host_edges(o, scale, ef=EF):
    """The RMAT edges of the device generator as int32, generated in chunks (int64 temporaries stay small)."""
    m = ef << scale
    s32 = np.empty(m, np.int32)
    d32 = np.empty(m, np.int32)
    step = 1 << 26
    for e0 in range(0, m, step):
        c = min(step, m - e0)
        s, d = o.rmat_edges(scale, ef, seed_of(scale), e0, c)
        s32[e0:e0 + c] = s
        d32[e0:e0 + c] = d
    return s32, d32


def pick_sources(ptr, k, seed):
    """Seeded uniform pick among vertices with at least one BOTH entry."""
    cand = np.flatnonzero(np.diff(ptr) > 0)
    return np.random.default_rng(seed).choice(cand, k, replace=False).astype(np.int64)


# ---------------- configs[1]: BFS RMAT-20 ----------------

def test_config1_bfs_rmat20(oracle_lib):
    import janusgraph_amd as jg
    o = oracle_lib
    scale = 20
    n = 1 << scale
    s, d = host_edges(o, scale)
    ptr, adj = o.csr_unordered(n, s, d, both=True)
    ctx = jg.Context((0,))
    g = ctx.build_rmat(scale, EF, seed_of(scale), flags=jg.ADJ_BOTH)
    for sv in pick_sources(ptr, 3, scale):
        got = g.bfs([int(sv)], jg.DIR_BOTH)[0]
        want = o.bfs_csr(n, ptr, adj, int(sv))
        np.testing.assert_array_equal(got, want)
        err, edges = o.bfs_validate(n, s, d, got, int(sv))
        assert err == 0 and edges > 0
        bounded = g.bfs([int(sv)], jg.DIR_BOTH, max_depth=2)[0]
        np.testing.assert_array_equal(bounded, o.bfs_csr(n, ptr, adj, int(sv), 2))
    g.close()
    ctx.close()


# ---------------- configs[2]: PageRank RMAT-24 ----------------

@pytest.fixture(scope="module")
def pr24(oracle_lib):
    o = oracle_lib
    scale = 24
    n = 1 << scale
    s, d = host_edges(o, scale)
    ec = np.bincount(s, minlength=n).astype(np.float64)
    ip, isrc = o.csr_unordered(n, d, s)
    del s, d
    want = o.pagerank_csr(n, ip, isrc, ec, 0.85, n, 30)
    return n, ec, want


def assert_pr(rank, ec, want, ec_want):
    np.testing.assert_array_equal(ec, ec_want)
    rel = np.abs(rank - want) / np.abs(want)
    assert rel.max() <= PR_RTOL, f"max rel err {rel.max()}"


@pytest.mark.parametrize("shards", [1, 2, 4, 8])
def test_config2_pagerank_rmat24(pr24, shards):
    import janusgraph_amd as jg
    n, ec_want, want = pr24
    ctx = jg.Context((0,) * shards)
    g = ctx.build_rmat(24, EF, seed_of(24), flags=jg.ADJ_IN)
    rank, ec = g.pagerank(0.85, n, 30)
    assert ctx.stats()["supersteps"] == 30
    assert_pr(rank, ec, want, ec_want)
    g.close()
    ctx.close()


# ---------------- configs[3], configs[4]: RMAT-26 ----------------

@pytest.fixture(scope="module")
def rmat26(oracle_lib):
    o = oracle_lib
    scale = 26
    n = 1 << scale
    s, d = host_edges(o, scale)
    ptr, adj = o.csr_unordered(n, s, d, both=True)
    lex = o.lex_rank_iota(n)
    label, it = o.cc_csr(n, ptr, adj, lex)
    vid_of_rank = np.empty(n, np.int64)
    vid_of_rank[lex] = np.arange(n, dtype=np.int64)
    del lex
    return {"n": n, "s": s, "d": d, "ptr": ptr, "adj": adj, "label": label, "cc_it": it,
            "vid_of_rank": vid_of_rank}


def test_config3_cc_rmat26(rmat26):
    import janusgraph_amd as jg
    r = rmat26
    ctx = jg.Context((0,))
    g = ctx.build_rmat(26, EF, seed_of(26), flags=jg.ADJ_BOTH)
    comp, it = g.connected_components()
    assert it == r["cc_it"]
    assert it < 99  # Fulgora's 100-iteration cap does not bind
    np.testing.assert_array_equal(comp, r["vid_of_rank"][r["label"]])
    g.close()
    ctx.close()


def test_config3_dobfs_rmat26_one_gpu(oracle_lib, rmat26):
    """The single-GPU DO-BFS at RMAT-26 that bench.py's rmat26.bfs block times: one shard, BOTH CSR of
    2.15 G entries (past 2^31: int64 row offsets, the 2^31-entry boundary inside the hub rows).  Sources
    are the bench's first candidates (same seeded pick among degree > 0 vertices), one depth-bounded;
    depths bit-exact against the oracle, Graph500 validation of one (SPVP's forced BOTH scope,
    FulgoraGraphComputer.java:249-253)."""
    import janusgraph_amd as jg
    o = oracle_lib
    r = rmat26
    n = r["n"]
    ctx = jg.Context((0,))
    g = ctx.build_rmat(26, EF, seed_of(26), flags=jg.ADJ_BOTH)
    assert g.info()["num_shards"] == 1
    deg = np.diff(r["ptr"])
    cand = np.flatnonzero(deg > 0)
    srcs = np.random.default_rng(26).choice(cand, 16, replace=False)[:3]  # bench.py bfs_block's first draws
    for k, sv in enumerate(srcs.tolist()):
        got = g.bfs([sv], jg.DIR_BOTH)[0]
        want = o.bfs_csr(n, r["ptr"], r["adj"], sv)
        np.testing.assert_array_equal(got, want, err_msg=f"one GPU: DO-BFS from {sv}")
        if k == 0:
            err, edges = o.bfs_validate(n, r["s"], r["d"], got, sv, r["label"])
            assert err == 0 and edges > 0, f"Graph500 validation bits {err} for source {sv}"
        del got
        if k == 1:
            bounded = g.bfs([sv], jg.DIR_BOTH, max_depth=3)[0]
            np.testing.assert_array_equal(bounded, o.bfs_csr(n, r["ptr"], r["adj"], sv, 3),
                                          err_msg=f"one GPU: DO-BFS from {sv}, maxDepth 3")
            del bounded
        del want
    g.close()
    ctx.close()


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_config3_sharded_cc_and_dobfs_rmat26(oracle_lib, rmat26, shards):
    """The code paths 2..8 GPUs run at configs[3]'s size: CC by label propagation over the BOTH halo
    (not the one-shard union-find), and single-source DO-BFS by dobfs_sharded (halo refresh for
    bottom-up levels, stamps and the reverse exchange for top-down levels)."""
    import janusgraph_amd as jg
    o = oracle_lib
    r = rmat26
    n = r["n"]
    ctx = jg.Context((0,) * shards)
    g = ctx.build_rmat(26, EF, seed_of(26), flags=jg.ADJ_BOTH)
    assert g.info()["num_shards"] == shards and g.info()["exchange_values"] > 0
    comp, it = g.connected_components()
    assert it == r["cc_it"], f"{shards} shards: {it} supersteps, oracle {r['cc_it']}"
    np.testing.assert_array_equal(comp, r["vid_of_rank"][r["label"]])
    del comp
    for sv in pick_sources(r["ptr"], 3, 126 + shards):
        got = g.bfs([int(sv)], jg.DIR_BOTH)[0]
        np.testing.assert_array_equal(got, o.bfs_csr(n, r["ptr"], r["adj"], int(sv)),
                                      err_msg=f"{shards} shards: DO-BFS from {sv}")
        assert ctx.stats()["levels"] > 2
    g.close()
    ctx.close()


def test_config4_msbfs64_rmat26(oracle_lib, rmat26):
    """8 logical shards and one shard: top-down levels for small frontiers (sharded: own frontier rows
    pushed, the peers' bits returned by the reverse halo exchange), split pull levels between them."""
    import janusgraph_amd as jg
    o = oracle_lib
    r = rmat26
    n = r["n"]
    srcs = pick_sources(r["ptr"], 64, 26)
    want = o.msbfs_csr(n, r["ptr"], r["adj"], srcs)
    for shards in (8, 1):
        ctx = jg.Context((0,) * shards)
        g = ctx.build_rmat(26, EF, seed_of(26), flags=jg.ADJ_BOTH)
        assert g.info()["num_shards"] == shards
        got = g.bfs(srcs, jg.DIR_BOTH)
        g.close()
        ctx.close()
        for k in range(64):
            assert np.array_equal(got[k], want[k]), f"{shards} shards: source {k} ({srcs[k]}) differs"
        for k in (0, 31, 63):
            err, _ = o.bfs_validate(n, r["s"], r["d"], got[k], int(srcs[k]), r["label"])
            assert err == 0, f"{shards} shards: Graph500 validation bits {err} for source {k}"
        del got
