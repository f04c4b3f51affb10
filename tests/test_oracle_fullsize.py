"""Pins the oracle's parallel full-size checkers (used by tests/test_gpu_configs.py at RMAT-20..26) to
its serial restatements, which the reference's OLAPTest KATs pin (tests/test_oracle_kats.py)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def g12(oracle_lib):
    o = oracle_lib
    n = 1 << 12
    s, t = o.rmat_edges(12, 16, 3)
    s = np.concatenate([s, [7, 7, 9]])  # a self-loop and a multi-edge beyond the generator's own
    t = np.concatenate([t, [7, 9, 7]])
    ptr, adj = o.csr_unordered(n, s, t, both=True)
    return n, s.astype(np.int32), t.astype(np.int32), ptr, adj


def test_csr_unordered_matches_bincount(oracle_lib, g12):
    n, s, t, ptr, adj = g12
    deg = np.bincount(s, minlength=n) + np.bincount(t, minlength=n)
    np.testing.assert_array_equal(np.diff(ptr), deg)
    ip, isrc = oracle_lib.csr_unordered(n, t, s)
    np.testing.assert_array_equal(np.diff(ip), np.bincount(t, minlength=n))
    for v in (0, 7, 9, 100):  # same multiset of neighbours per row
        np.testing.assert_array_equal(np.sort(isrc[ip[v]:ip[v + 1]]), np.sort(s[t == v]))


@pytest.mark.parametrize("max_depth", [-1, 0, 1, 3])
def test_bfs_csr_matches_serial(oracle_lib, g12, max_depth):
    o = oracle_lib
    n, s, t, ptr, adj = g12
    for src in (0, 7, 123, n - 1):
        np.testing.assert_array_equal(o.bfs_csr(n, ptr, adj, src, max_depth),
                                      o.bfs(n, s, t, src, o.DIR_BOTH, max_depth))


@pytest.mark.parametrize("max_depth", [-1, 0, 2])
def test_msbfs_csr_matches_serial(oracle_lib, g12, max_depth):
    o = oracle_lib
    n, s, t, ptr, adj = g12
    srcs = np.random.default_rng(5).integers(0, n, 64)
    srcs[1] = srcs[0]  # a duplicate source gets its own row
    got = o.msbfs_csr(n, ptr, adj, srcs, max_depth)
    for k, sv in enumerate(srcs):
        np.testing.assert_array_equal(got[k], o.bfs(n, s, t, int(sv), o.DIR_BOTH, max_depth))


@pytest.mark.parametrize("n", [1, 2, 9, 10, 11, 99, 100, 101, 1000, 4097])
def test_lex_rank_iota(oracle_lib, n):
    np.testing.assert_array_equal(oracle_lib.lex_rank_iota(n), oracle_lib.lex_rank(np.arange(n)))


def test_cc_csr_matches_serial(oracle_lib, g12):
    o = oracle_lib
    n, s, t, ptr, adj = g12
    lex = o.lex_rank_iota(n)
    label, it = o.cc_csr(n, ptr, adj, lex)
    inv = np.empty(n, np.int64)
    inv[lex] = np.arange(n)
    want, it_want = o.connected_components(n, s, t, np.arange(n, dtype=np.int64))
    np.testing.assert_array_equal(inv[label], want)
    assert it == it_want


def test_pagerank_csr_matches_serial(oracle_lib, g12):
    o = oracle_lib
    n, s, t, _, _ = g12
    ip, isrc = o.csr_unordered(n, t, s)
    ec = np.bincount(s, minlength=n).astype(np.float64)
    for vc, k in ((n, 30), (1, 10), (n + 5, 2)):
        got = o.pagerank_csr(n, ip, isrc, ec, 0.85, vc, k)
        want, ec_want = o.pagerank(n, s, t, 0.85, vc, k)
        np.testing.assert_array_equal(ec, ec_want)
        ok = ~np.isnan(want)
        assert (np.isnan(got) == ~ok).all()
        rel = np.abs(got[ok] - want[ok]) / np.abs(want[ok])
        assert rel.max() <= 1e-12


def test_bfs_validate_flags_bad_depths(oracle_lib, g12):
    o = oracle_lib
    n, s, t, ptr, adj = g12
    d = o.bfs_csr(n, ptr, adj, 7)
    assert o.bfs_validate(n, s, t, d, 7)[0] == 0
    bad = d.copy()
    bad[bad == 2] = 3
    assert o.bfs_validate(n, s, t, bad, 7)[0] != 0
    cut = d.copy()
    cut[np.flatnonzero(d == 1)[0]] = -1
    assert o.bfs_validate(n, s, t, cut, 7)[0] & 2
