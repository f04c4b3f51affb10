"""The in-process multi-device layout, checked on one GPU.

The Java computer shards with `computer.gpu.devices=0,1,...`: one process, one context over several
devices (jg_ctx_create with distinct devices, ncclCommInitAll).  No box here has two GPUs, and logical
shards (every shard on device 0) hide a buffer placed on the wrong device: it still works.  With
JG_VDEV_CHECK=1 every logical shard is a virtual device: a DevBuf records the shard whose guard was
current at its allocation, and a DevBuf handed to a kernel or copy under another shard's guard fails the
call with JG_ERR_STATE (jg_common.h).  Every sharded program runs here under the check, against the oracle,
on 2, 3 and 8 shards; JG_VDEV_FAULT=1 misplaces one buffer (a per-shard PageRank vector allocated under
the first shard's guard, the ADVICE r03 bug class) and the check must catch it.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PR_RTOL = 1e-9


def rmat_graph(o, scale):
    s, t = o.rmat_edges(scale, 16, 11)
    n = 1 << scale
    vid = (np.random.default_rng(scale).permutation(n).astype(np.int64) + 1) << 8
    w = (np.arange(len(s)) % 7 + 1).astype(np.int32)
    return n, vid, s, t, w


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_sharded_programs_under_virtual_device_check(oracle_lib, monkeypatch, shards):
    import janusgraph_amd as jg
    o = oracle_lib
    monkeypatch.setenv("JG_VDEV_CHECK", "1")
    n, vid, s, t, w = rmat_graph(o, 14)
    c = jg.Context((0,) * shards)
    try:
        g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
        assert g.info()["num_shards"] == shards
        rank, _ = g.pagerank(0.85, n, 10)
        want, _ = o.pagerank(n, s, t, 0.85, n, 10)
        rel = np.abs(rank - want) / np.maximum(np.abs(want), 1e-300)
        assert rel.max() <= PR_RTOL
        comp, it = g.connected_components()
        comp_ref, it_ref = o.connected_components(n, s, t, vid)
        np.testing.assert_array_equal(comp, comp_ref)
        assert it == it_ref
        deg = np.bincount(s, minlength=n) + np.bincount(t, minlength=n)
        cand = np.flatnonzero(deg > 0)
        src = int(cand[len(cand) // 3])
        np.testing.assert_array_equal(g.bfs([vid[src]], jg.DIR_BOTH)[0], o.bfs(n, s, t, src, o.DIR_BOTH))
        srcs = cand[::max(len(cand) // 64, 1)][:64]
        got = g.bfs(vid[srcs], jg.DIR_BOTH)
        for k in (0, 31, len(srcs) - 1):
            np.testing.assert_array_equal(got[k], o.bfs(n, s, t, int(srcs[k]), o.DIR_BOTH))
        dist = g.shortest_distance(vid[src], 4)
        np.testing.assert_array_equal(dist, o.shortest_distance(n, s, t, src, 4))
        g.close()
        gw = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT, weight=w)
        np.testing.assert_array_equal(gw.shortest_distance(vid[src], 5), o.shortest_distance(n, s, t, src, 5, w))
        gw.close()
    finally:
        c.close()


def test_virtual_device_check_catches_a_misplaced_buffer(oracle_lib, monkeypatch):
    import janusgraph_amd as jg
    o = oracle_lib
    monkeypatch.setenv("JG_VDEV_CHECK", "1")
    monkeypatch.setenv("JG_VDEV_FAULT", "1")
    n, vid, s, t, _ = rmat_graph(o, 12)
    c = jg.Context((0,) * 3)
    try:
        g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN)
        with pytest.raises(jg.JanusGpuError) as e:
            g.pagerank(0.85, n, 3)
        assert e.value.code == -6 and "virtual-device check" in str(e.value)
    finally:
        c.close()  # (closes g first)
    # the same misplacement without the check goes unnoticed on one device (what the check is for)
    monkeypatch.delenv("JG_VDEV_CHECK")
    c = jg.Context((0,) * 3)
    try:
        g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN)
        rank, _ = g.pagerank(0.85, n, 3)
        want, _ = o.pagerank(n, s, t, 0.85, n, 3)
        assert np.allclose(rank, want, rtol=PR_RTOL, atol=0)
        g.close()
    finally:
        c.close()
