"""CPU model of the near-far delta-stepping queue discipline (jg_traverse.hip sd_delta_stepping,
sd_near_kernel, sd_far_split_kernel) against the oracle's supersteps (oracle/jg_oracle.c
jo_shortest_distance), no GPU: the pass stamps, the far flags, the drop of far entries below the previous
threshold and the jump past an empty bucket are restated here step for step, with the passes' relaxations
applied in a shuffled order (the kernel's lanes race; the result must not depend on the order)."""
import numpy as np
import pytest

DEPTH_INF = 2**31 - 1
INF = np.iinfo(np.int64).max


def in_csr(n, s, t, w):
    """Row x's entries: the sources u of the edges u -> x (the IN adjacency sd_near_kernel walks)."""
    order = np.argsort(t, kind="stable")
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, t + 1, 1)
    return np.cumsum(rp), s[order], w[order]


def delta_stepping_model(n, s, t, w, seed, delta, rng):
    rp, col, wt = in_csr(n, s, t, w)
    dist = np.full(n, INF, np.int64)
    stamp = np.zeros(n, np.int64)
    far_flag = np.zeros(n, bool)
    dist[seed] = 0
    near, far = [seed], []
    T, npass = delta, 0
    while True:
        while near:  # sd_near_kernel passes
            npass += 1
            edges = [(x, j) for x in near for j in range(rp[x], rp[x + 1])]
            rng.shuffle(edges)
            nxt = []
            for x, j in edges:
                u, nd = col[j], dist[x] + int(wt[j])
                if nd < dist[u]:
                    dist[u] = nd
                    if nd < T:
                        if stamp[u] != npass:
                            stamp[u] = npass
                            nxt.append(u)
                    elif not far_flag[u]:
                        far_flag[u] = True
                        far.append(u)
            near = nxt
        if not far:
            break
        T2 = T + delta
        for _ in range(2):  # sd_far_split_kernel, again past the smallest kept distance if the bucket is empty
            if near or not far:
                break
            keep, minkept = [], INF
            for u in far:
                d = dist[u]
                if d >= T2:
                    keep.append(u)
                    minkept = min(minkept, d)
                else:
                    far_flag[u] = False
                    if d >= T:
                        near.append(u)
            far = keep
            if not near and far:
                T2 = (minkept // delta + 1) * delta
        T = T2
    out = dist.copy()
    out[out == INF] = np.iinfo(np.int64).min
    return out, npass


@pytest.mark.parametrize("delta", [1, 2, 5, 17, 1000])
@pytest.mark.parametrize("case", ["random", "zero_weights", "path"])
def test_delta_stepping_model_matches_oracle(oracle_lib, delta, case):
    rng = np.random.default_rng(delta * 7 + len(case))
    if case == "path":
        n = 40
        s, t = np.arange(1, n, dtype=np.int32), np.arange(0, n - 1, dtype=np.int32)
        w = rng.integers(0, 5, n - 1).astype(np.int32)
    else:
        n, m = 300, 1500
        s, t = rng.integers(0, n, m).astype(np.int32), rng.integers(0, n, m).astype(np.int32)
        w = rng.integers(0 if case == "zero_weights" else 1, 4 if case == "zero_weights" else 60, m).astype(np.int32)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    for trial in range(3):
        got, _ = delta_stepping_model(n, s, t, w, 0, delta, np.random.default_rng(trial))
        np.testing.assert_array_equal(got, want)


def test_delta_one_is_one_pass_per_distance(oracle_lib):
    """Weights >= 1 and delta = 1: each pass settles exactly one distance value (what
    tests/test_gpu_sssp_delta.py::test_delta_path_runs checks on the GPU's pass count)."""
    rng = np.random.default_rng(4)
    n, m = 200, 1200
    s, t = rng.integers(0, n, m).astype(np.int32), rng.integers(0, n, m).astype(np.int32)
    w = rng.integers(1, 9, m).astype(np.int32)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    got, npass = delta_stepping_model(n, s, t, w, 0, 1, rng)
    np.testing.assert_array_equal(got, want)
    assert npass == len(np.unique(want[want >= 0]))
