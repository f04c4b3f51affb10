"""CPU model of the near-far delta-stepping step discipline (jg_traverse.hip sd_delta_stepping_t,
sd_decide, sd_split_kernel, sd_near_kernel: the passes controlled on the device, round 6) against the
oracle's supersteps (oracle/jg_oracle.c jo_shortest_distance), no GPU: each step relaxes its near queue
when that has entries, else stops when the far pile is empty, else moves the far pile with the threshold
past the previous one by delta or at the bucket of the smallest far distance seen (the split's kept
minimum and every far relaxation since); pass stamps, far flags and the drop of far entries below the
previous threshold are restated step for step, with each pass's relaxations applied in a shuffled order
(the kernel's lanes race; the result must not depend on the order)."""
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
    T, npass, step, fmin_prev = delta, 0, 0, INF
    while True:
        # sd_decide / sd_split_kernel
        if sum(rp[x + 1] - rp[x] for x in near) > 0:
            fmin = fmin_prev  # no split: the far minimum carries over
        elif not far:
            break
        else:
            t2 = T + delta
            if fmin_prev != INF:
                t2 = max(t2, (fmin_prev // delta + 1) * delta)
            keep, fmin = [], INF
            for u in far:
                d = dist[u]
                if d >= t2:
                    keep.append(u)
                    fmin = min(fmin, d)
                else:
                    far_flag[u] = False
                    if d >= T:
                        near.append(u)
            far, T = keep, t2
        # sd_near_kernel (pass = step + 1); a queue with rows counts as a pass
        if near:
            npass += 1
        edges = [(x, j) for x in near for j in range(rp[x], rp[x + 1])]
        rng.shuffle(edges)
        nxt = []
        for x, j in edges:
            u, nd = col[j], dist[x] + int(wt[j])
            if nd < dist[u]:
                dist[u] = nd
                if nd < T:
                    if stamp[u] != step + 1:
                        stamp[u] = step + 1
                        nxt.append(u)
                else:
                    fmin = min(fmin, nd)
                    if not far_flag[u]:
                        far_flag[u] = True
                        far.append(u)
        near, fmin_prev = nxt, fmin
        step += 1
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
    tests/test_gpu_sssp_delta.py::test_delta_path_runs checks on the GPU's pass count: at least one pass per
    distinct distance)."""
    rng = np.random.default_rng(4)
    n, m = 200, 1200
    s, t = rng.integers(0, n, m).astype(np.int32), rng.integers(0, n, m).astype(np.int32)
    w = rng.integers(1, 9, m).astype(np.int32)
    want = oracle_lib.shortest_distance(n, s, t, 0, DEPTH_INF, w)
    got, npass = delta_stepping_model(n, s, t, w, 0, 1, rng)
    np.testing.assert_array_equal(got, want)
    assert npass == len(np.unique(want[want >= 0]))
