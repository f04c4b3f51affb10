"""CPU count of what a 64-source BFS pull level scans with and without a per-row early exit (numpy; the
study behind msbfs_exit).  A row's gain is the OR of its neighbours' frontier words masked
by need = ~visited & live (live: every source with a frontier bit); once the running OR covers need no
further entry can add a bit.  Per level and degree band (>= 128, 8..127, < 8 entries) it prints the
entries of rows that can still gain a bit (what the merge engine's live-task skip keeps, at row
granularity) and the entries scanned up to each row's exit.

    python tools/msbfs_exit_sim.py --scale 22

The graph is a numpy Graph500-style Kronecker RMAT (a, b, c = 0.57, 0.19, 0.19; both directions, self
loops dropped), statistically the library's jg_build_rmat graph, not the same edges; sources are a seeded
uniform pick among vertices with an entry (bench.pick_sources' rule).  Memory: ~40 B per entry (RMAT-22:
134 M entries, ~6 GB).
"""
import argparse

import numpy as np


def rmat(scale, ef, seed):
    rng = np.random.default_rng(seed)
    m = ef << scale
    src = np.zeros(m, np.int64)
    dst = np.zeros(m, np.int64)
    for bit in range(scale):
        r = rng.random(m)
        # quadrant: a (0,0) 0.57, b (0,1) 0.19, c (1,0) 0.19, d (1,1) 0.05
        sbit = r >= 0.76
        dbit = ((r >= 0.57) & (r < 0.76)) | (r >= 0.95)
        src |= sbit.astype(np.int64) << bit
        dst |= dbit.astype(np.int64) << bit
    perm = rng.permutation(1 << scale)  # Graph500 scrambles the vertex ids
    return perm[src], perm[dst]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    n = 1 << a.scale
    src, dst = rmat(a.scale, 16, a.seed)
    keep = src != dst
    s = np.concatenate([src[keep], dst[keep]])
    d = np.concatenate([dst[keep], src[keep]])
    order = np.lexsort((d, s))
    s, col = s[order], d[order]
    m = len(col)
    deg = np.bincount(s, minlength=n)
    ptr = np.concatenate([[0], np.cumsum(deg)])
    cand = np.flatnonzero(deg > 0)
    srcs = np.random.default_rng(a.seed).choice(cand, min(64, len(cand)), replace=False)
    F = np.zeros(n, np.uint64)
    for b, v in enumerate(srcs):
        F[v] |= np.uint64(1) << np.uint64(b)
    vis = F.copy()
    rowid = np.repeat(np.arange(n), deg)
    pos = np.arange(m) - ptr[rowid]
    band = np.where(deg >= 128, 0, np.where(deg >= 8, 1, 2))
    for level in range(16):
        live = np.bitwise_or.reduce(F)
        if live == 0:
            break
        need = ~vis & live
        g = F[col]
        acc = g.copy()
        step = 1
        while step < deg.max():  # segmented inclusive OR scan (Hillis-Steele within rows)
            sh = np.zeros_like(acc)
            sh[step:] = acc[:-step]
            acc = np.where(pos >= step, acc | sh, acc)
            step <<= 1
        nr = need[rowid]
        active = nr != 0
        notcov = ((acc & nr) != nr) & active
        scanned = np.bincount(rowid, weights=notcov, minlength=n)
        covered = np.bincount(rowid, weights=(~notcov) & active, minlength=n) > 0
        exit_scan = scanned + covered
        parts = []
        for b in range(3):
            rb = band == b
            parts.append("band %d %.1f%% -> %.1f%%" % (b, 100 * deg[rb & (need != 0)].sum() / m, 100 * exit_scan[rb].sum() / m))
        print("level %d: frontier %d rows | entries of rows that can gain: %.1f%% of m, with the exit %.1f%% | %s" % (
            level, int((F != 0).sum()), 100 * deg[need != 0].sum() / m, 100 * exit_scan.sum() / m, "; ".join(parts)))
        newF = np.zeros(n, np.uint64)
        np.bitwise_or.at(newF, rowid, g)
        newF &= ~vis
        vis |= newF
        F = newF


if __name__ == "__main__":
    main()
