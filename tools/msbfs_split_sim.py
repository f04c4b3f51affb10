"""CPU count behind msbfs_srcsplit: on each level of a 64-source BFS, the entries the
split's rows would scan with a per-row early exit when `need` covers every live source, against only the
sources whose frontier holds at least --permille of the entries (the others pushed top-down, whose push
entries are printed too).  numpy; the graph and sources as tools/msbfs_exit_sim.py, rows in degree order.

    python tools/msbfs_split_sim.py --scale 22 --permille 20
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from msbfs_exit_sim import rmat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--permille", type=float, default=20)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    n = 1 << a.scale
    src, dst = rmat(a.scale, 16, a.seed)
    keep = src != dst
    s = np.concatenate([src[keep], dst[keep]])
    d = np.concatenate([dst[keep], src[keep]])
    deg = np.bincount(s, minlength=n)
    order = np.argsort(-deg, kind="stable")  # the relabel: rows by degree, columns ascending (hubs first)
    newid = np.empty(n, np.int64)
    newid[order] = np.arange(n)
    s, d, deg = newid[s], newid[d], deg[order]
    o = np.lexsort((d, s))
    s, col = s[o], d[o]
    ptr = np.concatenate([[0], np.cumsum(deg)])
    m = len(col)
    cand = np.flatnonzero(deg > 0)
    srcs = np.random.default_rng(a.seed).choice(cand, 64, replace=False)
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
        fe = np.zeros(64)
        nz = np.flatnonzero(F)
        for b in range(64):
            mask = ((F[nz] >> np.uint64(b)) & np.uint64(1)).astype(bool)
            fe[b] = deg[nz[mask]].sum()
        big = fe >= a.permille / 1000.0 * m
        live_big = np.uint64(0)
        for b in np.flatnonzero(big):
            live_big |= np.uint64(1) << np.uint64(int(b))
        g = F[col]

        def exit_scan(lv):
            need = ~vis & lv
            acc = g & lv
            step = 1
            while step < deg.max():
                sh = np.zeros_like(acc)
                sh[step:] = acc[:-step]
                acc = np.where(pos >= step, acc | sh, acc)
                step <<= 1
            nr = need[rowid]
            active = nr != 0
            notcov = ((acc & nr) != nr) & active
            ex = np.bincount(rowid, weights=notcov, minlength=n) + (np.bincount(rowid, weights=(~notcov) & active, minlength=n) > 0)
            return [100 * ex[band == b].sum() / m for b in range(3)]

        e_all = exit_scan(live)
        e_big = exit_scan(live_big) if big.any() else [0.0, 0.0, 0.0]
        print("level %d: %d of %d live sources big | exit, all live: bands %.1f / %.1f / %.1f%% of m | big only: %.1f / %.1f / %.1f%% "
              "| the small sources' push: %.1f%% of m" % (level, int(big.sum()), int((fe > 0).sum()), *e_all, *e_big,
                                                          100 * fe[~big].sum() / m))
        newF = np.zeros(n, np.uint64)
        np.bitwise_or.at(newF, rowid, g)
        newF &= ~vis
        vis |= newF
        F = newF


if __name__ == "__main__":
    main()
