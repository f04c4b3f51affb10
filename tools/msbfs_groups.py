"""Replicated graph, partitioned sources: the bench's 64 sources (bench.pick_sources(deg, 64,
7)) split into G groups of 64/G; each group is one bit-parallel BFS on the full graph, as one GPU of a G-GPU node
holding the whole snapshot would run it.  The modelled G-GPU time is the slowest group (no exchange at all);
the 1-GPU time is the 64-source traversal.  One JSON line per (groups, repetition).
    python tools/msbfs_groups.py --scale 26 --groups 1 8
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_groups(g, ctx, jg, parts, G, a, key, val):
    for part in parts:
        g.bfs(part, jg.DIR_BOTH, want=False)  # warm every group once
    for rep in range(a.reps):
        ms, lv, ex = [], [], []
        for part in parts:
            g.bfs(part, jg.DIR_BOTH, want=False)
            st = ctx.stats()
            ms.append(st["compute_ms"])
            lv.append(st["levels"])
            ex.append(st["edges_traversed"])
        print(json.dumps({"scale": a.scale, "groups": G, "rep": rep, "max_ms": round(max(ms), 3),
                          "sum_ms": round(sum(ms), 3), "ms": [round(x, 3) for x in ms], "levels": lv,
                          "examined_M": [round(x / 1e6, 1) for x in ex], "tune": a.tune,
                          "sweep": [key, val] if key else None}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--groups", type=int, nargs="+", default=[1, 8])
    p.add_argument("--tune", action="append", default=[], help="a fixed jg_tune_set knob (key=value; repeatable)")
    p.add_argument("--sweep", nargs="+", default=None, help="key v1 v2 ...: one set of lines per value")
    a = p.parse_args()
    import bench
    import janusgraph_amd as jg
    for kv in a.tune:
        k, _, v = kv.partition("=")
        jg._lib.tune_set(k, int(v))
    ctx = jg.Context((0,))
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    srcs = bench.pick_sources(g.degrees(jg.DIR_BOTH), 64, 7)
    sweep = [(a.sweep[0], int(v)) for v in a.sweep[1:]] if a.sweep else [(None, None)]
    for key, val in sweep:
        if key:
            jg._lib.tune_set(key, val)
        for G in a.groups:
            run_groups(g, ctx, jg, np.array_split(srcs, G), G, a, key, val)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
