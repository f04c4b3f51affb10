"""Sweep the XCD-split threshold (rows of degree >= D are split over the 8 XCD column ranges).

For each D: build RMAT-`scale`, then time PageRank supersteps with the split off / per-XCD queues /
static mapping, interleaved in one process.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402
from janusgraph_amd import _lib  # noqa: E402


def time_steps(g, n, steps):
    g.pagerank_begin(0.85, n)
    g.pagerank_step(2)
    g.sync()
    t0 = time.perf_counter()
    g.pagerank_step(steps)
    g.sync()
    dt = (time.perf_counter() - t0) / steps * 1e3
    g.pagerank_end(want=False)
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--degrees", default="512,1024,2048,4096,8192")
    args = ap.parse_args()
    ctx = jg.Context((0,))
    n = 1 << args.scale
    out = {}
    for d in [int(x) for x in args.degrees.split(",")]:
        _lib.tune_set("split_min_degree", d)
        _lib.tune_set("pull_split", 1)  # build the split plan
        g = ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=jg.ADJ_IN)
        res = {0: [], 1: [], 2: []}
        for _ in range(args.rounds):
            for mode in (0, 1, 2):
                _lib.tune_set("pull_split", mode)
                res[mode].append(time_steps(g, n, args.steps))
        out[d] = {f"split{m}": round(float(np.median(v)), 4) for m, v in res.items()}
        g.close()
    _lib.tune_set("pull_split", 0)
    print(json.dumps({"scale": args.scale, "ms_per_step": out}))


if __name__ == "__main__":
    main()
