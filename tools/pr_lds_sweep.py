"""Sweep the LDS-staged hot prefix size of the pull superstep (one process, interleaved rounds)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402
from janusgraph_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sizes", default="0,4096,8192,16384,20480")
    args = ap.parse_args()
    ctx = jg.Context((0,))
    n = 1 << args.scale
    g = ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=jg.ADJ_IN)
    _lib.tune_set("pull_split", 0)
    sizes = [int(x) for x in args.sizes.split(",")]
    res = {s: [] for s in sizes}
    ranks = {}
    for r in range(args.rounds):
        for s in sizes:
            _lib.tune_set("pull_lds", s)
            g.pagerank_begin(0.85, n)
            g.pagerank_step(2)
            g.sync()
            t0 = time.perf_counter()
            g.pagerank_step(args.steps)
            g.sync()
            res[s].append((time.perf_counter() - t0) / args.steps * 1e3)
            rank, _ = g.pagerank_end(want=(r == 0))
            if r == 0:
                ranks[s] = rank
    base = ranks[sizes[0]]
    out = {s: {"median_ms": round(float(np.median(v)), 4),
               "max_rel_vs_off": float(np.max(np.abs(ranks[s] - base) / base))} for s, v in res.items()}
    _lib.tune_set("pull_lds", 0)
    _lib.tune_set("pull_split", 0)
    print(json.dumps({"scale": args.scale, "lds": out}))


if __name__ == "__main__":
    main()
