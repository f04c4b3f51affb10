"""Is the PageRank pull superstep bound by gather locality?  (diagnostic, not a benchmark)

Same rows as RMAT-`scale` (dst from the Graph500 generator), sources replaced by uniform picks among
the top-2^k vertices by in-degree (= the first 2^k relabelled ids, since the build sorts by
in-degree): k small => every gather hits L1/L2; k = scale => no reuse.  Prints ms per superstep.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import janusgraph_amd as jg  # noqa: E402
from janusgraph_amd import _lib  # noqa: E402
from oracle import oracle as o  # noqa: E402  (generator only)


def time_steps(g, n, steps=10):
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
    ap.add_argument("--ks", default="10,14,18,20,22,24")
    args = ap.parse_args()
    _lib.tune_set("pull_split", 0)
    n = 1 << args.scale
    src, dst = o.rmat_edges(args.scale, 16, 0x5EED + args.scale)
    order = np.argsort(-np.bincount(dst, minlength=n), kind="stable")
    vid = np.arange(n, dtype=np.int64)
    ctx = jg.Context((0,))
    out = {}
    g = ctx.build(vid, src, dst, flags=jg.ADJ_IN)
    out["rmat"] = round(time_steps(g, n), 4)
    g.close()
    rng = np.random.default_rng(1)
    for k in [int(x) for x in args.ks.split(",")]:
        s2 = order[rng.integers(0, 1 << k, len(dst))].astype(np.int64)
        g = ctx.build(vid, s2, dst, flags=jg.ADJ_IN)
        out[f"top2^{k}"] = round(time_steps(g, n), 4)
        g.close()
        print(json.dumps(out), flush=True)
    print(json.dumps({"scale": args.scale, "ms_per_step": out}))


if __name__ == "__main__":
    main()
