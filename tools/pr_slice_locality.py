"""Does the XCD slice split turn L2 misses into hits?  (diagnostic, not a benchmark)

Rows of RMAT-`scale` (dst from the Graph500 generator), sources replaced by uniform picks among the
top-2^k vertices by in-degree: at 2^k x 8 B larger than one XCD's 4 MiB L2 but at most 8 x that, the
unsliced pull misses L2 while the static slice split (each XCD gathers 1/8 of the lines) should hit.
Prints ms per superstep for: unsliced, sliced split, sliced split + LDS hot slice, sliced rows unsplit.
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
    ap.add_argument("--ks", default="14,18,20,22")
    args = ap.parse_args()
    n = 1 << args.scale
    src, dst = o.rmat_edges(args.scale, 16, 0x5EED + args.scale)
    order = np.argsort(-np.bincount(dst, minlength=n), kind="stable")
    vid = np.arange(n, dtype=np.int64)
    ctx = jg.Context((0,))
    rng = np.random.default_rng(1)
    out = {}
    for k in [int(x) for x in args.ks.split(",")]:
        s2 = order[rng.integers(0, 1 << k, len(dst))].astype(np.int64)
        r = {}
        _lib.tune_set("pull_split", 0)
        g = ctx.build(vid, s2, dst, flags=jg.ADJ_IN)
        r["unsliced"] = round(time_steps(g, n), 4)
        g.close()
        _lib.tune_set("pull_split", 1)
        g = ctx.build(vid, s2, dst, flags=jg.ADJ_IN)
        r["split_lds"] = round(time_steps(g, n), 4)  # (the split without LDS images was removed in round 5)
        _lib.tune_set("pull_split", 0)
        r["sliced_nosplit"] = round(time_steps(g, n), 4)
        _lib.tune_set("pull_split", 1)
        g.close()
        out[f"top2^{k}"] = r
        print(json.dumps(out), flush=True)
    print(json.dumps({"scale": args.scale, "ms_per_step": out}))


if __name__ == "__main__":
    main()
