"""A/B the pull-kernel variants in ONE process (interleaved rounds; cdna_hip_programming.md §5.4 rule 24).

python tools/pr_variants.py [--scale 24] [--rounds 5] [--steps 10]
Prints per-variant median / min ms per PageRank superstep and checks the ranks are bit-identical.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--variants", default="4:0:0,4:0:1,4:1:1,8:0:1")
    args = ap.parse_args()
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    ctx = jg.Context((0,))
    n = 1 << args.scale
    g = ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=jg.ADJ_IN)
    times = {v: [] for v in variants}
    ranks = {}
    for r in range(args.rounds):
        for v in variants:
            _lib.tune_set("pull_unroll", v[0])
            _lib.tune_set("pull_nt", v[1])
            _lib.tune_set("pull_split", v[2] if len(v) > 2 else 1)
            g.pagerank_begin(0.85, n)
            g.pagerank_step(2)
            g.sync()
            t0 = time.perf_counter()
            g.pagerank_step(args.steps)
            g.sync()
            times[v].append((time.perf_counter() - t0) / args.steps * 1e3)
            if r == 0:
                rank, _ = g.pagerank_end()
                ranks[v] = rank
            else:
                g.pagerank_end(want=False)
    base = ranks[variants[0]]
    out = {}
    for v in variants:
        t = np.array(times[v])
        out[f"unroll{v[0]}_nt{v[1]}_split{v[2] if len(v) > 2 else 1}"] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                                         "identical": bool(np.array_equal(ranks[v], base)),
                                         "max_rel_vs_first": float(np.max(np.abs(ranks[v] - base) / base))}
    print(json.dumps({"scale": args.scale, "steps": args.steps, "variants": out}))


if __name__ == "__main__":
    main()
