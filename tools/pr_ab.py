"""A/B timing of PageRank pull-engine variants on one RMAT graph shape (diagnostic, not a benchmark).

Each variant is "name:key=value,key=value" of jg_tune_set knobs, applied before its graph is built
(build-time knobs: pull_split, band<i>_deg, band<i>_bit) and while it runs.  All variants are
built once and timed in interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
Reports the median ms per superstep and the max relative difference of the ranks vs the first.
  python tools/pr_ab.py --scale 24 plain:pull_split=0 split:pull_split=1
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

DEFAULTS = {"pull_split": 1, "merge_temporal": 1, "merge_pack": 1, "merge_stage0": -1, "merge_stage1": -1,
            "merge_stage2": -1, "merge_stage3": -1,
            "band0_deg": 96, "band0_bit": 0, "band1_deg": -1, "band1_bit": 0, "band2_deg": -1, "band2_bit": 0,
            "band3_deg": 0, "band3_bit": 3}


def apply(knobs):
    for k, v in {**DEFAULTS, **knobs}.items():
        _lib.tune_set(k, v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shared-graph", action="store_true",
                    help="one graph built with the defaults for every variant (run-time knobs only): the "
                         "variants then differ by nothing but their knobs, not by the graph's memory placement")
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    ctx = jg.Context((0,))
    n = 1 << args.scale
    vs = []
    shared = None
    if args.shared_graph:
        apply({})
        shared = ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=jg.ADJ_IN)
    for spec in args.variants:
        name, _, kv = spec.partition(":")
        knobs = {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}
        apply(knobs)
        vs.append((name, knobs, shared if shared is not None else ctx.build_rmat(args.scale, 16, 0x5EED + args.scale,
                                                                                  flags=jg.ADJ_IN)))
    times = {name: [] for name, _, _ in vs}
    ranks = {}
    for r in range(args.rounds):
        for name, knobs, g in vs:
            apply(knobs)
            g.pagerank_begin(0.85, n)
            g.pagerank_step(2)
            g.sync()
            t0 = time.perf_counter()
            g.pagerank_step(args.steps)
            g.sync()
            times[name].append((time.perf_counter() - t0) / args.steps * 1e3)
            rank, _ = g.pagerank_end(want=(r == 0))
            if r == 0:
                ranks[name] = rank
    base = ranks[vs[0][0]]
    out = {name: {"median_ms": round(float(np.median(t)), 4),
                  "max_rel_vs_first": float(np.max(np.abs(ranks[name] - base) / base))} for name, t in times.items()}
    apply({})
    print(json.dumps({"scale": args.scale, "steps": args.steps, "variants": out}))


if __name__ == "__main__":
    main()
