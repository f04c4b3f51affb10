"""A/B timing of connected-components variants (build-time band knobs) on one RMAT graph (diagnostic).

Variants are "name:key=value,..." of jg_tune_set knobs, as in tools/pr_ab.py; every variant builds its
BOTH adjacency, then all are timed in interleaved rounds.  Reports the median CC time and whether
every variant's labels equal the first's.
  python tools/cc_ab.py --scale 26 b5:band0_bit=5 b6:band0_bit=6
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402
from pr_ab import apply  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    ctx = jg.Context((0,))
    vs = []
    for spec in args.variants:
        name, _, kv = spec.partition(":")
        knobs = {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}
        apply(knobs)
        vs.append((name, knobs, ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=jg.ADJ_BOTH)))
    times = {name: [] for name, _, _ in vs}
    comps = {}
    for r in range(args.rounds):
        for name, knobs, g in vs:
            apply(knobs)
            comp, _ = g.connected_components()
            times[name].append(ctx.stats()["compute_ms"])
            if r == 0:
                comps[name] = comp
    first = vs[0][0]
    out = {name: {"median_ms": round(float(np.median(t)), 3),
                  "same_labels": bool(np.array_equal(comps[name], comps[first]))} for name, t in times.items()}
    print(json.dumps({"scale": args.scale, "variants": out}))


if __name__ == "__main__":
    main()
