"""A/B of build-time knobs on the BOTH-adjacency programs (diagnostic): every variant builds its own
RMAT graph (jg_tune_set knobs "name:key=value,..." applied before the build, as in tools/pr_ab.py),
then CC and the bench's 64-source BFS are timed in interleaved rounds.  Reports median HIP-event ms and
whether every variant's CC labels and BFS depths equal the first's.
    python tools/build_ab.py --scale 26 col: nopack:merge_pack=0
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
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    ctx = jg.Context((0,))
    vs = []
    for spec in a.variants:
        name, _, kv = spec.partition(":")
        knobs = {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}
        apply(knobs)
        g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
        vs.append((name, knobs, g, ctx.stats()["build_ms"]))
    apply({})
    srcs = bench.pick_sources(vs[0][2].degrees(jg.DIR_BOTH), 64, 7)
    cc_ms = {v[0]: [] for v in vs}
    ms_ms = {v[0]: [] for v in vs}
    first = {}
    same = {v[0]: True for v in vs}
    for r in range(a.rounds):
        for name, knobs, g, _ in vs:
            apply(knobs)
            comp, _ = g.connected_components()
            cc_ms[name].append(ctx.stats()["compute_ms"])
            depth = g.bfs(srcs[:8], jg.DIR_BOTH) if r == 0 else None
            g.bfs(srcs, jg.DIR_BOTH, want=False)
            ms_ms[name].append(ctx.stats()["compute_ms"])
            if r == 0:
                if not first:
                    first = {"comp": comp, "depth": depth}
                else:
                    same[name] = bool(np.array_equal(comp, first["comp"]) and np.array_equal(depth, first["depth"]))
    apply({})
    print(json.dumps({"scale": a.scale, "variants": {
        name: {"build_ms": round(b, 1), "cc_ms": round(float(np.median(cc_ms[name])), 4),
               "msbfs64_ms": round(float(np.median(ms_ms[name])), 4), "same_results_as_first": same[name]}
        for name, _, _, b in vs}}))


if __name__ == "__main__":
    main()
