"""Combiner program (jg_combine_steps, the DegreeCounter family) on an RMAT graph: time per superstep
(HIP events), GTEPS and achieved GB/s against the 12 B/entry + 16 B/row model; spot parity of one
DegreeCounter(2) run against the numpy oracle on a sample of vertices.
Usage: python tools/combine_bench.py [--scale 24] [--steps 10]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--direction", choices=["out", "in", "both"], default="out")
    args = ap.parse_args()
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    d = {"out": (jg.DIR_OUT, jg.ADJ_OUT), "in": (jg.DIR_IN, jg.ADJ_IN), "both": (jg.DIR_BOTH, jg.ADJ_BOTH)}[args.direction]
    g = ctx.build_rmat(args.scale, 16, 0x5EED + args.scale, flags=d[1])
    g.combine_steps(d[0], jg.COMBINE_SUM, 1)  # warm-up
    x, _ = g.combine_steps(d[0], jg.COMBINE_SUM, args.steps)
    st = ctx.stats()
    ms = st["compute_ms"] / args.steps
    m = (16 << args.scale) * (2 if args.direction == "both" else 1)
    line = {"workload": f"combiner_sum_{args.direction}_rmat{args.scale}_ef16", "steps": args.steps,
            "ms_per_superstep": round(ms, 4), "gteps": round(m / (ms * 1e-3) / 1e9, 2),
            "achieved_gbs": round(st["algorithmic_bytes"] / (st["compute_ms"] * 1e-3) / 1e9, 1),
            "frac_of_8tbs": round(st["algorithmic_bytes"] / (st["compute_ms"] * 1e-3) / 1e9 / 8000.0, 4)}
    if args.scale <= 20:
        from oracle import oracle as o
        s, t = o.rmat_edges(args.scale, 16, 0x5EED + args.scale)
        ref, _ = o.combine_steps(1 << args.scale, s, t, d[0], 0, args.steps)
        line["parity"] = bool(np.array_equal(x, ref))
    print(json.dumps(line), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
