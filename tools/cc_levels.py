"""ConnectedComponentVertexProgram (configs[3]) on RMAT-<scale> for a kernel trace: prints supersteps
and time.  python tools/cc_levels.py [--scale 26] [--reps 2] [knob=value ...]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402
from janusgraph_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("knobs", nargs="*")
    a = ap.parse_args()
    for kv in a.knobs:
        k, v = kv.split("=")
        _lib.tune_set(k, int(v))
    ctx = jg.Context((0,))
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    out = []
    for _ in range(a.reps):
        _, it = g.connected_components()
        out.append({"ms": round(ctx.stats()["compute_ms"], 3), "iterations": it})
    print(json.dumps({"scale": a.scale, "knobs": a.knobs, "runs": out}), flush=True)


if __name__ == "__main__":
    main()
