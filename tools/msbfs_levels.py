"""64-source bit-parallel BFS (configs[4]) on RMAT-<scale> with the bench's sources, for a kernel trace:
prints levels and time; run under rocprofv3 --kernel-trace to see each level's launches.
  python tools/msbfs_levels.py [--scale 26] [--reps 2] [knob=value ...]"""
import argparse
import json
import os
import sys

import numpy as np

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
    n = 1 << a.scale
    ctx = jg.Context((0,))
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    rng = np.random.default_rng(7)
    srcs = np.unique(rng.integers(0, n, 4 * 64))[:64]
    out = []
    for _ in range(a.reps):
        g.bfs(srcs, jg.DIR_BOTH, want=False)
        st = ctx.stats()
        out.append({"ms": round(st["compute_ms"], 3), "levels": st["levels"]})
    print(json.dumps({"scale": a.scale, "knobs": a.knobs, "runs": out}), flush=True)


if __name__ == "__main__":
    main()
