"""Single-source DO-BFS runs on an RMAT graph, for per-level rocprofv3 kernel traces (diagnostic).
Prints, per run, the source, levels, edges traversed and ms."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=20)
ap.add_argument("--runs", type=int, default=4)
ap.add_argument("--shards", type=int, default=1, help="logical shards on device 0 (sharded DO-BFS when > 1)")
ap.add_argument("--tune", nargs="*", default=[], help="jg_tune_set knobs, key=value")
a = ap.parse_args()
for kv in a.tune:
    k, v = kv.split("=")
    jg._lib.tune_set(k, int(v))
ctx = jg.Context((0,) * a.shards)
g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
rng = np.random.default_rng(1)
for k in range(a.runs):
    s = int(rng.integers(0, 1 << a.scale))
    g.bfs([s], jg.DIR_BOTH, want=False)
    st = ctx.stats()
    print(s, st["levels"], st["edges_traversed"], round(st["compute_ms"], 4), flush=True)
