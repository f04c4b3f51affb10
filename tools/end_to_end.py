"""Wall-clock of a whole program call as a user sees it (build, run, results copied out in the
caller's vertex order) on RMAT-<scale>: PageRank (K supersteps), single-source BFS, CC, 64-source BFS.
  python tools/end_to_end.py [--scale 24] [--iterations 30]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--iterations", type=int, default=30)
    a = ap.parse_args()
    n = 1 << a.scale
    ctx = jg.Context((0,))
    out = {"scale": a.scale}
    t = time.perf_counter()
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_IN)
    out["build_in_s"] = round(time.perf_counter() - t, 3)
    for rep in range(2):
        t = time.perf_counter()
        rank, _ = g.pagerank(0.85, n, a.iterations)
        out[f"pagerank_{a.iterations}_s"] = round(time.perf_counter() - t, 3)
        out["pagerank_compute_ms"] = round(ctx.stats()["compute_ms"], 1)
    g.close()
    t = time.perf_counter()
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    out["build_both_s"] = round(time.perf_counter() - t, 3)
    for rep in range(2):
        t = time.perf_counter()
        d = g.bfs([1], jg.DIR_BOTH)
        out["bfs_s"] = round(time.perf_counter() - t, 3)
        t = time.perf_counter()
        comp, it = g.connected_components()
        out["cc_s"] = round(time.perf_counter() - t, 3)
        srcs = np.arange(64) * 7 + 1
        t = time.perf_counter()
        d = g.bfs(srcs, jg.DIR_BOTH)
        out["msbfs64_s"] = round(time.perf_counter() - t, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
