"""Sweep a BFS knob on the bench's RMAT-20 single-source BFS (bench.py's procedure: 6 sources,
Graph500 resampling of tiny components, first run dropped).  Usage: python tools/bfs_sweep.py
[--scale S] bfs_grid 1024 2048 4096"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import janusgraph_amd as jg
    args = sys.argv[1:]
    scale = 20
    if args[0] == "--scale":
        scale, args = int(args[1]), args[2:]
    key, values = args[0], [int(v) for v in args[1:]]
    ctx = jg.Context((0,))
    g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_BOTH)
    for v in values:
        jg._lib.tune_set(key, v)
        ms = []
        rng = np.random.default_rng(1)
        for rep in range(3):
            for k in range(6):
                src = int(rng.integers(0, 1 << scale))
                g.bfs([src], jg.DIR_BOTH, want=False)
                s = ctx.stats()
                if s["edges_traversed"] < (16 << scale) // 100 or (rep == 0 and k == 0):
                    continue
                ms.append((s["compute_ms"], s["edges_traversed"] / (s["compute_ms"] * 1e-3) / 1e9))
        ms = np.array(ms)
        print(json.dumps({key: v, "ms_median": round(float(np.median(ms[:, 0])), 4),
                          "gteps_median": round(float(np.median(ms[:, 1])), 2), "runs": len(ms)}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
