"""A/B of DO-BFS knob settings on the bench's own sources (bench.pick_sources, Graph500 resampling of tiny
components), interleaved over rounds so box drift hits every setting alike.  Timing only (parity:
tests/test_gpu_parity.py).  One line per setting: median HIP-event ms over all rounds and sources, and
the per-source medians.

    python tools/bfs_ab.py --scale 20 "bfs_td_split=0" "bfs_td_split=2,bfs_td_split_levels=6"
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(setting):
    return [(k, int(v)) for k, v in (kv.split("=") for kv in setting.split(",") if kv)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--nsrc", type=int, default=6)
    p.add_argument("settings", nargs="+")
    a = p.parse_args()
    import bench
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    m = 16 << a.scale
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    srcs = []
    for sv in bench.pick_sources(g.degrees(jg.DIR_BOTH), 4 * a.nsrc, a.scale).tolist():
        if len(srcs) == a.nsrc:
            break
        g.bfs([sv], jg.DIR_BOTH, want=False)
        if ctx.stats()["edges_traversed"] >= m // 100:
            srcs.append(sv)
    times = {s: {sv: [] for sv in srcs} for s in a.settings}
    wall = {s: [] for s in a.settings}  # host wall time of the call (launches, read-backs, no depth output)
    levels = {}
    for _ in range(a.rounds):
        for s in a.settings:
            kv = parse(s)
            for k, v in kv:
                jg._lib.tune_set(k, v)
            for sv in srcs:
                g.bfs([sv], jg.DIR_BOTH, want=False)  # warm (the bench drops the first run too)
                t = time.perf_counter()
                g.bfs([sv], jg.DIR_BOTH, want=False)
                wall[s].append((time.perf_counter() - t) * 1e3)
                st = ctx.stats()
                times[s][sv].append(st["compute_ms"])
                levels[sv] = st["levels"]
    for s in a.settings:
        allv = [x for v in times[s].values() for x in v]
        print(json.dumps({"setting": s, "scale": a.scale, "ms_median": round(float(np.median(allv)), 4),
                          "wall_ms_median": round(float(np.median(wall[s])), 4),
                          "per_source": {str(sv): round(float(np.median(v)), 4) for sv, v in times[s].items()},
                          "levels": {str(sv): levels[sv] for sv in srcs}}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
