"""A/B of 64-source bit-parallel BFS settings on the bench's own graph and sources (bench.py
rmat26_both_blocks: RMAT-<scale> BOTH, bench.pick_sources(deg, 64, 7)), interleaved over rounds so box
drift hits every setting alike.  Timing only (parity: tests/test_gpu_parity.py).  A setting is
comma-separated `knob=value` (jg_tune_set) and `env:NAME=value` (set in the environment before its
runs, removed after).  Knobs stay set after a setting's runs: give every setting that shares a knob its
value explicitly.  One line per setting: median HIP-event ms and call wall ms.

    python tools/msbfs_ab.py --scale 26 "" "msbfs_exit_first=8"
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
    knobs, env = [], []
    for kv in (x for x in setting.split(",") if x):
        k, v = kv.split("=")
        (env if k.startswith("env:") else knobs).append((k[4:] if k.startswith("env:") else k, v))
    return [(k, int(v)) for k, v in knobs], env


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("settings", nargs="+")
    a = p.parse_args()
    import bench
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    srcs = bench.pick_sources(g.degrees(jg.DIR_BOTH), 64, 7)
    times = {s: [] for s in a.settings}
    wall = {s: [] for s in a.settings}
    for r in range(a.rounds):
        for s in a.settings:
            knobs, env = parse(s)
            for k, v in knobs:
                jg._lib.tune_set(k, v)
            for k, v in env:
                os.environ[k] = v
            g.bfs(srcs, jg.DIR_BOTH, want=False)  # warm
            t = time.perf_counter()
            g.bfs(srcs, jg.DIR_BOTH, want=False)
            wall[s].append((time.perf_counter() - t) * 1e3)
            times[s].append(ctx.stats()["compute_ms"])
            for k, _ in env:
                del os.environ[k]
        print(f"round {r} done", file=sys.stderr, flush=True)
    for s in a.settings:
        print(json.dumps({"setting": s, "scale": a.scale, "ms_median": round(float(np.median(times[s])), 4),
                          "wall_ms_median": round(float(np.median(wall[s])), 4),
                          "ms": [round(x, 4) for x in times[s]]}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
