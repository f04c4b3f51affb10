"""A/B of bit-parallel BFS knobs on the bench's 64-source workload (bench.pick_sources(deg, 64, 7)),
timing only (parity: tests/test_gpu_configs.py, tests/test_gpu_parity.py).  One line per setting:
median HIP-event ms over `reps` runs after one warm run, levels, entries examined.
    python tools/msbfs_ab.py --scale 26 msbfs_exit 0 1 2
    python tools/msbfs_ab.py --scale 26 --tune msbfs_exit=1 msbfs_exit_live 0 700 1000
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--tune", action="append", default=[], help="a fixed jg_tune_set knob (key=value; repeatable)")
    p.add_argument("key")
    p.add_argument("values", type=int, nargs="+")
    a = p.parse_args()
    import bench
    import janusgraph_amd as jg
    for kv in a.tune:
        k, _, v = kv.partition("=")
        jg._lib.tune_set(k, int(v))
    ctx = jg.Context((0,))
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    srcs = bench.pick_sources(g.degrees(jg.DIR_BOTH), 64, 7)
    for v in a.values:
        jg._lib.tune_set(a.key, v)
        g.bfs(srcs, jg.DIR_BOTH, want=False)
        ms, st = [], None
        for _ in range(a.reps):
            g.bfs(srcs, jg.DIR_BOTH, want=False)
            st = ctx.stats()
            ms.append(st["compute_ms"])
        print(json.dumps({a.key: v, "scale": a.scale, "ms_median": round(float(np.median(ms)), 3),
                          "ms": [round(x, 3) for x in ms], "levels": st["levels"],
                          "entries_examined": st["edges_traversed"], "bytes": st["algorithmic_bytes"]}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
