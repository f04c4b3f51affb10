"""Per-level cost of a level boundary: the launch-per-level DO-BFS (one kernel boundary per level) against
the persistent one (bfs_persistent: one grid barrier per level), at equal grids, on a traversal whose
levels do almost no work: a 1000-vertex path in a graph of 2^20 rows (so the level grid is the RMAT-20
one, sqrt(rows) = 1024 workgroups).  ms / levels of each setting is the boundary (or barrier) plus one
level's fixed work, which is the same in both.  VERDICT r04 item 4; GPU.

    python tools/bfs_barrier_cost.py [--rows-log 20] [--path 1000] [--rounds 5]
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
    p.add_argument("--rows-log", type=int, default=20)
    p.add_argument("--path", type=int, default=1000)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    import janusgraph_amd as jg
    n = 1 << a.rows_log
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    s = np.arange(a.path - 1, dtype=np.int64)
    ctx = jg.Context((0,))
    g = ctx.build(vid, vid[s], vid[s + 1], flags=jg.ADJ_BOTH)
    settings = [("launch", {"bfs_persistent": 0, "bfs_grid": 8192}),
                ("launch_g256", {"bfs_persistent": 0, "bfs_grid": 256})]
    settings += [(f"persistent_g{pg}", {"bfs_persistent": pg, "bfs_grid": 8192})
                 for pg in (1024, 512, 256, 64)]
    jg._lib.tune_set("bfs_tail_grid", 0)  # every launch at the level grid
    res = {name: [] for name, _ in settings}
    lv = {}
    for _ in range(a.rounds):
        for name, kv in settings:
            for k, v in kv.items():
                jg._lib.tune_set(k, v)
            g.bfs([vid[0]], jg.DIR_BOTH, want=False)
            g.bfs([vid[0]], jg.DIR_BOTH, want=False)
            st = ctx.stats()
            res[name].append(st["compute_ms"])
            lv[name] = st["levels"]
    for k, v in (("bfs_persistent", 0), ("bfs_grid", 8192), ("bfs_tail_grid", 64)):
        jg._lib.tune_set(k, v)
    for name, _ in settings:
        ms = float(np.median(res[name]))
        print(json.dumps({"setting": name, "rows": n, "levels": lv[name], "ms_median": round(ms, 4),
                          "us_per_level": round(ms * 1e3 / max(lv[name], 1), 3),
                          "ms_all": [round(x, 4) for x in res[name]]}), flush=True)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
