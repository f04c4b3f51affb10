"""Every program on logical shards under the virtual-device check in report mode (JG_VDEV_CHECK=2 prints
each distinct violation with its return addresses as libjanusgpu.so offsets and continues;
llvm-symbolizer --obj=janusgraph_amd/libjanusgpu.so <offset> names the line).  GPU.
    JG_VDEV_CHECK=2 python tools/vdev_probe.py [shards ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("JG_VDEV_CHECK", "2")


def main():
    import janusgraph_amd as jg
    from oracle import oracle as o
    o.build()
    s, t = o.rmat_edges(12, 16, 11)
    n = 1 << 12
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    w = (np.arange(len(s)) % 7 + 1).astype(np.int32)
    for shards in [int(x) for x in sys.argv[1:]] or [2, 3]:
        c = jg.Context((0,) * shards)
        g = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT | jg.ADJ_BOTH)
        steps = [("pagerank", lambda: g.pagerank(0.85, n, 3)), ("cc", g.connected_components),
                 ("bfs1", lambda: g.bfs([vid[5]], jg.DIR_BOTH)), ("msbfs", lambda: g.bfs(vid[:64], jg.DIR_BOTH)),
                 ("msbfs_out", lambda: g.bfs(vid[:64], jg.DIR_OUT)), ("sd", lambda: g.shortest_distance(vid[5], 4)),
                 ("keep", lambda: (g.bfs_keep(vid[:3], jg.DIR_BOTH), g.bfs_kept_row(1))),
                 ("combine", lambda: g.combine_steps(jg.DIR_IN, steps=2)),
                 ("neighbors", lambda: g.neighbors(np.arange(10), jg.DIR_BOTH))]
        for name, f in steps:
            try:
                f()
                print(f"{shards} shards {name}: ok", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"{shards} shards {name}: {e}", flush=True)
        gw = c.build(vid, vid[s], vid[t], flags=jg.ADJ_IN | jg.ADJ_OUT, weight=w)
        try:
            gw.shortest_distance(vid[5], 5)
            print(f"{shards} shards sd weighted: ok", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{shards} shards sd weighted: {e}", flush=True)
        c.close()


if __name__ == "__main__":
    main()
