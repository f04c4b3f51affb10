"""Snapshot build from decoded id arrays (jg_graph_build, the path GpuSnapshot's id mode and the
edgestore decoder feed), repeated, for a rocprofv3 kernel / copy / HIP API trace (diagnostic).

    python tools/build_trace.py [--scale 20] [--flags 4] [--reps 3]

Prints one JSON line with every build's build_ms and wall time."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--flags", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rmat", action="store_true", help="the on-device RMAT generator (bench.py's build) instead of host ids")
    a = ap.parse_args()
    import janusgraph_amd as jg
    n = 1 << a.scale
    if not a.rmat:
        from oracle import oracle as o  # input generator only: the RMAT edge list
        s, t = o.rmat_edges(a.scale, 16, 0x5EED + a.scale)
        vid = (np.arange(n, dtype=np.int64) + 1) << 8
        src, dst = vid[np.asarray(s)], vid[np.asarray(t)]
    ctx = jg.Context((0,))
    out = {"scale": a.scale, "flags": a.flags, "rmat": a.rmat, "build_ms": [], "wall_ms": []}
    for _ in range(a.reps):
        t0 = time.perf_counter()
        if a.rmat:
            g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=a.flags)
        else:
            g = ctx.build(vid, src, dst, flags=a.flags)
        out["wall_ms"].append(round((time.perf_counter() - t0) * 1e3, 2))
        out["build_ms"].append(round(ctx.stats()["build_ms"], 2))
        g.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
