"""Weighted ShortestDistance with an unbounded hop count on an RMAT graph: the frontier Bellman-Ford
supersteps (sd_delta = 0) against near-far delta-stepping at several deltas (-1: automatic), one GPU.
Prints one JSON line: per delta the HIP-event times of `runs` calls, the pass / superstep count, and
whether the distances equal the supersteps' bit for bit.

  python tools/sd_bench.py [--scale 20] [--runs 5] [--deltas 0,-1,8,32,128] [--wmax 255] [--tune k=v ...]

The graph: Graph500 Kronecker edges (A, B, C = 0.57, 0.19, 0.19) drawn here with numpy, weights uniform
in [1, wmax] (Graph500 SSSP style), built with JG_ADJ_IN; the seed is the row of largest in-degree.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEPTH_INF = 2**31 - 1


def kronecker(scale, ef, seed):
    rng = np.random.default_rng(seed)
    m = ef << scale
    a, b, c = 0.57, 0.19, 0.19
    src = np.zeros(m, np.int64)
    dst = np.zeros(m, np.int64)
    for i in range(scale):
        r1 = rng.random(m, dtype=np.float32)
        r2 = rng.random(m, dtype=np.float32)
        ib = r1 > a + b
        jb = r2 > np.where(ib, c / (1 - a - b), a / (a + b))
        src |= ib.astype(np.int64) << i
        dst |= jb.astype(np.int64) << i
    perm = rng.permutation(1 << scale)
    return perm[src], perm[dst]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=20)
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--runs", type=int, default=5)
    p.add_argument("--deltas", default="0,-1,8,32,128")
    p.add_argument("--wmax", type=int, default=255)
    p.add_argument("--tune", nargs="*", default=[], help="jg_tune_set knobs key=value applied first (e.g. sd_dist32=0)")
    a = p.parse_args()
    import janusgraph_amd as jg
    n = 1 << a.scale
    s, t = kronecker(a.scale, a.ef, 0x55D + a.scale)
    w = np.random.default_rng(a.scale).integers(1, a.wmax + 1, len(s)).astype(np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    seed = int(np.bincount(t, minlength=n).argmax())
    ctx = jg.Context((0,))
    for kv in a.tune:
        k, v = kv.split("=")
        jg._lib.tune_set(k, int(v))
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN)
    out = {"workload": f"sssp_unbounded_rmat{a.scale}_ef{a.ef}_w1-{a.wmax}", "n": n, "m": len(s), "seed_row": seed,
           "runs": a.runs, "tune": a.tune, "results": []}
    ref = None
    for d in [int(x) for x in a.deltas.split(",")]:
        jg._lib.tune_set("sd_delta", d)
        dist = g.shortest_distance(vid[seed], DEPTH_INF)  # warm (the delta path's weight statistics)
        ms = []
        for _ in range(a.runs):
            dist = g.shortest_distance(vid[seed], DEPTH_INF)
            ms.append(ctx.stats()["compute_ms"])
        st = ctx.stats()
        if d == 0:
            ref = dist
        out["results"].append({"sd_delta": d, "ms": ms, "ms_median": float(np.median(ms)), "passes": st["levels"],
                               "reached": int((dist != jg.DIST_ABSENT).sum()),
                               "equal_to_supersteps": None if ref is None else bool(np.array_equal(dist, ref))})
        print(json.dumps(out["results"][-1]), flush=True)
    jg._lib.tune_set("sd_delta", -1)
    g.close()
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
