"""Sharded PageRank on ONE GPU: P logical shards (exchange by device copies), halo exchange vs the
dense allgather.  Estimates the per-shard superstep compute of a P-GPU run (the shards run one after
another on one stream) and prints the halo volume each shard would receive over xGMI.

    python tools/shard_sim.py --scale 22 --shards 8 [--steps 10]
Run with JG_DEBUG_PLAN=1 2> file to also get the per-shard halo sizes from the build.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(jg, scale, shards, halo, steps, warmup):
    jg._lib.tune_set("halo", halo)
    ctx = jg.Context((0,) * shards)
    try:
        g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_IN)
    finally:
        jg._lib.tune_set("halo", 1)
    build_ms = ctx.stats()["build_ms"]
    n, m = 1 << scale, 16 << scale
    g.pagerank_begin(0.85, n)
    g.pagerank_step(warmup)
    g.sync()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    g.pagerank_step(steps)
    g.sync()
    dt = time.perf_counter() - t0
    rank, _ = g.pagerank_end()  # collects the profiling events
    st = ctx.stats()
    ctx.set_profiling(False)
    g.close()
    ctx.close()
    launches = max(st["kernel_launches"], 1)
    return {"shards": shards, "halo": halo, "build_ms": round(build_ms, 1),
            "ms_per_step_all_shards": round(dt / steps * 1e3, 4),
            "compute_ms_per_shard_step": round(st["kernel_ms_total"] / launches, 4),
            "exchange_ms_per_step": round(dt / steps * 1e3 - st["kernel_ms_total"] / steps, 4),
            "gteps_single_gpu_equiv": round(m / (dt / steps) / 1e9, 2)}, rank


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--shards", type=int, nargs="+", default=[1, 8])
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--halo", type=int, nargs="+", default=[1, 0], help="halo settings tried for P > 1")
    a = p.parse_args()
    import numpy as np
    import janusgraph_amd as jg
    ref = None
    for P in a.shards:
        for halo in (a.halo if P > 1 else [1]):
            r, rank = run(jg, a.scale, P, halo, a.steps, a.warmup)
            if ref is None:
                ref = rank
            r["max_rel_vs_first"] = float(np.max(np.abs(rank - ref) / np.maximum(np.abs(ref), 1e-300)))
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
