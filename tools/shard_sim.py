"""Sharded programs on ONE GPU: P logical shards (exchange by device copies) to estimate a P-GPU run.
The shards run one after another on one stream, so the kernel time per shard is the P-GPU compute
estimate; the halo volume is what each shard would receive over xGMI per exchange step.

    python tools/shard_sim.py --scale 26 --shards 1 8 [--program pr|bfs|cc|msbfs|sd] [--steps 10]

pr:    PageRank supersteps (halo vs the dense allgather layout), per-shard superstep kernel time
bfs:   sharded single-source DO-BFS from the bench's sources: levels, exchange steps, kernel time
cc:    the sharded CC propagation (one shard: the union-find path), supersteps and time
msbfs: the 64-source bit-parallel BFS, levels and time
sd:    weighted shortest distance, 6 hops (the supersteps; sharded over the IN halo plan), weights 1..255
Each line carries exchange_values (values all shards receive per exchange step) and its bytes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_pr(jg, scale, shards, halo, steps, warmup):
    jg._lib.tune_set("halo", halo)
    ctx = jg.Context((0,) * shards)
    try:
        g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_IN)
    finally:
        jg._lib.tune_set("halo", 1)
    build_ms = ctx.stats()["build_ms"]
    xv = g.info()["exchange_values"]
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
    return {"program": "pr", "shards": shards, "halo": halo, "build_ms": round(build_ms, 1),
            "ms_per_step_all_shards": round(dt / steps * 1e3, 4),
            "compute_ms_per_shard_step": round(st["kernel_ms_total"] / launches, 4),
            "exchange_ms_per_step": round(dt / steps * 1e3 - st["kernel_ms_total"] / steps, 4),
            "exchange_values_all_shards": xv, "exchange_bytes_per_shard": 8 * xv / max(shards, 1),
            "gteps_single_gpu_equiv": round(m / (dt / steps) / 1e9, 2)}, rank


def run_both(jg, program, scale, shards, reps, groups=1, group=0):
    import bench
    ctx = jg.Context((0,) * shards)
    g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_BOTH)
    xv = g.info()["exchange_values"]
    deg = g.degrees(jg.DIR_BOTH)
    out = {"program": program, "shards": shards, "exchange_values_all_shards": xv,
           "exchange_values_per_shard": xv / max(shards, 1)}
    rows = []
    if program == "bfs":
        m = 16 << scale
        for sv in bench.pick_sources(deg, 16, scale).tolist():
            g.bfs([sv], jg.DIR_BOTH, want=False)
            if ctx.stats()["edges_traversed"] < m // 100:
                continue
            for _ in range(reps):
                ctx.set_profiling(True)
                g.bfs([sv], jg.DIR_BOTH, want=False)
                st = ctx.stats()
                ctx.set_profiling(False)
                rows.append((st["compute_ms"], st["exchange_ms"], st["levels"]))
            if len(rows) >= 3 * reps:
                break
    else:
        # msbfs --groups G: the bench's 64 sources split into G groups of 64 / G (a 2D plan: G source
        # groups x P vertex shards); this run is group `group`
        srcs = np.array_split(bench.pick_sources(deg, 64, 7), groups)[group]
        out.update({"sources": int(len(srcs)), "groups": groups, "group": group})
        call = g.connected_components if program == "cc" else (
            lambda: g.bfs(srcs, jg.DIR_BOTH, want=False))
        call()
        for _ in range(reps):
            ctx.set_profiling(True)
            call()
            st = ctx.stats()
            ctx.set_profiling(False)
            rows.append((st["compute_ms"], st["exchange_ms"], st["levels"]))
    g.close()
    ctx.close()
    r = np.array(rows)
    out.update({"runs": len(rows), "compute_ms_all_shards": round(float(np.median(r[:, 0])), 4),
                "exchange_ms_all_shards": round(float(np.median(r[:, 1])), 4),
                "levels": int(np.median(r[:, 2])),
                "kernel_ms_per_shard": round(float(np.median(r[:, 0] - r[:, 1])) / shards, 4)})
    return out


def run_sd(jg, scale, shards, reps, max_depth=6):
    """Weighted shortest distance, hop-bounded (the supersteps; sharded: the IN halo plan with the reverse
    exchange of candidates), Graph500 Kronecker edges with weights 1..255 as tools/sd_bench.py draws them,
    seeded at the row of largest in-degree."""
    from sd_bench import kronecker
    n = 1 << scale
    s, t = kronecker(scale, 16, 0x55D + scale)
    w = np.random.default_rng(scale).integers(1, 256, len(s)).astype(np.int32)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    seed = int(np.bincount(t, minlength=n).argmax())
    ctx = jg.Context((0,) * shards)
    g = ctx.build(vid, vid[s], vid[t], weight=w, flags=jg.ADJ_IN)
    xv = g.info()["exchange_values"]
    g.shortest_distance(vid[seed], max_depth)
    rows = []
    for _ in range(reps):
        ctx.set_profiling(True)
        g.shortest_distance(vid[seed], max_depth)
        st = ctx.stats()
        ctx.set_profiling(False)
        rows.append((st["compute_ms"], st["exchange_ms"], st["levels"]))
    g.close()
    ctx.close()
    r = np.array(rows)
    return {"program": "sd", "shards": shards, "max_depth": max_depth, "exchange_values_all_shards": xv,
            "runs": len(rows), "compute_ms_all_shards": round(float(np.median(r[:, 0])), 4),
            "exchange_ms_all_shards": round(float(np.median(r[:, 1])), 4), "levels": int(np.median(r[:, 2])),
            "kernel_ms_per_shard": round(float(np.median(r[:, 0] - r[:, 1])) / shards, 4)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--shards", type=int, nargs="+", default=[1, 8])
    p.add_argument("--program", default="pr", choices=["pr", "bfs", "cc", "msbfs", "sd"])
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--halo", type=int, nargs="+", default=[1, 0], help="halo settings tried for P > 1 (pr)")
    p.add_argument("--tune", nargs="*", default=[], help="jg_tune_set knobs key=value applied first")
    p.add_argument("--groups", type=int, default=1, help="msbfs: split the 64 sources into this many groups "
                                                          "and run each (a groups x shards 2D plan)")
    p.add_argument("--only-group", type=int, default=-1, help="msbfs --groups: run this group alone (traces)")
    a = p.parse_args()
    import janusgraph_amd as jg
    for kv in a.tune:
        k, v = kv.split("=")
        jg._lib.tune_set(k, int(v))
    if a.program == "sd":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        for P in a.shards:
            print(json.dumps(run_sd(jg, a.scale, P, a.reps)), flush=True)
        return
    if a.program != "pr":
        for P in a.shards:
            for grp in range(a.groups if a.program == "msbfs" else 1):
                if a.only_group >= 0 and grp != a.only_group:
                    continue
                print(json.dumps(run_both(jg, a.program, a.scale, P, a.reps, a.groups, grp)), flush=True)
        return
    ref = None
    for P in a.shards:
        for halo in (a.halo if P > 1 else [1]):
            r, rank = run_pr(jg, a.scale, P, halo, a.steps, a.warmup)
            if ref is None:
                ref = rank
            r["max_rel_vs_first"] = float(np.max(np.abs(rank - ref) / np.maximum(np.abs(ref), 1e-300)))
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
