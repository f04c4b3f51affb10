"""Benchmark: GpuGraphComputer supersteps on synthetic Graph500 RMAT graphs (BASELINE.json metric).

Headline (value): PageRank fp64 on RMAT scale-24 edgefactor-16 (BASELINE.json configs[2]), one
"step" = one power superstep of JanusGraph's PageRankVertexProgram over the whole graph (pull SpMV
over the in-CSR + contribution write + RCCL allgather of the rank-contribution vector when N > 1).
value = directed edges processed per second over all GPUs (GTEPS), inputs resident in HBM.
Secondary blocks (same JSON line, one GPU): "bfs" = DO-BFS (SPVP depth, undirected) from one source on
RMAT scale-20 (configs[1]) as Graph500 TEPS with its roofline and CPU baseline; "rmat26" = PageRank
(with roofline), DO-BFS, ConnectedComponent (configs[3]) and 64-source MS-BFS (configs[4]) at scale 26.
With N > 1: "per_rank" = each rank's superstep kernel time, exchange time, halo volume and roofline.

Run:  python bench.py [--gpus N --steps K --warmup W]
      N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

# Host-clock windows of every timed region (block, start ns, end ns, runs), CLOCK_MONOTONIC: printed with
# --trace-windows so tools/bench_trace.py can cut a rocprofv3 kernel trace of this same process into the
# blocks' timed runs
WINDOWS = []


def window_start():
    return time.monotonic_ns()


def window_end(block, t0, runs=1):
    WINDOWS.append([block, t0, time.monotonic_ns(), runs])


def code_identity():
    """What this line was measured with: the commit the tree was at (JG_BENCH_HEAD, set by the GPU scripts:
    the box gets the tree without .git) and content hashes of bench.py and the library it loaded."""
    import hashlib

    def sha16(path):
        try:
            with open(path, "rb") as f:
                return hashlib.sha256(f.read()).hexdigest()[:16]
        except OSError:
            return None
    return os.environ.get("JG_BENCH_HEAD"), {"bench_py_sha16": sha16(os.path.join(ROOT, "bench.py")),
                                             "libjanusgpu_sha16": sha16(os.path.join(ROOT, "janusgraph_amd",
                                                                                     "libjanusgpu.so"))}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--scale", type=int, default=24)
    p.add_argument("--edgefactor", type=int, default=16)
    p.add_argument("--seed", type=int, default=0x5EED + 24)
    p.add_argument("--bfs-scale", type=int, default=20)
    p.add_argument("--no-bfs", action="store_true")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="CPU work of each cpu_baseline sample (whole supersteps / BFS rounds until then)")
    p.add_argument("--no-big", action="store_true", help="skip the RMAT-26 blocks (PageRank, BFS, CC, MS-BFS)")
    p.add_argument("--big-scale", type=int, default=26)
    p.add_argument("--big-steps", type=int, default=10)
    p.add_argument("--cc-plan", choices=["replicated", "sharded"], default="replicated",
                   help="N > 1: CC on a whole-graph copy per GPU (default) or over the ranks' shards")
    p.add_argument("--trace-windows", action="store_true",
                   help="add the timed regions' host-clock windows to the JSON line (tools/bench_trace.py)")
    p.add_argument("--host-transport", action="store_true",
                   help="N > 1 rehearsal on one GPU: every rank on device 0, exchanges over gloo through the "
                        "library's host transport instead of RCCL (not a performance measurement)")
    return p.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


class Control:
    """Control plane for N ranks (gloo): unique-id broadcast, barriers, max-over-ranks."""

    def __init__(self, ws, rank):
        self.ws, self.rank = ws, rank
        self.dist = None
        if ws > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=ws)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def sum_array(self, a):
        if not self.dist:
            return a
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a, np.int64))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.numpy()

    def min_array(self, a):
        if not self.dist:
            return a
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a, np.int64))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return t.numpy()

    def gather(self, row):
        """Every rank's list of floats, on every rank (rank order)."""
        if not self.dist:
            return [row]
        import torch
        t = torch.tensor(row, dtype=torch.float64)
        out = [torch.zeros_like(t) for _ in range(self.ws)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def pmc_traffic(workload):
    """Fabric bytes per run of a workload from the newest committed rocprofv3 PMC summary whose "workload"
    matches (profiles/<round>/**/summary.json, made by tools/pmc_workloads.sh + tools/pmc_summary.py from
    runs of tools/workload.py / bench.py on the same workload).  (None, None) when there is none."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    for rnd in sorted(os.listdir(pdir), reverse=True):
        rdir = os.path.join(pdir, rnd)
        if not os.path.isdir(rdir):
            continue
        for dirpath, _, files in sorted(os.walk(rdir)):
            if "summary.json" not in files:
                continue
            with open(os.path.join(dirpath, "summary.json")) as f:
                s = json.load(f)
            wl = s.get("workload")
            if wl is None and os.path.exists(os.path.join(dirpath, "bench.json")):
                with open(os.path.join(dirpath, "bench.json")) as f:
                    wl = json.load(f).get("config", {}).get("workload")  # round-2 summaries
            if wl != workload or s.get("traffic_bytes_per_launch") is None:
                continue
            rel = os.path.relpath(os.path.join(dirpath, "summary.json"), ROOT)
            return s["traffic_bytes_per_launch"], f"{rel} ({s.get('read_bytes_method', '')})"
    return None, None


def trace_kernel_ms(workload):
    """Kernel time per run of a workload from the newest committed counter-free rocprofv3 trace summary
    (profiles/<round>/trace/<name>/summary.json, made by tools/gpu_steps.sh "trace" steps with
    tools/trace_summary.py): the check that a block's kernel_ms is not inflated by counter collection
    (VERDICT r03 item 6).  None when there is none."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for rnd in sorted(os.listdir(pdir), reverse=True):
        tdir = os.path.join(pdir, rnd, "trace")
        if not os.path.isdir(tdir):
            continue
        for dirpath, _, files in sorted(os.walk(tdir)):
            if "summary.json" not in files:
                continue
            with open(os.path.join(dirpath, "summary.json")) as f:
                s = json.load(f)
            if s.get("workload") != workload:
                continue
            return {"kernel_ms_per_run": s.get("kernel_ms_per_run"), "kernel_ms_per_run_steady": s.get("kernel_ms_per_run_steady"),
                    "event_ms_per_run": s.get("event_ms_per_run"),
                    "source": os.path.relpath(os.path.join(dirpath, "summary.json"), ROOT)}
    return None


def bench_trace_block(workload):
    """This workload's block from the newest committed trace of a whole bench process
    (profiles/<round>/bench_trace/summary.json, tools/bench_trace.py): the trace's span and kernel sum per
    run against that process's own event figure, and the roofline fraction on each.
    None when there is none."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for rnd in sorted(os.listdir(pdir), reverse=True):
        fn = os.path.join(pdir, rnd, "bench_trace", "summary.json")
        if not os.path.exists(fn):
            continue
        with open(fn) as f:
            blk = json.load(f).get("blocks", {}).get(workload)
        if blk is None:
            continue
        keep = ("event_ms", "trace_span_ms", "trace_kernel_ms", "frac_event", "frac_trace_span", "frac_trace_kernel",
                "span_over_event", "agree", "within_step")
        out = {k: blk[k] for k in keep if k in blk}
        out["source"] = os.path.relpath(fn, ROOT)
        return out
    return None


def cpu_baseline(scale, ef, seed, seconds, min_steps=2):
    """The oracle's PageRank superstep (OpenMP) on the same RMAT graph, rank 0 only: whole supersteps until
    `seconds` of CPU work (a bounded sample of the workload)."""
    from oracle import oracle as o
    o.build()
    n, m = 1 << scale, ef << scale
    src, dst = o.rmat_edges(scale, ef, seed)
    s32, d32 = src.astype(np.int32), dst.astype(np.int32)
    del src, dst
    ptr, col = o.build_in_csr(n, s32, d32)
    outdeg = np.bincount(s32, minlength=n).astype(np.float64)
    del s32, d32
    with np.errstate(divide="ignore"):  # sinks: never gathered (no out-edges), as in the kernels
        contrib = (1.0 / n) / outdeg
    t0 = time.perf_counter()
    steps = 0
    while steps < min_steps or time.perf_counter() - t0 < seconds:
        contrib = o.pagerank_superstep_csr(n, ptr, col, contrib, outdeg, 0.85, n)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": round(m * steps / dt / 1e9, 4), "unit": "GTEPS", "cores": o.num_threads(), "kind": "port",
            "sample": f"oracle/jg_oracle.c jo_pagerank_superstep_csr (OpenMP), {steps} full power supersteps on "
                      f"the same RMAT-{scale} ef{ef} graph (seed {seed}), {dt:.1f} s; CSR build untimed"}


def cpu_baseline_bfs(scale, ef, seed, sources, seconds):
    """The oracle's level-synchronous parallel BFS (jo_bfs_csr, OpenMP) from the bench's sources on the same
    symmetrised RMAT graph, Graph500 TEPS (input edges of the source's component / time), rounds over the
    sources until `seconds` of CPU work."""
    from oracle import oracle as o
    o.build()
    n = 1 << scale
    s, d = o.rmat_edges(scale, ef, seed)
    s, d = s.astype(np.int32), d.astype(np.int32)
    ptr, adj = o.csr_unordered(n, s, d, both=True)
    teps, total, rounds = [], 0.0, 0
    while rounds == 0 or total < seconds:
        for sv in sources:
            t0 = time.perf_counter()
            depth = o.bfs_csr(n, ptr, adj, int(sv))
            dt = time.perf_counter() - t0
            total += dt
            teps.append(int(np.count_nonzero(depth[s] >= 0)) / dt / 1e9)
        rounds += 1
    return {"value": round(float(np.median(teps)), 4), "unit": "GTEPS", "cores": o.num_threads(), "kind": "port",
            "sample": f"oracle/jg_oracle.c jo_bfs_csr (OpenMP, top-down level-synchronous), {rounds} rounds over the "
                      f"{len(sources)} bench sources on the same RMAT-{scale} ef{ef} graph, {total:.1f} s of CPU BFS; "
                      f"CSR build untimed"}


def hbm_roofline(alg_bytes, ms, kernel, workload=None, model=None):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(workload) if workload else (None, None)
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
         "kernel": kernel, "kernel_ms": round(ms, 4), "bytes_per_launch": alg_bytes}
    if traffic:
        # the fabric bytes the counters saw per run over this run's time: the HBM efficiency itself, where
        # `frac` is the model's work-equivalent (the BFS's "one full pass", CC's pass model; VERDICT r05
        # weak 5).  The PMC run is the committed summary named in traffic_source, not this process.
        r["frac_fabric"] = round(traffic / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if workload:
        r["trace"] = trace_kernel_ms(workload)
        r["bench_trace"] = bench_trace_block(workload)
    if model:
        r["model"] = model
    return r


def pick_sources(degree, k, seed):
    """Seeded uniform pick among vertices with at least one BOTH entry."""
    cand = np.flatnonzero(degree > 0)
    return np.random.default_rng(seed).choice(cand, min(k, len(cand)), replace=False).astype(np.int64)


def both_degrees(jg, ctl, g):
    """Entries per vertex of the BOTH adjacency (rank mode: each rank's rows, summed over ranks)."""
    deg = g.degrees(jg.DIR_BOTH)
    return ctl.sum_array(deg) if ctl.ws > 1 else deg


def bfs_block(jg, ctx, ctl, scale, ef, nsrc=6, cpu=True, cpu_seconds=10.0):
    """Single-source DO-BFS (SPVP depth, BOTH edges) from seeded sources of degree > 0, Graph500 TEPS (input
    edges of the source's component / time); roofline of one traversal: 8*m + 12*n algorithmic bytes
    (one full pass) / its HIP-event time.  N > 1: the sharded DO-BFS (dobfs_sharded)."""
    n, m = 1 << scale, ef << scale
    gb = ctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_BOTH)
    deg = both_degrees(jg, ctl, gb)
    cand = pick_sources(deg, 4 * nsrc, scale)
    times, teps, srcs, ranks, walls, keep_ms, keep_walls = [], [], [], [], [], [], []
    for sv in cand.tolist():
        if len(srcs) == nsrc:
            break
        gb.bfs([sv], jg.DIR_BOTH, want=False)
        if ctx.stats()["edges_traversed"] < m // 100:
            continue  # a source in a tiny component: Graph500 resamples
        ctx.set_profiling(ctl.ws > 1)  # N > 1: exchange_ms from events around every exchange step
        ctl.barrier()
        w0 = window_start()
        t0 = time.perf_counter()
        gb.bfs([sv], jg.DIR_BOTH, want=False)  # timed run (the first touched cold pages)
        wall = (time.perf_counter() - t0) * 1e3
        window_end(f"bfs_spvp_rmat{scale}_ef{ef}", w0)
        st = ctx.stats()
        ctx.set_profiling(False)
        ms = ctl.max(st["compute_ms"])
        srcs.append(sv)
        times.append(ms)
        walls.append(ctl.max(wall))
        teps.append(st["edges_traversed"] / (ms * 1e-3) / 1e9)
        ranks.append(ctl.gather([st["compute_ms"], st["exchange_ms"]]))
        # the ShortestPathVertexProgram drop-in's call (GpuGraphComputer: jg_bfs_keep, the depth row kept on
        # the device for the walk-back), entry to return
        ctl.barrier()
        t0 = time.perf_counter()
        gb.bfs_keep([sv], jg.DIR_BOTH)
        keep_walls.append(ctl.max((time.perf_counter() - t0) * 1e3))
        keep_ms.append(ctl.max(ctx.stats()["compute_ms"]))
    gb.close()
    ms = float(np.median(times))
    workload = f"bfs_spvp_rmat{scale}_ef{ef}"
    blk = {"workload": workload, "gteps_median": round(float(np.median(teps)), 3), "ms_median": round(ms, 4),
           "wall_ms_median": round(float(np.median(walls)), 4),
           "runs": len(times), "sources": [int(x) for x in srcs],
           "timed_region": "ms: HIP events from the init launch to the end of the last level batch (the depth init "
                           "covers every row a BOTH traversal can reach; the empty suffix keeps -1 between calls); "
                           "wall_ms: the call from entry to return (source id lookup, level launches, the host's "
                           "read of the final level state), max over ranks",
           "spvp_keep": {"ms_median": round(float(np.median(keep_ms)), 4),
                         "wall_ms_median": round(float(np.median(keep_walls)), 4),
                         "call": "jg_bfs_keep (GpuGraphComputer's ShortestPathVertexProgram path: the depth row kept "
                                 "on the device), same sources; wall_ms from entry to return"}}
    if ctl.ws == 1:
        blk["roofline"] = hbm_roofline(8.0 * m + 12.0 * n, ms, "direction-optimising BFS, one traversal "
                                       "(bfs_init_kernel + bfs_level_kernel launches)", workload,
                                       "8*m + 12*n: every symmetrised entry (4 B) once, row_ptr (8 B) and depth "
                                       "(4 B) per vertex (SURVEY.md 8d)")
    else:
        blk["per_rank"] = per_rank_rows(ranks[len(ranks) // 2])
    if cpu and ctl.ws == 1:
        blk["cpu_baseline"] = cpu_baseline_bfs(scale, ef, 0x5EED + scale, srcs, cpu_seconds)
    return blk


def per_rank_rows(rows):
    """Each rank's (compute_ms, exchange_ms) of a program call.  The exchange pairs are recorded inside the
    call's timed region only (prof_discard_exchanges at its start), so exchange_ms <= compute_ms must hold;
    a row that breaks it is flagged `timing_suspect` (the other blocks' results stay), and
    tests/test_bench_host.py fails on such a row."""
    out = [{"rank": r, "compute_ms": round(x[0], 4), "exchange_ms": round(x[1], 4)} for r, x in enumerate(rows)]
    for o in out:
        if o["exchange_ms"] > o["compute_ms"] * 1.001 + 0.01:
            o["timing_suspect"] = "exchange_ms exceeds the call's compute_ms"
    return out


def pagerank_block(jg, ctx, scale, ef, steps, warmup):
    n, m = 1 << scale, ef << scale
    g = ctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_IN)
    build_ms = ctx.stats()["build_ms"]
    live = int(np.count_nonzero(g.degrees(jg.DIR_IN)))
    g.pagerank_begin(0.85, n)
    g.pagerank_step(warmup)
    g.sync()
    ctx.set_profiling(True)
    w0 = window_start()
    t0 = time.perf_counter()
    g.pagerank_step(steps)
    g.sync()
    dt = time.perf_counter() - t0
    window_end(f"pagerank_fp64_rmat{scale}_ef{ef}", w0, steps)
    g.pagerank_end(want=False)
    st = ctx.stats()
    ctx.set_profiling(False)
    g.close()
    kern_ms = st["kernel_ms_total"] / max(st["kernel_launches"], 1)
    workload = f"pagerank_fp64_rmat{scale}_ef{ef}"
    return {"workload": workload, "ms_per_step": round(dt / steps * 1e3, 4),
            "gteps": round(m * steps / dt / 1e9, 3), "steps": steps, "build_ms": round(build_ms, 1),
            "roofline": hbm_roofline(12.0 * m + 32.0 * n, kern_ms, "PageRank superstep (same launch sequence "
                                     "as the headline)", workload, PR_MODEL),
            "required": required_roofline(m, live, kern_ms)}


PR_MODEL = ("12*m + 32*n per superstep (SURVEY.md 8d): col (4 B) and gathered contribution (8 B) per edge; "
            "row_ptr, 1/outdeg, rank write, contribution write (8 B each) per vertex")


def required_roofline(m, live, ms):
    """The bytes a superstep needs once the rows without in-edges are constant (written in the first two
    power steps only) and the rank is stored on the last superstep only: 12*m + 24*live (row_ptr,
    1/outdeg and the contribution write per row with an in-edge)."""
    b = 12.0 * m + 24.0 * live
    a = b / (ms * 1e-3) / 1e9
    return {"bytes_per_launch": b, "rows_with_in_edges": live, "achieved": round(a, 1),
            "frac": round(a / HBM_PEAK_GBS, 4)}


def rmat26_both_blocks(jg, ctx, ctl, scale, ef, local=0, cc_plan="replicated"):
    """CC (configs[3]) and 64-source MS-BFS (configs[4]) on the BOTH adjacency.  N > 1: every rank holds
    its shard and MS-BFS runs the sharded bit-parallel levels; CC runs replicated: every GPU builds the
    whole BOTH graph (9 GB of 288 GB at RMAT-26) and runs the one-GPU union-find, because the sharded CC
    (local union-finds, tree labels over the halo, a multi-root sharded DO-BFS: jg_cc.hip
    cc_union_find_sharded) models below one GPU's time at P = 8."""
    n, m = 1 << scale, ef << scale
    g = ctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_BOTH)
    build_ms = ctx.stats()["build_ms"]
    deg = both_degrees(jg, ctl, g)
    cctx, cg = ctx, g
    replicated = ctl.ws > 1 and cc_plan == "replicated"
    if replicated:
        cctx = jg.Context((local,))
        cg = cctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_BOTH)
    cg.connected_components()  # warm
    cctx.set_profiling(ctl.ws > 1 and not replicated)  # sharded: exchange_ms from events around every exchange
    ctl.barrier()
    w0 = window_start()
    t0 = time.perf_counter()
    comp, it = cg.connected_components()
    cc_wall = ctl.max((time.perf_counter() - t0) * 1e3)
    window_end(f"cc_rmat{scale}_ef{ef}", w0)
    st = cctx.stats()
    cctx.set_profiling(False)
    cc_ms = ctl.max(st["compute_ms"])
    cc_rank = ctl.gather([st["compute_ms"], st["exchange_ms"]])
    if replicated:
        cg.close()
        cctx.close()
    elif ctl.ws > 1:
        comp = ctl.min_array(comp)  # each rank filled its own rows (the others hold INT64_MAX)
    counts = np.bincount(comp, minlength=n)  # RMAT ids are 0..n-1: labels are vertex ids
    wl_cc = f"cc_rmat{scale}_ef{ef}"
    cc = {"workload": wl_cc, "ms": round(cc_ms, 3), "iterations": it, "wall_ms": round(cc_wall, 3),
          "timed_region": "ms: HIP events around the union-find passes, the superstep-count BFS and (one GPU) the "
                          "caller-order output (cc_output_kernel: every vertex's component id, edgeless rows "
                          "included, gathered into caller order on the device, queued behind the BFS start); one "
                          "GPU: the end event follows the BFS's last level batch, before the host reads its final "
                          "level state (as the DO-BFS's); wall_ms: the call from entry to return, which adds that "
                          "read and the copy of the n int64 ids to the caller's host array",
          "components": int(np.count_nonzero(counts)), "build_ms": round(build_ms, 1),
          "algorithm": "one shard: union-find + one DO-BFS from every component's minimum-rank vertex "
                       "(jg_cc.hip cc_union_find), labels and superstep count identical to the propagation"
          if ctl.ws == 1 else "replicated: every GPU holds the whole BOTH graph and runs the one-GPU union-find "
                              "+ DO-BFS (the sharded cc_union_find_sharded models at 0.85-0.9x of one GPU at P = 8, "
                              "DESIGN.md section 7)" if replicated else
                              "sharded: local Afforest union-finds, tree labels over forward and reverse halo "
                              "exchanges (pairs of the labels that fell after the first rounds), one multi-root "
                              "sharded DO-BFS for the superstep count (jg_cc.hip cc_union_find_sharded)"}
    if ctl.ws == 1:
        cc["roofline"] = hbm_roofline(st["algorithmic_bytes"], cc_ms, "ConnectedComponent run (uf_* kernels + "
                                      "bfs_init_roots_kernel + bfs_level_kernel)", wl_cc,
                                      "58 B per row with an edge (union-find passes + BFS start), 12 B per entry "
                                      "linked in the second round, 4 B per entry of the rows the BFS reached "
                                      "(jg_cc.hip cc_union_find); the caller-order output: 4 B per row with an edge (giant-component bits) + "
                                      "12 B per vertex")
    else:
        cc["per_rank"] = per_rank_rows(cc_rank)
    # 64 sources among the degree > 0 vertices; TEPS counts each source's component edges
    srcs = pick_sources(deg, 64, 7)
    comp_edges = np.bincount(comp, weights=deg.astype(np.float64), minlength=n) / 2.0
    edges = float(comp_edges[comp[srcs]].sum())
    del comp, counts, comp_edges
    g.bfs(srcs, jg.DIR_BOTH, want=False)  # warm
    ctx.set_profiling(ctl.ws > 1)
    ctl.barrier()
    w0 = window_start()
    t0 = time.perf_counter()
    g.bfs(srcs, jg.DIR_BOTH, want=False)
    ms_wall = ctl.max((time.perf_counter() - t0) * 1e3)
    window_end(f"msbfs64_rmat{scale}_ef{ef}", w0)
    st = ctx.stats()
    ctx.set_profiling(False)
    ms = ctl.max(st["compute_ms"])
    wl_ms = f"msbfs64_rmat{scale}_ef{ef}"
    msb = {"workload": wl_ms, "sources": int(len(srcs)), "ms": round(ms, 3), "levels": st["levels"],
           "wall_ms": round(ms_wall, 3),
           "timed_region": "ms: HIP events from the state fills to the last level; the depth rows (want=False: not "
                           "materialised; the per-level words are an exact encoding) are outside; wall_ms: the call "
                           "from entry to return (the sources' id lookup, launches, level-control reads)",
           "gteps": round(edges / (ms * 1e-3) / 1e9, 1),
           "gteps_note": "sum over the 64 sources (degree > 0) of the input edges in the source's component / time"}
    if ctl.ws == 1:
        msb["roofline"] = hbm_roofline(st["algorithmic_bytes"], ms, "64-source bit-parallel BFS (MsBfsOp merge / "
                                       "light kernels + msbfs_* kernels)", wl_ms,
                                       "per pull level 12 B per entry of a live merge task and of the light rows "
                                       "+ 32 B per row (incl. the level's new-bit word: the depths); per top-down "
                                       "level 12 B per frontier entry + 24 B per touched word + 8 B per queued vertex")
        msb["entries_examined"] = st["edges_traversed"]
    else:
        msb["per_rank"] = per_rank_rows(ctl.gather([st["compute_ms"], st["exchange_ms"]]))
    g.close()
    return cc, msb


def main():
    args = parse()
    ws, rank, local = dist_env()
    if ws != args.gpus:
        args.gpus = ws if ws > 1 else args.gpus
    ctl = Control(ws, rank)
    import janusgraph_amd as jg

    if ws > 1 and args.host_transport:
        from janusgraph_amd.transport import GlooTransport
        ctx = jg.Context((0,), rank=rank, nranks=ws, transport=GlooTransport(ctl.dist, ws))
    else:
        uid = jg._lib.comm_unique_id() if (ws > 1 and rank == 0) else None
        uid = ctl.bcast_bytes(uid)
        ctx = jg.Context((local,), rank=rank if ws > 1 else None, nranks=ws, unique_id=uid)
    n = 1 << args.scale
    m = args.edgefactor << args.scale

    g = ctx.build_rmat(args.scale, args.edgefactor, args.seed, flags=jg.ADJ_IN)
    build_ms = ctx.stats()["build_ms"]
    info = g.info()
    live = int(ctl.sum(float(np.count_nonzero(g.degrees(jg.DIR_IN)))))  # rows with an in-edge, all ranks
    g.pagerank_begin(0.85, n)
    g.pagerank_step(args.warmup)
    g.sync()
    ctl.barrier()
    ctx.set_profiling(True)
    w0 = window_start()
    t0 = time.perf_counter()
    g.pagerank_step(args.steps)
    g.sync()
    t1 = time.perf_counter()
    window_end(f"pagerank_fp64_rmat{args.scale}_ef{args.edgefactor}", w0, args.steps)
    ctl.barrier()
    elapsed = ctl.max(t1 - t0)
    g.pagerank_end(want=False)
    st = ctx.stats()
    ctx.set_profiling(False)
    ms_per_step = elapsed / args.steps * 1e3
    value = m * args.steps / elapsed / 1e9  # GTEPS, all ranks

    # roofline of the dominant kernel (the superstep's launch sequence), HIP events on its stream, this
    # rank's launches; with N > 1 the exchange step is outside these events
    launches = max(st["kernel_launches"], 1)
    kern_ms = st["kernel_ms_total"] / launches
    in_nnz = info["num_edges"] if ws == 1 else None
    alg_bytes_launch = 12.0 * m + 32.0 * n  # SURVEY §8d per-edge/per-vertex bytes
    if ws > 1:
        alg_bytes_launch = (12.0 * m + 32.0 * n) / ws  # this rank's share (rows and entries are balanced)
    workload = f"pagerank_fp64_rmat{args.scale}_ef{args.edgefactor}"
    roofline = hbm_roofline(alg_bytes_launch, kern_ms, "PageRank superstep (pull_merge_kernel x bands + fixup + "
                            "fused light-row/finalize kernel, PrOp)", workload if ws == 1 else None, PR_MODEL)
    if ws == 1:
        roofline["required"] = required_roofline(m, live, kern_ms)
    per_rank = None
    if ws > 1:
        # every rank's own numbers, gathered on rank 0: superstep kernel time, exchange time, halo volume
        mine = [float(rank), kern_ms, st["exchange_ms"] / max(args.steps, 1), float(info["exchange_values"]),
                alg_bytes_launch / (kern_ms * 1e-3) / 1e9]
        rows = ctl.gather(mine)
        per_rank = [{"rank": int(r[0]), "kernel_ms": round(r[1], 4), "exchange_ms": round(r[2], 4),
                     "halo_values": int(r[3]), "halo_bytes": int(r[3]) * 8,
                     "roofline_frac": round(r[4] / HBM_PEAK_GBS, 4)} for r in rows]
    g.close()

    extra = {}
    if not args.no_bfs and ws == 1:
        extra["bfs"] = bfs_block(jg, ctx, ctl, args.bfs_scale, args.edgefactor, cpu=not args.no_cpu,
                                 cpu_seconds=args.cpu_seconds)
    if not args.no_big:
        # N > 1: the configs[3] / [4] workloads on N GPUs (sharded DO-BFS, CC propagation, sharded MS-BFS)
        big = args.big_scale
        blk = {}
        if ws == 1:
            blk["pagerank"] = pagerank_block(jg, ctx, big, args.edgefactor, args.big_steps, 3)
        blk["bfs"] = bfs_block(jg, ctx, ctl, big, args.edgefactor, nsrc=4, cpu=False)
        blk["cc"], blk["msbfs64"] = rmat26_both_blocks(jg, ctx, ctl, big, args.edgefactor,
                                                       0 if args.host_transport else local, args.cc_plan)
        extra[f"rmat{big}"] = blk

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.scale, args.edgefactor, args.seed, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "GTEPS for PageRank iter + BFS, RMAT-24/26, 1/2/4/8 GPUs; % of HBM peak",
            "value": round(value, 3), "unit": "GTEPS", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (Graph500 Kronecker RMAT, on-device generator)",
            "config": {"workload": workload, "n": n, "m": m,
                       "parallelism": (f"1d-vertex-partition x{ws}, " + ("host-transport rehearsal on one GPU (not a "
                                       "measurement)" if args.host_transport else "RCCL halo send/recv"))
                       if ws > 1 else "single GPU",
                       "build_ms": round(build_ms, 1), "truncated_vertices": info["truncated_vertices"],
                       "in_entries": in_nnz},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if per_rank is not None:
            line["per_rank"] = per_rank
        line["head"], line["code"] = code_identity()
        line.update(extra)
        if args.trace_windows:
            line["trace_windows"] = {"clock": "CLOCK_MONOTONIC ns", "windows": WINDOWS}
        print(json.dumps(line), flush=True)
    ctx.close()
    ctl.close()


if __name__ == "__main__":
    main()
