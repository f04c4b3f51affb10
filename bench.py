"""Benchmark: GpuGraphComputer supersteps on synthetic Graph500 RMAT graphs (BASELINE.json metric).

Headline (value): PageRank fp64 on RMAT scale-24 edgefactor-16 (BASELINE.json configs[2]), one
"step" = one power superstep of JanusGraph's PageRankVertexProgram over the whole graph (pull SpMV
over the in-CSR + contribution write + RCCL allgather of the rank-contribution vector when N > 1).
value = directed edges processed per second over all GPUs (GTEPS), inputs resident in HBM.
Secondary (same JSON line): BFS (SPVP depth, undirected) from one source on RMAT scale-20
(configs[1]) as Graph500 TEPS.

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
    p.add_argument("--cpu-steps", type=int, default=2)
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

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def pmc_traffic(kernel_tag="PrOp", workload=None):
    """HBM bytes per launch of the dominant kernel from the newest committed rocprofv3 PMC summary
    (profiles/<round>/summary.json, made by tools/profile_round.sh + tools/pmc_summary.py on the same
    bench workload).  None when no summary exists."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    for rnd in sorted(os.listdir(pdir), reverse=True):
        path = os.path.join(pdir, rnd, "summary.json")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            s = json.load(f)
        if kernel_tag not in s.get("kernel", "") or s.get("traffic_bytes_per_launch") is None:
            continue
        bj = os.path.join(pdir, rnd, "bench.json")
        if workload and os.path.exists(bj):
            with open(bj) as f:
                if json.load(f).get("config", {}).get("workload") != workload:
                    continue
        return s["traffic_bytes_per_launch"], f"profiles/{rnd}/summary.json ({s.get('read_bytes_method', '')})"
    return None, None


def cpu_baseline(scale, ef, seed, steps):
    """The oracle's PageRank superstep (OpenMP) on the same RMAT graph, rank 0 only."""
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
    for _ in range(steps):
        contrib = o.pagerank_superstep_csr(n, ptr, col, contrib, outdeg, 0.85, n)
    dt = time.perf_counter() - t0
    return {"value": round(m * steps / dt / 1e9, 4), "unit": "GTEPS", "cores": o.num_threads(), "kind": "port",
            "sample": f"oracle/jg_oracle.c jo_pagerank_superstep_csr (OpenMP), {steps} full power supersteps on "
                      f"the same RMAT-{scale} ef{ef} graph (seed {seed}); CSR build untimed"}


def main():
    args = parse()
    ws, rank, local = dist_env()
    if ws != args.gpus:
        args.gpus = ws if ws > 1 else args.gpus
    ctl = Control(ws, rank)
    import janusgraph_amd as jg

    uid = jg._lib.comm_unique_id() if (ws > 1 and rank == 0) else None
    uid = ctl.bcast_bytes(uid)
    ctx = jg.Context((local,), rank=rank if ws > 1 else None, nranks=ws, unique_id=uid)
    n = 1 << args.scale
    m = args.edgefactor << args.scale

    g = ctx.build_rmat(args.scale, args.edgefactor, args.seed, flags=jg.ADJ_IN)
    build_ms = ctx.stats()["build_ms"]
    info = g.info()
    g.pagerank_begin(0.85, n)
    g.pagerank_step(args.warmup)
    g.sync()
    ctl.barrier()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    g.pagerank_step(args.steps)
    g.sync()
    t1 = time.perf_counter()
    ctl.barrier()
    elapsed = ctl.max(t1 - t0)
    g.pagerank_end(want=False)
    st = ctx.stats()
    ctx.set_profiling(False)
    ms_per_step = elapsed / args.steps * 1e3
    value = m * args.steps / elapsed / 1e9  # GTEPS, all ranks

    # roofline of the dominant kernel (pull SpMV), HIP events on its stream, this rank's launches
    launches = max(st["kernel_launches"], 1)
    kern_ms = st["kernel_ms_total"] / launches
    alg_bytes_launch = 12.0 * m / ws + 32.0 * n / ws  # SURVEY §8d per-edge/per-vertex bytes x this rank's share
    if ws == 1:
        alg_bytes_launch = 12.0 * m + 32.0 * n
    achieved = alg_bytes_launch / (kern_ms * 1e-3) / 1e9
    workload = f"pagerank_fp64_rmat{args.scale}_ef{args.edgefactor}"
    traffic, traffic_src = pmc_traffic("PrOp", workload) if ws == 1 else (None, None)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": "PageRank superstep (pull_merge_kernel x bands + fixups + light-row pull_kernel + finalize kernels, PrOp)", "kernel_ms": round(kern_ms, 4),
                "bytes_per_launch": alg_bytes_launch}

    bfs = None
    if not args.no_bfs and ws == 1:
        gb = ctx.build_rmat(args.bfs_scale, args.edgefactor, 0x5EED + args.bfs_scale, flags=jg.ADJ_BOTH)
        rng = np.random.default_rng(1)
        times, teps = [], []
        for k in range(6):
            srcv = int(rng.integers(0, 1 << args.bfs_scale))
            gb.bfs([srcv], jg.DIR_BOTH, want=False)
            s = ctx.stats()
            if s["edges_traversed"] < (args.edgefactor << args.bfs_scale) // 100:
                continue  # source in a tiny component: Graph500 resamples
            if k == 0:
                continue
            times.append(s["compute_ms"])
            teps.append(s["edges_traversed"] / (s["compute_ms"] * 1e-3) / 1e9)
        bfs = {"workload": f"bfs_spvp_rmat{args.bfs_scale}_ef{args.edgefactor}", "gteps_median": round(float(np.median(teps)), 3) if teps else None,
               "ms_median": round(float(np.median(times)), 4) if times else None, "runs": len(times)}
        gb.close()

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.scale, args.edgefactor, args.seed, args.cpu_steps)

    if rank == 0:
        line = {
            "metric": "GTEPS for PageRank iter + BFS, RMAT-24/26, 1/2/4/8 GPUs; % of HBM peak",
            "value": round(value, 3), "unit": "GTEPS", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (Graph500 Kronecker RMAT, on-device generator)",
            "config": {"workload": f"pagerank_fp64_rmat{args.scale}_ef{args.edgefactor}", "n": n, "m": m,
                       "parallelism": f"1d-vertex-partition x{ws}, RCCL halo send/recv" if ws > 1 else "single GPU",
                       "build_ms": round(build_ms, 1), "truncated_vertices": info["truncated_vertices"]},
            "roofline": roofline, "cpu_baseline": cpu, "bfs": bfs,
        }
        print(json.dumps(line), flush=True)
    g.close()
    ctx.close()
    ctl.close()


if __name__ == "__main__":
    main()
