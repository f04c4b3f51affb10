"""One bench workload, repeated, for rocprofv3 (kernel trace or PMC passes): the same graph, sources and
calls as bench.py's block, `runs` times after one warm run.  Prints one JSON line with the HIP-event
time and the library's algorithmic bytes of every run.  tools/pmc_workloads.sh profiles each workload,
tools/pmc_summary.py turns the counters into bytes per run (profiles/<round>/<workload>/summary.json),
which bench.py reads for the block's roofline "traffic".

  python tools/workload.py bfs20|bfs26|cc26|msbfs26|pr24|pr26 [--runs R] [--tune key=value ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# kernels of each workload's timed region (name substrings; tools/pmc_summary.py filters on them)
KERNELS = {
    "bfs": ["bfs_init_kernel", "bfs_level_kernel", "bfs_td_claim_kernel"],
    "cc": ["uf_init_kernel", "uf_link_first_kernel", "uf_hook_first_kernel", "uf_link_up_compress_kernel",
           "uf_link_rest_kernel", "uf_compress_kernel", "uf_sample_kernel", "uf_minrank_kernel",
           "heavy_rows_kernel", "bfs_init_roots_kernel", "bfs_level_kernel", "bfs_td_claim_kernel",
           "cc_giant_bits_kernel", "cc_output_kernel"],  # (round 6: the caller-order output is in the region)
    "msbfs": ["MsBfsOp", "msbfs_live_kernel", "msbfs_scan_kernel", "msbfs_todo_kernel", "msbfs_task_live_kernel",
              "msbfs_init_kernel", "msbfs_frontier_kernel", "msbfs_source_queue_kernel", "msbfs_td_kernel",
              "msbfs_td_apply_kernel", "msbfs_zero_list_kernel", "msbfs_td_recv_kernel", "msbfs_td_record_kernel",
              "msbfs_exit_first_kernel", "msbfs_exit_rest_kernel", "zero_words_kernel", "msbfs_frontier_live_kernel",
              "msbfs_td_apply_rows_kernel", "msbfs_zero_tail_sources_kernel"],
    "pr": ["PrOp"],
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("workload", choices=["bfs20", "bfs26", "cc26", "msbfs26", "pr24", "pr26"])
    p.add_argument("--runs", type=int, default=5)
    p.add_argument("--tune", action="append", default=[], help="a jg_tune_set knob (key=value; repeatable) applied before the build")
    a = p.parse_args()
    import janusgraph_amd as jg
    for kv in a.tune:
        k, _, v = kv.partition("=")
        jg._lib.tune_set(k, int(v))
    ctx = jg.Context((0,))
    kind, scale = a.workload.rstrip("0123456789"), int(a.workload[-2:])
    ef = 16
    n, m = 1 << scale, ef << scale
    out = {"workload": a.workload, "tune": a.tune, "runs": a.runs, "warm_runs": 1, "kernels": KERNELS[kind], "ms": [], "bytes": []}
    if kind == "pr":
        g = ctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_IN)
        g.pagerank_begin(0.85, n)
        g.pagerank_step(1 + a.runs)  # one warm superstep + runs: each run is one superstep
        g.sync()
        g.pagerank_end(want=False)
        out["workload_name"] = f"pagerank_fp64_rmat{scale}_ef{ef}"
        out["runs_note"] = "supersteps 0, 1 (pagerank_begin) run other kernels; runs = the power supersteps"
        out["runs_total"] = 1 + a.runs
    else:
        g = ctx.build_rmat(scale, ef, 0x5EED + scale, flags=jg.ADJ_BOTH)
        deg = g.degrees(jg.DIR_BOTH)
        if kind == "bfs":
            # bench.bfs_block's first source: the same candidates, the first whose component is not tiny
            # (the accepted trial is the warm run; rejected trials traverse tiny components)
            trials = 0
            for sv in bench.pick_sources(deg, 4 * (6 if scale == 20 else 4), scale).tolist():
                g.bfs([sv], jg.DIR_BOTH, want=False)
                trials += 1
                if ctx.stats()["edges_traversed"] >= m // 100:
                    break
            out["source"] = sv
            out["warm_runs"] = trials
            out["runs_total"] = trials + a.runs
            call = lambda: g.bfs([sv], jg.DIR_BOTH, want=False)  # noqa: E731
            out["workload_name"] = f"bfs_spvp_rmat{scale}_ef{ef}"
        elif kind == "cc":
            out["runs_total"] = 1 + a.runs
            call = g.connected_components
            out["workload_name"] = f"cc_rmat{scale}_ef{ef}"
        else:
            srcs = bench.pick_sources(deg, 64, 7)
            out["runs_total"] = 1 + a.runs
            call = lambda: g.bfs(srcs, jg.DIR_BOTH, want=False)  # noqa: E731
            out["workload_name"] = f"msbfs64_rmat{scale}_ef{ef}"
        for r in range(a.runs + (0 if kind == "bfs" else 1)):
            call()
            st = ctx.stats()
            if kind == "bfs" or r:
                out["ms"].append(st["compute_ms"])
                out["bytes"].append(st["algorithmic_bytes"])
    g.close()
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
