"""Per-level kernel times of single-source DO-BFS traversals under two knob settings (RMAT, the bench's
sources), for a counter-free rocprofv3 kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d DIR -o t -- python3 tools/bfs_level_trace.py run --scale 26 A B
    python3 tools/bfs_level_trace.py show DIR            # one line per traversal: level kernel durations (us)

`run` does, for each setting, one warm and one traced traversal per source; with JG_DEBUG_BFS=1 the library
prints each level's direction and frontier to stderr.
"""
import argparse
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import bench
    import janusgraph_amd as jg
    ctx = jg.Context((0,))
    m = 16 << a.scale
    g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_BOTH)
    srcs = []
    for sv in bench.pick_sources(g.degrees(jg.DIR_BOTH), 4 * a.nsrc, a.scale).tolist():
        if len(srcs) == a.nsrc:
            break
        g.bfs([sv], jg.DIR_BOTH, want=False)
        if ctx.stats()["edges_traversed"] >= m // 100:
            srcs.append(sv)
    for s in a.settings:
        for kv in s.split(","):
            k, v = kv.split("=")
            jg._lib.tune_set(k, int(v))
        for sv in srcs:
            g.bfs([sv], jg.DIR_BOTH, want=False)
            g.bfs([sv], jg.DIR_BOTH, want=False)
            print(s, sv, round(ctx.stats()["compute_ms"], 4), ctx.stats()["levels"], flush=True)
    g.close()
    ctx.close()


def show(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    cur = None
    out = []
    for r in rows:
        n = r["Kernel_Name"]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "bfs_init_kernel" in n:
            cur = []
            out.append(cur)
        elif cur is not None and ("bfs_level_kernel" in n or "bfs_td_claim_kernel" in n):
            cur.append(("c" if "claim" in n else "") + f"{us:.1f}")
    for t in out[-16:]:
        print(" ".join(t))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=["run", "show"])
    p.add_argument("args", nargs="*")
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--nsrc", type=int, default=4)
    a = p.parse_intermixed_args()
    if a.cmd == "run":
        a.settings = a.args
        run(a)
    else:
        show(a.args[0])


if __name__ == "__main__":
    main()
