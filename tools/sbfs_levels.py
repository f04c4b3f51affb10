"""Per-level kernel time of the sharded DO-BFS from a counter-free rocprofv3 kernel trace of
`tools/shard_sim.py --program bfs --shards P` (logical shards on one device):

    python tools/sbfs_levels.py <trace dir> [--shards 8] [--out levels.json]

Takes the last traversal in the trace (its P `sbfs_init_kernel` launches), then per level the P pre, P mid
and P post launches (the one `sbfs_copy_kernel` stands in for the exchange and is reported apart), and
prints µs per shard: pre (pack / push), mid (stamps -> mark words), post (probes / claims), their sum.
"""
import argparse
import csv
import glob
import json
import os


def kernel_rows(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        name = name.replace("jg::", "").split("<")[0]
        out.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


def levels(rows, P):
    inits = [i for i, (n, _) in enumerate(rows) if n in ("sbfs_init_kernel", "sbfs_init_roots_kernel")]
    if len(inits) < P:
        raise SystemExit("fewer init launches than shards")
    start = inits[-P]
    init_us = sum(d for n, d in rows[start:start + P]) / P
    table, lv, cur = [], 0, None
    for n, d in rows[start + P:]:
        if n in ("sbfs_init_kernel", "sbfs_init_roots_kernel"):
            break
        if n == "sbfs_pre_kernel":
            if cur is None or cur["pre_n"] == P:
                cur = {"level": lv, "pre": 0.0, "mid": 0.0, "post": 0.0, "copy": 0.0, "pre_n": 0}
                table.append(cur)
                lv += 1
            cur["pre"] += d / P
            cur["pre_n"] += 1
        elif cur is not None and n == "sbfs_mid_kernel":
            cur["mid"] += d / P
        elif cur is not None and n == "sbfs_post_kernel":
            cur["post"] += d / P
        elif cur is not None and n == "sbfs_copy_kernel":
            cur["copy"] += d
    for t in table:
        del t["pre_n"]
        t["sum"] = t["pre"] + t["mid"] + t["post"]
    return init_us, table


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--out")
    a = p.parse_args()
    init_us, table = levels(kernel_rows(a.trace), a.shards)
    total = init_us + sum(t["sum"] for t in table)
    print(f"{'level':>5} {'pre':>7} {'mid':>7} {'post':>7} {'sum':>7}   (us per shard; copy = exchange stand-in)")
    print(f"{'init':>5} {'':>7} {'':>7} {'':>7} {init_us:7.1f}")
    for t in table:
        print(f"{t['level']:5d} {t['pre']:7.1f} {t['mid']:7.1f} {t['post']:7.1f} {t['sum']:7.1f}   copy {t['copy']:.1f}")
    print(f"total {total / 1e3:.4f} ms per shard")
    if a.out:
        json.dump({"shards": a.shards, "init_us": init_us, "levels": table, "ms_per_shard": total / 1e3},
                  open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
