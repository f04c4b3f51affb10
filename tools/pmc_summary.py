"""Summarise a tools/profile_round.sh output directory into profiles/<tag>/summary.json.

HBM traffic per launch of the dominant kernel follows MI355X_MICROARCH.md §HBM / rocprofv3:
  FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE = TCC_EA0_RDREQ x 64 B on gfx950, which under-counts
  128-B requests by 2x, so when the TCC_EA0_RDREQ_{32B,64B,128B} split is present the read bytes
  are recomputed as 32*n32 + 64*n64 + 128*n128 (n64 = RDREQ - n32 - n128 if no 64B counter).
Usage: python tools/pmc_summary.py gpurun_out/r01 profiles/r01 [kernel-substring]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def per_kernel(path, kernel):
    vals = defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "pull_kernel"
    os.makedirs(dst, exist_ok=True)
    out = {"kernel": kernel}
    stats = os.path.join(src, "stats", "bench_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        out["kernel_stats_top"] = [{"name": r["Name"][:120], "calls": int(r["Calls"]),
                                    "avg_us": round(float(r["AverageNs"]) / 1e3, 2), "pct": float(r["Percentage"])}
                                   for r in rows[:12]]
        dom = [r for r in rows if kernel in r["Name"]]
        if dom:
            out["dominant_avg_us"] = round(float(dom[0]["AverageNs"]) / 1e3, 2)
            out["dominant_calls"] = int(dom[0]["Calls"])
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    c = {}
    for sub in ["pmc_fetch/fetch_counter_collection.csv", "pmc_write/write_counter_collection.csv",
                "pmc_rdreq/rdreq_counter_collection.csv", "pmc_wrreq/wrreq_counter_collection.csv"]:
        c.update(per_kernel(os.path.join(src, sub), kernel))
    out["counters_per_launch"] = c
    rd = None
    if "TCC_EA0_RDREQ_sum" in c and "TCC_EA0_RDREQ_128B_sum" in c:
        n = c["TCC_EA0_RDREQ_sum"]
        n32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        n128 = c.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        n64 = c.get("TCC_EA0_RDREQ_64B_sum", n - n32 - n128)
        rd = 32 * n32 + 64 * n64 + 128 * n128
        out["read_bytes_method"] = "TCC_EA0_RDREQ 32/64/128B split"
    elif "FETCH_SIZE" in c:
        rd = c["FETCH_SIZE"] * 1024
        out["read_bytes_method"] = "FETCH_SIZE x 1024 (64-B tally; uncalibrated for this access width)"
    wr = c["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in c else None
    out["read_bytes_per_launch"] = rd
    out["write_bytes_per_launch"] = wr
    out["traffic_bytes_per_launch"] = (rd or 0) + (wr or 0) if rd is not None else None
    b = os.path.join(src, "bench.json")
    if os.path.exists(b):
        shutil.copy(b, os.path.join(dst, "bench.json"))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
