"""Summarise a tools/profile_round.sh output directory into profiles/<tag>/summary.json.

Traffic per PageRank superstep = the sum over every kernel of the superstep (pull_merge_kernel,
pull_merge_fixup_kernel, pull_kernel, the fused light+finalize and the finalize kernels; PrOp instantiations) of the L2 <-> fabric
bytes, from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE = TCC_EA0_RDREQ x 64 B on
gfx950 and under-counts 128-B requests by 2x, so the reads are recomputed from the request-size
split: 32*n32 + 64*n64 + 128*n128; writes: 64*n64 + 32*(n - n64)).  Infinity-Cache hits are counted
by these counters, so this is fabric traffic beyond L2 (HBM + MALL), an upper bound on HBM bytes.
Usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<tag> [steps]
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

SUPERSTEP = ("pull_merge_kernel", "pull_merge_fixup_kernel", "pull_kernel", "pull_slice_finalize_kernel",
             "pull_hub_finalize_kernel", "pull_lds_kernel", "pull_light_finalize_kernel")


def counters(path):
    """{counter: total over the superstep kernels}, {kernel: dispatches}"""
    tot, calls = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "PrOp" not in k or not any(s in k for s in SUPERSTEP):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k.split("(")[0]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return tot, {k: len(v) for k, v in calls.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6  # --steps 5 --warmup 1
    os.makedirs(dst, exist_ok=True)
    out = {"kernel": "PageRank superstep (PrOp): " + ", ".join(SUPERSTEP), "supersteps_profiled": steps}
    stats = os.path.join(src, "stats", "bench_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        out["kernel_stats_top"] = [{"name": r["Name"][:120], "calls": int(r["Calls"]),
                                    "avg_us": round(float(r["AverageNs"]) / 1e3, 2), "pct": float(r["Percentage"])}
                                   for r in rows[:14]]
        ss = [r for r in rows if "PrOp" in r["Name"] and any(s in r["Name"] for s in SUPERSTEP)]
        # template instantiations (e.g. the merge kernel's packed widths, one per band) stay apart:
        # the kernel name plus its template arguments
        out["superstep_kernel_avg_us"] = {r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]:
                                          round(float(r["AverageNs"]) / 1e3, 2) for r in ss}
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    rd, rd_calls = counters(os.path.join(src, "pmc_rd"))
    wr, _ = counters(os.path.join(src, "pmc_wr"))
    fe, _ = counters(os.path.join(src, "pmc_fetch"))
    out["pmc_dispatches"] = rd_calls
    per = {k: v / steps for k, v in {**rd, **wr, **fe}.items()}
    out["counters_per_superstep"] = per
    read = write = None
    if "TCC_EA0_RDREQ_sum" in per:
        n, n32 = per["TCC_EA0_RDREQ_sum"], per.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        n128 = per.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        n64 = per.get("TCC_EA0_RDREQ_64B_sum", n - n32 - n128)
        read = 32 * n32 + 64 * n64 + 128 * n128
    if "TCC_EA0_WRREQ_sum" in per:
        n, n64 = per["TCC_EA0_WRREQ_sum"], per.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        write = 64 * n64 + 32 * (n - n64)
    out["read_bytes_per_superstep"] = read
    out["write_bytes_per_superstep"] = write
    out["read_bytes_method"] = "TCC_EA0_RDREQ 32/64/128B request split (fabric reads beyond L2)"
    out["traffic_bytes_per_launch"] = (read or 0) + (write or 0) if read is not None else None
    for f in ("bench.json",):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("read_bytes_per_superstep", "write_bytes_per_superstep",
                                          "traffic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
