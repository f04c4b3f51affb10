"""Summarise tools/pmc_workloads.sh output into profiles/<round>/pmc/<workload>/summary.json.

For each workload: the kernels of its timed region (tools/workload.py KERNELS, name substrings) are
selected in every counter CSV, their counters summed and divided by the runs the command made
(workload.json "runs_total": warm and rejected-source runs included, all the same kind of work).  Bytes
follow MI355X_MICROARCH.md's HBM section (FETCH_SIZE under-counts 128-B requests 2x on gfx950, so reads
come from the TCC_EA0_RDREQ 32/64/128-B split: 32*n32 + 64*n64 + 128*n128; writes 64*n64 + 32*(n - n64));
Infinity-Cache hits are counted, so this is fabric traffic beyond L2, an upper bound on HBM bytes.
Usage: python tools/pmc_workload_summary.py gpurun_out/<tag> profiles/<round>/pmc
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def selected(name, kernels):
    return any(k in name for k in kernels)


def counters(path, kernels):
    tot, calls = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not selected(k, kernels):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k.split("(")[0]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return tot, {k: len(v) for k, v in calls.items()}


def summarise(src, dst):
    wl = json.loads(open(os.path.join(src, "workload.json")).read().strip().splitlines()[-1])
    kernels, runs = wl["kernels"], wl["runs_total"]
    out = {"workload": wl["workload_name"], "command": f"python3 tools/workload.py {wl['workload']}",
           "kernels": kernels, "runs_profiled": runs,
           "ms_per_run": wl["ms"], "algorithmic_bytes_per_run": wl["bytes"]}
    stats = os.path.join(src, "stats", "wl_kernel_stats.csv")
    if os.path.exists(stats):
        rows = [r for r in csv.DictReader(open(stats)) if selected(r["Name"], kernels)]
        out["kernel_us_per_run"] = {r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]:
                                    round(float(r["TotalDurationNs"]) / 1e3 / runs, 2) for r in rows}
        out["kernel_ms_per_run"] = round(sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / runs, 4)
        os.makedirs(dst, exist_ok=True)
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    rd, calls = counters(os.path.join(src, "pmc_rd"), kernels)
    wr, _ = counters(os.path.join(src, "pmc_wr"), kernels)
    fe, _ = counters(os.path.join(src, "pmc_fetch"), kernels)
    per = {k: v / runs for k, v in {**rd, **wr, **fe}.items()}
    out["pmc_dispatches"] = calls
    out["counters_per_run"] = per
    read = write = None
    if "TCC_EA0_RDREQ_sum" in per:
        n, n32 = per["TCC_EA0_RDREQ_sum"], per.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        n128 = per.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        n64 = per.get("TCC_EA0_RDREQ_64B_sum", n - n32 - n128)
        read = 32 * n32 + 64 * n64 + 128 * n128
    if "TCC_EA0_WRREQ_sum" in per:
        n, n64 = per["TCC_EA0_WRREQ_sum"], per.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        write = 64 * n64 + 32 * (n - n64)
    out["read_bytes_per_run"] = read
    out["write_bytes_per_run"] = write
    out["read_bytes_method"] = "TCC_EA0_RDREQ 32/64/128B request split (fabric reads beyond L2)"
    out["traffic_bytes_per_launch"] = (read or 0) + (write or 0) if read is not None else None
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "workload.json"), os.path.join(dst, "workload.json"))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    for d in sorted(os.listdir(src)):
        if os.path.exists(os.path.join(src, d, "workload.json")):
            o = summarise(os.path.join(src, d), os.path.join(dst, d))
            print(d, o["workload"], "traffic/run", o["traffic_bytes_per_launch"], "kernel ms/run",
                  o.get("kernel_ms_per_run"), "alg bytes/run", o["algorithmic_bytes_per_run"][:1])


if __name__ == "__main__":
    main()
