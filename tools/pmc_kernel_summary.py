"""Per-kernel counters from rocprofv3 --pmc passes (tools/gpu_pmc_kernels.sh): every counter summed per
kernel name over the profiled dispatches, divided by the workload's runs_total (the tools/workload.py
line), with the derived fabric bytes (reads: 32/64/128-B request split; writes: 64-B and 32-B requests)
and the L2 hit rate.
    python tools/pmc_kernel_summary.py <dir with pmc_*/ subdirs and trace.json> [--top N]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def name_of(k):
    return k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    runs = 1
    for f in ("trace.json", "pmc_rd.json", "workload.json"):
        p = os.path.join(a.dir, f)
        if os.path.exists(p):
            try:
                runs = json.load(open(p)).get("runs_total", 1)
                break
            except ValueError:
                pass
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(a.dir, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[name_of(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, c in per.items():
        d = {n: v / runs for n, v in c.items()}
        if "TCC_EA0_RDREQ_sum" in d:
            d["read_bytes"] = 32 * d.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * d.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                128 * d.get("TCC_EA0_RDREQ_128B_sum", 0)
        if "TCC_EA0_WRREQ_sum" in d:
            w64 = d.get("TCC_EA0_WRREQ_64B_sum", 0)
            d["write_bytes"] = 64 * w64 + 32 * (d["TCC_EA0_WRREQ_sum"] - w64)
        if "TCC_HIT_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d.get("TCC_MISS_sum", 0), 1)
        out[k] = {n: round(v, 4) for n, v in d.items()}
    order = sorted(out, key=lambda k: -(out[k].get("read_bytes", 0) + out[k].get("write_bytes", 0)))
    print(json.dumps({"dir": a.dir, "runs_total": runs, "kernels": {k: out[k] for k in order[:a.top]}}, indent=1))


if __name__ == "__main__":
    main()
