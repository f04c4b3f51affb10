"""Summarise a counter-free rocprofv3 kernel trace of one tools/workload.py run.

  python tools/trace_summary.py <trace dir> <workload>      (tools/gpu_steps.sh "trace" steps run it)

Reads <dir>/**/*kernel_trace.csv (one row per dispatch, no --pmc: no counter-collection inflation) and
the workload's JSON line (the HIP-event ms of each timed run, printed by tools/workload.py into the
step's log, <dir>.log).  Writes <dir>/summary.json:
  kernel_ms_per_run         the workload's kernels (tools/workload.py KERNELS) summed over the trace ÷ the
                            runs the command made (warm runs included: the same work each time)
  kernel_ms_per_run_steady  per kernel name the median dispatch duration × its dispatches per run: the
                            steady state, without the first (cold) dispatches' outliers
  event_ms_per_run          the library's own HIP-event time of every timed run (what bench.py reports)
  kernel_us                 per kernel name: dispatches per run, median and mean µs
bench.py cites these next to the PMC traffic of the same workload (roofline "trace_source").
"""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from workload import KERNELS  # noqa: E402


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0][:100]


def main():
    d, wl = sys.argv[1], sys.argv[2]
    kind = wl.rstrip("0123456789")
    kernels = KERNELS[kind]
    info = None
    log = d.rstrip("/") + ".log"
    if os.path.exists(log):
        for line in open(log):
            line = line.strip()
            if line.startswith("{") and '"workload"' in line:
                info = json.loads(line)
    durs = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(k in name for k in kernels):
                continue
            durs.setdefault(short(name), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    runs = info["runs_total"] if info else 1
    total_us = sum(sum(v) for v in durs.values())
    steady_us = sum(statistics.median(v) * len(v) / runs for v in durs.values())
    out = {"workload": info.get("workload_name") if info else wl, "command": f"python3 tools/workload.py {wl}",
           "profiler": "rocprofv3 --kernel-trace --stats (no counters)", "kernels": kernels, "runs_profiled": runs,
           "kernel_ms_per_run": round(total_us / 1e3 / runs, 4),
           "kernel_ms_per_run_steady": round(steady_us / 1e3, 4),
           "event_ms_per_run": info["ms"] if info else None,
           "kernel_us": {k: {"dispatches_per_run": round(len(v) / runs, 2), "median_us": round(statistics.median(v), 2),
                             "mean_us": round(sum(v) / len(v), 2)} for k, v in sorted(durs.items())}}
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("workload", "kernel_ms_per_run", "kernel_ms_per_run_steady",
                                          "event_ms_per_run")}))


if __name__ == "__main__":
    main()
