"""Per-kernel time of one workload window in a rocprofv3 kernel trace (diagnostic).

    python tools/trace_window.py <kernel_trace.csv> [--match msbfs] [--runs 2]

The window spans the first to the last kernel whose name contains --match; times are divided by
--runs (the calls inside the window)."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="msbfs")
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    hit = [r for r in rows if a.match in r["Kernel_Name"]]
    t0 = min(int(r["Start_Timestamp"]) for r in hit)
    t1 = max(int(r["End_Timestamp"]) for r in hit)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or e > t1:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:100]
        agg[name][0] += e - s
        agg[name][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"window {(t1 - t0) / a.runs / 1e6:.3f} ms per run, kernels {tot / a.runs / 1e6:.3f} ms per run")
    for k, v in sorted(agg.items(), key=lambda x: -x[1][0]):
        print(f"{v[0] / a.runs / 1e6:9.3f} ms {v[1] // a.runs:6d}  {k}")


if __name__ == "__main__":
    main()
