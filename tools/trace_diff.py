"""Kernel time of ONE program call from two counter-free rocprofv3 traces of the same command that differ
only in how many calls they time (build kernels and warm-up calls cancel out):

    python tools/trace_diff.py <trace dir A> <runs A> <trace dir B> <runs B> [--shards P] [--out f.json]

Each dir holds the rocprofv3 --kernel-trace --stats output (*kernel_stats.csv) of e.g.
`tools/shard_sim.py --program msbfs --shards 8 --reps R`; `runs` is the "runs" field of that command's
JSON line.  Per kernel name: (total B - total A) / (runs B - runs A) µs per call; with --shards P the
sum over kernels divided by P is the per-shard kernel time of a P-GPU run (logical shards run one after
another on one stream).  The simulation's device copies (`__amd_rocclr_copyBuffer`: the
halo runs copied between logical shards, the counters read back) stand in for the RCCL exchange and are
reported apart (copy_ms_per_call), not in kernel_ms_per_shard; memsets (fillBuffer) are shard work and
stay in.  The exchange itself is modelled separately.
"""
import argparse
import csv
import glob
import json
import os


def totals(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:110]
            t, c = out.get(name, (0.0, 0))
            out[name] = (t + float(r["TotalDurationNs"]) / 1e3, c + int(r["Calls"]))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("a")
    p.add_argument("runs_a", type=int)
    p.add_argument("b")
    p.add_argument("runs_b", type=int)
    p.add_argument("--shards", type=int, default=1)
    p.add_argument("--out")
    a = p.parse_args()
    ta, tb = totals(a.a), totals(a.b)
    dr = a.runs_b - a.runs_a
    if dr <= 0:
        raise SystemExit("runs B must exceed runs A")
    per = {}
    for k in set(ta) | set(tb):
        us = (tb.get(k, (0.0, 0))[0] - ta.get(k, (0.0, 0))[0]) / dr
        calls = (tb.get(k, (0.0, 0))[1] - ta.get(k, (0.0, 0))[1]) / dr
        if calls > 0 and us > 0.05:
            per[k] = {"us_per_call": round(us, 2), "launches_per_call": round(calls, 2)}
    copy = sum(v["us_per_call"] for k, v in per.items() if "copyBuffer" in k)
    total = sum(v["us_per_call"] for k, v in per.items() if "copyBuffer" not in k)
    out = {"runs_a": a.runs_a, "runs_b": a.runs_b, "shards": a.shards, "kernel_ms_per_call": round(total / 1e3, 4),
           "kernel_ms_per_shard": round(total / 1e3 / a.shards, 4), "copy_ms_per_call": round(copy / 1e3, 4),
           "kernels": dict(sorted(per.items(), key=lambda kv: -kv[1]["us_per_call"]))}
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(json.dumps({k: out[k] for k in ("shards", "kernel_ms_per_call", "kernel_ms_per_shard", "copy_ms_per_call")}))


if __name__ == "__main__":
    main()
