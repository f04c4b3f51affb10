"""The roofline of every bench block from a counter-free kernel trace of the bench process itself (VERDICT r04
item 5).  Run the bench under the profiler with its timed regions' host-clock windows in the JSON line:

    JG_TRACE_MARKS=1 rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o bench -- python3 bench.py \
        --gpus 1 --steps 20 --warmup 5 --trace-windows > OUT/bench.json
    python tools/bench_trace.py OUT bench OUT/bench.json [--out profiles/r05/bench_trace/summary.json]

Each window (a block's timed call, or the K supersteps of a PageRank block) selects the dispatches that
started inside it, cut to the library's event-timed region when the run had JG_TRACE_MARKS=1 (marker
dispatches around t0 / t1; the call's id lookups, argument copies and output kernels fall outside).  Per
run (per superstep for PageRank) it reports the kernel-time sum and the span (first start to last end of the
region's dispatches: the interval the block's HIP events bracket), against the block's event figure from the
same process, and the HBM-roofline fraction of the block's algorithmic bytes on each.  `agree` = the
trace span within 3% of the event figure; `within_step` = neither exceeds the block's ms_per_step (for the
blocks that have one).  No GPU.
"""
import argparse
import csv
import glob
import gzip
import json
import os
import sys

import numpy as np

PEAK_GBS = 8000.0


def bench_line(path):
    with open(path) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                return json.loads(ln)
    raise SystemExit(f"no bench JSON line in {path}")


def event_figures(line):
    """workload -> (event ms per run, algorithmic bytes per run, ms_per_step or None)"""
    out = {}
    r = line["roofline"]
    out[line["config"]["workload"]] = (r["kernel_ms"], r["bytes_per_launch"], line["ms_per_step"])
    if "bfs" in line and "roofline" in line["bfs"]:
        b = line["bfs"]
        out[b["workload"]] = (b["ms_median"], b["roofline"]["bytes_per_launch"], None)
    for key, blk in line.items():
        if not (key.startswith("rmat") and isinstance(blk, dict)):
            continue
        for name, b in blk.items():
            if not isinstance(b, dict) or "roofline" not in b:
                continue
            ms = b["roofline"]["kernel_ms"]
            out[b["workload"]] = (ms, b["roofline"]["bytes_per_launch"], b.get("ms_per_step"))
    return out


def is_mark(name, which):
    return f"region_{which}_kernel" in name


def segments(ks):
    """The event-timed parts of a window: with the library's markers (JG_TRACE_MARKS=1: region_begin_kernel
    before t0, region_end_kernel after t1, one after every level batch for the DO-BFS), each begin mark to
    the last end mark before the next begin -> (begin mark's end, end mark's start, dispatches between);
    without markers the whole window -> (None, None, dispatches)."""
    b = [i for i, k in enumerate(ks) if is_mark(k[2], "begin")]
    if not b:
        return [(None, None, ks)]
    out = []
    for j, i in enumerate(b):
        nxt = b[j + 1] if j + 1 < len(b) else len(ks)
        ends = [x for x in range(i + 1, nxt) if is_mark(ks[x][2], "end")]
        if not ends:
            continue
        e = ends[-1]
        body = [k for k in ks[i + 1:e] if not is_mark(k[2], "end")]
        out.append((ks[i][1], ks[e][0], body))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("name", help="the rocprofv3 -o name")
    p.add_argument("bench_json")
    p.add_argument("--out")
    a = p.parse_args()
    files = [f for ext in ("csv", "csv.gz")
             for f in glob.glob(os.path.join(a.trace_dir, "**", f"{a.name}_kernel_trace.{ext}"), recursive=True)]
    if not files:
        raise SystemExit(f"no {a.name}_kernel_trace.csv(.gz) under {a.trace_dir}")
    rows = []
    for fn in files:
        with (gzip.open(fn, "rt") if fn.endswith(".gz") else open(fn)) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    start = np.array([r[0] for r in rows], dtype=np.int64)
    line = bench_line(a.bench_json)
    wins = line.get("trace_windows", {}).get("windows")
    if not wins:
        raise SystemExit("the bench line has no trace_windows (run bench.py --trace-windows)")
    ev = event_figures(line)
    per = {}
    for name, t0, t1, runs in wins:
        i0, i1 = np.searchsorted(start, t0), np.searchsorted(start, t1)
        ks = rows[i0:i1]
        if not ks:
            raise SystemExit(f"window {name}: no dispatch started inside it (clock mismatch?)")
        kern, span, nd, marked = 0, 0, 0, False
        for seg in segments(ks):
            marked |= seg[0] is not None
            body = seg[2]
            kern += sum(e - s for s, e, _ in body)
            nd += len(body)
            if body:  # the events sit right before the first dispatch and right after the last
                span += max(e for _, e, _ in body) - body[0][0]
        d = per.setdefault(name, {"kernel": [], "span": [], "dispatches": [], "runs": runs, "marked": marked})
        d["kernel"].append(kern / runs / 1e6)
        d["span"].append(span / runs / 1e6)
        d["dispatches"].append(nd / runs)
    out = {"bench_head": line.get("head"), "bench_code": line.get("code"), "trace_files": [os.path.relpath(x) for x in files], "blocks": {}}
    for name, d in per.items():
        kern, span = float(np.median(d["kernel"])), float(np.median(d["span"]))
        blk = {"windows": len(d["kernel"]), "runs_per_window": d["runs"], "marked": d["marked"],
               "dispatches_per_run": float(np.median(d["dispatches"])),
               "trace_kernel_ms": round(kern, 4), "trace_span_ms": round(span, 4)}
        if name in ev:
            ems, byt, step = ev[name]
            blk.update({"event_ms": round(ems, 4), "bytes": byt,
                        "frac_event": round(byt / (ems * 1e-3) / 1e9 / PEAK_GBS, 4),
                        "frac_trace_span": round(byt / (span * 1e-3) / 1e9 / PEAK_GBS, 4),
                        "frac_trace_kernel": round(byt / (kern * 1e-3) / 1e9 / PEAK_GBS, 4),
                        "span_over_event": round(span / ems, 4),
                        "agree": bool(abs(span / ems - 1.0) <= 0.03)})
            if step is not None:
                blk["ms_per_step"] = step
                blk["within_step"] = bool(span <= step and ems <= step)
        out["blocks"][name] = blk
    text = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    sys.exit(main())
