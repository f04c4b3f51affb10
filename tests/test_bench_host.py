"""bench.py host helpers (CPU): the CPU-baseline leg, the PMC traffic lookup and the source pick."""
import os

import numpy as np
import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_small():
    cpu = bench.cpu_baseline(12, 16, 7, 0.0, min_steps=1)
    assert set(cpu) >= {"value", "unit", "cores", "kind", "sample"}
    assert cpu["kind"] == "port" and cpu["unit"] == "GTEPS" and cpu["value"] > 0 and cpu["cores"] >= 1


def test_cpu_baseline_bfs_rounds_until_the_budget():
    b = bench.cpu_baseline_bfs(12, 16, 7, [1, 2], 0.0)
    assert b["value"] > 0 and "1 rounds over the 2 bench sources" in b["sample"]


def test_pmc_traffic_lookup():
    """Every committed summary is found by its workload (round-2 ones through their bench.json)."""
    t, src = bench.pmc_traffic("pagerank_fp64_rmat24_ef16")
    assert t is not None and t > 1e9 and src.startswith("profiles/")
    t26, src26 = bench.pmc_traffic("pagerank_fp64_rmat26_ef16")
    assert t26 is not None and t26 > t and src26 != src
    assert bench.pmc_traffic("no_such_workload") == (None, None)


def test_sources_have_edges():
    deg = np.array([0, 3, 0, 1, 5, 0, 2], np.int64)
    s = bench.pick_sources(deg, 3, 1)
    assert len(set(s.tolist())) == 3 and (deg[s] > 0).all()
    assert len(bench.pick_sources(deg, 10, 1)) == 4  # all candidates when fewer than asked


def test_required_bytes_below_model():
    m, n, live = 16 << 24, 1 << 24, 9_000_000
    r = bench.required_roofline(m, live, 0.8)
    assert r["bytes_per_launch"] == 12.0 * m + 24.0 * live < 12.0 * m + 32.0 * n
    assert abs(r["frac"] - r["bytes_per_launch"] / 0.8e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-4


def test_per_rank_rows_flag_exchange_beyond_compute():
    """a rank's exchange time inside a call cannot exceed the call's time; such a row
    is flagged (the other blocks' results are kept) and this test is where it fails."""
    rows = bench.per_rank_rows([[10.0, 2.5], [9.5, 3.0]])
    assert rows[1] == {"rank": 1, "compute_ms": 9.5, "exchange_ms": 3.0}
    assert not any("timing_suspect" in r for r in rows)
    bad = bench.per_rank_rows([[936.9, 1302.0]])
    assert "timing_suspect" in bad[0]


def test_bench_trace_cuts_windows_at_the_markers(tmp_path):
    """tools/bench_trace.py: a window's dispatches outside the library's region markers (id lookups,
    argument copies, output kernels) do not count; the span runs from the begin mark to the last end mark
    (the DO-BFS marks the end of every level batch); a window without marks counts whole."""
    import csv
    import json
    import subprocess
    import sys
    us = 1000
    rows = [("id_lookup_kernel", 0, 2), ("jg::region_begin_kernel()", 3, 4), ("bfs_init_kernel", 5, 8),
            ("bfs_level_kernel", 9, 19), ("jg::region_end_kernel()", 20, 21), ("copyBuffer", 22, 24),
            ("bfs_level_kernel", 25, 30), ("jg::region_end_kernel()", 31, 32), ("cc_output_kernel", 33, 90),
            ("pull_merge_kernel", 100, 110), ("pull_light_finalize_kernel", 111, 120),
            ("pull_merge_kernel", 121, 131), ("pull_light_finalize_kernel", 132, 140)]
    with open(tmp_path / "b_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for n, s, e in rows:
            w.writerow([n, s * us, e * us])
    line = {"metric": "m", "ms_per_step": 0.02, "config": {"workload": "pr"},
            "roofline": {"kernel_ms": 0.02, "bytes_per_launch": 8e6},
            "bfs": {"workload": "bfs", "ms_median": 0.025, "roofline": {"bytes_per_launch": 1e6}},
            "trace_windows": {"windows": [["bfs", 0, 95 * us, 1], ["pr", 99 * us, 141 * us, 2]]}}
    (tmp_path / "b.json").write_text(json.dumps(line) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_trace.py"), str(tmp_path), "b",
                          str(tmp_path / "b.json")], capture_output=True, text=True, check=True).stdout
    blk = json.loads(out)["blocks"]
    b = blk["bfs"]
    assert b["marked"] and b["dispatches_per_run"] == 4  # init, two levels, the copy between batches
    assert b["trace_span_ms"] == pytest.approx(0.025)  # init start 5 -> last level end 30 us
    assert b["trace_kernel_ms"] == pytest.approx((3 + 10 + 2 + 5) / 1000)
    assert b["agree"]
    p = blk["pr"]
    assert not p["marked"] and p["dispatches_per_run"] == 2
    assert p["trace_span_ms"] == pytest.approx(0.020) and p["within_step"]


def test_roofline_reports_fabric_fraction_beside_the_model():
    """a block whose workload has a committed PMC summary carries frac_fabric (the
    counters' fabric bytes over the run's time) beside the model's work-equivalent frac."""
    r = bench.hbm_roofline(3.758e9, 0.75, "k", "pagerank_fp64_rmat24_ef16", "m")
    assert r["traffic"] is not None and "frac_fabric" in r
    assert abs(r["frac_fabric"] - r["traffic"] / 0.75e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-4
    assert "frac_fabric" not in bench.hbm_roofline(1e9, 1.0, "k")


def test_code_identity(monkeypatch):
    """The bench line names what it measured: JG_BENCH_HEAD (the GPU box gets the tree without .git) and
    content hashes of bench.py and the library (bench_trace.py copies both into its summary)."""
    monkeypatch.setenv("JG_BENCH_HEAD", "abc1234")
    head, code = bench.code_identity()
    assert head == "abc1234" and len(code["bench_py_sha16"]) == 16
    assert set(code) == {"bench_py_sha16", "libjanusgpu_sha16"}
