"""bench.py host helpers (CPU): the CPU-baseline leg, the PMC traffic lookup and the source pick."""
import numpy as np

import bench


def test_cpu_baseline_small():
    cpu = bench.cpu_baseline(12, 16, 7, 1)
    assert set(cpu) >= {"value", "unit", "cores", "kind", "sample"}
    assert cpu["kind"] == "port" and cpu["unit"] == "GTEPS" and cpu["value"] > 0 and cpu["cores"] >= 1


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
