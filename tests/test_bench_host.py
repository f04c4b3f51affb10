"""bench.py host helpers (CPU): the CPU-baseline leg and the PMC traffic lookup."""
import bench


def test_cpu_baseline_small():
    cpu = bench.cpu_baseline(12, 16, 7, 1)
    assert set(cpu) >= {"value", "unit", "cores", "kind", "sample"}
    assert cpu["kind"] == "port" and cpu["unit"] == "GTEPS" and cpu["value"] > 0 and cpu["cores"] >= 1


def test_pmc_traffic_lookup():
    t, src = bench.pmc_traffic("PrOp", "pagerank_fp64_rmat24_ef16")
    if t is not None:
        assert t > 1e9 and src.startswith("profiles/")
    assert bench.pmc_traffic("NoSuchKernel")[0] is None
