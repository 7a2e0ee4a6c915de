"""The roofline's time basis on CPU: the union of compositing-launch
intervals (bench.busy_union_ms over in-kernel spans, tools/busy_union.py over
a rocprofv3 kernel trace).  Overlapping launches count once, disjoint ones
add, and the trace tool groups launches into regions and keeps only regions
of the bench's shape (4 launches: one per group of 5 views)."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_bench_busy_union_ms():
    import bench
    # 100 MHz ticks: [0, 100) and [50, 150) overlap -> 150 ticks; [300, 400) apart -> +100
    assert bench.busy_union_ms([(0, 100), (50, 150), (300, 400)]) == pytest.approx(250e-5)
    assert bench.busy_union_ms([(10, 20)]) == pytest.approx(10e-5)
    assert bench.busy_union_ms([]) == 0.0
    # nested and touching intervals
    assert bench.busy_union_ms([(0, 100), (10, 20), (100, 130)]) == pytest.approx(130e-5)


def test_busy_union_tool(tmp_path):
    import busy_union
    assert busy_union.union_ns([(0, 10), (5, 20), (30, 40)]) == 30
    # two regions of 4 launches (the bench's shape) and one stray launch region
    name = "void gsr::(anonymous namespace)::k_composite_views<0>(gsr::(anonymous namespace)::CompViews)"
    rows = []
    for r0 in (0, 10_000_000):  # ns; regions 10 ms apart
        for i in range(4):
            rows.append((name, r0 + i * 100_000, r0 + i * 100_000 + 300_000))  # overlapping 300 us launches
    rows.append((name, 30_000_000, 30_050_000))
    rows.append(("void other_kernel()", 0, 5_000_000))
    trace = tmp_path / "kernel_trace.csv"
    with open(trace, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "busy_union.py"), str(trace), "--views", "20"],
                         check=True, capture_output=True, text=True).stdout
    got = json.loads(out)
    assert got["regions_of_the_bench_shape"] == 2
    # each region: launches at 0, 100, 200, 300 us lasting 300 us -> union [0, 600) us
    assert got["busy_us_per_region_median"] == pytest.approx(600.0)
    assert got["us_per_view"] == pytest.approx(30.0)
