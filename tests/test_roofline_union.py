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


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)


def test_region_kernels_tool(tmp_path):
    """tools/region_kernels.py finds the timed region (the first idle-gap
    segment with 4 group compositing launches and no frame-alone compositor)
    and reports each kernel's busy union per frame."""
    cv = "void gsr::(anonymous namespace)::k_composite_views<0>(gsr::(anonymous namespace)::CompViews)"
    pre = "void gsr::(anonymous namespace)::k_preprocess_fc_views<3, false>(gsr::(anonymous namespace)::PreFc)"
    alone = "void gsr::(anonymous namespace)::k_composite<0, false>(uint4 const*)"
    us = 1000
    rows = []
    # warm-up segment: 8 group launches
    rows += [(cv, i * 10 * us, i * 10 * us + 20 * us) for i in range(8)]
    # timed region at 1 ms: preprocess 0..100 us, 4 overlapping compositing launches 100..400 us
    t0 = 1_000 * us
    rows += [(pre, t0, t0 + 100 * us)] + [(cv, t0 + 100 * us + 50 * us * i, t0 + 250 * us + 50 * us * i)
                                          for i in range(4)]
    # frame-alone segment, then the instrumented repeat
    rows += [(alone, 2_000 * us, 2_100 * us)]
    rows += [(cv, 3_000 * us + 40 * us * i, 3_000 * us + 100 * us + 40 * us * i) for i in range(4)]
    tr = tmp_path / "kt.csv"
    _trace(tr, rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "region_kernels.py"), str(tr), "--frames", "20"],
                         check=True, capture_output=True, text=True).stdout
    got = json.loads(out)
    k = got["timed_region"]["kernels"]
    assert k["k_composite_views<0>"]["launches"] == 4
    assert k["k_composite_views<0>"]["busy_us"] == pytest.approx(300.0)  # [100, 400) us
    assert k["k_composite_views<0>"]["busy_us_per_frame"] == pytest.approx(15.0)
    assert k["k_preprocess_fc_views<3, false>"]["busy_us"] == pytest.approx(100.0)
    assert got["timed_region"]["span_us"] == pytest.approx(400.0)
    assert got["instrumented_repeat"]["kernels"]["k_composite_views<0>"]["busy_us"] == pytest.approx(220.0)


def test_bench_roofline_tables(tmp_path, monkeypatch):
    """bench.py's per-kernel table and resource fractions from a committed
    profile (profiles/LATEST): bytes per stage, GB/s over the busy time, and
    the frame's VALU / LDS / HBM demand over its time."""
    import argparse

    import bench
    by = bench.stage_bytes(1000, 800, 2000, 10, 32, 16, 236, share=5, depth_passes=4)
    assert by["composite"] == 2000 * 52 + 10 * 8 + 32 * 16 * 12
    assert by["tile_sort"] == 2000 * 16
    assert by["depth_sort"] == 1000 * 12 + 800 * 12 + 3 * 800 * 24
    assert by["preprocess"] == pytest.approx((1000 * 16 + 800 * 224) / 5 + 1000 * 12 + 800 * 48)
    prof = tmp_path / "profiles" / "rX"
    prof.mkdir(parents=True)
    (tmp_path / "profiles" / "LATEST").write_text("rX\n")
    region = {"timed_region": {"span_us_per_frame": 150.0, "busy_us": 3000.0, "kernels": {
        "k_composite_views<0>": {"launches": 4, "busy_us": 1600.0, "busy_us_per_frame": 80.0},
        "k_rs_offsets_views": {"launches": 24, "busy_us": 300.0, "busy_us_per_frame": 15.0}}}}
    t = bench.per_kernel_table(region, 1000, 800, 2000, 10, 32, 16, 236, 5)
    row = t["kernels"]["k_composite_views<0>"]
    assert row["stage"] == "composite" and row["GBps"] == pytest.approx(by["composite"] / 80e-6 / 1e9, abs=0.06)
    assert "stage" not in t["kernels"]["k_rs_offsets_views"]
    # PMC summary: one compositing launch per group of 5 views
    with open(prof / "pmc_summary.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "dispatches", "mean", "value_per_dispatch"])
        w.writerow(["k_composite_views<0>", "SQ_INSTS_VALU", 4, 0, 5e7])
        w.writerow(["k_composite_views<0>", "SQ_INSTS_VALU_TRANS_F32", 4, 0, 5e6])
        w.writerow(["k_composite_views<0>", "SQ_LDS_IDX_ACTIVE", 4, 0, 1e8])
        w.writerow(["k_rs_scatter_views<8, true, 8>", "SQ_INSTS_VALU", 16, 0, 1e6])
        w.writerow(["k_preprocess_fc_views<3, true>", "SQ_INSTS_VALU", 60, 0, 9e9])  # frame alone: excluded
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "PMC_PROFILE", str(tmp_path / "profiles" / "LATEST"))
    args = argparse.Namespace(config="c2", n=None, width=None, height=None, box="none")
    fr = bench.frame_resources(args, 5, 0.15, 260e6, 1 / 0.15e-3)
    valu = (5e7 * 4 + 1e6 * 16) / 4 / 5
    trans = 5e6 * 4 / 4 / 5
    want = (bench.VALU_NS * (valu - trans) + bench.TRANS_NS * trans) * 1e-9 / bench.SIMDS / 0.15e-3
    assert fr["fractions"]["VALU issue"] == pytest.approx(want, rel=1e-3)
    assert fr["fractions"]["LDS"] == pytest.approx(1e8 * 4 / 4 / 5 / (256 * 2.4e9) / 0.15e-3, rel=1e-3)
    assert fr["fractions"]["HBM (B_frame)"] == pytest.approx(260e6 / 0.15e-3 / 8e12, rel=1e-3)
