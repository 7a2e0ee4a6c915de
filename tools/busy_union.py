"""Busy time of one kernel over the regions of a rocprofv3 kernel trace: the
union of its launches' [start, end) intervals, so launches that overlap (the
bench's four group streams composite concurrently at the end of a region)
are counted once.  Launches closer than --gap-ms belong to one region.

bench.py reads the output (profiles/LATEST/composite_busy.json) as the
profiler's cross-check of its live figure: the same union over the in-kernel
spans of a repeat of the timed region (roofline.us_per_view).
usage: python tools/busy_union.py KERNEL_TRACE.csv [--kernel 'k_composite_views<0>'] [--views 20]"""
import argparse
import csv
import json
import re


def union_ns(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_composite_views<0>")
    ap.add_argument("--views", type=int, default=20, help="views composited per region (the bench's --steps)")
    ap.add_argument("--launches", type=int, default=4, help="launches per region (groups)")
    ap.add_argument("--gap-ms", type=float, default=1.0)
    a = ap.parse_args()
    clean = lambda n: re.sub(r"\(.*", "", n.replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(a.trace))
                if clean(r["Kernel_Name"]) == a.kernel)
    regions, cur = [], []
    for s, e in iv:
        if cur and s - max(x[1] for x in cur) > a.gap_ms * 1e6:
            regions.append(cur)
            cur = []
        cur.append((s, e))
    if cur:
        regions.append(cur)
    rows = [{"launches": len(r), "busy_us": union_ns(r) / 1e3, "sum_us": sum(e - s for s, e in r) / 1e3,
             "first_to_last_us": (max(e for _, e in r) - min(s for s, _ in r)) / 1e3} for r in regions]
    full = [r for r in rows if r["launches"] == a.launches]
    busy = sorted(r["busy_us"] for r in full)
    med = busy[len(busy) // 2] if busy else None
    out = {"kernel": a.kernel, "source": a.trace, "regions": rows,
           "regions_of_the_bench_shape": len(full),
           "busy_us_per_region_median": med,
           "us_per_view": med / a.views if med is not None else None,
           "views_per_region": a.views,
           "method": "union of the launches' [start, end) per region (launches within --gap-ms of the region's "
                     "last end), median over the regions with --launches launches"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
