"""Per-kernel busy time of bench.py's timed region, from a rocprofv3 kernel
trace of `bench.py --steps 20 --warmup 5` (tools/gpu_round.sh).

The trace is cut into segments at idle gaps (no kernel running for more than
--gap-us); the timed region is the first segment after the warm-up that runs
exactly --groups compositing launches of a group (k_composite_views) and no
frame-alone compositor (the repeat of the region that bench.py instruments
comes later and looks the same: it is reported beside it).  For every kernel:
launches, the union of its launches' [start, end) (overlapping launches of
the four group streams counted once), the sum of their durations, and both
per frame (the region's frames = --frames).  bench.py reads the output
(profiles/LATEST/region_kernels.json) for its per-kernel roofline table.
usage: python tools/region_kernels.py KERNEL_TRACE.csv[.gz] [--frames 20] [--groups 4]"""
import argparse
import csv
import gzip
import json
import re


def clean(n):
    return re.sub(r"\(.*", "", n.replace("gsr::(anonymous namespace)::", "").replace("void ", ""))


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


def segments(rows, gap_ns):
    rows = sorted(rows, key=lambda r: r[1])
    out, cur, end = [], [], None
    for r in rows:
        if cur and r[1] - end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(r)
        end = r[2] if end is None or not cur[:-1] else max(end, r[2])
    if cur:
        out.append(cur)
    return out


def summarise(seg, frames):
    names = sorted({n for n, _, _ in seg})
    per = {}
    for k in names:
        iv = [(s, e) for n, s, e in seg if n == k]
        per[k] = {"launches": len(iv), "busy_us": union_ns(iv) / 1e3, "sum_us": sum(e - s for s, e in iv) / 1e3}
        per[k]["busy_us_per_frame"] = per[k]["busy_us"] / frames
    span = (max(e for _, _, e in seg) - min(s for _, s, _ in seg)) / 1e3
    return {"span_us": span, "span_us_per_frame": span / frames,
            "busy_us": union_ns([(s, e) for _, s, e in seg]) / 1e3, "kernels": per}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--groups", type=int, default=4)
    ap.add_argument("--gap-us", type=float, default=100.0)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    with op(a.trace, "rt") as fh:
        rows = [(clean(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(fh)]
    segs = segments(rows, a.gap_us * 1e3)
    found = []
    for sg in segs:
        names = [n for n, _, _ in sg]
        views = sum(1 for n in names if n.startswith("k_composite_views"))
        alone = sum(1 for n in names if n.startswith("k_composite<"))
        if views == a.groups and alone == 0:
            found.append(summarise(sg, a.frames))
    if not found:
        raise SystemExit("no segment with the timed region's shape")
    out = {"source": a.trace, "frames": a.frames, "groups": a.groups, "timed_region": found[0],
           "instrumented_repeat": found[1] if len(found) > 1 else None,
           "method": "segments of the trace split at idle gaps > gap_us; the first with `groups` k_composite_views "
                     "launches and no frame-alone compositor is the timed region; per kernel the union of its "
                     "launches' [start, end) and the sum of their durations", "gap_us": a.gap_us}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
