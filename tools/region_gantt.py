"""Per-group timeline of the last region of views in flight in a rocprofv3
kernel trace (tooling): for each of the last G group frames, when its
preprocess, depth sort, finish chain (binning .. chunks) and compositing ran,
relative to the region's first launch.  usage:
python tools/region_gantt.py KERNEL_TRACE.csv [G]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r), r.get("Stream_Id", r.get("Queue_Id")))
            for r in rows)
views = [e for e in ev if "_views" in e[2] and not e[2].endswith(", true>")]
pre = [i for i, e in enumerate(views) if e[2].startswith("k_preprocess_fc_views")]
first = pre[-G]
reg = views[first:]
t0 = reg[0][0]
groups = []  # a group frame runs from its preprocess to its compositing
cur = defaultdict(list)
by_stream = defaultdict(list)
for e in reg:
    by_stream[e[3]].append(e)
print(f"region: {len(reg)} launches, span {(max(e[1] for e in reg) - t0) / 1e3:.1f} us")
for s, es in by_stream.items():
    stage = lambda pred: [e for e in es if pred(e[2])]
    p = stage(lambda n: n.startswith("k_preprocess"))
    c = stage(lambda n: n.startswith("k_composite"))
    rs = stage(lambda n: n.startswith("k_rs_") or n.startswith("k_bin") or n.startswith("k_tile") or n.startswith("k_chunk"))
    line = [f"stream {s}:"]
    for lab, xs in (("pre", p), ("sort+bin+chunks", rs), ("comp", c)):
        if xs:
            line.append(f"{lab} {(xs[0][0] - t0) / 1e3:7.1f}-{(max(x[1] for x in xs) - t0) / 1e3:7.1f}")
    print("  ".join(line))
busy = sorted((e[0], e[1]) for e in reg)
tot, cs, ce = 0, None, None
for s, e in busy:
    if cs is None or s > ce:
        if cs is not None:
            tot += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
tot += ce - cs
print(f"GPU busy (any kernel) {tot / 1e3:.1f} us of {(max(e[1] for e in reg) - t0) / 1e3:.1f}")
for lab, pred in (("preprocess", lambda n: n.startswith("k_preprocess")), ("composite", lambda n: n.startswith("k_composite"))):
    xs = [e for e in reg if pred(e[2])]
    print(lab, " ".join(f"{(e[0] - t0) / 1e3:.0f}-{(e[1] - t0) / 1e3:.0f}" for e in xs))
