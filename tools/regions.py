"""Regions of a bench trace (tooling): the group launches (`*_views` kernels of
views in flight) split where the GPU idles > GAP us (the bench's synchronize
points), one line per region, and for region R a per-stream timeline: when each
group's preprocess, depth sort, finish chain and compositing ran.
usage: python tools/regions.py KERNEL_TRACE.csv [R] [GAP_US]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
want = int(sys.argv[2]) if len(sys.argv) > 2 else None
gap_us = float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r), r["Stream_Id"]) for r in rows)
ev = [e for e in ev if "_views" in e[2] and not e[2].endswith(", true>")]
regions, cur, end = [], [], None
for e in ev:
    if cur and e[0] - end > gap_us * 1e3:
        regions.append(cur)
        cur = []
    cur.append(e)
    end = e[1] if end is None or not cur[:-1] else max(end, e[1])
regions.append(cur)
for i, rg in enumerate(regions):
    t0, t1 = rg[0][0], max(e[1] for e in rg)
    nc = sum(1 for e in rg if e[2].startswith("k_composite_views"))
    print(f"region {i}: {len(rg)} launches, span {(t1 - t0) / 1e3:.1f} us, compositing launches {nc}")
if want is None:
    sys.exit(0)
rg = regions[want]
t0 = rg[0][0]
by_stream = defaultdict(list)
for e in rg:
    by_stream[e[3]].append(e)
for sid, es in sorted(by_stream.items()):
    print(f"stream {sid}:")
    phase, ps, pe = None, None, None
    def flush():
        if phase:
            print(f"   {phase:10s} {(ps - t0) / 1e3:8.1f} .. {(pe - t0) / 1e3:8.1f} us  ({(pe - ps) / 1e3:6.1f})")
    for s, e_, n, _ in es:
        ph = ("preprocess" if n.startswith(("k_preprocess", "k_cull")) else
              "composite" if n.startswith("k_composite") else
              "depth sort" if n.startswith(("k_rs_upsweep_views<8", "k_rs_scatter_views<8")) or
              (n.startswith("k_rs_offsets") and phase in ("preprocess", "depth sort")) else "finish")
        if ph != phase:
            flush()
            phase, ps = ph, s
        pe = e_
    flush()
