"""Median per-kernel duration and gap of single-view frames (gsr_render) in a
rocprofv3 kernel_trace.csv; a frame runs from its cull (k_cull, or the fused
preprocess k_preprocess_fc_views<DEG, true> of a frame alone) to its k_merge.
usage: python tools/frame_kernels.py KERNEL_TRACE.csv"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r)) for r in rows)
frames, cur = [], None
for i, e in enumerate(ev):
    if e[2] == "k_cull" or (e[2].startswith("k_preprocess_fc_views<") and e[2].endswith(", true>")):
        cur = [e]
        continue
    if cur is None:
        continue
    if "_views" in e[2] and not e[2].endswith(", true>"):
        cur = None
        continue
    cur.append(e)
    if e[2] == "k_merge":
        frames.append(cur)
        cur = None
dur, gap = defaultdict(list), defaultdict(list)
spans = []
for fr in frames:
    spans.append((fr[-1][1] - fr[0][0]) / 1e3)
    seen = defaultdict(int)
    prev = None
    for e in fr:
        key = f"{e[2]}#{seen[e[2]]}"
        seen[e[2]] += 1
        dur[key].append((e[1] - e[0]) / 1e3)
        gap[key].append(((e[0] - prev) / 1e3) if prev is not None else 0.0)
        prev = e[1]
order = list(dict.fromkeys(f"{e[2]}#{k}" for fr in frames[:1] for k, e in
                           [(sum(1 for x in fr[:j] if x[2] == e[2]), e) for j, e in enumerate(fr)]))
print(f"{len(frames)} single-view frames: span median {np.median(spans):.1f} us (min {np.min(spans):.1f})")
tot_d = tot_g = 0.0
for k in order:
    d, g = np.median(dur[k]), np.median(gap[k])
    tot_d += d
    tot_g += g
    print(f"  {k:34s} dur {d:7.2f}  gap {g:6.2f}")
print(f"  sum of medians: kernels {tot_d:.1f} us, gaps {tot_g:.1f} us")
