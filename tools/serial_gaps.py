"""GPU idle gaps of single-view frames (tooling): per frame (k_cull or the fused preprocess ... k_merge,
non-batched kernels; k_preprocess_fc_views with k = 1 for the fused cull) the span, the kernel busy time and the idle gaps between
consecutive kernels, by the kernel that follows the gap.
usage: python tools/serial_gaps.py prof_kernel_trace.csv [frames]"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20


def short(n):
    n = n.split("(anonymous namespace)::", 1)[-1]
    return n.split("(")[0]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
# a frame alone with the fused cull starts with k_preprocess_fc_views<DEG, true>
ev = [(e[0], e[1], "k_preprocess_fc") if e[2].startswith("k_preprocess_fc_views<") and e[2].endswith(", true>")
      else e for e in ev]
ev = [e for e in ev if "_views" not in e[2] and "rocclr" not in e[2] and "repack" not in e[2]]
starts = [i for i, e in enumerate(ev) if e[2] in ("k_cull", "k_preprocess_fc")]
frames = []
for a, b in zip(starts, starts[1:] + [len(ev)]):
    fr = ev[a:b]
    if any(e[2] == "k_merge" for e in fr):
        frames.append(fr)
frames = frames[-last:]
spans, busy, gaps = [], [], defaultdict(list)
period = []
for i, fr in enumerate(frames):
    spans.append((fr[-1][1] - fr[0][0]) / 1e3)
    busy.append(sum(e[1] - e[0] for e in fr) / 1e3)
    for p, q in zip(fr, fr[1:]):
        gaps[q[2]].append(max(0, q[0] - p[1]) / 1e3)
    if i:
        period.append((fr[0][0] - frames[i - 1][0][0]) / 1e3)
print(f"frames {len(frames)}: period {np.mean(period):.1f} us, span {np.mean(spans):.1f} us, "
      f"kernel busy {np.mean(busy):.1f} us, idle inside frame {np.mean(spans) - np.mean(busy):.1f} us, "
      f"between frames {np.mean(period) - np.mean(spans):.1f} us")
for n, v in sorted(gaps.items(), key=lambda x: -np.sum(x[1])):
    print(f"  gap before {n:26s} mean {np.mean(v):6.2f} us  max {np.max(v):6.2f}")
