"""Busy fraction and concurrency of the views-in-flight region of a rocprofv3
kernel trace (tooling): python tools/timeline.py prof_kernel_trace.csv [groups] [views_per_group]"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))


def short(n):
    n = n.split("(anonymous namespace)::", 1)[-1]
    return n.split("(")[0]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
# group launches (the <DEG, true> preprocess is a frame alone's)
views = [e for e in ev if "_views" in e[2] and not e[2].endswith(", true>")]
# the timed region: the last `groups` groups of views (default 10 = 50 frames of 5-view groups)
groups = int(sys.argv[2]) if len(sys.argv) > 2 else 10
vpg = int(sys.argv[3]) if len(sys.argv) > 3 else 5
culls = [e for e in views if e[2].startswith(("k_cull_views", "k_preprocess_fc_views"))]
# a group ends with its merge launch, or with its compositing launch (tail merge)
ends = [e for e in views if e[2].startswith(("k_merge_views", "k_composite_views"))]
t0, t1 = culls[-groups][0], ends[-1][1]
seg = [e for e in ev if e[0] >= t0 and e[1] <= t1]
busy, cs, ce = 0, None, None
for s, e, n in seg:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
span = t1 - t0
tot = sum(e - s for s, e, n in seg)
nc = sum(1 for e in seg if e[2].startswith("k_composite_views"))
print(f"span {span/1e3:.1f} us, busy {busy/span:.3f}, sum(kernel)/span {tot/span:.2f}, frames {vpg*nc}, "
      f"us/frame {span/1e3/(vpg*nc):.1f}")
d = defaultdict(int)
for s, e, n in seg:
    d[n] += e - s
for n, v in sorted(d.items(), key=lambda x: -x[1])[:16]:
    print(f"  {n:28s} share {v/tot:.3f}  {v/1e3/(vpg*nc):7.1f} us/frame of kernel time")
ts = np.linspace(t0, t1, 4000)
st = np.array([s for s, e, n in seg])
en = np.array([e for s, e, n in seg])
conc = np.array([((st <= t) & (en > t)).sum() for t in ts])
print("concurrency mean", conc.mean().round(2), "hist", np.bincount(conc).tolist())
comp = np.array([n.startswith("k_composite") for s, e, n in seg])
on = np.array([((st[comp] <= t) & (en[comp] > t)).any() for t in ts])
print("fraction of time a compositor runs", on.mean().round(3))
