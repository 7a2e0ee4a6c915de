"""Concurrency of a multi-stream run from a rocprofv3 kernel trace: over a
window of dispatches (in start order), the fraction of time each kernel
family is running and how many dispatches overlap.
usage: python tools/overlap.py KERNEL_TRACE.csv [FIRST LAST]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
name = lambda r: re.sub(r"[<(].*", "", r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r)) for r in rows if "repack" not in r["Kernel_Name"]]
ev.sort()
a, b = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (int(len(ev) * 0.4), len(ev))
ev = ev[a:b]
t_lo = ev[0][0]
t_hi = max(e for _, e, _ in ev)
span = t_hi - t_lo
fam_time = collections.defaultdict(int)
points = []
for s, e, n in ev:
    points += [(s, 1, n), (e, -1, n)]
points.sort()
active = collections.Counter()
depth_time = collections.Counter()
last = t_lo
for t, d, n in points:
    dt = t - last
    if dt > 0:
        depth_time[sum(active.values())] += dt
        for f in active:
            if active[f] > 0:
                fam_time[f] += dt
    active[n] += d
    last = t
print(f"steady-state span {span / 1e3:.1f} us, {len(ev)} dispatches")
for f, t in sorted(fam_time.items(), key=lambda x: -x[1]):
    print(f"  {f:18s} running {100.0 * t / span:5.1f}% of the time")
print("  concurrent dispatches: " + ", ".join(f"{k}: {100.0 * v / span:.1f}%" for k, v in sorted(depth_time.items())))
