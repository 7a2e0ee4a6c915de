"""One frame's kernel timeline from a rocprofv3 kernel_trace.csv: duration of
each launch and the gap before it (launch/boundary overhead).
usage: python tools/ktrace.py KERNEL_TRACE.csv [FRAME_INDEX]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
# frames start at k_cull, or (fused cull) at a k_preprocess_fc_views launch
starts = [i for i, r in enumerate(rows) if name(r).startswith("k_cull") or name(r).startswith("k_preprocess_fc")]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
a, b = starts[k], starts[k + 1] if k + 1 < len(starts) else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
busy = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:8.2f}us  +gap {gap:6.2f}  dur {(e - s) / 1e3:7.2f}  grid {r['Grid_Size_X']:>9s}  {name(r)}")
    prev_end = e
print(f"frame span {(prev_end - t0) / 1e3:.2f}us, busy {busy / 1e3:.2f}us")
