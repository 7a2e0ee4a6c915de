"""Per-queue kernel sequence of the last views-in-flight region of a rocprofv3
kernel trace (tooling): python tools/gantt.py prof_kernel_trace.csv GROUPS [hip_api_trace.csv]
Prints start/end (us from the region's first k_cull_views), queue, kernel; with
the HIP API trace (rocprofv3 --hip-runtime-trace) also when the host enqueued it."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
groups = int(sys.argv[2])
enq = {}
if len(sys.argv) > 3:
    for r in csv.DictReader(open(sys.argv[3])):
        if "Launch" in r.get("Function", ""):
            enq[r["Correlation_Id"]] = int(r["Start_Timestamp"])


def short(n):
    n = n.split("(anonymous namespace)::", 1)[-1]
    return n.split("(")[0]


qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
             r.get(qkey, "?") if qkey else "?", enq.get(r["Correlation_Id"])) for r in rows)
culls = [e for e in ev if e[2].startswith(("k_cull_views", "k_preprocess_fc_views"))]
merges = [e for e in ev if e[2].startswith("k_merge_views")]
t0 = culls[-groups][0]
t1 = max(e[1] for e in merges[-groups:])
print(f"region {(t1 - t0) / 1e3:.1f} us; columns: start end dur queue [enqueued] kernel")
for s, e, n, q, h in ev:
    if s >= t0 and e <= t1:
        hs = "" if h is None else f"{(h - t0) / 1e3:8.1f} "
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {q:>4} {hs}{n}")
