"""Per-frame kernel time table from a rocprofv3 kernel_stats.csv.
usage: python tools/kstats.py KERNEL_STATS.csv FRAMES"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = float(sys.argv[2])
tot = 0.0
for r in rows:
    n = re.sub(r"\(.*", "", r["Name"].replace("gsr::(anonymous namespace)::", "").replace("void ", ""))
    per = float(r["TotalDurationNs"]) / frames / 1000
    if "repack" in n:
        continue
    tot += per
    print(f"{n:32s} calls={r['Calls']:6s} avg={float(r['AverageNs']) / 1000:8.2f}us per-frame={per:8.2f}us")
print(f"{'total per frame':32s} {tot:.2f}us")
