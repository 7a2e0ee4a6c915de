"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin), one line per kernel."""
import re
import subprocess
import sys

rows, cur = [], None
keys = {"VGPRs": "vgpr", "SGPRs": "sgpr", "LDS Size [bytes/block]": "lds", "Occupancy [waves/SIMD]": "occ",
        "ScratchSize [bytes/lane]": "scratch"}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name.replace("gsr::(anonymous namespace)::", ""))
        cur = {"name": name}
        rows.append(cur)
        continue
    for k, short in keys.items():
        m = re.search(re.escape(k) + r": (\d+)", line)
        if m and cur is not None:
            cur[short] = m.group(1)
for r in rows:
    print(f"{r['name']:56s} " + " ".join(f"{s} {r.get(s, '?'):>5}" for s in keys.values()))
