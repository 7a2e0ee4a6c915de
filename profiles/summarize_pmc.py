"""Summarise rocprofv3 --pmc CSVs into per-kernel means per dispatch.

FETCH_SIZE / WRITE_SIZE are in KB; gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE reports half of the bytes of wide coalesced
streaming reads -> doubled here; WRITE_SIZE is exact for 16-B-per-lane
stores.  Other counters (SQ_*) are plain event counts ("value" column).
usage: python profiles/summarize_pmc.py OUT.csv pmc_dir1 [pmc_dir2 ...]
"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("gsr::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def main(out, dirs):
    with open(out, "w") as f:
        f.write("kernel,counter,dispatches,mean,value_per_dispatch\n")
        for d in dirs:
            rows = list(csv.DictReader(open(f"{d}/pmc_counter_collection.csv")))
            agg = collections.defaultdict(list)
            for r in rows:
                agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
            for (k, c), v in sorted(agg.items()):
                m = sum(v) / len(v)
                corr = m * 1024 * (2 if c == "FETCH_SIZE" else 1) if c in ("FETCH_SIZE", "WRITE_SIZE") else m
                f.write(f'"{k}",{c},{len(v)},{m:.1f},{corr:.0f}\n')


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
