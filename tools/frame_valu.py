"""VALU budget of the frame in flight from a PMC summary (tooling):
python tools/frame_valu.py profiles/<round>/pmc_summary.csv [views_per_group] [frame_ms]

Sums SQ_INSTS_VALU (which counts the SQ_INSTS_VALU_TRANS_F32 too) of the view-batched kernels
(`*_views`: the bench's timed region), weighted by their dispatch counts per
group (the depth sort runs 4 radix steps per group, the tile sort 2), per
view-frame.  Issue time: 1.6 ns per VALU and 3.5 ns per transcendental
instruction per SIMD (the compositor calibration bench.py reports as
roofline.valu_issue), over 1024 SIMDs."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
vpg = int(sys.argv[2]) if len(sys.argv) > 2 else 5
frame_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
valu, trans, disp = defaultdict(float), defaultdict(float), {}
for r in csv.DictReader(open(path)):
    k = r["kernel"]
    if "_views" not in k or k.endswith(", true>"):  # (<DEG, true>: the fused preprocess of a frame alone)
        continue
    if r["counter"] == "SQ_INSTS_VALU":
        valu[k] = float(r["value_per_dispatch"])
        disp[k] = int(r["dispatches"])
    elif r["counter"] == "SQ_INSTS_VALU_TRANS_F32":
        trans[k] = float(r["value_per_dispatch"])
groups = disp.get("k_composite_views<0>", 1)
rows = []
for k in valu:
    w = disp[k] / groups / vpg  # dispatches per group, per view
    rows.append((k, valu[k] * w, trans[k] * w))
rows.sort(key=lambda r: -r[1])
tv = sum(r[1] for r in rows)
tt = sum(r[2] for r in rows)
print(f"{'kernel':40s} {'VALU M':>8s} {'trans M':>8s} {'share':>6s}")
for k, v, t in rows:
    print(f"{k[:40]:40s} {v / 1e6:8.2f} {t / 1e6:8.2f} {v / tv:6.1%}")
issue_us = ((tv - tt) * 1.6 + tt * 3.5) / 1024 / 1e3  # (SQ_INSTS_VALU counts the transcendentals too)
print(f"per view-frame: VALU {tv / 1e6:.1f} M (of them trans {tt / 1e6:.2f} M) -> issue {issue_us:.1f} us "
      f"over 1024 SIMDs")
if frame_ms:
    print(f"frame {frame_ms * 1e3:.1f} us -> VALU pipes busy {issue_us / (frame_ms * 1e3):.0%} on average")
