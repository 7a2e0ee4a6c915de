"""Compositor work analysis (not a test; lives under tests/ because it uses the
CPU oracle): on the bench workload (garden stand-in, 1M, 1080p, default
camera) counts the 16x4 slice evaluations the compositor performs, how many
of them hold a kept fragment, and the kept pixels per 64-lane evaluation.
    python tests/analysis_slice_occupancy.py [N]"""
import os
import sys
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(_HERE))
sys.path.insert(0, _HERE)
from gsviewer_amd.gaussian_data import garden_standin
from gsviewer_amd.camera import Camera
from oracle import gl_oracle as O
import helpers as Hh

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
g = garden_standin(n, seed=1, sh_degree=3)
cam = Camera(1080, 1920)
U = Hh.uniforms_for(cam)
t = time.time()
vs = O.vertex_stage(g.flat(), g.sh_dim, U)
print("vertex", time.time() - t)
W, H = 1920, 1080
vis = vs["visible"]
qa, qb, qc = Hh.expected_quadratic(vs)
op = vs["opacity"].astype(np.float64)
with np.errstate(all="ignore"):
    thr = -np.log2(255.0 * op)
rec = dict(qa=qa, qb=qb, qc=qc, center=vs["center"], mid=(thr / 2).astype(np.float32))
rects = O.splat_rects(vs, U)
x0, x1, r0, r1 = Hh.alpha_box_rects(rec, rects, H)
ok = vis & (x0 <= x1) & (r0 <= r1)
idx = np.nonzero(ok)[0]
x0, x1, r0, r1 = x0[idx], x1[idx], r0[idx], r1[idx]
qa, qb, qc = qa[idx].astype(np.float64), qb[idx].astype(np.float64), qc[idx].astype(np.float64)
cx, cy = vs["center"][idx, 0].astype(np.float64), vs["center"][idx, 1].astype(np.float64)
thr = thr[idx]
print("splats", len(idx), "mean rect w", (x1 - x0 + 1).mean(), "h", (r1 - r0 + 1).mean())
hgt = r1 - r0 + 1
sp = np.repeat(np.arange(len(idx)), hgt)
row = r0[sp] + (np.arange(hgt.sum()) - np.repeat(np.cumsum(hgt) - hgt, hgt))
dy = (H - 1 - row + 0.5) - cy[sp]
A = qa[sp]; B = qb[sp] * dy; C = qc[sp] * dy * dy - thr[sp]
disc = B * B - 4 * A * C
has = disc >= 0
sq = np.sqrt(np.maximum(disc, 0))
lo = (-B + sq) / (2 * A); hi = (-B - sq) / (2 * A)
kc0 = np.ceil(cx[sp] + lo - 0.5 - 1e-3); kc1 = np.floor(cx[sp] + hi - 0.5 + 1e-3)
kc0 = np.maximum(kc0, x0[sp]); kc1 = np.minimum(kc1, x1[sp])
rowkept = has & (kc0 <= kc1)
print("rows", len(sp), "rows with kept", rowkept.mean())
ntx = x1 // 16 - x0 // 16 + 1
inst = (ntx * (r1 // 16 - r0 // 16 + 1)).sum()
# slice evals: per (splat, tile column) the bands [r0//4, r1//4] (band = 4 image rows; tiles are 16 rows)
evald = (ntx * (r1 // 4 - r0 // 4 + 1)).sum()
print("instances", inst, "slice evals", evald, "per inst", evald / inst)
band = row // 4
key_rows = np.nonzero(rowkept)[0]
s = sp[key_rows]; b = band[key_rows]; c0 = kc0[key_rows].astype(np.int64); c1 = kc1[key_rows].astype(np.int64)
t0 = c0 // 16; t1 = c1 // 16
nt = t1 - t0 + 1
rs = np.repeat(np.arange(len(s)), nt)
tt = t0[rs] + (np.arange(nt.sum()) - np.repeat(np.cumsum(nt) - nt, nt))
keys = (s[rs].astype(np.int64) * 300 + b[rs]) * 130 + tt
useful = len(np.unique(keys))
print("useful slices", useful, "frac", useful / evald)
keys2 = (s[rs].astype(np.int64) * 300 + b[rs] // 4) * 130 + tt
print("useful instances", len(np.unique(keys2)), "frac", len(np.unique(keys2)) / inst)
kp = (kc1 - kc0 + 1)[rowkept].sum()
print("kept px", kp, "per slice eval", kp / evald, "lane util", kp / evald / 64)
