"""Per-block timeline of the per-tile depth sort on the C2 frame alone (GPU box).

GSR_DEBUG_TDS=8 makes k_tile_depth_sort write, per block of view 0, its
start, the end of its long runs (part A), the end of finding its span's runs
and its end (100 MHz s_memrealtime), with the long runs it sorted, their
instances, its span's runs and the instances of those it sorted.
usage: python tools/tds_stamps.py [--config c2|c3|c5] [--coarse-bits B]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gsviewer_amd import _lib  # noqa: E402
from gsviewer_amd.camera import Camera  # noqa: E402
from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--coarse-bits", default=None)
a = ap.parse_args()
n, seed, (h, w) = {"c2": (1_000_000, 1, (1080, 1920)), "c3": (6_000_000, 2, (1080, 1920)),
                   "c5": (1_000_000, 1, (2160, 3840))}[a.config]
os.environ["GSR_DEBUG_TDS"] = "8"
if a.coarse_bits is not None:
    os.environ["GSR_TDS_COARSE_BITS"] = a.coarse_bits
g = garden_standin(n, seed=seed, sh_degree=3)
scene = HipScene.from_gaussian_data(g)
cam = camera_from(Camera(h, w))
out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
lib = _lib.load()
ctx = HipContext()
st = RenderSettings(t_min=1e-4, out_layout=1)
for _ in range(3):
    render_into(ctx, scene, cam, st, out)
torch.cuda.synchronize()
nd = ctx.stats()["n_instances"]
blocks = (nd + 8191) // 8192
buf = torch.empty(8 * (blocks + 1) * 2, dtype=torch.int32, device="cuda")
got = lib.gsr_debug_copy(ctx.handle, 5, ctypes.c_void_p(buf.data_ptr()), 8 * 8 * blocks, None)
torch.cuda.synchronize()
s = buf.cpu().numpy().view(np.uint64)[: got // 8].reshape(-1, 8)[:blocks].astype(np.int64)
t0 = s[:, 0].min()
us = lambda x: x / 100.0  # 100 MHz ticks -> us
start, a_end, f_end, end = (us(s[:, i] - t0) for i in range(4))
print(f"blocks {blocks}, instances {nd}, coarse bits {a.coarse_bits or 'default'}")
print(f"kernel span (first start .. last end) {end.max():.1f} us; block start spread {start.max():.1f} us")
for name, d in (("part A (long runs)", a_end - start), ("find runs", f_end - a_end), ("part B (short runs)", end - f_end),
                ("whole block", end - start)):
    print(f"  {name:22s} median {np.median(d):6.1f}  p90 {np.percentile(d, 90):6.1f}  max {d.max():6.1f} us")
print(f"  long runs per block: mean {s[:, 4].mean():.2f} max {s[:, 4].max()}, instances max {s[:, 5].max()}")
print(f"  span runs per block: mean {s[:, 6].mean():.1f} max {s[:, 6].max()}; short-run instances total {s[:, 7].sum()}")
worst = np.argsort(-(end - start))[:8]
for b in worst:
    print(f"  block {b}: start {start[b]:.1f} A {a_end[b] - start[b]:.1f} find {f_end[b] - a_end[b]:.1f} "
          f"B {end[b] - f_end[b]:.1f} | long runs {s[b, 4]} ({s[b, 5]} inst) span runs {s[b, 6]} short inst {s[b, 7]}")
