"""Per-tile depth sort probe on the C2 frame alone (GPU box).

Stage times (gsr_context_set_profiling 1) of gsr_render frames for each
GSR_DEBUG_TDS setting given on the command line (timing-only knob of
tile_sort.hip: 1 skips the workgroup-class lists, 2 the wave-class lists, 4
sorts one digit pass), then the tile-length and per-list key-width census of
the frame (default form).
usage: python tools/tds_probe.py [--config c2|c3|c5] [--frames 30] DEBUG[:COARSE_BITS[:FORM]] ...
(FORM 0: the exact global depth sort, GSR_TILE_DEPTH_SORT=0)"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from gsviewer_amd import _lib  # noqa: E402
from gsviewer_amd.camera import Camera  # noqa: E402
from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--frames", type=int, default=30)
ap.add_argument("debug", nargs="*", default=["0"])
a = ap.parse_args()
n, seed, (h, w) = {"c2": (1_000_000, 1, (1080, 1920)), "c3": (6_000_000, 2, (1080, 1920)),
                   "c5": (1_000_000, 1, (2160, 3840))}[a.config]
g = garden_standin(n, seed=seed, sh_degree=3)
scene = HipScene.from_gaussian_data(g)
cam = camera_from(Camera(h, w))
out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
lib = _lib.load()
for arg in a.debug:  # DEBUG[:COARSE_BITS[:TILE_DEPTH_SORT]]
    parts = arg.split(":")
    dbg = parts[0]
    os.environ["GSR_DEBUG_TDS"] = dbg
    if len(parts) > 1:
        os.environ["GSR_TDS_COARSE_BITS"] = parts[1]
    else:
        os.environ.pop("GSR_TDS_COARSE_BITS", None)
    os.environ["GSR_TILE_DEPTH_SORT"] = parts[2] if len(parts) > 2 else "1"
    ctx = HipContext()
    st = RenderSettings(t_min=1e-4, out_layout=1)
    for _ in range(5):
        render_into(ctx, scene, cam, st, out)
    torch.cuda.synchronize()
    _lib.check(lib.gsr_context_set_profiling(ctx.handle, 1), "set_profiling")
    for _ in range(a.frames):
        render_into(ctx, scene, cam, st, out)
    torch.cuda.synchronize()
    ms = (ctypes.c_double * len(_lib.STAGES))()
    fr = ctypes.c_int64()
    _lib.check(lib.gsr_context_stage_times(ctx.handle, ms, ctypes.byref(fr)), "stage_times")
    print(f"{arg}: " + " ".join(f"{k} {1e3 * ms[i] / max(fr.value, 1):.1f}"
                                               for i, k in enumerate(_lib.STAGES)), flush=True)
    ctx.close()
os.environ["GSR_DEBUG_TDS"] = "0"
os.environ["GSR_TILE_DEPTH_SORT"] = "1"
os.environ.pop("GSR_TDS_COARSE_BITS", None)
ctx = HipContext()
render_into(ctx, scene, cam, RenderSettings(t_min=1e-4, out_layout=1), out)
torch.cuda.synchronize()
from helpers import grab_debug  # noqa: E402
stt = ctx.stats()
d = grab_debug(ctx, stt)
keys = torch.empty(n + 1, dtype=torch.int32, device="cuda")
got = lib.gsr_debug_copy(ctx.handle, _lib.GSR_DEBUG_SLOT_KEYS, ctypes.c_void_p(keys.data_ptr()), n * 4, None)
torch.cuda.synchronize()
slot_keys = keys.cpu().numpy().view(np.uint32)[:got // 4]
vis_slots = np.nonzero(slot_keys != 0xFFFFFFFF)[0]
r = d["ranges"].astype(np.int64)
lens = r[:, 1] - r[:, 0]
tl = vis_slots[d["tile_list"]]
bits = []
for t in np.nonzero(lens >= 2)[0]:
    k = slot_keys[tl[r[t, 0]:r[t, 1]]].astype(np.int64)
    bits.append((int(lens[t]), int(k.max() - k.min()).bit_length()))
bits = np.asarray(bits)
print("stats", stt)
print("tiles >= 2:", len(bits), "instances", int(lens.sum()), "max", int(lens.max()))
for lo, hi in ((2, 65), (65, 257), (257, 1025), (1025, 2049), (2049, 8193), (8193, 24577), (24577, 1 << 40)):
    m = (bits[:, 0] >= lo) & (bits[:, 0] < hi)
    if m.any():
        print(f"  len [{lo},{hi}): tiles {m.sum()} inst {bits[m, 0].sum()} key bits median {np.median(bits[m, 1]):.0f}"
              f" max {bits[m, 1].max()}")
