"""Debug aid: where does a t_min > 0 frame differ from the oracle?  (tooling)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from helpers import gpu_frame, uniforms_for  # noqa: E402

from gsviewer_amd.camera import Camera  # noqa: E402
from gsviewer_amd.gaussian_data import random_scene  # noqa: E402
from gsviewer_amd.rasterizer import RenderSettings  # noqa: E402
from oracle import gl_oracle as O  # noqa: E402

chunk = int(os.environ.get("GSR_CHUNK", "192"))
g = random_scene(3000, sh_degree=3, seed=11, scale_range=(0.02, 0.1))
cam = Camera(96, 128)
st = RenderSettings(t_min=1e-4)
res = gpu_frame(g, cam, st, with_debug=True)
U = uniforms_for(cam, st)
vs = O.vertex_stage(g.flat().astype(np.float32), g.sh_dim, U)
ref = O.composite(vs, U)
d = np.abs(res["image"] - ref).max(-1)
ranges = res["ranges"]
lens = (ranges[:, 1] - ranges[:, 0]).astype(np.int64)
tx_n = (cam.w + 15) // 16
bad = np.argwhere(d > 2e-4)
print("lib", os.environ.get("GSR_LIB_PATH"), "bad px", len(bad), "max", d.max())
tiles = {}
for r, c in bad:
    t = (r // 16) * tx_n + c // 16
    tiles.setdefault(t, []).append(float(d[r, c]))
for t, v in sorted(tiles.items()):
    print(f"tile {t} len {lens[t]} chunks {max(1, -(-lens[t] // chunk))} bad {len(v)} max {max(v):.4f}")
print("multi-chunk tiles", int((lens > chunk).sum()), "of", len(lens))
