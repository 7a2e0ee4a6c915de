"""Frame time of the near-cluster scene (tests/test_gpu_large_splats.py) at
1080p, for A/B of the binning across library builds (GSR_LIB_PATH).
usage: python tools/large_splats_time.py [frames]"""
import os
import sys
import time

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
from test_gpu_large_splats import near_cluster_scene  # noqa: E402

from gsviewer_amd.camera import Camera  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
g = near_cluster_scene()
scene = HipScene.from_gaussian_data(g)
cam = Camera(1080, 1920)
ctx = HipContext()
out = torch.empty((3, cam.h, cam.w), dtype=torch.float32, device="cuda")
st = RenderSettings(out_layout=0)
render_into(ctx, scene, camera_from(cam), st, out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(frames):
    render_into(ctx, scene, camera_from(cam), st, out)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / frames
print(f"lib={os.environ.get('GSR_LIB_PATH', 'in-tree')} ms/frame={dt * 1e3:.3f} stats={ctx.stats()}", flush=True)
