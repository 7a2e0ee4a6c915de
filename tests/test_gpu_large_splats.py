"""Large splats close to the camera: the binning's balanced enumeration.

A block of 1024 depth-adjacent splats that each cover hundreds of tiles (what
a camera close to a scene's large splats produces: they sit together at the
front of the depth order) used to be enumerated by each thread walking its
own splats' rectangles, window after window: nearly single-lane work
(ADVICE r3).  Blocks with a splat over kSerialTiles tiles now enumerate their
instances balanced (composite.hip instance_at).  Checked here:

* parity with the C oracle on a frame where every block of the near cluster
  takes the balanced path (stated tolerances of tests/helpers.py);
* the fused binning (balanced) and the separate binning + full tile sort give
  bit-identical frames and tile lists at 1080p;
* that 1080p frame (1.9 M tile instances, ~900 tiles per near splat) renders
  in bounded time.
"""
import time

import numpy as np
import pytest
import torch

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import GaussianData, random_scene
from helpers import TOL_EXACT, TOL_MAX, compare_images, gpu_frame, uniforms_for
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu


def near_cluster_scene(n_big=2048, n_small=20000, seed=3):
    """n_big wide, fairly opaque splats in a slab 1.3-1.8 units in front of the
    default camera (z in [3.2, 3.7], camera at z = 5), over a field of small
    ones."""
    rng = np.random.default_rng(seed)
    small = random_scene(n_small, sh_degree=1, seed=seed)
    xyz = np.stack([rng.uniform(-1.2, 1.2, n_big), rng.uniform(-0.7, 0.7, n_big), rng.uniform(3.2, 3.7, n_big)],
                   1).astype(np.float32)
    rot = rng.normal(0, 1, (n_big, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    scale = np.exp(rng.uniform(np.log(0.1), np.log(0.35), (n_big, 3))).astype(np.float32)
    opacity = rng.uniform(0.3, 0.9, (n_big, 1)).astype(np.float32)
    sh = rng.normal(0, 0.5, (n_big, 12)).astype(np.float32)
    return GaussianData(np.concatenate([small.xyz, xyz]), np.concatenate([small.rot, rot]),
                        np.concatenate([small.scale, scale]), np.concatenate([small.opacity, opacity]),
                        np.concatenate([small.sh, sh]))


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def test_near_cluster_parity(gpu):
    g = near_cluster_scene()
    cam = Camera(270, 480)
    st = _settings(t_min=0.0)
    res = gpu_frame(g, cam, st)
    # the near cluster covers many tiles per splat: the balanced path runs
    assert res["stats"]["n_instances"] > 100_000
    ref = C.render(g.flat(), g.sh_dim, uniforms_for(cam, st), threads=16)
    compare_images(res["image"], ref, tol=TOL_EXACT, tol_max=TOL_MAX)


def test_near_cluster_fused_equals_unfused_binning(gpu, monkeypatch):
    from gsviewer_amd.rasterizer import HipContext, HipScene, camera_from, render_into
    g = near_cluster_scene()
    scene = HipScene.from_gaussian_data(g)
    cam = Camera(1080, 1920)
    imgs, times = [], []
    for fused in ("1", "0"):
        monkeypatch.setenv("GSR_BIN_FUSED", fused)
        ctx = HipContext()
        out = torch.empty((cam.h, cam.w, 3), dtype=torch.float32, device="cuda")
        st = _settings(t_min=0.0, out_layout=1)
        render_into(ctx, scene, camera_from(cam), st, out)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            render_into(ctx, scene, camera_from(cam), st, out)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) / 3)
        imgs.append(out.cpu().numpy())
        stats = ctx.stats()
        ctx.close()
    scene.close()
    assert stats["n_instances"] > 1_500_000, stats
    np.testing.assert_array_equal(imgs[0], imgs[1])
    # ~1.9 M instances: milliseconds, not the near single-lane enumeration
    assert times[0] < 0.05, times
