"""The coarse depth order of a frame alone (api.hip kDepthCoarseAlone, GSR_DEPTH_COARSE).

A frame's depth sort orders only the top bits of its key range (2 radix
passes) and keeps equal coarse keys in slot order; k_tile_ranges then puts
every run of one tile's instances with equal coarse keys into the exact
(key, slot) order (composite.hip fix_run; runs longer than 16 in
long_runs.h k_long_runs, tests/test_gpu_long_runs.py).  What the compositor reads -- the
tile lists, their ranges, the records -- and so the image must be exactly the
exact sort's:

* against the oracle (the tile lists of the GL draw order restricted to each
  tile, tests/test_gpu_scale.check_frame_order) with the default 16 coarse
  bits and with 12 and 8 (256 coarse keys: runs with descents in most
  tiles), alone and (exact) in a group;
* bit for bit against the exact sort (GSR_DEPTH_COARSE=0) at C2 (1M
  Gaussians, 1080p) and on a tilted plane seen edge-on (deep tiles, long
  runs).
"""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import GaussianData, garden_standin, random_scene
from helpers import batched_frames, gpu_frame, uniforms_for
from oracle import gl_oracle as O
from test_gpu_scale import _plane_scene, check_frame_order

pytestmark = pytest.mark.gpu


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def _tilted_plane(n, seed):
    """Splats on a plane almost parallel to the view ray: a narrow band of the
    image holds them all, and their depths differ in the low key bits."""
    rng = np.random.default_rng(seed)
    xyz = np.empty((n, 3), np.float32)
    xyz[:, 0] = rng.uniform(-0.3, 0.3, n)
    xyz[:, 2] = rng.uniform(-2.0, 2.0, n)
    xyz[:, 1] = 0.01 * xyz[:, 2]
    rot = np.tile(np.array([1, 0, 0, 0], np.float32), (n, 1))
    scale = np.full((n, 3), 0.004, np.float32)
    opacity = np.full((n, 1), 0.3, np.float32)
    sh = rng.normal(0, 0.5, (n, 3)).astype(np.float32)
    return GaussianData(xyz, rot, scale, opacity, sh)


@pytest.mark.parametrize("coarse", [None, "12", "8"])
def test_coarse_tile_lists_match_oracle(gpu, monkeypatch, coarse):
    from gsviewer_amd.rasterizer import HipScene
    if coarse is None:
        monkeypatch.delenv("GSR_DEPTH_COARSE", raising=False)
    else:
        monkeypatch.setenv("GSR_DEPTH_COARSE", coarse)
    g = random_scene(300_000, sh_degree=0, seed=3, scale_range=(0.003, 0.03))
    cam = Camera(270, 480).yaw(10)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    check_frame_order(res, vs, U)
    scene = HipScene.from_gaussian_data(g)
    got = batched_frames(scene, [cam, Camera(270, 480).yaw(100)], _settings(t_min=0.0), group=2,
                         debug_views=(0,))
    scene.close()
    check_frame_order(got[0], vs, U)


@pytest.mark.parametrize("zvals", [[0.0, 1e-6], [0.0, 0.25, -0.75]])
def test_coarse_planes_match_oracle(gpu, monkeypatch, zvals):
    monkeypatch.setenv("GSR_DEPTH_COARSE", "8")
    g = _plane_scene(50_000, zvals, seed=len(zvals))
    cam = Camera(240, 320)
    U = uniforms_for(cam)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    check_frame_order(res, O.vertex_stage(g.flat(), g.sh_dim, U), U)


def test_coarse_long_runs_match_oracle(gpu, monkeypatch):
    monkeypatch.setenv("GSR_DEPTH_COARSE", "8")
    g = _tilted_plane(20_000, seed=7)
    cam = Camera(120, 160)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    res = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    lens = res["ranges"][:, 1].astype(np.int64) - res["ranges"][:, 0]
    assert lens.max() > 200  # deep tiles, many instances per coarse key
    check_frame_order(res, vs, U)


def _frames(monkeypatch, coarse, g, scene, cams):
    monkeypatch.setenv("GSR_DEPTH_COARSE", coarse)
    alone = gpu_frame(g, cams[0], _settings(), with_debug=True)
    group = batched_frames(scene, cams, _settings(), group=len(cams), debug_views=(0,))
    return alone, group


@pytest.mark.parametrize("h,w,n", [(360, 640, 60_000), (1080, 1920, 1_000_000)])
def test_coarse_equals_exact(gpu, monkeypatch, h, w, n):
    from gsviewer_amd.rasterizer import HipScene
    g = garden_standin(n, seed=1, sh_degree=0 if n < 1_000_000 else 3)
    scene = HipScene.from_gaussian_data(g)
    cams = [Camera(h, w).yaw(45.0 * v) for v in range(3)]
    ref = _frames(monkeypatch, "0", g, scene, cams)
    for coarse in ("16", "12", "8"):
        alone, group = _frames(monkeypatch, coarse, g, scene, cams)
        for a, b in ((ref[0], alone), (ref[1][0], group[0])):
            for key in ("tile_list", "ranges", "records"):
                np.testing.assert_array_equal(a[key], b[key], err_msg=f"coarse {coarse} {key}")
            np.testing.assert_array_equal(a["image"], b["image"], err_msg=f"coarse {coarse} image")
        for v in range(1, len(cams)):
            np.testing.assert_array_equal(ref[1][v]["image"], group[v]["image"], err_msg=f"coarse {coarse} view {v}")
    scene.close()


def test_coarse_equals_exact_tilted_plane(gpu, monkeypatch):
    from gsviewer_amd.rasterizer import HipScene
    g = _tilted_plane(20_000, seed=8)
    scene = HipScene.from_gaussian_data(g)
    cams = [Camera(120, 160), Camera(120, 160).yaw(3.0)]
    ref = _frames(monkeypatch, "0", g, scene, cams)
    got = _frames(monkeypatch, "8", g, scene, cams)
    for a, b in ((ref[0], got[0]), (ref[1][0], got[1][0])):
        for key in ("tile_list", "ranges", "image"):
            np.testing.assert_array_equal(a[key], b[key], err_msg=key)
    np.testing.assert_array_equal(ref[1][1]["image"], got[1][1]["image"])
    scene.close()
