"""Culling fused into the preprocess (the default; GSR_FUSED_CULL=0 keeps the
separate cull + compaction scan).  The fused form keeps one slot per Gaussian,
drops the culled ones in the depth sort's first pass, and derives each frame's
visible count and depth-key range from sequence-tagged shards
(csrc/preprocess.hip).  These tests aim at what that adds: views of one group
with very different visibility (none, a few, all), a context whose frames
alternate between key ranges and empty frames (stale shard entries must never
count), heavy box culls, and both forms giving the same frames."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin
from helpers import gpu_frame

pytestmark = pytest.mark.gpu


def _cams(h, w):
    """Views of the garden stand-in: the default camera, one that sees
    nothing (the scene beyond the far plane), one inside the scene (a part
    visible, depths from ~0 up) and two yawed."""
    near = Camera(h, w)
    near.target_dist = 0.4
    far = Camera(h, w)
    far.target_dist = 2000.0  # zfar = 500
    return [Camera(h, w), far, near, Camera(h, w).yaw(60.0), Camera(h, w).yaw(-120.0)]


def _render_alone(scene, cam, st):
    import torch

    from gsviewer_amd.rasterizer import HipContext, camera_from, render_into
    ctx = HipContext()
    out = torch.full((cam.h, cam.w, 3), -1.0, dtype=torch.float32, device="cuda")
    render_into(ctx, scene, camera_from(cam), st, out)
    torch.cuda.synchronize()
    res = out.cpu().numpy(), ctx.stats()
    ctx.close()
    return res


def test_group_views_of_mixed_visibility(gpu, monkeypatch):
    """One group (shared scene pass, batched sorts and finish) whose views see
    nothing, a part and all of the scene: every view bit-identical to the
    same view rendered alone, with the same counts."""
    import torch

    from gsviewer_amd.multiview import ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from
    monkeypatch.setenv("GSR_CHUNK", "256")
    monkeypatch.setenv("GSR_CHUNK_VIEWS", "256")
    h, w = 180, 320
    g = garden_standin(50_000, seed=11, sh_degree=3)
    scene = HipScene.from_gaussian_data(g)
    st = RenderSettings(t_min=1e-4, out_layout=1)
    cams = _cams(h, w)
    want = [_render_alone(scene, c, st) for c in cams]
    vis = [s["n_visible"] for _, s in want]
    assert vis[1] == 0 and 0 < vis[2] < len(g) and vis[0] > 0, vis
    ctxs = [HipContext() for _ in cams]
    outs = [torch.full((h, w, 3), -1.0, dtype=torch.float32, device="cuda") for _ in cams]
    pipe = ViewBatchPipeline([(ctxs, [camera_from(c) for c in cams], outs, torch.cuda.Stream())], scene, st)
    for _ in range(3):  # the same frames again: shards hold the previous frame's entries
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    for k, (img, stats) in enumerate(want):
        np.testing.assert_array_equal(outs[k].cpu().numpy(), img, err_msg=f"view {k}")
        got = ctxs[k].stats()
        for f in ("n_visible", "n_instances"):
            assert got[f] == stats[f], (k, f)
    for c in ctxs:
        c.close()
    scene.close()


def test_context_alternating_key_ranges(gpu):
    """One context renders frames whose visible depth ranges differ (wide,
    narrow, none, wide again, ...): each frame bit-identical to a fresh
    context's render of it.  A stale key-range shard of an earlier frame that
    counted would widen or, worse, narrow the range the depth sort keeps."""
    import torch

    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    h, w = 144, 256
    g = garden_standin(40_000, seed=12, sh_degree=1)
    scene = HipScene.from_gaussian_data(g)
    st = RenderSettings(t_min=0.0, out_layout=1)
    cams = _cams(h, w)
    seq = [0, 2, 1, 2, 0, 1, 3, 4, 1, 0]
    want = {k: _render_alone(scene, cams[k], st) for k in set(seq)}
    ctx = HipContext()
    out = torch.empty((h, w, 3), dtype=torch.float32, device="cuda")
    for k in seq:
        render_into(ctx, scene, camera_from(cams[k]), st, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), want[k][0], err_msg=f"camera {k}")
        assert ctx.stats()["n_visible"] == want[k][1]["n_visible"]
    ctx.close()
    scene.close()


@pytest.mark.parametrize("box", ["aabb", "obb"])
def test_fused_and_separate_cull_identical_under_box_cull(gpu, monkeypatch, box):
    """A box cull that removes most of the scene: the fused and the separate
    cull give identical images, records, depth order and tile lists."""
    from gsviewer_amd.rasterizer import RenderSettings
    g = garden_standin(60_000, seed=13, sh_degree=2)
    cam = Camera(270, 480).yaw(30.0)
    c = np.asarray(g.xyz, np.float64).mean(axis=0).astype(np.float32)

    def settings():
        st = RenderSettings(t_min=1e-4)
        st.points_center = [float(v) for v in c]
        if box == "aabb":
            st.enable_aabb = 1
            st.cube_min = [-0.6, -0.5, -0.6]
            st.cube_max = [0.5, 0.6, 0.4]
        else:
            st.enable_obb = 1
            st.set_cube_rotation_euler([25.0, 40.0, 10.0])
            st.cube_min = [-0.7, -0.4, -0.5]
            st.cube_max = [0.6, 0.5, 0.7]
        return st

    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("GSR_FUSED_CULL", fused)
        res[fused] = gpu_frame(g, cam, settings(), with_debug=True, radii=True)
    a, b = res["1"], res["0"]
    nv = a["stats"]["n_visible"]
    assert 0 < nv < len(g) // 2, nv
    assert a["stats"] == b["stats"]
    for key in ("image", "records", "depth_order", "tile_list", "ranges", "radii"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
