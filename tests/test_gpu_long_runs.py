"""The coarse depth order's long runs (gsviewer_amd/csrc/long_runs.h k_long_runs).

A frame alone sorts depth by the top GSR_DEPTH_COARSE bits of its key range
(default 16); the stable binning and tile sort leave each tile's list in runs
of equal coarse key, in slot order, which must end in (full key, slot) order:
the GL draw order restricted to the tile, the one
/root/reference/render/renderer_ogl.py:16-26 draws back to front (read front
to back; ties in descending Gaussian id).  Runs of up to 16 are repaired in
k_tile_ranges; longer ones are listed and sorted by k_long_runs (one wave up
to 1024 instances, a workgroup in registers up to 24576, a workgroup through
global scratch beyond).  Checked bit for bit (tile lists, ranges, records,
images) against the exact sort (GSR_DEPTH_COARSE=0; tests/test_gpu_parity.py
checks that form's global order and tile lists against the oracle):

* every run path: a fronto-parallel plane whose density falls off to the
  right, one far splat stretching the key range (so that, with 8 coarse bits,
  each tile's list is one run) -- runs of every length class;
* a single run of ~60k instances in one tile;
* lists whose keys are all equal, or take two values (ties by slot only);
* round 4's adversarial case: a dense plane plus one far splat at 1080p (runs
  as long as the tile lists; round 4 spent ~5e8 serial steps there), whose
  frame must stay within 1.5x the exact form's time;
* a group of views (exact sort) against the same views alone (coarse).
"""

import numpy as np
import pytest
import torch

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import GaussianData
from helpers import batched_frames, check_depth_order, compare_images, gpu_frame, uniforms_for
from oracle import c_oracle as C
from oracle import gl_oracle as O

pytestmark = pytest.mark.gpu

CAP_WAVE, CAP_BLOCK, FIX_MAX = 1024, 24576, 16  # long_runs.h kTdsCapWave / kTdsCapBlock, kFixRunMax


def run_class(lens):
    """Run classes by length: 0 global path, 1-3 workgroup, 4-6 wave, 7 the
    in-thread repair, 8 nothing to sort."""
    lens = np.asarray(lens, np.int64)
    return np.select([lens > CAP_BLOCK, lens > 8192, lens > 2048, lens > CAP_WAVE, lens > 256, lens > 64,
                      lens > FIX_MAX, lens >= 2], [0, 1, 2, 3, 4, 5, 6, 7], 8)


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def _scene(xyz, scale, seed, opacity=(0.05, 0.6)):
    rng = np.random.default_rng(seed)
    n = len(xyz)
    rot = rng.normal(0, 1, (n, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    return GaussianData(np.asarray(xyz, np.float32), rot, np.asarray(scale, np.float32),
                        rng.uniform(*opacity, (n, 1)).astype(np.float32),
                        rng.normal(0, 0.5, (n, 3)).astype(np.float32))


def graded_plane(n=400_000, seed=11, far=True):
    """A fronto-parallel plane (depth jitter 1e-4) whose density falls off
    exponentially to the right of the frame: tile lists from a few instances
    to > 24576; with the far splat and 8 coarse bits each list is one run."""
    rng = np.random.default_rng(seed)
    x = -1.6 + rng.exponential(0.35, n)
    y = rng.uniform(-1.0, 1.0, n)
    z = rng.uniform(-1e-4, 1e-4, n)
    scale = np.exp(rng.uniform(np.log(0.004), np.log(0.03), (n, 3)))
    scale[:, 2] = 1e-4
    xyz = np.stack([x, y, z], 1)
    if far:
        xyz = np.concatenate([xyz, [[0.0, 0.0, -400.0]]])
        scale = np.concatenate([scale, [[2.0, 2.0, 2.0]]])
    return _scene(xyz, scale, seed, opacity=(0.02, 0.2))


def plane_scene(n=250_000, seed=12, far=True, levels=0):
    """A dense fronto-parallel plane (z = 0 facing the default camera): with
    levels = 0 a jitter of 1e-4 in depth, else exactly `levels` distinct
    depths; plus (far) one splat 400 units behind it, which stretches the
    frame's depth-key range."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1.0, 1.0, n)
    y = rng.uniform(-0.6, 0.6, n)
    z = rng.uniform(-1e-4, 1e-4, n) if levels == 0 else rng.integers(0, levels, n) * 0.01
    scale = np.exp(rng.uniform(np.log(0.004), np.log(0.02), (n, 3)))
    scale[:, 2] = 1e-4
    xyz = np.stack([x, y, z], 1)
    if far:
        xyz = np.concatenate([xyz, [[0.0, 0.0, -400.0]]])
        scale = np.concatenate([scale, [[2.0, 2.0, 2.0]]])
    return _scene(xyz, scale, seed, opacity=(0.02, 0.2))


def _coarse(monkeypatch, form):
    monkeypatch.setenv("GSR_DEPTH_COARSE", {"exact": "0", "coarse": "16", "coarse8": "8"}[form])


def _frames(monkeypatch, g, cam, st, form):
    _coarse(monkeypatch, form)
    return gpu_frame(g, cam, st, with_debug=True)


def _same(a, b, what=""):
    for key in ("tile_list", "ranges", "records", "image"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=f"{what} {key}")
    assert a["stats"] == b["stats"], what


@pytest.mark.parametrize("form", ["coarse8", "coarse"])
def test_every_class_matches_exact_form(gpu, monkeypatch, form):
    g = graded_plane()
    cam = Camera(540, 960)
    st = _settings(t_min=0.0)
    got = _frames(monkeypatch, g, cam, st, form)
    exact = _frames(monkeypatch, g, cam, st, "exact")
    _same(got, exact)
    assert check_depth_order(exact, O.vertex_stage(g.flat(), g.sh_dim, uniforms_for(cam)))
    lens = (got["ranges"][:, 1] - got["ranges"][:, 0]).astype(np.int64)
    classes = set(run_class(lens).tolist())
    assert {0, 1, 2, 3, 4, 5, 6, 7} <= classes, sorted(classes)
    assert lens.max() > 2 * 12288, lens.max()  # several sub-blocks per pass on the global path


def test_deep_lists_image_against_oracle(gpu, monkeypatch):
    """The global path's frame against the C oracle at the stated tolerances
    (small frame: every tile deep)."""
    g = graded_plane(n=120_000, seed=5)
    cam = Camera(96, 160)
    st = _settings(t_min=0.0)
    res = _frames(monkeypatch, g, cam, st, "coarse8")
    lens = res["ranges"][:, 1].astype(np.int64) - res["ranges"][:, 0]
    assert lens.max() > CAP_BLOCK, lens.max()
    ref = C.render(g.flat(), g.sh_dim, uniforms_for(cam), mode="float")
    compare_images(res["image"], ref)


def test_single_long_run(gpu, monkeypatch):
    """~60k instances in one tile and one coarse bucket: a plane of jittered
    depth in front of the camera, one far splat stretching the key range."""
    rng = np.random.default_rng(21)
    n = 60_000
    # (centred on a tile of the 160x96 frame: 9.6 px per unit at z = 0, tile centres 8 px off the image centre)
    xyz = np.stack([0.83 + rng.uniform(-0.15, 0.15, n), 0.83 + rng.uniform(-0.1, 0.1, n),
                    rng.uniform(-1e-4, 1e-4, n)], 1)
    scale = np.exp(rng.uniform(np.log(0.002), np.log(0.006), (n, 3)))
    scale[:, 2] = 1e-4
    xyz = np.concatenate([xyz, [[0.0, 0.0, -400.0]]])
    scale = np.concatenate([scale, [[2.0, 2.0, 2.0]]])
    g = _scene(xyz, scale, 21, opacity=(0.01, 0.05))
    cam = Camera(96, 160)
    st = _settings(t_min=0.0)
    tile = _frames(monkeypatch, g, cam, st, "coarse")
    exact = _frames(monkeypatch, g, cam, st, "exact")
    _same(tile, exact)
    lens = tile["ranges"][:, 1].astype(np.int64) - tile["ranges"][:, 0]
    assert lens.max() > 2 * 12288, lens.max()
    ref = C.render(g.flat(), g.sh_dim, uniforms_for(cam), mode="float")
    compare_images(tile["image"], ref)


@pytest.mark.parametrize("levels", [1, 2])
def test_equal_depths(gpu, monkeypatch, levels):
    """Lists whose depth keys are all equal (nothing to sort: slot order) or
    take two values."""
    g = plane_scene(n=60_000, far=False, levels=levels)
    cam = Camera(270, 480)
    st = _settings(t_min=1e-4)
    tile = _frames(monkeypatch, g, cam, st, "coarse")
    exact = _frames(monkeypatch, g, cam, st, "exact")
    _same(tile, exact, f"levels {levels}")
    assert tile["stats"]["n_instances"] > 50_000


def _frame_ms(monkeypatch, g, cam, st, form, reps=10):
    from gsviewer_amd.rasterizer import HipContext, HipScene, camera_from, render_into
    _coarse(monkeypatch, form)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    out = torch.empty((cam.h, cam.w, 3), dtype=torch.float32, device="cuda")
    c = camera_from(cam)
    st.out_layout = 1
    render_into(ctx, scene, c, st, out)
    torch.cuda.synchronize()
    # device time by HIP events on the frames' stream (host timers
    # at 0.2 ms a frame measure mostly the host), median over the frames
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        render_into(ctx, scene, c, st, out)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ctx.close()
    scene.close()
    return float(np.median(ts))


def test_plane_with_far_splat(gpu, monkeypatch):
    """Round 4's adversarial case for the coarse depth order:
    a dense fronto-parallel plane plus one far splat at 1080p.  Bit-identical
    to the exact form, and its frame within 1.5x the exact form's."""
    g = plane_scene()
    cam = Camera(1080, 1920)
    st = _settings(t_min=1e-4)
    got = _frames(monkeypatch, g, cam, st, "coarse")
    exact = _frames(monkeypatch, g, cam, st, "exact")
    _same(got, exact)
    lens = got["ranges"][:, 1].astype(np.int64) - got["ranges"][:, 0]
    assert lens.max() > 1000, lens.max()
    ms_coarse = _frame_ms(monkeypatch, g, cam, _settings(t_min=1e-4), "coarse", reps=15)
    ms_exact = _frame_ms(monkeypatch, g, cam, _settings(t_min=1e-4), "exact", reps=15)
    print(f"plane + far splat, 1080p: coarse {ms_coarse:.3f} ms, exact {ms_exact:.3f} ms")
    assert ms_coarse <= 1.5 * ms_exact, (ms_coarse, ms_exact)


@pytest.mark.parametrize("scene_kind", ["graded", "plane"])
def test_group_matches_frames_alone(gpu, monkeypatch, scene_kind):
    """A group's frames (exact sort, gsr_render_finish_views) against the same
    views rendered alone (coarse order + long runs), deep lists included.
    (One chunk length for both: with t_min > 0 it decides where a pixel
    stops, tests/test_gpu_multiview.py.)"""
    from gsviewer_amd.rasterizer import HipScene
    monkeypatch.setenv("GSR_CHUNK", "256")
    monkeypatch.setenv("GSR_CHUNK_VIEWS", "256")
    g = graded_plane(n=200_000) if scene_kind == "graded" else plane_scene(n=100_000)
    cams = [Camera(270, 480).yaw(v * 20.0) for v in range(3)]
    st = _settings(t_min=1e-4)
    scene = HipScene.from_gaussian_data(g)
    group = batched_frames(scene, cams, st, group=3, debug_views=(0, 1, 2))
    scene.close()
    for v in range(3):
        alone = _frames(monkeypatch, g, cams[v], st, "coarse8")
        for key in ("tile_list", "ranges", "records", "image"):
            np.testing.assert_array_equal(alone[key], group[v][key], err_msg=f"view {v} {key}")


def test_unorm8_long_runs(gpu, monkeypatch):
    """The RGBA8 framebuffer (GSR_BLEND_UNORM8: whole lists back to front, no
    chunks) sorts the long runs in a launch of its own: tile lists and image
    bit-identical to the exact sort's."""
    g = graded_plane(n=120_000, seed=6)
    cam = Camera(270, 480)
    st = _settings(blend=1)
    got = _frames(monkeypatch, g, cam, st, "coarse8")
    exact = _frames(monkeypatch, g, cam, _settings(blend=1), "exact")
    for key in ("tile_list", "ranges", "image"):
        np.testing.assert_array_equal(got[key], exact[key], err_msg=key)
    lens = got["ranges"][:, 1].astype(np.int64) - got["ranges"][:, 0]
    assert lens.max() > CAP_BLOCK, lens.max()
