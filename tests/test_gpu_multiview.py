"""Several independent views in flight on one GPU (gsr_render_begin/finish,
one context and stream per view, gsviewer_amd.multiview.ViewPipeline): every
image must be bit-identical to the same view rendered alone, and the
begin/finish protocol must reject misuse with the reference's error style."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _same_chunk_length(monkeypatch):
    """Frames finished alone use GSR_CHUNK (default 192) and a group's frames
    GSR_CHUNK_VIEWS (default 3072); with t_min > 0 the chunking decides where
    compositing stops (within t_min), so the bit-identity checks here give
    both paths one length, short enough that busy tiles take the multi-chunk
    merge in both."""
    monkeypatch.setenv("GSR_CHUNK", "256")
    monkeypatch.setenv("GSR_CHUNK_VIEWS", "256")


def _setup(n_views, h=180, w=320, n=60_000):
    import torch

    from gsviewer_amd.multiview import view_of
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from
    g = garden_standin(n, seed=3, sh_degree=3)
    scene = HipScene.from_gaussian_data(g)
    st = RenderSettings(t_min=1e-4, out_layout=1)
    cams = [camera_from(view_of(k, h, w)) for k in range(n_views)]
    ctxs = [HipContext() for _ in range(n_views)]
    streams = [torch.cuda.Stream() for _ in range(n_views)]
    outs = [torch.full((h, w, 3), -1.0, dtype=torch.float32, device="cuda") for _ in range(n_views)]
    return scene, st, cams, ctxs, streams, outs


def test_pipelined_views_match_serial_renders(gpu):
    import torch

    from gsviewer_amd.multiview import ViewPipeline
    from gsviewer_amd.rasterizer import HipContext, render_into
    K = 4
    scene, st, cams, ctxs, streams, outs = _setup(K)
    want = []
    ref_ctx = HipContext()
    for k in range(K):
        o = torch.empty_like(outs[k])
        render_into(ref_ctx, scene, cams[k], st, o)
        want.append(o)
    torch.cuda.synchronize()
    pipe = ViewPipeline(ctxs, streams, scene, cams, st, outs)
    for _ in range(3 * K + 1):  # every view several times, one view a frame ahead
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    for k in range(K):
        np.testing.assert_array_equal(outs[k].cpu().numpy(), want[k].cpu().numpy(), err_msg=f"view {k}")
    for c in ctxs + [ref_ctx]:
        c.close()
    scene.close()


def test_begin_finish_protocol_errors(gpu):
    import torch

    from gsviewer_amd.rasterizer import camera_from, render_begin, render_finish
    scene, st, cams, ctxs, streams, outs = _setup(2, n=2000)
    from gsviewer_amd.rasterizer import render_wait_counts
    with pytest.raises(RuntimeError, match="no frame was begun"):
        render_finish(ctxs[0], streams[0])
    with pytest.raises(RuntimeError, match="no frame was begun"):
        render_wait_counts(ctxs[0])
    render_begin(ctxs[0], scene, cams[0], st, outs[0], stream=streams[0])
    render_wait_counts(ctxs[0])  # the frame stays pending: waiting twice, then finishing, is fine
    render_wait_counts(ctxs[0])
    with pytest.raises(RuntimeError, match="not finished"):
        render_begin(ctxs[0], scene, cams[0], st, outs[0], stream=streams[0])
    with pytest.raises(RuntimeError, match="stream"):
        render_finish(ctxs[0], streams[1])
    render_finish(ctxs[0], streams[0])
    torch.cuda.synchronize()
    assert np.isfinite(outs[0].cpu().numpy()).all()
    for c in ctxs:
        c.close()
    scene.close()


def test_contexts_share_one_scene_concurrently(gpu):
    """Two contexts on two streams rendering different views of one scene at
    once (the scene handle is immutable after create)."""
    import torch

    from gsviewer_amd.rasterizer import HipContext, render_begin, render_finish, render_into
    scene, st, cams, ctxs, streams, outs = _setup(2)
    render_begin(ctxs[0], scene, cams[0], st, outs[0], stream=streams[0])
    render_begin(ctxs[1], scene, cams[1], st, outs[1], stream=streams[1])
    render_finish(ctxs[1], streams[1])
    render_finish(ctxs[0], streams[0])
    torch.cuda.synchronize()
    ref = HipContext()
    for k in range(2):
        o = torch.empty_like(outs[k])
        render_into(ref, scene, cams[k], st, o)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(outs[k].cpu().numpy(), o.cpu().numpy())
    for c in ctxs + [ref]:
        c.close()
    scene.close()


@pytest.mark.parametrize("batched_sorts,batched_finish,mode", [(True, True, "serial"), (True, False, "serial"),
                                                                (False, True, "serial"), (False, False, "serial"),
                                                                (True, True, "lookahead1"), (True, True, "lookahead0"),
                                                                (True, True, "threads"), (True, True, "exact"),
                                                                (True, False, "exact"), (False, True, "exact")])
def test_shared_scene_pass_matches_serial_renders(gpu, monkeypatch, batched_sorts, batched_finish, mode):
    """gsr_render_begin_views (one cull + preprocess pass over the scene for a
    group of views) through ViewBatchPipeline with two groups: images, radii
    and counts identical to each view rendered alone (a frame alone sorts
    depth coarsely and repairs the tile lists' runs; a group's frames sort
    exactly); with the group's sort step and finish batched or per view in
    every combination; also with one group finished a step after it began
    (lookahead 1), with one host thread per group (ThreadedViewBatchPipeline),
    and against frames alone sorted exactly too (GSR_DEPTH_COARSE=0)."""
    import torch

    monkeypatch.setenv("GSR_DEPTH_COARSE", "0" if mode == "exact" else "16")

    from gsviewer_amd.multiview import ThreadedViewBatchPipeline, ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, render_into
    K, G = 3, 2
    scene, st, cams, ctxs, streams, outs = _setup(K * G)
    want, want_stats = [], []
    ref_ctx = HipContext()
    for k in range(K * G):
        o = torch.empty_like(outs[k])
        render_into(ref_ctx, scene, cams[k], st, o)
        torch.cuda.synchronize()
        want.append(o)
        want_stats.append(ref_ctx.stats())
    groups = [(ctxs[g * K:(g + 1) * K], cams[g * K:(g + 1) * K], outs[g * K:(g + 1) * K], streams[g])
              for g in range(G)]
    if mode == "threads":
        pipe = ThreadedViewBatchPipeline(groups, scene, st, batched_sorts=batched_sorts,
                                         batched_finish=batched_finish)
    else:
        pipe = ViewBatchPipeline(groups, scene, st, batched_sorts=batched_sorts, batched_finish=batched_finish,
                                 lookahead={"lookahead1": 1, "lookahead0": 0}.get(mode))
    for _ in range(3 * G + 1):  # every group several times, one group a step ahead
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    if mode == "threads":
        pipe.close()
    for k in range(K * G):
        np.testing.assert_array_equal(outs[k].cpu().numpy(), want[k].cpu().numpy(), err_msg=f"view {k}")
        got = ctxs[k].stats()
        for f in ("n_visible", "n_instances"):
            assert got[f] == want_stats[k][f], (k, f)
    for c in ctxs + [ref_ctx]:
        c.close()
    scene.close()


@pytest.mark.parametrize("interleave,classes,k,first", [("0", "2", 3, "1"), ("1", "2", 3, "1"), ("1", "8", 5, "1"),
                                                        ("1", "16", 3, "1"), ("1", "16", 5, "1"), ("1", "8", 5, "0"),
                                                        ("0", "8", 3, "0")])
def test_compositing_dispatch_orders(gpu, monkeypatch, interleave, classes, k, first):
    """The compositor's dispatch order (chunk length classes; a group's views
    interleaved class-major, or view after view; k * classes > 64 falls back to
    view after view; first chunks before later ones, or full chunks first)
    moves no pixel: a group's images equal each view rendered alone.  Short
    chunks so that deep tiles have many and partials span the classes."""
    import torch

    from gsviewer_amd.multiview import ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, render_into
    monkeypatch.setenv("GSR_CHUNK", "64")
    monkeypatch.setenv("GSR_CHUNK_VIEWS", "64")
    monkeypatch.setenv("GSR_LEN_CLASSES", classes)
    monkeypatch.setenv("GSR_VIEWS_INTERLEAVE", interleave)
    monkeypatch.setenv("GSR_FIRST_MAJOR", first)
    scene, st, cams, ctxs, streams, outs = _setup(k)
    ref_ctx = HipContext()
    want = []
    for v in range(k):
        o = torch.empty_like(outs[v])
        render_into(ref_ctx, scene, cams[v], st, o)
        want.append(o)
    pipe = ViewBatchPipeline([(ctxs, cams, outs, streams[0])], scene, st)
    for _ in range(2):
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()
    for v in range(k):
        np.testing.assert_array_equal(outs[v].cpu().numpy(), want[v].cpu().numpy(), err_msg=f"view {v}")
    for c in ctxs + [ref_ctx]:
        c.close()
    scene.close()


def test_shared_scene_pass_radii_and_errors(gpu):
    import torch

    from gsviewer_amd.rasterizer import (HipContext, render_begin_sort, render_begin_views, render_finish,
                                         render_into)
    scene, st, cams, ctxs, streams, outs = _setup(2, n=5000)
    n = 5000
    radii = [torch.full((n,), -7, dtype=torch.int32, device="cuda") for _ in range(2)]
    with pytest.raises(RuntimeError, match="no gsr_render_begin_views frame"):
        render_begin_sort(ctxs[0], streams[0])
    with pytest.raises(RuntimeError, match="contexts must differ"):
        render_begin_views([ctxs[0], ctxs[0]], scene, cams[:2], st, outs[:2])
    from gsviewer_amd.rasterizer import render_begin_sorts
    with pytest.raises(RuntimeError, match="no gsr_render_begin_views frame"):
        render_begin_sorts(ctxs, streams[0])
    s = torch.cuda.Stream()
    render_begin_views(ctxs, scene, cams[:2], st, outs, radii=radii, stream=s)
    with pytest.raises(RuntimeError, match="not finished"):
        render_begin_views(ctxs, scene, cams[:2], st, outs, stream=s)
    s.synchronize()
    for c, vs in zip(ctxs, streams):
        render_begin_sort(c, vs)
        render_finish(c, vs)
    torch.cuda.synchronize()
    ref = HipContext()
    for k in range(2):
        o = torch.empty_like(outs[k])
        r = torch.empty_like(radii[k])
        render_into(ref, scene, cams[k], st, o, r)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(outs[k].cpu().numpy(), o.cpu().numpy())
        np.testing.assert_array_equal(radii[k].cpu().numpy(), r.cpu().numpy())
    for c in ctxs + [ref]:
        c.close()
    scene.close()


def test_finish_views_mixed_frames(gpu):
    """gsr_render_finish_views over frames begun one by one (gsr_render_begin)
    on one stream, of two different scenes, one of them with no visible
    Gaussian: identical to finishing each alone; protocol errors."""
    import torch

    from gsviewer_amd.rasterizer import HipContext, HipScene, render_begin, render_finish_views, render_into
    scene, st, cams, ctxs, streams, outs = _setup(3)
    g = garden_standin(3000, seed=5, sh_degree=3)
    g.xyz = g.xyz + np.float32(1e8)  # beyond the far plane: nothing visible
    far = HipScene.from_gaussian_data(g)
    scenes = [scene, far, scene]
    s = torch.cuda.Stream()
    with pytest.raises(RuntimeError, match="no frame was begun"):
        render_finish_views(ctxs, s)
    for _ in range(2):  # twice: buffers sized by the first frames are reused
        for k in range(3):
            render_begin(ctxs[k], scenes[k], cams[k], st, outs[k], stream=s)
        render_finish_views(ctxs, s)
    torch.cuda.synchronize()
    ref = HipContext()
    for k in range(3):
        o = torch.empty_like(outs[k])
        render_into(ref, scenes[k], cams[k], st, o)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(outs[k].cpu().numpy(), o.cpu().numpy(), err_msg=f"view {k}")
        want = ref.stats()
        got = ctxs[k].stats()
        for f in ("n_visible", "n_instances"):
            assert got[f] == want[f], (k, f)
    assert ctxs[1].stats()["n_visible"] == 0
    # misuse: the same context twice; frames of different sizes; another stream
    render_begin(ctxs[0], scene, cams[0], st, outs[0], stream=s)
    with pytest.raises(RuntimeError, match="contexts must differ"):
        render_finish_views([ctxs[0], ctxs[0]], s)
    with pytest.raises(RuntimeError, match="not the frames' stream"):
        render_finish_views([ctxs[0]], streams[0])
    from gsviewer_amd.multiview import view_of
    from gsviewer_amd.rasterizer import camera_from
    small = camera_from(view_of(1, 90, 160))
    o_small = torch.empty((90, 160, 3), dtype=torch.float32, device="cuda")
    render_begin(ctxs[1], scene, small, st, o_small, stream=s)
    with pytest.raises(RuntimeError, match="differ in frame size"):
        render_finish_views([ctxs[0], ctxs[1]], s)
    render_finish_views([ctxs[0]], s)
    render_finish_views([ctxs[1]], s)
    torch.cuda.synchronize()
    for c in ctxs + [ref]:
        c.close()
    scene.close()
    far.close()


def test_rect_payload_matches_gathered_rects(gpu, monkeypatch):
    """The depth sort carrying the packed tile rectangles (default for frames
    of <= 256 x 256 tiles) bins exactly as the by-id gather of the rectangles
    (GSR_NO_RECT_PAYLOAD): same images and counts, single view and a batched
    group.  One view sits inside the scene (part of it visible): with the
    fused cull's uncompacted slots the gathered ids reach past V."""
    import torch

    from gsviewer_amd.multiview import ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, camera_from, render_into
    scene, st, cams, ctxs, streams, outs = _setup(4)
    near = Camera(180, 320)
    near.target_dist = 0.4
    cams[3] = camera_from(near)
    got = {}
    for mode in ("payload", "gather"):
        if mode == "gather":
            # the knob is read at context creation: fresh contexts
            monkeypatch.setenv("GSR_NO_RECT_PAYLOAD", "1")
            for c in ctxs:
                c.close()
            ctxs = [HipContext() for _ in ctxs]
        o = torch.empty_like(outs[0])
        render_into(ctxs[0], scene, cams[3], st, o)
        assert 0 < ctxs[0].stats()["n_visible"] < scene.n
        assert ctxs[0].knob("frame_packed") == (mode == "payload")  # the form this frame took
        # the context moves to another stream: its frame on this one must be done
        torch.cuda.synchronize()
        pipe = ViewBatchPipeline([(ctxs, cams, outs, streams[0])], scene, st)
        pipe.step()
        pipe.drain()
        torch.cuda.synchronize()
        assert [c.knob("frame_packed") for c in ctxs] == [mode == "payload"] * len(ctxs)
        got[mode] = ([o.cpu().numpy()] + [x.cpu().numpy() for x in outs], [c.stats() for c in ctxs])
    for a, b in zip(got["payload"][0], got["gather"][0]):
        np.testing.assert_array_equal(a, b)
    assert got["payload"][1] == got["gather"][1]
    for c in ctxs:
        c.close()
    scene.close()


@pytest.mark.parametrize("wh", [(16, 16), (13, 9)])
def test_single_tile_frames(gpu, wh):
    """A frame of one 16x16 tile has no tile sort; its range [0, D) is set
    directly (single_tile_range).  Alone and batched, against the oracle."""
    import sys

    from gsviewer_amd.camera import view_for_rank
    from gsviewer_amd.gaussian_data import random_scene
    from gsviewer_amd.rasterizer import HipScene, RenderSettings
    from helpers import TOL_MAX, batched_frames, compare_images, gpu_frame, uniforms_for
    sys.path.insert(0, __file__.rsplit("/tests/", 1)[0])
    from oracle import gl_oracle as O
    w, h = wh
    g = random_scene(800, sh_degree=1, seed=11, scale_range=(0.02, 0.08))
    cams = [view_for_rank(h, w, k) for k in range(4)]
    st = RenderSettings(t_min=0.0)
    scene = HipScene.from_gaussian_data(g)
    res = batched_frames(scene, cams, st, group=4)
    for cam, r in zip(cams, res):
        U = uniforms_for(cam, st)
        ref = O.composite(O.vertex_stage(g.flat().astype(np.float32), g.sh_dim, U), U)
        assert r["stats"]["n_instances"] > 0
        compare_images(r["image"], ref, tol_max=TOL_MAX)
        alone = gpu_frame(g, cam, RenderSettings(t_min=0.0))
        compare_images(alone["image"], ref, tol_max=TOL_MAX)
    scene.close()
