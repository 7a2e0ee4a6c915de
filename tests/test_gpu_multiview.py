"""Several independent views in flight on one GPU (gsr_render_begin/finish,
one context and stream per view, gsviewer_amd.multiview.ViewPipeline): every
image must be bit-identical to the same view rendered alone, and the
begin/finish protocol must reject misuse with the reference's error style."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin

pytestmark = pytest.mark.gpu


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
    with pytest.raises(RuntimeError, match="no frame was begun"):
        render_finish(ctxs[0], streams[0])
    render_begin(ctxs[0], scene, cams[0], st, outs[0], stream=streams[0])
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
