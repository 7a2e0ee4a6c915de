"""GSR_BLEND_UNORM8: the reference viewer's RGBA8 framebuffer as a GPU output
mode, against the oracle's RGBA8 blend (oracle/gl_oracle.c mode "gl8": GL
SRC_ALPHA / ONE_MINUS_SRC_ALPHA in draw order in unorm8 fixed point as Mesa
llvmpipe performs it, pinned by tests/golden/llvmpipe_golden.npz;
renderer_ogl.py:178-180, main.py:197-198).

Both sides run the same integer blend on the same 8-bit colour and alpha; the
per-fragment alpha comes from the record's log2-scaled quadratic on the GPU
and from expf(power) in the oracle, which can differ by an ulp and then,
rarely, move its 8-bit value by one step.  So the check is exact equality
(values k/255) on at least 99.9 % of the channels, at most 1e-4 of the
channels off by more than one step, none by more than 4."""
import numpy as np
import pytest
import torch

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin, random_scene
from oracle import c_oracle as C
from helpers import batched_frames, gpu_frame, uniforms_for

pytestmark = pytest.mark.gpu

FRAC_EQUAL = 0.999
FRAC_OVER_1LSB = 1e-4
MAX_LSB = 4


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(blend=1, **kw)


def _check8(img, ref):
    steps = np.rint(np.abs(img.astype(np.float64) - ref.astype(np.float64)) * 255.0)
    assert np.all(np.abs(img * 255.0 - np.rint(img * 255.0)) < 1e-3), "output is not on the unorm8 grid"
    info = dict(equal=float((steps == 0).mean()), over1=float((steps > 1).mean()), max=int(steps.max()))
    assert info["equal"] >= FRAC_EQUAL, info
    assert info["over1"] <= FRAC_OVER_1LSB, info
    assert info["max"] <= MAX_LSB, info
    return info


@pytest.mark.parametrize("mode", [-6, -5, -4, -3, -2, -1, 0, 1, 3, 6])
def test_unorm8_modes(gpu, mode):
    g = random_scene(2000, sh_degree=3, seed=80, scale_range=(0.01, 0.07))
    cam = Camera(96, 128).yaw(10)
    st = _settings(render_mod=mode, bg=[0.1, 0.3, 0.7])
    res = gpu_frame(g, cam, st)
    ref = C.render(g.flat(), g.sh_dim, uniforms_for(cam, st), mode="gl8", threads=8)
    _check8(res["image"], ref)


def test_unorm8_garden_1080p_full_size(gpu):
    """C2 at full size (1M garden stand-in, SH 3, 1920x1080), one view."""
    g = garden_standin(1_000_000, seed=1, sh_degree=3)
    cam = Camera(1080, 1920).yaw(30)
    st = _settings()
    res = gpu_frame(g, cam, st)
    ref = C.render(g.flat(), g.sh_dim, uniforms_for(cam, st), mode="gl8", threads=16)
    info = _check8(res["image"], ref)
    print("unorm8 C2:", info)


def test_unorm8_through_the_batched_path(gpu):
    """The bench's path (shared preprocess, batched sorts and finish) in
    unorm8 mode: every view equals its single-view render bit for bit."""
    from gsviewer_amd.rasterizer import HipScene
    g = garden_standin(60_000, seed=3, sh_degree=1)
    scene = HipScene.from_gaussian_data(g)
    cams = [Camera(180, 320).yaw(45.0 * v) for v in range(4)]
    res = batched_frames(scene, cams, _settings(), group=4)
    for cam, r in zip(cams, res):
        single = gpu_frame(g, cam, _settings())["image"]
        np.testing.assert_array_equal(r["image"], single)
    scene.close()


def test_unorm8_rejects_bad_blend(gpu):
    import ctypes
    from gsviewer_amd import _lib
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from
    g = random_scene(100, sh_degree=0, seed=1)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    out = torch.empty((3, 16, 16), dtype=torch.float32, device="cuda")
    st = RenderSettings().to_c()
    st.blend = 7
    lib = _lib.load()
    rc = lib.gsr_render(ctx.handle, scene.handle, ctypes.byref(camera_from(Camera(16, 16))), ctypes.byref(st),
                        ctypes.c_void_p(out.data_ptr()), None, None)
    assert rc == _lib.GSR_ERR_INVALID and b"blend" in lib.gsr_last_error()
    ctx.close()
    scene.close()
