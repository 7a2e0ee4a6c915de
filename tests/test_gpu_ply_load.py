"""The viewer's "Open ply" straight into a device scene (gsr_scene_load_ply,
SURVEY.md §8(f) row 2) against the oracle of the host path it replaces:
oracle/ply_oracle.load_ply (the PLY vertex reader and load_ply's activations,
util_gau.py:236-305, restated in the reference's own NumPy expressions), then
GaussianData.scale_data(5.0) (util_gau.py:44-53, bit-exact against the
reference-run fixture in tests/golden) and points_center, as
gs_elements_control.py:41-44 does.  The product's own host loader is not
the reference here.

xyz, rot and sh are bit-identical; scale and opacity go through exp, which
NumPy evaluates with its own float32 SIMD polynomial (up to ~2.5 ulp from the
exact value) and the GPU with its exp (within 1 ulp), so they are checked to
a few ulps; points_center and the rescale factor are bit-identical."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import GaussianData
from oracle import ply_oracle as P
from helpers import compare_images, TOL_EXACT
from test_ply import vertex_array, write

pytestmark = pytest.mark.gpu

EXP_ULPS = 4


def _host(path, interval):
    g = GaussianData(*P.load_ply(path))
    if interval > 0:
        g.scale_data(interval)
    return g


def _check(path, interval=5.0):
    from gsviewer_amd.rasterizer import HipScene
    g = _host(path, interval)
    scene = HipScene.from_ply(path, scale_to_interval=interval)
    got = scene.read_flat().cpu().numpy()
    want = g.flat().astype(np.float32)
    assert scene.n == len(g) and got.shape == want.shape
    np.testing.assert_array_equal(got[:, 0:3], want[:, 0:3])      # xyz (rescaled)
    np.testing.assert_array_equal(got[:, 3:7], want[:, 3:7])      # rot (normalised twice)
    np.testing.assert_array_equal(got[:, 11:], want[:, 11:])      # sh
    np.testing.assert_array_max_ulp(got[:, 7:11], want[:, 7:11], maxulp=EXP_ULPS)  # exp(scale)*f, sigmoid
    np.testing.assert_array_equal(scene.points_center, np.mean(want[:, 0:3], axis=0).astype(np.float32))
    return g, scene


@pytest.mark.parametrize("deg,fmt,xyz_type", [(3, "binary_little_endian", "f4"), (0, "binary_big_endian", "f8"),
                                              (0, "ascii", "f4"), (3, "binary_little_endian", "f8")])
def test_load_ply_to_device_matches_host(gpu, tmp_path, deg, fmt, xyz_type):
    path = write(tmp_path, vertex_array(3001, deg=deg, seed=7 + deg, xyz_type=xyz_type), fmt)
    g, scene = _check(path)
    scene.close()


def test_load_ply_to_device_many_chunks_and_render(gpu, tmp_path):
    """300K rows (three staging chunks); the loaded scene renders like the
    host-loaded one."""
    import torch
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into
    path = write(tmp_path, vertex_array(300_000, deg=3, seed=3))
    g, dev_scene = _check(path)
    host_scene = HipScene.from_gaussian_data(g)
    cam = Camera(360, 640).yaw(25.0)
    st = RenderSettings(t_min=0.0, out_layout=1, points_center=list(dev_scene.points_center))
    imgs = []
    for sc in (host_scene, dev_scene):
        out = torch.empty((cam.h, cam.w, 3), dtype=torch.float32, device="cuda")
        ctx = HipContext()
        render_into(ctx, sc, camera_from(cam), st, out)
        torch.cuda.synchronize()
        imgs.append(out.cpu().numpy())
        ctx.close()
    compare_images(imgs[1], imgs[0], tol=TOL_EXACT)
    host_scene.close()
    dev_scene.close()


def test_load_ply_without_rescale_and_tiny(gpu, tmp_path):
    path = write(tmp_path, vertex_array(1, deg=0, seed=1), name="one.ply")
    g, scene = _check(path, interval=0.0)
    assert scene.scale_factor == 1.0
    scene.close()
    path = write(tmp_path, vertex_array(500, deg=3, seed=2), name="five.ply")
    g, scene = _check(path, interval=0.0)
    scene.close()


def test_load_ply_errors(gpu, tmp_path):
    from gsviewer_amd.rasterizer import HipScene
    with pytest.raises(RuntimeError, match="cannot open"):
        HipScene.from_ply(str(tmp_path / "missing.ply"))
    bad = tmp_path / "bad.ply"
    bad.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement face 0\nend_header\n")
    with pytest.raises(RuntimeError, match="vertex"):
        HipScene.from_ply(str(bad))
