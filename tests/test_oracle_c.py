"""The C restatement (bench CPU baseline, large-size checker) agrees with the
NumPy restatement of the reference OpenGL path."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera, euler_to_rotation_matrix
from gsviewer_amd.gaussian_data import naive_gaussian, random_scene
from oracle import c_oracle as C
from oracle import gl_oracle as O
from helpers import uniforms_for


def _both(g, cam, mode="float", **over):
    U = uniforms_for(cam, **over)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    ref = O.composite(vs, U, mode=mode)
    img, order = C.render(g.flat(), g.sh_dim, U, mode=mode, threads=4, return_order=True)
    return ref, img, order, vs


@pytest.mark.parametrize("deg", [0, 3])
def test_c_matches_numpy_float(deg):
    g = random_scene(1500, sh_degree=deg, seed=40 + deg)
    ref, img, order, vs = _both(g, Camera(72, 96).yaw(10))
    np.testing.assert_array_equal(order, O.sort_back_to_front(vs["view_z"], vs["visible"]))
    # same arithmetic; exp() may differ by an ulp between libm and numpy
    assert np.abs(ref - img).max() <= 1e-5


@pytest.mark.parametrize("mode", [-6, -5, -4, -3, -2, -1, 1, 2])
def test_c_matches_numpy_modes(mode):
    g = random_scene(800, sh_degree=3, seed=50)
    ref, img, _, _ = _both(g, Camera(64, 80), render_mod=mode)
    assert np.abs(ref - img).max() <= 1e-5


def test_c_matches_numpy_gl8_and_boxes():
    g = random_scene(1200, sh_degree=1, seed=60)
    ref, img, _, _ = _both(g, Camera(64, 80), mode="gl8")
    assert (np.abs(ref - img) > 1.5 / 255).mean() < 1e-3
    c = g.points_center.astype(np.float32)
    ref, img, _, vs = _both(g, Camera(64, 80), enable_obb=1, points_center=c,
                            cube_rotation=euler_to_rotation_matrix([30, 15, 0]).astype(np.float32),
                            cubeMin=np.full(3, -1.2, np.float32), cubeMax=np.full(3, 1.2, np.float32))
    assert 0 < vs["visible"].sum() < len(g)
    assert np.abs(ref - img).max() <= 1e-5


def test_naive_scene_known_answers():
    """Hand-derivable values for the reference's built-in scene at the default
    camera (util_gau.naive_gaussian, util.Camera defaults)."""
    g = naive_gaussian()
    cam = Camera(720, 1280)
    U = uniforms_for(cam)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    assert vs["visible"].all()
    # Gaussian 0 at the origin projects to the image centre
    np.testing.assert_allclose(vs["center"][0], [640, 360], atol=1e-3)
    # isotropic sigma 0.03 at depth 5, focal 360 px: var = (0.03*360/5)^2 + 0.3
    np.testing.assert_allclose(vs["cov2d"][0], [(0.03 * 72) ** 2 + 0.3, 0, (0.03 * 72) ** 2 + 0.3], rtol=1e-5,
                               atol=1e-6)
    # colour = C0 * (c - 0.5)/0.28209 + 0.5 ~= c
    np.testing.assert_allclose(vs["color"], [[1, 0, 1], [1, 0, 0], [0, 1, 0], [0, 0, 1]], atol=2e-4)
    img = C.render(g.flat(), g.sh_dim, U)
    # centre pixel: Gaussian 3 (z=1, front) covers it at alpha 0.99 over Gaussian 0
    assert img[359:361, 639:641].max() > 0.9


@pytest.mark.parametrize("n", [0, 1, 2, 1000, 300_000])
@pytest.mark.parametrize("threads", [1, 4])
def test_c_depth_sort_is_stable_argsort(n, threads):
    """oracle_sort_depth (the parallel radix sort the CPU baseline times) gives
    the reference's _sort_gaussian_cpu order: ascending view z, equal keys in
    ascending id (renderer_ogl.py:16-26), -0.0 equal to +0.0."""
    rng = np.random.default_rng(n + threads)
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    if n > 10:
        xyz[::7] = xyz[3]                      # exact ties
        xyz[5] = [0.0, 0.0, 0.0]               # z = +0.0 ...
        xyz[9] = [-0.0, 0.0, 0.0]              # ... and -0.0 (equal keys)
    V = np.eye(4, dtype=np.float32)
    V[2, :3] = [0.3, -0.5, 0.8]
    z = ((V[2, 0] * xyz[:, 0] + V[2, 1] * xyz[:, 1]) + V[2, 2] * xyz[:, 2]) + V[2, 3]
    np.testing.assert_array_equal(C.sort_depth(xyz, V, threads=threads), np.argsort(z, kind="stable"))
