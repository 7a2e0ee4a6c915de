"""Camera matrices against GLM's closed forms (PyGLM is absent here).

``util.Camera`` builds its matrices with ``glm.lookAt``, ``glm.perspective``
and, with the orthographic checkbox (gui/camera_control.py:25-26),
``glm.ortho`` (util.py:61-93).  GLM's default clip space is right-handed with
z in [-1, 1] (lookAtRH, perspectiveRH_NO, orthoRH_NO); these are their
element formulas, written out in float64 in math orientation (row, column),
against ``gsviewer_amd/camera.py``'s float32 restatement.  The llvmpipe frames
(tests/golden/llvmpipe_golden.npz, cases ``*ortho*``) then pin what the
shaders do with an orthographic P: computeCov2D still applies the perspective
Jacobian from hfovxy_focal (gau_vert.glsl:97-122, util.py:181-185).
"""
import math

import numpy as np
import pytest

from gsviewer_amd import camera as C


def glm_look_at_rh(eye, center, up):
    eye, center, up = (np.asarray(v, np.float64) for v in (eye, center, up))
    f = center - eye
    f /= np.linalg.norm(f)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    M = np.eye(4)
    M[0, :3], M[1, :3], M[2, :3] = s, u, -f
    M[0, 3], M[1, 3], M[2, 3] = -s @ eye, -u @ eye, f @ eye
    return M


def glm_perspective_rh_no(fovy, aspect, n, f):
    t = math.tan(fovy / 2)
    M = np.zeros((4, 4))
    M[0, 0] = 1 / (aspect * t)
    M[1, 1] = 1 / t
    M[2, 2] = -(f + n) / (f - n)
    M[3, 2] = -1.0
    M[2, 3] = -(2 * f * n) / (f - n)
    return M


def glm_ortho_rh_no(l, r, b, t, n, f):
    M = np.eye(4)
    M[0, 0] = 2 / (r - l)
    M[1, 1] = 2 / (t - b)
    M[2, 2] = -2 / (f - n)
    M[0, 3] = -(r + l) / (r - l)
    M[1, 3] = -(t + b) / (t - b)
    M[2, 3] = -(f + n) / (f - n)
    return M


def close(a, b, rtol=2e-6):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.allclose(a, b, rtol=rtol, atol=rtol * max(1.0, np.abs(b).max()))


@pytest.mark.parametrize("args", [(-4.0, 4.0, -3.0, 3.0, 0.001, 500.0), (-1.0, 3.0, -2.5, 0.5, 0.1, 10.0)])
def test_ortho_is_glm_ortho(args):
    assert close(C.ortho(*args), glm_ortho_rh_no(*args))


@pytest.mark.parametrize("args", [(math.pi / 2, 16 / 9, 0.001, 500.0), (0.7, 0.75, 0.1, 100.0)])
def test_perspective_is_glm_perspective(args):
    assert close(C.perspective(*args), glm_perspective_rh_no(*args))


@pytest.mark.parametrize("eye,center,up", [((0, 0, 5), (0, 0, 0), (0, 1, 0)),
                                           ((1.5, -2.0, 3.0), (0.2, 0.1, -0.4), (0.1, 1.0, 0.2))])
def test_look_at_is_glm_look_at(eye, center, up):
    assert close(C.look_at(eye, center, up), glm_look_at_rh(eye, center, up))


@pytest.mark.parametrize("h,w,scale", [(1080, 1920, 5.0), (150, 200, 2.5)])
def test_camera_orthographic_projection(h, w, scale):
    """util.py:79-85: glm.ortho(-s*ar, s*ar, -s, s, znear, zfar), ar = w / h;
    the perspective branch is unchanged by the flag's absence."""
    cam = C.Camera(h, w)
    cam.use_orthographic = True
    cam.ortho_scale = scale
    ar = w / h
    P = cam.get_project_matrix()
    assert close(P, glm_ortho_rh_no(-scale * ar, scale * ar, -scale, scale, 0.001, 500.0))
    # a view-space point at the frustum's right edge lands on ndc.x = 1 at any depth
    for z in (-1.0, -50.0):
        p = P @ np.array([scale * ar, 0.0, z, 1.0], np.float32)
        assert abs(p[0] / p[3] - 1.0) < 1e-6
    cam.use_orthographic = False
    assert close(cam.get_project_matrix(), glm_perspective_rh_no(math.pi / 2, ar, 0.001, 500.0))


def test_default_view_is_glm_look_at():
    """util.py:61-76 with the free-rotation defaults: pos = target - R (0,0,-1) dist."""
    cam = C.Camera(120, 160)
    V = cam.get_view_matrix()
    assert close(V, glm_look_at_rh((0, 0, 5), (0, 0, 0), (0, 1, 0)))
    cam = C.Camera(120, 160).yaw(30.0)
    V = cam.get_view_matrix()
    a = math.radians(30.0)
    eye = (5 * math.sin(a), 0.0, 5 * math.cos(a))
    assert close(cam.position, eye, rtol=1e-5)
    assert close(V, glm_look_at_rh(eye, (0, 0, 0), (0, 1, 0)), rtol=1e-5)
