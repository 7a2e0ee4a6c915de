"""Frames rendered by the reference's own shaders on a real GL driver (Mesa
llvmpipe) -- the cases behind ``tests/golden/llvmpipe_golden.npz``.

``tests/golden/make_gl_golden.py`` renders each case through
``oracle/gl_ref/llvmpipe_gl.c`` (build container only); the tests rebuild the
same scene, camera and uniforms from this file and compare the oracle
(``test_oracle_gl_golden.py``) and the HIP path (``test_gpu_gl_golden.py``)
with the stored framebuffers.  Scenes are regenerated from their seeds; the
fixture stores a SHA-256 of each ``flat()`` buffer so a changed generator
fails loudly instead of comparing different scenes.
"""
from __future__ import annotations

import hashlib

import numpy as np

from gsviewer_amd.camera import Camera, euler_to_quaternion, euler_to_rotation_matrix
from gsviewer_amd.gaussian_data import garden_standin, naive_gaussian, random_scene

F = np.float32

SCENES = {
    # name: (kind, n, sh_degree, seed, scale_range)
    "naive": ("naive", 4, 0, 0, None),
    "sh0": ("random", 3000, 0, 13, (0.005, 0.05)),
    "sh1": ("random", 3000, 1, 12, (0.005, 0.05)),
    "sh3": ("random", 3000, 3, 11, (0.005, 0.05)),
    "sh3_big": ("random", 1500, 3, 14, (0.03, 0.25)),
    "garden": ("garden", 100_000, 3, 1, None),  # the bench's scene generator (C2's stand-in), 1/10 size
}

# name: (scene, (h, w), yaw_deg, target_dist, orthographic, uniform overrides)
CASES = {
    "naive": ("naive", (120, 160), 0.0, 5.0, False, {}),
    "naive_yaw": ("naive", (120, 160), 35.0, 3.0, False, {}),
    "sh0_m6": ("sh0", (150, 200), 20.0, 5.0, False, {}),
    "sh1_m6": ("sh1", (150, 200), -30.0, 5.0, False, {}),
    "sh3_m6": ("sh3", (150, 200), 20.0, 5.0, False, {}),
    "sh3_m0": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": 0}),
    "sh3_m1": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": 1}),
    "sh3_m2": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": 2}),
    "sh3_depth": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -3}),
    "sh3_normal": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -2}),
    "sh3_bb_normal": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -1}),
    "sh3_billboard": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -4}),
    "sh3_flat_ball": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -5}),
    "sh3_gauss_ball": ("sh3", (150, 200), 20.0, 5.0, False, {"render_mod": -6}),
    "sh3_appearance": ("sh3", (150, 200), 20.0, 5.0, False, {
        "gaussian_scale_factor": 1.4, "screen_display_scale_factor": 0.75, "dc_factor": 1.3,
        "extra_factor": 0.6, "color_scale_factors": (1.2, 0.8, 1.0), "rot_modifier_euler": (10.0, 20.0, 30.0),
        "light_rotation": (30.0, -45.0, 10.0)}),
    "sh3_aabb": ("sh3", (150, 200), 20.0, 5.0, False, {"enable_aabb": 1, "aabb_frac": 0.5}),
    "sh3_obb": ("sh3", (150, 200), 20.0, 5.0, False, {
        "enable_obb": 1, "cube_rotation_euler": (30.0, 15.0, 0.0), "cubeMin": (-1.0, -1.0, -1.0),
        "cubeMax": (1.0, 1.0, 1.0)}),
    "sh3_ortho": ("sh3", (150, 200), 20.0, 5.0, True, {}),
    "sh3_ortho_depth": ("sh3", (150, 200), 20.0, 5.0, True, {"render_mod": -3}),
    "sh3_ortho_normal": ("sh3", (150, 200), 20.0, 5.0, True, {"render_mod": -2}),
    "big_close": ("sh3_big", (144, 176), 60.0, 2.5, False, {}),
    "garden_100k": ("garden", (180, 320), 0.0, 5.0, False, {}),
}

# cases the CPU test checks with the C oracle (oracle/gl_oracle.c) instead of the NumPy one (too slow there)
LARGE = {"garden_100k"}


def scene(name):
    kind, n, deg, seed, sr = SCENES[name]
    if kind == "naive":
        return naive_gaussian()
    if kind == "garden":
        return garden_standin(n, seed=seed, sh_degree=deg)
    return random_scene(n, sh_degree=deg, seed=seed, scale_range=sr)


def flat_sha(g) -> str:
    return hashlib.sha256(np.ascontiguousarray(g.flat(), F).tobytes()).hexdigest()


def camera(case):
    _, (h, w), yaw, dist, ortho, _ = CASES[case]
    cam = Camera(h, w)
    cam.target_dist = dist
    if yaw:
        cam.yaw(yaw)
    cam.use_orthographic = bool(ortho)
    return cam


def uniform_overrides(case, g):
    """Oracle ``default_uniforms`` overrides for a case (the reference setters'
    arguments resolved: Euler -> quaternion via util.euler_to_quaternion,
    Euler -> matrix via util.convert_euler_angles_to_rotation_matrix, AABB from
    compute_aabb as SURVEY 8d C5 does)."""
    over = dict(CASES[case][5])
    kw = {}
    for k, v in over.items():
        if k == "rot_modifier_euler":
            kw["rot_modifier"] = np.asarray(euler_to_quaternion(*v), F)
        elif k == "cube_rotation_euler":
            kw["cube_rotation"] = np.asarray(euler_to_rotation_matrix(v), F)
        elif k == "aabb_frac":
            mn, mx, _ = g.compute_aabb
            kw["points_center"] = np.asarray(g.points_center, F)
            kw["cubeMin"] = (np.asarray(mn, F) * F(v)).astype(F)
            kw["cubeMax"] = (np.asarray(mx, F) * F(v)).astype(F)
        elif isinstance(v, (tuple, list)):
            kw[k] = np.asarray(v, F)
        elif isinstance(v, float):
            kw[k] = F(v)
        else:
            kw[k] = v
    return kw


def uniforms(case, g):
    from oracle import gl_oracle as O

    cam = camera(case)
    V = cam.get_view_matrix()
    P = cam.get_project_matrix()
    return cam, O.default_uniforms(V, P, np.asarray(cam.get_htanfovxy_focal(), F), cam.position, cam.w, cam.h,
                                   **uniform_overrides(case, g))


def settings_from_uniforms(U):
    """RenderSettings carrying the same uniform state (for the HIP path)."""
    from gsviewer_amd.rasterizer import RenderSettings

    return RenderSettings(
        scale_modifier=float(U["gaussian_scale_factor"]), screen_scale=float(U["screen_display_scale_factor"]),
        render_mod=int(U["render_mod"]), dc_factor=float(U["dc_factor"]), extra_factor=float(U["extra_factor"]),
        color_scale=[float(v) for v in U["color_scale_factors"]],
        rot_modifier=[float(v) for v in U["rot_modifier"]],
        light_rotation=[float(v) for v in U["light_rotation"]],
        enable_aabb=int(U["enable_aabb"]), enable_obb=int(U["enable_obb"]),
        cube_rotation=np.asarray(U["cube_rotation"], F), cube_min=[float(v) for v in U["cubeMin"]],
        cube_max=[float(v) for v in U["cubeMax"]], points_center=[float(v) for v in U["points_center"]],
        bg=[0.0, 0.0, 0.0])
