"""Generate golden vectors from the reference's pure-NumPy functions.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

The reference modules ``util_gau``, ``util`` and ``render/renderer_ogl`` import
PyOpenGL / PyGLM / plyfile at module level; none is installed here and none is
used by the functions exercised below, so empty stand-in modules are placed in
``sys.modules`` before the import.  Only data (inputs and
outputs) is written, to ``tests/golden/reference_golden.npz``; no reference
source travels.

Functions pinned (reference file:line):
  util_gau.naive_gaussian            util_gau.py:149-184
  util_gau.GaussianData.flat         util_gau.py:40-42
  util_gau.GaussianData.scale_data   util_gau.py:44-53
  util_gau.GaussianData.sh_dim / points_center / compute_aabb  :76-111
  renderer_ogl._sort_gaussian_cpu    renderer_ogl.py:16-26
  util.convert_euler_angles_to_rotation_matrix  util.py:453-479
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_golden.npz")


def _stub(name):
    m = types.ModuleType(name)
    m.__path__ = []  # importable as a package
    sys.modules[name] = m
    return m


def import_reference():
    sys.dont_write_bytecode = True
    for name in ["plyfile", "OpenGL", "OpenGL.GL", "OpenGL.GL.shaders", "OpenGL.raw",
                 "OpenGL.raw.WGL", "OpenGL.raw.WGL.EXT", "glm"]:
        _stub(name)
    sys.modules["plyfile"].PlyData = object
    sys.modules["plyfile"].PlyElement = object
    sys.modules["OpenGL"].GL = sys.modules["OpenGL.GL"]
    sys.modules["OpenGL.GL"].shaders = sys.modules["OpenGL.GL.shaders"]
    sys.path[:0] = [REF, os.path.join(REF, "render")]
    import util_gau  # noqa: E402
    import util  # noqa: E402
    import renderer_ogl  # noqa: E402
    return util_gau, util, renderer_ogl


def lookat_translate(dz):
    V = np.eye(4, dtype=np.float32)
    V[2, 3] = -dz
    return V


def main():
    util_gau, util, renderer_ogl = import_reference()
    assert renderer_ogl._sort_gaussian is renderer_ogl._sort_gaussian_cpu
    out = {}

    g = util_gau.naive_gaussian()
    out["naive_xyz"] = g.xyz
    out["naive_rot"] = g.rot
    out["naive_scale"] = g.scale
    out["naive_opacity"] = g.opacity
    out["naive_sh"] = g.sh
    out["naive_flat"] = g.flat()
    out["naive_sh_dim"] = np.array(g.sh_dim)

    rng = np.random.default_rng(1234)
    n = 3000
    xyz = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    rot = rng.normal(0, 1, (n, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=-1, keepdims=True)
    scale = np.exp(rng.uniform(np.log(0.005), np.log(0.05), (n, 3))).astype(np.float32)
    opacity = (1 / (1 + np.exp(-rng.normal(0, 1.5, (n, 1))))).astype(np.float32)
    sh = rng.normal(0, 0.6, (n, 48)).astype(np.float32)
    out["rand_xyz"], out["rand_rot"], out["rand_scale"] = xyz, rot, scale
    out["rand_opacity"], out["rand_sh"] = opacity, sh
    gr = util_gau.GaussianData(xyz.copy(), rot.copy(), scale.copy(), opacity.copy(), sh.copy())
    out["rand_flat"] = gr.flat()
    out["rand_points_center"] = gr.points_center
    mn, mx, corners = gr.compute_aabb
    out["rand_aabb_min"], out["rand_aabb_max"], out["rand_aabb_corners"] = mn, mx, corners

    # scale_data(5.0) as on PLY load (gs_elements_control.py:41-42)
    xyz2 = (rng.uniform(-7, 3, (n, 3)) * np.array([1.0, 0.3, 2.0])).astype(np.float32)
    rot2 = rng.normal(0, 2, (n, 4)).astype(np.float32)
    gs = util_gau.GaussianData(xyz2.copy(), rot2.copy(), scale.copy(), opacity.copy(), sh.copy())
    gs.scale_data(5.0)
    out["scale_in_xyz"], out["scale_in_rot"] = xyz2, rot2
    out["scale_out_xyz"], out["scale_out_rot"], out["scale_out_scale"] = gs.xyz, gs.rot, gs.scale

    # _sort_gaussian_cpu for several view matrices (math orientation, float32)
    views = []
    V0 = lookat_translate(5.0)
    views.append(V0)
    for k, ang in enumerate([0.3, 1.1, -2.0]):
        c, s = np.cos(ang), np.sin(ang)
        R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]]) @ np.array(
            [[1, 0, 0], [0, np.cos(ang / 2), -np.sin(ang / 2)], [0, np.sin(ang / 2), np.cos(ang / 2)]])
        V = np.eye(4)
        V[:3, :3] = R
        V[:3, 3] = [0.1 * k, -0.2, -4.0 - k]
        views.append(V.astype(np.float32))
    out["sort_views"] = np.stack(views)
    out["sort_index"] = np.stack([renderer_ogl._sort_gaussian_cpu(gr, V)[:, 0] for V in views])

    # Euler -> rotation matrix (used for the OBB uniform, renderer_ogl.py:308-310)
    angles = np.array([[0, 0, 0], [30, 15, 0], [-45, 10, 170], [90, -90, 33.3]], np.float64)
    out["euler_angles"] = angles
    out["euler_R"] = np.stack([util.convert_euler_angles_to_rotation_matrix(a) for a in angles])

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
