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
  util.convert_rotation_matrix_to_euler_angles  util.py:494-501
  util_gau.GaussianData.compute_obb  util_gau.py:114-138
  util_gau.export_ply's mask and bbox  util_gau.py:388-413 (the downstream
      gsconverter call is replaced by a function that records its convertargs;
      the reference's computation is untouched)
  gsconverter BaseConverter.crop_by_bbox  tools/gsconverter/utils/base_converter.py:175-191
      (run on a structured array of the original positions plus a row index)
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

    # matrix -> Euler angles (scipy Rotation.as_euler('xyz', degrees=True)), util.py:494-501
    mats = list(out["euler_R"])
    rr = np.random.default_rng(77)
    for _ in range(12):
        q = rr.normal(size=4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        mats.append(np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                              [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                              [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]))
    out["r2e_R"] = np.stack(mats)
    out["r2e_euler"] = np.stack([util.convert_rotation_matrix_to_euler_angles(R) for R in mats])

    # compute_obb (pandas mean / cov, SVD), util_gau.py:114-138, on three point sets
    obb_sets = [xyz, xyz2, (rng.normal(0, 1, (5000, 3)) @ np.array([[3.0, 0.4, 0.1], [0.0, 1.0, -0.5],
                                                                       [0.2, 0.0, 0.3]])).astype(np.float32)]
    for k, pts in enumerate(obb_sets):
        go = util_gau.GaussianData(pts.copy(), rot[: len(pts)].copy() if len(pts) == n else
                                   np.tile([1, 0, 0, 0], (len(pts), 1)).astype(np.float32),
                                   np.ones((len(pts), 3), np.float32), np.ones((len(pts), 1), np.float32),
                                   np.zeros((len(pts), 3), np.float32))
        omin, omax, U, corners = go.compute_obb
        out[f"obb{k}_xyz"], out[f"obb{k}_min"], out[f"obb{k}_max"] = pts, omin, omax
        out[f"obb{k}_U"], out[f"obb{k}_corners"] = U, corners

    # export_ply (util_gau.py:388-431): the mask and bbox, with the box acting on
    # the current (rescaled) positions and the bbox taken over the original ones
    captured = {}

    def capture(convertargs):
        captured["args"] = dict(convertargs)
        return True

    util_gau.gsconverter = capture
    from tools.gsconverter.utils.base_converter import BaseConverter  # noqa: E402
    ne = 20_000
    er = np.random.default_rng(3)
    orig = er.normal(0, 2.0, (ne, 3)).astype(np.float32)
    cur = (orig * np.float32(0.5) + np.float32(0.05)).astype(np.float32)
    out["export_orig"], out["export_cur"] = orig, cur
    cases = [(0, 0, [-1, -1, -1], [1, 1, 1], [0, 0, 0]),
             (1, 0, [-0.8, -0.5, -0.6], [0.7, 0.9, 0.4], [0, 0, 0]),
             (0, 1, [-0.9, -0.4, -0.7], [0.6, 0.8, 0.5], [30.0, 15.0, 0.0]),
             (1, 1, [-0.9, -0.4, -0.7], [0.6, 0.8, 0.5], [10.0, -20.0, 45.0]),
             (1, 0, [50, 50, 50], [60, 60, 60], [0, 0, 0]),
             (0, 1, [-0.3, -2.0, -0.2], [0.25, 2.0, 0.3], [0.0, 0.0, 90.0])]
    rec = np.zeros(ne, dtype=[("x", "f4"), ("y", "f4"), ("z", "f4"), ("row", "i8")])
    rec["x"], rec["y"], rec["z"], rec["row"] = orig[:, 0], orig[:, 1], orig[:, 2], np.arange(ne)
    ex_params, ex_bbox, ex_rows = [], [], []
    for aabb, obb, cmin, cmax, erot in cases:
        ge = util_gau.GaussianData(orig.copy(), np.tile([1, 0, 0, 0], (ne, 1)).astype(np.float32),
                                   np.ones((ne, 3), np.float32), np.ones((ne, 1), np.float32),
                                   np.zeros((ne, 3), np.float32))
        ge.xyz = cur.copy()  # the viewer's current positions (scale_data); the original state stays
        captured.clear()
        assert util_gau.export_ply(ge, "unused", aabb, obb, cmin, cmax, erot)
        bbox = captured["args"]["bbox"]
        if bbox is None:
            ex_bbox.append(np.full(6, np.nan))
            ex_rows.append(np.arange(ne))  # gsconverter skips the crop without a bbox
        else:
            ex_bbox.append(np.array(bbox, np.float64))
            ex_rows.append(BaseConverter(rec.copy()).crop_by_bbox(*bbox)["row"])
        ex_params.append(np.array([aabb, obb, *cmin, *cmax, *erot], np.float64))
    out["export_params"] = np.stack(ex_params)
    out["export_bbox"] = np.stack(ex_bbox)
    out["export_nrows"] = np.array([len(r) for r in ex_rows])
    out["export_rows"] = np.concatenate(ex_rows)

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
